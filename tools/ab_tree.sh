#!/bin/bash
# A/B of trees on one box: each directory in $DIRS (worktrees with their own
# build; "." = this tree), alternating bench runs per config.
# usage: DIRS=". _r2" CONFIGS="3 4" ROUNDS=2 tools/ab_tree.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in ${CONFIGS:-3 4}; do
  for r in $(seq ${ROUNDS:-2}); do
    for d in ${DIRS:-. _r2}; do
      out=$( cd $d && timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} 2>/dev/null ) || { echo "FAIL $d config $c rc=$?"; exit 1; }
      echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('config $c $d', d['value'], d['ms_per_step'], d['config'].get('pipeline'), d['config'].get('work_order'), d['roofline'].get('grays_per_s'))" | tee -a gpurun_out/ab_tree.log
    done
  done
done
