#!/bin/bash
# A/B: current tree vs the worktree in _old (same box, alternating runs)
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for r in 1 2 3; do
  for t in . _old; do
    (cd $t && timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > /tmp/ab.json 2>/dev/null) || exit 1
    python -c "import json;d=json.load(open('/tmp/ab.json'));print('$t', d['value'], d['kernel_ms_per_step'])" >> gpurun_out/ab.log
  done
done
cat gpurun_out/ab.log
