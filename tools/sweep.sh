#!/bin/bash
# Knob sweep on the bench workload: each line "ENV=.. ENV=.." runs bench once.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
while read -r line; do
  [ -z "$line" ] && continue
  out=$(env $line timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-cpu-baseline 2>/dev/null)
  rc=$?
  v=$(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["kernel_ms_per_step"], d["roofline"]["busy_ms_per_step"])' 2>/dev/null)
  echo "$line -> rc=$rc $v" | tee -a gpurun_out/sweep.log
  if [ $rc -ge 124 ]; then exit $rc; fi
done
