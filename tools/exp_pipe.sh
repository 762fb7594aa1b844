#!/bin/bash
# wavefront vs fused pipeline per config (the current default build).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for c in 1 2 4; do
  for p in wavefront fused; do
    timeout -k 10 300 python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --pipeline $p > /tmp/p.json 2>/dev/null || exit $?
    python -c "import json;d=json.load(open('/tmp/p.json'));print('config $c $p', d['value'], d['ms_per_step'])" | tee -a gpurun_out/pipe.log
  done
done
