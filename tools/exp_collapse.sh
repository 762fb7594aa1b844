#!/bin/bash
# BVH8 collapse variants (spt_config.collapse via SPT_COLLAPSE=sah|greedy): traversal stats + bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for mode in ${COLLAPSE_VARIANTS:-greedy sah}; do
  echo "== collapse $mode" >> gpurun_out/exp_collapse.log
  env SPT_COLLAPSE=$mode timeout -k 10 300 python tools/trav_stats.py --depths 8 2>&1 | grep -v amdgpu.ids >> gpurun_out/exp_collapse.log || exit 1
  env SPT_COLLAPSE=$mode timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline 2>/dev/null \
    | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['roofline']['chip_busy'], d['bvh'])" >> gpurun_out/exp_collapse.log || exit 1
done
cat gpurun_out/exp_collapse.log
