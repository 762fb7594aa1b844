#!/bin/bash
# BVH8 collapse variants (SPT_BVH8_MODE / SPT_BVH8_CPRIM): traversal stats + bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for v in ${COLLAPSE_VARIANTS:-"1:0.3" "3:0.3" "3:0.15" "3:0.6"}; do
  mode=${v%%:*}; cp=${v#*:}
  echo "== mode $mode cprim $cp" >> gpurun_out/exp_collapse.log
  env SPT_BVH8_MODE=$mode SPT_BVH8_CPRIM=$cp timeout -k 10 300 python tools/trav_stats.py --depths 8 2>&1 | grep -v amdgpu.ids >> gpurun_out/exp_collapse.log || exit 1
  env SPT_BVH8_MODE=$mode SPT_BVH8_CPRIM=$cp timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline 2>/dev/null \
    | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['roofline']['grays_per_s'], d['bvh'])" >> gpurun_out/exp_collapse.log || exit 1
done
cat gpurun_out/exp_collapse.log
