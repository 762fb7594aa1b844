#!/bin/bash
# GPU builder sweep: PLOC radius vs SAH cost, build time and render speed.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for c in ${CONFIGS:-4 1}; do
  for r in ${RADII:-8 16 32 64}; do
    env SPT_BUILD=gpu SPT_PLOC_RADIUS=$r timeout -k 10 300 python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline 2>/dev/null \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('config $c radius $r', d['value'], d['bvh'])" >> gpurun_out/exp_build.log || exit 1
  done
  env SPT_BUILD=host timeout -k 10 300 python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline 2>/dev/null \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('config $c host', d['value'], d['bvh'])" >> gpurun_out/exp_build.log || exit 1
done
cat gpurun_out/exp_build.log
