#!/bin/bash
# Public spt_intersect kernels per node format (templated) + config-4 occupancy sensitivity.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/tests_api.log 2>&1; rc=$?
tail -2 gpurun_out/tests_api.log
[ $rc -ne 0 ] && exit $rc
for v in "" "SPT_PUBLIC_PERSISTENT=1" "SPT_BVH=8" "SPT_BVH=8 SPT_PUBLIC_PERSISTENT=1"; do
  echo "== $v" >> gpurun_out/api.log
  env $v timeout -k 10 200 python tools/isect_api_bench.py >> gpurun_out/api.log 2>&1 || exit $?
done
cat gpurun_out/api.log
VARIANTS="s0= s4=" ENVS="s0:SPT_STACK_SLACK=0 s4:SPT_STACK_SLACK=4" ROUNDS=2 BENCH_ARGS="--config 4 --steps 2" timeout -k 10 500 bash tools/ab.sh || exit $?
