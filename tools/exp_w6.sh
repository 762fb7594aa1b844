#!/bin/bash
# 64-B six-wide nodes (SPT_BVH=6) vs the 80-B BVH8: GPU suite under SPT_BVH=6,
# then alternating bench runs on configs 1 and 4.  Each step under a timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 600 env SPT_BVH=6 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > gpurun_out/tests_w6.log 2>&1; rc=$?
tail -5 gpurun_out/tests_w6.log
[ $rc -ge 124 ] && exit $rc
VARIANTS="w8= w6=" ENVS="w8:SPT_BVH=8 w6:SPT_BVH=6" ROUNDS=3 timeout -k 10 400 bash tools/ab.sh || exit $?
echo "== config 4" >> gpurun_out/ab.log
VARIANTS="w8= w6=" ENVS="w8:SPT_BVH=8 w6:SPT_BVH=6" ROUNDS=2 BENCH_ARGS="--config 4 --steps 2" timeout -k 10 500 bash tools/ab.sh || exit $?
