#!/bin/bash
# 64-B nodes at 8 waves/SIMD (default build) vs 7 waves (build_w67) vs the 80-B BVH8.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
P=smallpt-enoki-optix_amd
VARIANTS="w8= w6x8= w6x7=$P/build_w67/libspt.so" ENVS="w8:SPT_BVH=8 w6x8:SPT_BVH=6 w6x7:SPT_BVH=6" ROUNDS=3 \
  timeout -k 10 400 bash tools/ab.sh || exit $?
echo "== config 4" >> gpurun_out/ab.log
VARIANTS="w8= w6x8= w6x7=$P/build_w67/libspt.so" ENVS="w8:SPT_BVH=8 w6x8:SPT_BVH=6 w6x7:SPT_BVH=6" ROUNDS=2 \
  BENCH_ARGS="--config 4 --steps 2" timeout -k 10 500 bash tools/ab.sh || exit $?
