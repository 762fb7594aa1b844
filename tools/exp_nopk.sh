#!/bin/bash
# Device code without packed-fp32 instructions (build_nopk) vs the default build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
P=smallpt-enoki-optix_amd
VARIANTS="base= nopk=$P/build_nopk/libspt.so" ROUNDS=3 timeout -k 10 400 bash tools/ab.sh || exit $?
echo "== config 4" >> gpurun_out/ab.log
VARIANTS="base= nopk=$P/build_nopk/libspt.so" ROUNDS=2 BENCH_ARGS="--config 4 --steps 2" timeout -k 10 500 bash tools/ab.sh || exit $?
echo "== config 1 fused" >> gpurun_out/ab.log
VARIANTS="base= nopk=$P/build_nopk/libspt.so" ROUNDS=2 BENCH_ARGS="--pipeline fused" timeout -k 10 400 bash tools/ab.sh || exit $?
