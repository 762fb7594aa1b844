#!/bin/bash
# The working tree's build vs build_base (the previous commit): GPU suite, then
# alternating bench runs on configs 1 and 4 and the fused pipeline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
P=smallpt-enoki-optix_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/tests_ab.log 2>&1; rc=$?
tail -3 gpurun_out/tests_ab.log
[ $rc -ne 0 ] && exit $rc
VARIANTS="new= base=$P/build_base/libspt.so" ROUNDS=3 timeout -k 10 400 bash tools/ab.sh || exit $?
echo "== config 4" >> gpurun_out/ab.log
VARIANTS="new= base=$P/build_base/libspt.so" ROUNDS=2 BENCH_ARGS="--config 4 --steps 2" timeout -k 10 500 bash tools/ab.sh || exit $?
echo "== config 1 fused" >> gpurun_out/ab.log
VARIANTS="new= base=$P/build_base/libspt.so" ROUNDS=2 BENCH_ARGS="--pipeline fused" timeout -k 10 400 bash tools/ab.sh || exit $?
