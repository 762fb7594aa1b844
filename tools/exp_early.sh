#!/bin/bash
# Early finish (default build) vs a separate final step (build_base, SPT_EARLY_DONE=0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
P=smallpt-enoki-optix_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/tests_early.log 2>&1; rc=$?
tail -2 gpurun_out/tests_early.log
[ $rc -ne 0 ] && exit $rc
V="new= base=$P/build_base/libspt.so"
VARIANTS="$V" ROUNDS=3 timeout -k 10 400 bash tools/ab.sh || exit $?
echo "== fused" >> gpurun_out/ab.log
VARIANTS="$V" ROUNDS=2 BENCH_ARGS="--pipeline fused" timeout -k 10 300 bash tools/ab.sh || exit $?
echo "== config 2" >> gpurun_out/ab.log
VARIANTS="$V" ROUNDS=1 BENCH_ARGS="--config 2 --steps 1" timeout -k 10 300 bash tools/ab.sh || exit $?
echo "== config 4" >> gpurun_out/ab.log
VARIANTS="$V" ROUNDS=1 BENCH_ARGS="--config 4 --steps 2" timeout -k 10 400 bash tools/ab.sh || exit $?
