#!/bin/bash
# 56-B emit-mode path vs 64 B (build_base): parity tests with emitters, then config 2 A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
P=smallpt-enoki-optix_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/tests_e56.log 2>&1; rc=$?
tail -2 gpurun_out/tests_e56.log
[ $rc -ne 0 ] && exit $rc
VARIANTS="e56= e64=$P/build_base/libspt.so" ROUNDS=3 BENCH_ARGS="--config 2 --steps 1" timeout -k 10 700 bash tools/ab.sh || exit $?
