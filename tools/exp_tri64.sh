#!/bin/bash
# 64-B triangle records (build_t4) vs 48 B: parity, configs 1 and 4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
P=smallpt-enoki-optix_amd
SPT_LIB=$PWD/$P/build_t4/libspt.so timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/tests_t4.log 2>&1; rc=$?
tail -2 gpurun_out/tests_t4.log
[ $rc -ne 0 ] && exit $rc
V="t3= t4=$P/build_t4/libspt.so"
VARIANTS="$V" ROUNDS=2 BENCH_ARGS="--config 4 --steps 2" timeout -k 10 600 bash tools/ab.sh || exit $?
echo "== config 1" >> gpurun_out/ab.log
VARIANTS="$V" ROUNDS=3 timeout -k 10 400 bash tools/ab.sh || exit $?
