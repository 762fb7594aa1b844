#!/bin/bash
# Unit-mode shade, two paths per thread (default) vs one (build_base): suite, A/B, kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
P=smallpt-enoki-optix_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/tests_s2.log 2>&1; rc=$?
tail -2 gpurun_out/tests_s2.log
[ $rc -ne 0 ] && exit $rc
V="new= base=$P/build_base/libspt.so"
VARIANTS="$V" ROUNDS=3 timeout -k 10 400 bash tools/ab.sh || exit $?
echo "== config 3" >> gpurun_out/ab.log
VARIANTS="$V" ROUNDS=1 BENCH_ARGS="--config 3 --steps 1" timeout -k 10 300 bash tools/ab.sh || exit $?
export TMPDIR=/tmp
timeout -k 10 300 env SPT_STREAMS=1 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s2 -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_s2.log 2>&1 || exit $?
