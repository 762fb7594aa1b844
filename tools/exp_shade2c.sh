#!/bin/bash
# Unit-mode shade, two paths per thread held to 64 VGPRs (default) vs one path (build_base).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
P=smallpt-enoki-optix_amd
timeout -k 10 300 python -u -m pytest tests/test_gpu_render.py tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/tests_s2c.log 2>&1; rc=$?
tail -2 gpurun_out/tests_s2c.log
[ $rc -ne 0 ] && exit $rc
V="new= base=$P/build_base/libspt.so"
VARIANTS="$V" ROUNDS=3 timeout -k 10 400 bash tools/ab.sh || exit $?
echo "== config 3" >> gpurun_out/ab.log
VARIANTS="$V" ROUNDS=1 BENCH_ARGS="--config 3 --steps 1" timeout -k 10 300 bash tools/ab.sh || exit $?
