#!/bin/bash
# Unit-mode shade: two paths per thread with 128 / 256 (default) / 512-thread blocks vs one path (build_base).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
P=smallpt-enoki-optix_amd
timeout -k 10 300 python -u -m pytest tests/test_gpu_render.py tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/tests_s2b.log 2>&1; rc=$?
tail -2 gpurun_out/tests_s2b.log
[ $rc -ne 0 ] && exit $rc
V="s256= base=$P/build_base/libspt.so s128=$P/build_s2_128/libspt.so s512=$P/build_s2_512/libspt.so"
VARIANTS="$V" ROUNDS=3 timeout -k 10 600 bash tools/ab.sh || exit $?
