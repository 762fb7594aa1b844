#!/bin/bash
# Fused kernel: shade pending lanes at once after the pool drains (default) vs build_base.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
P=smallpt-enoki-optix_amd
timeout -k 10 300 python -u -m pytest tests/test_gpu_render.py tests/test_gpu_parity.py tests/test_gpu_spheres.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/tests_tail.log 2>&1; rc=$?
tail -2 gpurun_out/tests_tail.log
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do
for lib in "" "$PWD/$P/build_base/libspt.so"; do
  echo "== lib=${lib:-new}" >> gpurun_out/tail.log
  env SPT_LIB=$lib timeout -k 10 120 python tools/tile_sim.py --tiles 1 4 8 --pipeline fused >> gpurun_out/tail.log 2>&1 || exit $?
done
done
