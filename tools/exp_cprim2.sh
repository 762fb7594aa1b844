#!/bin/bash
# SAH collapse cost c_prim: 0.6 / 1.0 / 1.5 / 2.5 on config 1 (plus traversal statistics).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
P=smallpt-enoki-optix_amd
V="cp03= cp06=$P/build_cp06/libspt.so cp10=$P/build_cp10/libspt.so cp15=$P/build_cp15/libspt.so cp25=$P/build_cp25/libspt.so"
VARIANTS="$V" ROUNDS=3 timeout -k 10 700 bash tools/ab.sh || exit $?
for v in "$PWD/$P/build_cp15/libspt.so" "$PWD/$P/build_cp25/libspt.so"; do
  echo "== trav ${v:-default}" >> gpurun_out/ab.log
  SPT_LIB=$v timeout -k 10 120 python tools/trav_stats.py --depths 8 >> gpurun_out/ab.log 2>&1 || exit $?
done
echo "== config 2" >> gpurun_out/ab.log
VARIANTS="cp03= cp10=$P/build_cp10/libspt.so" ROUNDS=1 BENCH_ARGS="--config 2 --steps 1" timeout -k 10 600 bash tools/ab.sh || exit $?
