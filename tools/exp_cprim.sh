#!/bin/bash
# SAH collapse cost c_prim (triangle test vs node visit): 0.3 (default) vs 0.15 / 0.6 / 1.0, configs 1 and 4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
P=smallpt-enoki-optix_amd
V="cp03= cp015=$P/build_cp015/libspt.so cp06=$P/build_cp06/libspt.so cp10=$P/build_cp10/libspt.so"
VARIANTS="$V" ROUNDS=2 timeout -k 10 500 bash tools/ab.sh || exit $?
echo "== config 4" >> gpurun_out/ab.log
VARIANTS="$V" ROUNDS=1 BENCH_ARGS="--config 4 --steps 2" timeout -k 10 600 bash tools/ab.sh || exit $?
for v in "" "$PWD/$P/build_cp06/libspt.so" "$PWD/$P/build_cp10/libspt.so"; do
  echo "== trav ${v:-default}" >> gpurun_out/ab.log
  SPT_LIB=$v timeout -k 10 120 python tools/trav_stats.py --depths 8 >> gpurun_out/ab.log 2>&1 || exit $?
done
