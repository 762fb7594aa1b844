#!/bin/bash
# Fused kernel (unit mode, 64-B nodes) at 6 waves/SIMD (default) vs 5 (build_fw5):
# whole config 1 and the tiles of N = 1, 2, 4, 8 (tools/tile_sim.py), both pipelines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
P=smallpt-enoki-optix_amd
VARIANTS="fw6= fw5=$P/build_fw5/libspt.so" ROUNDS=2 BENCH_ARGS="--pipeline fused" timeout -k 10 300 bash tools/ab.sh || exit $?
for lib in "" "$PWD/$P/build_fw5/libspt.so"; do
  echo "== tile_sim lib=${lib:-default} fused" >> gpurun_out/tiles.log
  env SPT_LIB=$lib timeout -k 10 200 python tools/tile_sim.py --tiles 1 2 4 8 --pipeline fused >> gpurun_out/tiles.log 2>&1 || exit $?
done
echo "== tile_sim default wavefront" >> gpurun_out/tiles.log
timeout -k 10 200 python tools/tile_sim.py --tiles 1 2 4 8 --pipeline wavefront >> gpurun_out/tiles.log 2>&1 || exit $?
cat gpurun_out/tiles.log
