#!/bin/bash
# r02 experiment batch A: shade block size (256/512/1024) at 4 and 1 streams,
# fused kernel at 6 waves/SIMD on the N=8 tile.  Each step under a timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
P=smallpt-enoki-optix_amd
VARIANTS="base= sb256=$P/build_sb256/libspt.so sb1024=$P/build_sb1024/libspt.so" ROUNDS=2 \
  timeout -k 10 400 bash tools/ab.sh || exit $?
echo "== 1 stream" >> gpurun_out/ab.log
VARIANTS="base= sb256=$P/build_sb256/libspt.so sb1024=$P/build_sb1024/libspt.so" ROUNDS=1 \
  ENVS="base:SPT_STREAMS=1 sb256:SPT_STREAMS=1 sb1024:SPT_STREAMS=1" timeout -k 10 300 bash tools/ab.sh || exit $?
for lib in "" "$PWD/$P/build_fw6/libspt.so"; do
  echo "== tile_sim lib=${lib:-base}" >> gpurun_out/exp_a.log
  env SPT_LIB=$lib timeout -k 10 200 python tools/tile_sim.py --tiles 4 8 --timing >> gpurun_out/exp_a.log 2>&1 || exit $?
done
cat gpurun_out/ab.log gpurun_out/exp_a.log
