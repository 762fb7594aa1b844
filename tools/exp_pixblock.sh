#!/bin/bash
# A/B of the camera-path pixel order (spt_config.pixel_block): scanline (1)
# against B x B blocks, config 1 wavefront, config 1 fused, configs 2 and 4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
V="b1= b4= b8= b16="
E="b1:SPT_PIXEL_BLOCK=1 b4:SPT_PIXEL_BLOCK=4 b8:SPT_PIXEL_BLOCK=8 b16:SPT_PIXEL_BLOCK=16"
echo "== config 1 wavefront" >> gpurun_out/ab.log
VARIANTS="$V" ENVS="$E" ROUNDS=3 bash tools/ab.sh > /dev/null || exit $?
echo "== config 1 fused" >> gpurun_out/ab.log
VARIANTS="$V" ENVS="$E" ROUNDS=2 BENCH_ARGS="--pipeline fused" bash tools/ab.sh > /dev/null || exit $?
echo "== config 4" >> gpurun_out/ab.log
VARIANTS="b1= b8=" ENVS="$E" ROUNDS=2 BENCH_ARGS="--config 4" bash tools/ab.sh > /dev/null || exit $?
echo "== config 2" >> gpurun_out/ab.log
VARIANTS="b1= b8=" ENVS="$E" ROUNDS=2 BENCH_ARGS="--config 2" bash tools/ab.sh > /dev/null || exit $?
cat gpurun_out/ab.log
