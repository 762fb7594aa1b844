#!/bin/bash
# Confirm the per-pipeline pixel_block default (0) against scanline (1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
E="auto:SPT_PIXEL_BLOCK=0 b1:SPT_PIXEL_BLOCK=1 b2:SPT_PIXEL_BLOCK=2 b4:SPT_PIXEL_BLOCK=4"
echo "== config 1 wavefront" >> gpurun_out/ab.log
VARIANTS="auto= b1= b2= b4=" ENVS="$E" ROUNDS=3 bash tools/ab.sh > /dev/null || exit $?
echo "== config 3 (wavefront)" >> gpurun_out/ab.log
VARIANTS="auto= b1=" ENVS="$E" ROUNDS=2 BENCH_ARGS="--config 3 --steps 1" bash tools/ab.sh > /dev/null || exit $?
cat gpurun_out/ab.log
