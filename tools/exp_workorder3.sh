#!/bin/bash
# After the stream-share fix: sample- vs pixel-major on configs 1 (wavefront),
# 3 and 4, and the fused kernel on the N = 1..8 tiles of config 1.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
E="smaj:SPT_WORK_ORDER=1 pmaj:SPT_WORK_ORDER=2"
echo "== config 3" >> gpurun_out/ab.log
VARIANTS="smaj= pmaj=" ENVS="$E" ROUNDS=2 BENCH_ARGS="--config 3 --steps 1" bash tools/ab.sh > /dev/null || exit $?
echo "== config 4" >> gpurun_out/ab.log
VARIANTS="smaj= pmaj=" ENVS="$E" ROUNDS=2 BENCH_ARGS="--config 4" bash tools/ab.sh > /dev/null || exit $?
echo "== config 1 wavefront" >> gpurun_out/ab.log
VARIANTS="smaj= pmaj=" ENVS="$E" ROUNDS=2 bash tools/ab.sh > /dev/null || exit $?
for v in 1 2; do
  echo "== fused tiles SPT_WORK_ORDER=$v" >> gpurun_out/tiles.log
  SPT_WORK_ORDER=$v timeout -k 10 200 python tools/tile_sim.py --tiles 1 2 4 8 --pipeline fused >> gpurun_out/tiles.log 2>&1 || exit $?
done
cat gpurun_out/ab.log gpurun_out/tiles.log
