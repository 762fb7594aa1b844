#!/bin/bash
# Wavefront with pixel-major work split by samples across the streams.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
E="smaj:SPT_WORK_ORDER=1 pmaj:SPT_WORK_ORDER=2 auto:SPT_WORK_ORDER=0"
echo "== config 1 wavefront" >> gpurun_out/ab.log
VARIANTS="smaj= pmaj=" ENVS="$E" ROUNDS=3 bash tools/ab.sh > /dev/null || exit $?
echo "== config 3" >> gpurun_out/ab.log
VARIANTS="smaj= pmaj=" ENVS="$E" ROUNDS=2 BENCH_ARGS="--config 3 --steps 1" bash tools/ab.sh > /dev/null || exit $?
echo "== config 2" >> gpurun_out/ab.log
VARIANTS="smaj= pmaj=" ENVS="$E" ROUNDS=2 BENCH_ARGS="--config 2" bash tools/ab.sh > /dev/null || exit $?
echo "== config 1 fused" >> gpurun_out/ab.log
VARIANTS="smaj= auto=" ENVS="$E" ROUNDS=2 BENCH_ARGS="--pipeline fused" bash tools/ab.sh > /dev/null || exit $?
cat gpurun_out/ab.log
