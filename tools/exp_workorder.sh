#!/bin/bash
# A/B of the work-item order (spt_config.work_order): sample-major (0) against
# pixel-major (1), config 1 wavefront and fused, configs 3 and 4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
E="smaj:SPT_WORK_ORDER=1 pmaj:SPT_WORK_ORDER=2"
echo "== config 1 wavefront" >> gpurun_out/ab.log
VARIANTS="smaj= pmaj=" ENVS="$E" ROUNDS=3 bash tools/ab.sh > /dev/null || exit $?
echo "== config 1 fused" >> gpurun_out/ab.log
VARIANTS="smaj= pmaj=" ENVS="$E" ROUNDS=2 BENCH_ARGS="--pipeline fused" bash tools/ab.sh > /dev/null || exit $?
echo "== config 4" >> gpurun_out/ab.log
VARIANTS="smaj= pmaj=" ENVS="$E" ROUNDS=2 BENCH_ARGS="--config 4" bash tools/ab.sh > /dev/null || exit $?
echo "== config 3" >> gpurun_out/ab.log
VARIANTS="smaj= pmaj=" ENVS="$E" ROUNDS=2 BENCH_ARGS="--config 3 --steps 1" bash tools/ab.sh > /dev/null || exit $?
cat gpurun_out/ab.log
