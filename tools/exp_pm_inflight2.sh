#!/bin/bash
# Confirm: pixel-major at 20M-28M paths in flight (config 1), sample-major at
# 24M, and configs 3 / 4 at pixel-major 24M.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
E="pm24:SPT_WORK_ORDER=2,SPT_WAVEFRONT_PATHS=25165824 pm20:SPT_WORK_ORDER=2,SPT_WAVEFRONT_PATHS=20971520 pm28:SPT_WORK_ORDER=2,SPT_WAVEFRONT_PATHS=29360128 sm24:SPT_WORK_ORDER=1,SPT_WAVEFRONT_PATHS=25165824"
echo "== config 1" >> gpurun_out/ab.log
VARIANTS="base= pm24= pm20= pm28= sm24=" ENVS="$E" ROUNDS=2 bash tools/ab.sh > /dev/null || exit $?
echo "== config 3" >> gpurun_out/ab.log
VARIANTS="base= pm24=" ENVS="$E" ROUNDS=2 BENCH_ARGS="--config 3 --steps 1" bash tools/ab.sh > /dev/null || exit $?
echo "== config 4" >> gpurun_out/ab.log
VARIANTS="base= pm24=" ENVS="$E" ROUNDS=2 BENCH_ARGS="--config 4" bash tools/ab.sh > /dev/null || exit $?
cat gpurun_out/ab.log
