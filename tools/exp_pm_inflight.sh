#!/bin/bash
# Wavefront config 1: pixel-major work at 16M-48M paths in flight against the default.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
E="pm32:SPT_WORK_ORDER=2 pm16:SPT_WORK_ORDER=2,SPT_WAVEFRONT_PATHS=16777216 pm24:SPT_WORK_ORDER=2,SPT_WAVEFRONT_PATHS=25165824 pm48:SPT_WORK_ORDER=2,SPT_WAVEFRONT_PATHS=50331648 pm2s:SPT_WORK_ORDER=2,SPT_STREAMS=2"
VARIANTS="base= pm32= pm16= pm24= pm48= pm2s=" ENVS="$E" ROUNDS=2 bash tools/ab.sh
