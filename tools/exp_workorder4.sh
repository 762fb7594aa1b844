#!/bin/bash
# Fused kernel tiles at both work orders and AUTO (current build), config 1.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for v in 1 2 1 2; do
  echo "== fused tiles SPT_WORK_ORDER=$v" >> gpurun_out/tiles.log
  SPT_WORK_ORDER=$v timeout -k 10 200 python tools/tile_sim.py --tiles 1 2 4 8 --pipeline fused >> gpurun_out/tiles.log 2>&1 || exit $?
done
cat gpurun_out/tiles.log
