#!/bin/bash
# Round-2 refresh on the committed build: fused-knob check, tile projection,
# PMC passes (isect configs 1/2/4, shade), kernel stats, all bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for v in "SPT_FUSED_IDLE=32" "SPT_FUSED_IDLE=24" "SPT_FUSED_IDLE=40"; do
  echo "== $v" >> gpurun_out/fidle.log
  env $v timeout -k 10 120 python tools/tile_sim.py --tiles 1 8 --pipeline fused >> gpurun_out/fidle.log 2>&1 || exit $?
done
echo "== wavefront" >> gpurun_out/tiles.log
timeout -k 10 200 python tools/tile_sim.py --tiles 1 2 4 8 --pipeline wavefront >> gpurun_out/tiles.log 2>&1 || exit $?
echo "== fused" >> gpurun_out/tiles.log
timeout -k 10 200 python tools/tile_sim.py --tiles 1 2 4 8 --pipeline fused >> gpurun_out/tiles.log 2>&1 || exit $?
bash tools/gpu_run.sh pmc1 pmc2 pmc4 pmcshade prof prof1s prof2s smoke bench bench0 bench2 bench3 bench4
