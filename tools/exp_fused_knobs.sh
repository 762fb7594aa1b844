#!/bin/bash
# Fused-kernel knobs on one rank's tile at N = 8 and N = 4 (tools/tile_sim.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for v in "SPT_FUSED_IDLE=32" "SPT_FUSED_IDLE=16" "SPT_FUSED_IDLE=24" "SPT_FUSED_IDLE=40" "SPT_FUSED_IDLE=48" \
         "SPT_FUSED_STATIC_SHARE_Q8=16" "SPT_FUSED_STATIC_SHARE_Q8=48" "SPT_CHUNK=64" "SPT_CHUNK=32"; do
  echo "== $v" >> gpurun_out/fknobs.log
  env $v timeout -k 10 120 python tools/tile_sim.py --tiles 4 8 --pipeline fused >> gpurun_out/fknobs.log 2>&1 || exit $?
done
cat gpurun_out/fknobs.log
