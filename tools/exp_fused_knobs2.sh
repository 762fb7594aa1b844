#!/bin/bash
# Fused-kernel work grabs on the N = 1, 4, 8 tiles: chunk 64 with static shares 0 / 16 / 32.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for r in 1 2; do
for v in "SPT_CHUNK=128" "SPT_CHUNK=64" "SPT_CHUNK=64 SPT_FUSED_STATIC_SHARE_Q8=16" "SPT_CHUNK=64 SPT_FUSED_STATIC_SHARE_Q8=0" "SPT_CHUNK=96 SPT_FUSED_STATIC_SHARE_Q8=16"; do
  echo "== $v" >> gpurun_out/fknobs2.log
  env $v timeout -k 10 120 python tools/tile_sim.py --tiles 1 4 8 --pipeline fused >> gpurun_out/fknobs2.log 2>&1 || exit $?
done
done
