#!/bin/bash
# Fused-kernel knobs on one rank's tile (tools/tile_sim.py, queued renders as
# bench.py runs them), alternating variants (environment; commas join settings).
#   usage: TILES="8 4" ROUNDS=2 VARIANTS="X=0 SPT_FUSED_IDLE=16" tools/tile_sweep.sh
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
for r in $(seq ${ROUNDS:-2}); do for v in ${VARIANTS:-X=0}; do
  out=$(env ${v//,/ } timeout -k 10 300 python tools/tile_sim.py --tiles ${TILES:-8 4} --timing 2>/dev/null) || { echo FAIL; exit 1; }
  echo "$out" | python -c "
import json,sys
for l in sys.stdin:
    l=l.strip()
    if l.startswith('{'):
        d=json.loads(l); print('$v', 'tiles', d['tiles'], d['tile_mpaths_s'], d['projected_job_mpaths_s'], 'fused', d['fused'])" | tee -a gpurun_out/tile_sweep.log
done; done
