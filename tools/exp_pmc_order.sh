#!/bin/bash
# PMC passes on the fused kernel (config 1 whole image, --pipeline fused) at
# both work orders: why pixel-major is faster (L2 hits, bytes fetched).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for v in 1 2; do
  SPT_WORK_ORDER=$v KERNEL=render_fused BENCH_ARGS="--pipeline fused" bash tools/pmc_sweep.sh gpurun_out/pmc_fused_order$v \
    "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES" || exit $?
done
