#!/bin/bash
# PMC passes on the wavefront isect kernel (config 1) at sample-major 32M and
# the AUTO pixel-major 24M in flight.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
SPT_WORK_ORDER=1 bash tools/pmc_sweep.sh gpurun_out/pmc_wave_smaj "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES" || exit $?
SPT_WORK_ORDER=0 bash tools/pmc_sweep.sh gpurun_out/pmc_wave_auto "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES" || exit $?
