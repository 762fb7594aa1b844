#!/bin/bash
# SQ stall breakdown of isect_queue_kernel on the config-1 bench (one PMC pass each).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
i=0
for ctrs in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAVES SQ_BUSY_CYCLES" \
            "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $ctrs --kernel-include-regex isect_queue -d gpurun_out/pmcsq$i -o run --output-format csv \
      -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/pmcsq$i.log 2>&1 || exit 1
done
python tools/pmc_summary.py gpurun_out/pmcsq1/run_counter_collection.csv gpurun_out/pmcsq2/run_counter_collection.csv
