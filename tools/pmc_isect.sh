#!/bin/bash
# PMC passes on the isect kernel of the config-1 bench, one rocprofv3 run per
# pass (kernel-trace only, each under its own time limit), then
# tools/pmc_isect.py -> OUTDIR/isect_pmc.json.   usage: tools/pmc_isect.sh OUTDIR
set -u
out=${1:-gpurun_out/pmc}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p "$out"
export TMPDIR=/tmp
i=0
csvs=""
for ctrs in "FETCH_SIZE" "WRITE_SIZE" \
            "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES" \
            "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-include-regex isect_queue -d "$out/p$i" -o run --output-format csv \
      -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline > "$out/p$i.log" 2>&1
  rc=$?
  echo "== pass $i ($ctrs) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$out/p$i.log"; exit $rc; fi
  csvs="$csvs $out/p$i/run_counter_collection.csv"
done
python tools/pmc_isect.py "$out/isect_pmc.json" $csvs
