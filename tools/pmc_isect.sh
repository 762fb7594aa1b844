#!/bin/bash
# PMC passes on the isect kernel of one bench config, one rocprofv3 run per
# pass (kernel-trace only, each under its own time limit), then
# tools/pmc_isect.py merges the per-cast figures into OUTDIR/isect_pmc.json
# under "config<N>".
#   usage: CONFIG=1 [PIPE=fused] [KERNEL=drain] tools/pmc_isect.sh OUTDIR      (CONFIG default 1)
# PIPE=fused: the fused trace+shade kernel (--pipeline fused), key "config<N>_fused".
set -u
out=${1:-gpurun_out/pmc}
cfg=${CONFIG:-1}
pipe=${PIPE:-auto}
regex='isect_(queue|lockstep)|camera_cast'
key=config$cfg
if [ "$pipe" = fused ]; then regex=render_fused; key=config${cfg}_fused; fi
# KERNEL=drain: the wavefront's drain (render_fused_kernel<drain>), key "config<N>_drain"
if [ "${KERNEL:-isect}" = drain ]; then regex=render_fused; key=config${cfg}_drain; fi
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p "$out"
export TMPDIR=/tmp
i=0
csvs=""
for ctrs in "FETCH_SIZE" "WRITE_SIZE" \
            "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES" \
            "TCC_HIT_sum TCC_MISS_sum" \
            "TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $ctrs --kernel-include-regex "$regex" -d "$out/${key}_p$i" -o run \
      --output-format csv -- python bench.py --config "$cfg" --pipeline "$pipe" --steps 1 --warmup 1 \
      --no-cpu-baseline > "$out/${key}_p$i.log" 2>&1
  rc=$?
  echo "== $key pass $i ($ctrs) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$out/${key}_p$i.log"; exit $rc; fi
  csvs="$csvs $out/${key}_p$i/run_counter_collection.csv"
done
python tools/pmc_isect.py "$out/isect_pmc.json" "$key" "$out/${key}_p1.log" $csvs --kernel "$regex"
