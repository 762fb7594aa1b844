#!/bin/bash
# One rocprofv3 --pmc run per counter set (kernel-trace only, each under its
# own time limit) on the isect kernel of the config-1 bench, then a per-launch
# summary.  The caller's environment passes through (e.g. SPT_STREAMS=1 for a
# full-chip isect grid, so the serialised PMC launches keep the bench's occupancy).
#   usage: [KERNEL=shade_kernel] [CONFIG=1] tools/pmc_sweep.sh OUTDIR "CTR CTR .." ["CTR .." ...]
set -u
out=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p "$out"
export TMPDIR=/tmp
i=0
csvs=""
for ctrs in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-include-regex ${KERNEL:-isect_queue} -d "$out/p$i" -o run --output-format csv \
      -- python bench.py --config ${CONFIG:-1} --steps 1 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > "$out/p$i.log" 2>&1
  rc=$?
  echo "== pass $i ($ctrs) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$out/p$i.log"; exit $rc; fi
  csvs="$csvs $out/p$i/run_counter_collection.csv"
done
python tools/pmc_isect.py "$out/summary.json" "config${CONFIG:-1}" "$out/p1.log" $csvs --kernel ${KERNEL:-isect_queue}
