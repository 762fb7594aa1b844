#!/bin/bash
# Round-6 end measurements of the committed build, in two GPU calls (each step
# under its own time limit; the script stops at the first step that times out,
# faults or aborts).  Output: gpurun_out/r06_final/ (copied to profiles/).
#   bash tools/final_r06.sh a    suite, smoke, default bench (+ CPU baseline, parity),
#                                single-render bench, kernel trace of the default bench
#   bash tools/final_r06.sh b    configs 0, 2, 3, 4 (+ CPU baselines), tile projection x3
#                                (PMC=1: also the PMC passes of the config-2 / config-3 drains;
#                                the final build's passes of every config ran on their own:
#                                profiles/r06_pmc2/, r06_pmc3/)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06_final
mkdir -p $O
step() {  # name limit cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*" >> $O/steps.log
  local t0=$(date +%s)
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc $(( $(date +%s) - t0 ))s" >> $O/steps.log
  tail -n 3 "$O/$name.log"
  if [ $rc -ne 0 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
}
case "${1:-a}" in
  a)
    step tests 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
    step smoke 300 python __graft_entry__.py smoke
    step bench 400 python bench.py
    step bench_sync 300 env SPT_BENCH_SYNC=1 python bench.py --steps 10 --warmup 2 --no-cpu-baseline
    step prof 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
        python bench.py --steps 20 --warmup 2 --no-cpu-baseline
    python tools/trace_window_avg.py $O/prof/run_kernel_trace.csv --kernel render_fused --launches 20 \
        > $O/prof/timed_window.txt
    python tools/trace_window_avg.py $O/prof/run_kernel_trace.csv --kernel camera_cast --launches 20 \
        >> $O/prof/timed_window.txt
    cat $O/prof/timed_window.txt
    ;;
  b)
    for c in 0 2 3 4; do step bench$c 500 python bench.py --config $c --steps 2 --warmup 1; done
    if [ "${PMC:-0}" = 1 ]; then
      step pmcd2 600 env CONFIG=2 KERNEL=drain bash tools/pmc_isect.sh $O/pmc
      step pmcd3 600 env CONFIG=3 KERNEL=drain bash tools/pmc_isect.sh $O/pmc
    fi
    for r in 1 2 3; do step tiles$r 300 python tools/tile_sim.py --tiles 1 2 4 8 --steps 8; done
    ;;
esac
