#!/bin/bash
# GPU-box driver: each step under its own timeout; stop at the first step that
# faults / aborts / times out (exit 124, 134, 137, 139 or > 128).  Test
# failures (pytest exit 1) do not stop the later steps.
# usage: tools/gpu_run.sh step1 step2 ...   (steps: smoke tests bench prof pmc)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*" | tee -a gpurun_out/steps.log
  local t0=$(date +%s)
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc $(( $(date +%s) - t0 ))s" | tee -a gpurun_out/steps.log
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "STOP: $name ended with $rc" | tee -a gpurun_out/steps.log
    exit $rc
  fi
  return 0
}
for s in "$@"; do
  case "$s" in
    smoke) run smoke 300 python __graft_entry__.py smoke ;;
    tests) run tests 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread ;;
    testsnx) run testsnx 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ;;
    testsv) run testsv 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ;;
    testsall) run testsall 900 python -m pytest tests -m gpu -q ;;
    tests2) run tests2 900 env SPT_BVH=2 python -m pytest tests -m gpu -q -x ;;
    tests8) run tests8 900 env SPT_BVH=8 python -m pytest tests -m gpu -q -x ;;
    trav48) run trav48 600 env SPT_BVH=8 python tools/trav_stats.py --city --depths 8 --spp 8 ;;
    trav18) run trav18 600 env SPT_BVH=8 python tools/trav_stats.py --depths 8 ;;
    testsgb) run testsgb 900 env SPT_BUILD=gpu python -m pytest tests -m gpu -q -x ;;
    bench4gq) run bench4gq 600 env SPT_BUILD=gpu python bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline ;;
    bench1gq) run bench1gq 600 env SPT_BUILD=gpu python bench.py --config 1 --steps 3 --warmup 1 --no-cpu-baseline ;;
    bench) run bench 600 python bench.py ;;
    benchq) run benchq 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline ;;
    bench1x3) for r in 1 2 3; do run bench1_$r 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline; done ;;
    bench10) run bench10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline ;;
    bench1f) run bench1f 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --pipeline fused ;;
    bench0|bench2|bench3|bench4) run $s 600 python bench.py --config ${s#bench} --steps 2 --warmup 1 ;;
    bench2q|bench3q|bench4q) c=${s#bench}; run $s 600 python bench.py --config ${c%q} --steps 2 --warmup 1 --no-cpu-baseline ;;
    benchwf) for wf in ${WFS:-1048576 4194304 8388608}; do run benchwf$wf 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --wavefront $wf; done ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
    prof2s) run prof2s 600 env SPT_STREAMS=1 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2s -o run --output-format csv -- python bench.py --config 2 --steps 1 --warmup 1 --no-cpu-baseline ;;
    prof2|prof4) run $s 600 rocprofv3 --kernel-trace --stats -d gpurun_out/$s -o run --output-format csv -- python bench.py --config ${s#prof} --steps 1 --warmup 1 --no-cpu-baseline ;;
    pmcfetch) run pmcfetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex isect_queue -d gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
    pmcwrite) run pmcwrite 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex isect_queue -d gpurun_out/pmc_write -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
    pmc|pmc1|pmc2|pmc3|pmc4) c=${s#pmc}; run $s 900 env CONFIG=${c:-1} bash tools/pmc_isect.sh gpurun_out/pmc ;;
    pmcshade) run pmcshade 600 env KERNEL=shade_kernel bash tools/pmc_sweep.sh gpurun_out/pmc_shade "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES" ;;
    pmcshade1) run pmcshade1 600 env SPT_STREAMS=1 KERNEL=shade_kernel bash tools/pmc_sweep.sh gpurun_out/pmc_shade1 "FETCH_SIZE" "WRITE_SIZE" ;;
    pmc1s) run pmc1s 900 env SPT_STREAMS=1 CONFIG=1 bash tools/pmc_isect.sh gpurun_out/pmc1s ;;
    proff) run proff 600 rocprofv3 --kernel-trace --stats -d gpurun_out/proff -o run --output-format csv -- python bench.py --pipeline fused --steps 2 --warmup 1 --no-cpu-baseline ;;
    pmcd1|pmcd4) c=${s#pmcd}; run $s 900 env CONFIG=$c KERNEL=drain bash tools/pmc_isect.sh gpurun_out/pmc ;;
    pmcf) run pmcf 900 env CONFIG=1 PIPE=fused bash tools/pmc_isect.sh gpurun_out/pmc ;;
    prof1s) run prof1s 600 env SPT_STREAMS=1 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1s -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
    trav) run trav 600 python tools/trav_stats.py ;;
    trav4) run trav4 600 python tools/trav_stats.py --city --depths 8 --spp 8 ;;
    trav4h) run trav4h 600 env SPT_BUILD=host python tools/trav_stats.py --city --depths 8 --spp 8 ;;
    bench4h) run bench4h 600 env SPT_BUILD=host python bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline ;;
    proftile2|proftile4|proftile8) n=${s#proftile}; run $s 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$s -o run --output-format csv -- python tools/tile_sim.py --tiles $n --steps 4 --pipeline ${PIPE:-wavefront} ;;
    drainsweep) for dq in ${DRAINS:-0 256 512 1024 2048}; do run drain$dq 300 env SPT_DRAIN_Q8=$dq python tools/tile_sim.py --tiles 1 2 4 8 --pipeline wavefront --steps 8; done ;;
    sweep) run sweep 600 python tools/tile_sim.py --tiles ${TILES:-1 2 4 8} --pipeline ${PIPE:-wavefront} --steps ${STEPS:-8} --sweep $SWEEP ;;
    matrix) i=0; IFS=';' read -ra CFGS <<< "$MATRIX"; for c in "${CFGS[@]}"; do i=$((i+1)); run matrix$i 300 env ${c//,/ } python tools/tile_sim.py --tiles ${TILES:-1 2 4 8} --pipeline ${PIPE:-wavefront} --steps ${STEPS:-40} --sweep REP=${REPS:-1,2} TAG=m$i; done ;;
    benchm) i=0; IFS=';' read -ra CFGS <<< "$MATRIX"; for c in "${CFGS[@]}"; do i=$((i+1)); run benchm$i 400 env ${c//,/ } python bench.py --config ${CONFIG:-1} --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline; done ;;
    tilesimw) run tilesimw 400 python tools/tile_sim.py --tiles 1 2 4 8 --pipeline wavefront --timing ;;
    tilesima) run tilesima 400 python tools/tile_sim.py --tiles 1 2 4 8 --timing ;;
    tilesim) run tilesim 400 python tools/tile_sim.py ;;
    tilesimt) run tilesimt 400 python tools/tile_sim.py --timing ;;
    tilesimf) run tilesimf 400 python tools/tile_sim.py --pipeline fused ;;
    listctr) run listctr 300 rocprofv3 -L ;;
    pmcsq) run pmcsq 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD --kernel-include-regex isect_queue -d gpurun_out/pmc_sq -o run --output-format csv -- python tools/trav_stats.py --depths 8 --spp 8 ;;
    pmctcc) run pmctcc 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --kernel-include-regex isect_queue -d gpurun_out/pmc_tcc -o run --output-format csv -- python tools/trav_stats.py --depths 8 --spp 8 ;;
    pmctcp) run pmctcp 600 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr TA_TA_BUSY_sum --kernel-include-regex isect_queue -d gpurun_out/pmc_tcp -o run --output-format csv -- python tools/trav_stats.py --depths 8 --spp 8 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
