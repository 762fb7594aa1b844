#!/bin/bash
# Bench variants (environment) per config, alternating, ROUNDS rounds: e.g. the
# bench flow (SPT_BENCH_SETUP / SPT_BENCH_SYNC in bench.py) or library knobs
# (SPT_* -> spt_config, sptamd/_lib.py).  A variant with several settings joins
# them with commas: VARIANTS="X=0 SPT_STREAMS=3,SPT_ISECT_GRID_Q8=85".
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
for c in ${CONFIGS:-3 4 1}; do for r in $(seq ${ROUNDS:-1}); do for v in ${VARIANTS:-X=0 SPT_BENCH_SETUP=0 SPT_BENCH_SYNC=1}; do
  st=2; [ $c = 1 ] && st=20
  out=$(env ${v//,/ } timeout -k 10 300 python bench.py --config $c --steps $st --warmup 1 --no-cpu-baseline 2>gpurun_out/ov_err.log) || { echo "FAIL config $c $v"; tail -5 gpurun_out/ov_err.log; exit 1; }
  echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('config $c $v', d['value'], d['ms_per_step'], d['roofline'].get('grays_per_s'), d['config'].get('paths_in_flight'))" | tee -a gpurun_out/ov.log
done; done; done
