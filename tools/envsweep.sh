#!/bin/bash
# Env-knob sweep of bench.py on one box: each line of $SWEEP_LIST is
# "name [ENV=val ...]"; ROUNDS passes; one line per run to gpurun_out/envsweep.log.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for r in $(seq ${ROUNDS:-2}); do
  while read -r name envs; do
    [ -z "$name" ] && continue
    env $envs timeout -k 10 200 python bench.py --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/es.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/es.json'));print('$name', d['value'], d['kernel_ms_per_step'])" >> gpurun_out/envsweep.log
  done < "${SWEEP_LIST:?set SWEEP_LIST}"
done
cat gpurun_out/envsweep.log
