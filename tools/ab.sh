#!/bin/bash
# A/B on one box: alternate bench runs of library variants.
#   VARIANTS="base=  t4=smallpt-enoki-optix_amd/build_t4/libspt.so"  (empty = build/libspt.so)
#   ENVS may add per-variant env as name:VAR=val,VAR2=val
#   BENCH_ARGS extra bench.py flags; ROUNDS (3)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq ${ROUNDS:-3}); do
  for v in ${VARIANTS:-base=}; do
    name=${v%%=*}; lib=${v#*=}
    extra=""
    for e in ${ENVS:-}; do [ "${e%%:*}" = "$name" ] && extra=$(echo "${e#*:}" | tr ',' ' '); done
    env SPT_LIB=${lib:+$PWD/$lib} $extra timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > /tmp/ab.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('/tmp/ab.json'));print('$name', d['value'], d['kernel_ms_per_step'])" >> gpurun_out/ab.log
  done
done
cat gpurun_out/ab.log
