#!/bin/bash
# s_setprio around the step's load issue (build_sp1 / build_sp3) vs none.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
P=smallpt-enoki-optix_amd
V="base= sp1=$P/build_sp1/libspt.so sp3=$P/build_sp3/libspt.so"
VARIANTS="$V" ROUNDS=3 timeout -k 10 500 bash tools/ab.sh || exit $?
echo "== fused" >> gpurun_out/ab.log
VARIANTS="$V" ROUNDS=1 BENCH_ARGS="--pipeline fused" timeout -k 10 300 bash tools/ab.sh || exit $?
