#!/bin/bash
# Packed child groups (SPT_PACK=1, default) vs aligned groups of eight slots.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/tests_pack.log 2>&1; rc=$?
tail -3 gpurun_out/tests_pack.log
[ $rc -ne 0 ] && exit $rc
VARIANTS="p1= p0=" ENVS="p1:SPT_PACK=1 p0:SPT_PACK=0" ROUNDS=3 timeout -k 10 400 bash tools/ab.sh || exit $?
echo "== config 4" >> gpurun_out/ab.log
VARIANTS="p1= p0=" ENVS="p1:SPT_PACK=1 p0:SPT_PACK=0" ROUNDS=2 BENCH_ARGS="--config 4 --steps 2" timeout -k 10 500 bash tools/ab.sh || exit $?
for p in 1 0; do SPT_PACK=$p timeout -k 10 200 python tools/trav_stats.py --depths 8 | head -1 >> gpurun_out/ab.log; done
