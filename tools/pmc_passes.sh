#!/bin/bash
# Several rocprofv3 --pmc passes (each its own run, kernel-trace only) on the
# isect kernel.  usage: tools/pmc_passes.sh OUTDIR "CTR CTR .." "CTR .." ...
set -u
out=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p "$out"
export TMPDIR=/tmp
i=0
for ctrs in "$@"; do
  i=$((i+1))
  echo "== pass $i: $ctrs"
  timeout -k 10 300 rocprofv3 --pmc $ctrs --kernel-include-regex isect_queue -d "$out/p$i" -o run --output-format csv \
      -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline > "$out/p$i.log" 2>&1
  rc=$?
  echo "== pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$out/p$i.log"; fi
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
done
