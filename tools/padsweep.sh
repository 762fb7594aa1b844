#!/bin/bash
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for pad in 0 0 192 1088 4160 0; do
  echo "pad $pad" >> gpurun_out/pad.log
  SPT_PLANE_PAD=$pad timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pad_$pad.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/pad_$pad.json'));print($pad, d['value'], d['kernel_ms_per_step'])" >> gpurun_out/pad.log
done
cat gpurun_out/pad.log
