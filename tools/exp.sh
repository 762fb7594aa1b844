#!/bin/bash
# Env-variant sweep of tools/tile_sim.py on one box: each line of $EXP_LIST
# is "name ENV=val ..." ; output to gpurun_out/exp.log.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
while read -r name envs; do
  [ -z "$name" ] && continue
  echo "== $name $envs" >> gpurun_out/exp.log
  env $envs timeout -k 10 200 python tools/tile_sim.py --timing ${TS_ARGS:-} 2>&1 | grep -v amdgpu.ids >> gpurun_out/exp.log || exit 1
done < "${EXP_LIST:?set EXP_LIST to a file of lines: name ENV=val ...}"
