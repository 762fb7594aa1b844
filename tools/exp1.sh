cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for s in 1 2 3 4; do echo "streams $s" >> gpurun_out/exp1.log; SPT_STREAMS=$s timeout -k 10 200 python tools/tile_sim.py --timing >> gpurun_out/exp1.log 2>&1 || exit 1; done
for i in 16 32 48; do echo "fused idle $i" >> gpurun_out/exp1.log; SPT_FUSED_IDLE=$i timeout -k 10 200 python tools/tile_sim.py --timing --pipeline fused >> gpurun_out/exp1.log 2>&1 || exit 1; done
