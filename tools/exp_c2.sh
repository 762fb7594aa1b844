set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config 2 --steps 2 --warmup 1 > gpurun_out/bench2a.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config 2 --steps 2 --warmup 1 --pipeline fused --no-cpu-baseline > gpurun_out/bench2af.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config 2 --scene cornell_spheres --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench2c.log 2>&1 || exit $?
