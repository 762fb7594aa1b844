#!/bin/bash
# Rehearse bench.py's N-rank flow on a one-GPU box: N ranks share the GPU
# (SPT_REHEARSE_SHARED_GPU=1) and gather over gloo; the assembled image must
# equal the one-rank image bit for bit.  usage: [CONFIG=c] tools/rehearse_ranks.sh N...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
c=${CONFIG:-1}
img=${IMG_DIR:-gpurun_out}  # images (25 MB each at config 4): IMG_DIR=/tmp keeps them out of gpurun_out
mkdir -p "$img"
timeout -k 10 300 python bench.py --config $c --steps 1 --warmup 1 --no-cpu-baseline --save $img/img_n1.npy \
    > gpurun_out/rehearse_c${c}_n1.json 2> gpurun_out/rehearse_c${c}_n1.err || { tail -5 gpurun_out/rehearse_c${c}_n1.err; exit 1; }
for n in "$@"; do
  SPT_DIST_BACKEND=gloo SPT_REHEARSE_SHARED_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
      --nproc-per-node "$n" --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --config $c --gpus "$n" \
      --steps 1 --warmup 1 --save $img/img_n$n.npy > gpurun_out/rehearse_c${c}_n$n.json 2> gpurun_out/rehearse_c${c}_n$n.err
  rc=$?
  echo "== N=$n rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/rehearse_c${c}_n$n.err; exit $rc; fi
  cut -c1-400 gpurun_out/rehearse_c${c}_n$n.json
  python -c "import numpy as np,sys; a=np.load('$img/img_n1.npy'); b=np.load('$img/img_n$n.npy'); print('N=$n image bit-equal to N=1:', bool(np.array_equal(a,b))); sys.exit(0 if np.array_equal(a,b) else 1)" || exit 1
done
