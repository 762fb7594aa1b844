"""bench.py's N-rank flow on the GPU box: torch.distributed.run with N ranks
sharing the one GPU (SPT_REHEARSE_SHARED_GPU=1) and the tile gather over gloo;
the rank-0 image must equal the one-rank image bit for bit, and the rank-0
JSON line must report N GPUs.  (The 8-GPU node runs the same flow one rank per
device over RCCL.)"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--width", "256", "--height", "128", "--spp", "4", "--depth", "4", "--steps", "1", "--warmup", "1",
         "--no-cpu-baseline"]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(cmd, env):
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 3])
def test_bench_ranks_match_one_rank(tmp_path, n):
    env = dict(os.environ)
    one = _run([sys.executable, "bench.py", *SMALL, "--save", str(tmp_path / "one.npy")], env)
    assert one["n_gpus"] == 1
    env.update(SPT_DIST_BACKEND="gloo", SPT_REHEARSE_SHARED_GPU="1")
    rec = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
                "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", str(n),
                *SMALL, "--save", str(tmp_path / "n.npy")], env)
    assert rec["n_gpus"] == n and rec["value"] > 0
    assert rec["dist"] == {"backend": "gloo", "world_size": n}
    assert rec["work_check"]["paths_device_counted"] == rec["work_check"]["expected"] == 256 * 128 * 4
    # a tile this small (< 2^20 paths) runs fused (AUTO); the other pipeline
    # is timed beside it on the same tiles, with the same image
    assert rec["config"]["pipeline"] == "fused"
    leg = rec["wavefront_leg"]
    assert leg["value"] > 0 and leg["paths_device_counted"] == 256 * 128 * 4 and leg["image_equal"]
    np.testing.assert_array_equal(np.load(tmp_path / "n.npy"), np.load(tmp_path / "one.npy"))
