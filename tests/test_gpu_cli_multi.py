"""The C++ host's multi-GPU path (spt_render_cli --gpus N, csrc/main.cpp): one
host thread per device commits the scene and renders its interleaved
row-group tile, ONE ncclGather (RCCL over xGMI) brings the fp32 tiles to
device 0, and the rows are put back in place — the route a C++ caller
replacing main.cpp:354-446 takes to 8 GPUs.  On the one-GPU box: --gpus 1
runs the RCCL gather over one communicator; --rehearse-shared-gpu renders N
tiles on device 0 and gathers by device copies (tiling and assembly at any
N).  Every image must equal the single-device render and the oracle bit for
bit (the RNG is keyed by the global pixel)."""
import os
import subprocess

import numpy as np
import pytest

import oracle as O
from sptamd import _lib, scenes
from test_gpu_pbrt import read_pfm

pytestmark = pytest.mark.gpu

CLI = os.path.join(os.path.dirname(_lib.LIB_PATH), "spt_render_cli")
W, H, SPP, D = 72, 53, 4, 4


def run(args, out):
    r = subprocess.run([CLI] + args + ["-o", out], capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout + r.stderr
    return read_pfm(out)


@pytest.fixture(scope="module")
def obj(tmp_path_factory):
    m = scenes.mitsuba_synth(detail=0.1)
    path = str(tmp_path_factory.mktemp("cli") / "m.obj")
    scenes.write_obj(path, m)
    return path


def test_cli_multi_gpu_equals_single_and_oracle(obj, tmp_path):
    base = ["-w", str(W), "-h", str(H), "-s", str(SPP), "-d", str(D), obj]
    single = run(base, str(tmp_path / "single.pfm"))
    ref, _ = O.OracleScene(scenes.load_obj(obj)).render(O.reference_params(W, H, SPP, D))
    np.testing.assert_array_equal(single, ref)
    rccl1 = run(base + ["--gpus", "1"], str(tmp_path / "rccl1.pfm"))       # ncclGather, one communicator
    np.testing.assert_array_equal(rccl1, single)
    for n, rpg in ((2, 8), (3, 4), (8, 1)):                                  # N tiles on one device
        img = run(base + ["--gpus", str(n), "--rows-per-group", str(rpg), "--rehearse-shared-gpu"],
                  str(tmp_path / f"r{n}.pfm"))
        np.testing.assert_array_equal(img, single, err_msg=f"N={n} rows/group {rpg}")


def test_cli_multi_gpu_refuses_more_gpus_than_devices(obj, tmp_path):
    r = subprocess.run([CLI, "-w", "8", "-h", "8", "-s", "1", "-d", "1", obj, "--gpus", "64", "-o",
                        str(tmp_path / "x.pfm")], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "devices visible" in r.stderr
