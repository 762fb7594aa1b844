"""pbrt-v3 scenes on the GPU (the San-Miguel path of BASELINE configs[4]):
a scene written as pbrt + PLY and read back through spt_pbrt_load renders
bit-equal to the oracle, through the Python host and through the C++ CLI
(whose camera, film size and sky come from the .pbrt file)."""
import os
import subprocess

import numpy as np
import pytest
import torch

import oracle as O
import sptamd
from sptamd import _lib, scenes

pytestmark = pytest.mark.gpu


def test_pbrt_cornell_emitters_bitexact(tmp_path):
    m = scenes.cornell_spheres(detail=0.25)
    path = str(tmp_path / "cornell.pbrt")
    scenes.write_pbrt(path, m, camera=scenes.cornell_camera(), width=48, height=40)
    s = sptamd.Scene()
    s.add_triangle_mesh(path)
    s.commit(0)
    alb, emi = scenes.smallpt_materials(s.mesh)
    s.backend.set_albedo(alb)
    s.backend.set_emission(emi)
    cam = s.pbrt_info["camera"]
    kw = dict(camera=cam, rr_start_depth=5, env=(0.0, 0.0, 0.0))
    film, st = s.render(sptamd.make_params(48, 40, 8, 10, **kw))
    torch.cuda.synchronize()
    ref, casts = O.OracleScene(s.mesh, albedo=alb, emission=emi).render(O.reference_params(48, 40, 8, 10, **kw))
    np.testing.assert_array_equal(film.cpu().numpy(), ref)
    assert st["ray_casts"] == casts and film.cpu().numpy().max() > 0


def read_pfm(path):
    with open(path, "rb") as f:
        assert f.readline().strip() == b"PF"
        w, h = map(int, f.readline().split())
        assert float(f.readline()) < 0
        data = np.frombuffer(f.read(), "<f4").reshape(h, w, 3)[::-1]  # rows bottom-up (fimage.h:46-55)
    return np.ascontiguousarray(data.transpose(2, 0, 1))


def test_cli_renders_pbrt_scene(tmp_path):
    """spt_render_cli scene.pbrt: film size and camera from the file."""
    m = scenes.mitsuba_synth(detail=0.1)
    path = str(tmp_path / "m.pbrt")
    scenes.write_pbrt(path, m, width=40, height=30)
    cli = os.path.join(os.path.dirname(_lib.LIB_PATH), "spt_render_cli")
    out = str(tmp_path / "out.pfm")
    r = subprocess.run([cli, path, "-s", "4", "-d", "4", "-o", out], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    got = read_pfm(out)
    assert got.shape == (3, 30, 40)
    loaded, info = scenes.load_pbrt(path)
    ref, _ = O.OracleScene(loaded).render(O.reference_params(40, 30, 4, 4, camera=info["camera"]))
    np.testing.assert_array_equal(got, ref)
