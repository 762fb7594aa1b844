"""The binary scene cache (include/spt.h spt_scene_save /
spt_scene_load): a committed scene saved and loaded back — with no parse, no
BVH build and no re-layout — renders and intersects bit-identically to the
scene that was saved, for every node format and builder, with textures,
emitters, spheres and material kinds, the pbrt camera riding along as extra
bytes; damaged files are refused."""
import os

import numpy as np
import pytest
import torch

import oracle as O
import sptamd
from sptamd import _lib, scenes

pytestmark = pytest.mark.gpu

HOST, GPU = _lib.SPT_BUILD_HOST_SAH, _lib.SPT_BUILD_GPU_PLOC


def build(kind):
    """(scene, camera kwargs) of one cache case."""
    cfg = sptamd.default_config()
    kw = {}
    if kind == "smallpt":                       # spheres, mirror / glass kinds, emitters
        m = scenes.smallpt_analytic(detail=0.5)
        s = sptamd.Scene(cfg)
        s.add_arrays(m)
        s.commit(0)
        alb, emi = scenes.smallpt_materials(m)
        s.backend.set_albedo(alb)
        s.backend.set_emission(emi)
        kw = dict(camera=scenes.cornell_camera(), rr_start_depth=5, env=(0.0, 0.0, 0.0))
        return s, kw
    m = scenes.with_planar_uv(scenes.mitsuba_synth(detail=0.25))
    b = HOST
    if kind == "gpu8":
        cfg.bvh_width, cfg.pack_groups, b = 8, 0, GPU
    elif kind == "gpu6":
        b = GPU
    elif kind == "bvh2":
        cfg.bvh_width = 2
    elif kind == "empty":
        m = {"pos": np.zeros((0, 3), np.float32), "pos_tri": np.zeros((0, 3), np.int32)}
    s = sptamd.Scene(cfg)
    s.add_arrays(m)
    s.commit(0, build=b)
    if kind == "host6":                          # albedo, textures, emitters
        nm = len(m["kd"])
        s.backend.set_albedo(np.full((nm, 3), 0.8, np.float32))
        emi = np.zeros((nm, 3), np.float32)
        emi[4] = (3.0, 2.0, 1.0)
        s.backend.set_emission(emi)
        s.backend.set_texture(1, scenes.checker(8, 8, cell=1))
        s.backend.set_texture(3, scenes.checker(16, 4, cell=2))
        kw = dict(rr_start_depth=3, env=(0.2, 0.2, 0.3))
    return s, kw


def frame(s, kw, pipeline):
    film, st = s.render(sptamd.make_params(40, 32, 4, 6, pipeline=pipeline, **kw))
    torch.cuda.synchronize()
    return film.cpu().numpy(), st["ray_casts"]


def hits(s):
    rng = np.random.default_rng(5)
    o = rng.uniform(-2.5, 2.5, size=(3, 6000)).astype(np.float32)
    d = rng.normal(size=(3, 6000)).astype(np.float32)
    out = s.backend.intersect_raw(sptamd.Ray3.make(o, d))
    torch.cuda.synchronize()
    return [x.cpu().numpy() for x in out]


@pytest.mark.parametrize("kind", ["host6", "smallpt", "gpu8", "gpu6", "bvh2", "empty"])
def test_cache_roundtrip_bitexact(tmp_path, kind):
    if os.environ.get("SPT_BVH") or os.environ.get("SPT_PACK"):
        pytest.skip("SPT_BVH / SPT_PACK override the layout")
    s, kw = build(kind)
    path = str(tmp_path / "scene.sptc")
    s.save(path)
    info = sptamd.scene_cache_info(path)
    saved = dict(s.backend.stats)
    for st in (info["stats"], saved):
        st.pop("build_ms")
    assert info["stats"] == saved and info["config"] == s.backend.config and info["extra_bytes"] == 0
    t = sptamd.Scene.load(path)
    got = dict(t.backend.stats)
    assert got.pop("build_ms") > 0 and got == saved
    assert t.backend.config == s.backend.config and t.mesh is None
    for pipeline in ("wavefront", "fused"):
        a, ca = frame(s, kw, pipeline)
        b, cb = frame(t, kw, pipeline)
        np.testing.assert_array_equal(b, a)
        assert ca == cb
    for x, y in zip(hits(s), hits(t)):
        np.testing.assert_array_equal(y, x)
    if kind == "empty":
        assert (hits(t)[0] == -1).all()
    # the loaded scene owns its arrays: destroying the original changes nothing
    a, _ = frame(s, kw, "wavefront")
    del s
    b, _ = frame(t, kw, "wavefront")
    np.testing.assert_array_equal(b, a)


def test_cache_pbrt_camera_and_oracle(tmp_path):
    """A pbrt scene cached with its camera (Scene.save's extra bytes) renders
    from the cache bit-equal to the oracle."""
    m = scenes.cornell_spheres(detail=0.25)
    src = str(tmp_path / "cornell.pbrt")
    scenes.write_pbrt(src, m, camera=scenes.cornell_camera(), width=48, height=40)
    s = sptamd.Scene()
    s.add_triangle_mesh(src)
    s.commit(0)
    alb, emi = scenes.smallpt_materials(s.mesh)
    s.backend.set_albedo(alb)
    s.backend.set_emission(emi)
    path = str(tmp_path / "cornell.sptc")
    s.save(path)
    assert sptamd.scene_cache_info(path)["extra_bytes"] > 0
    t = sptamd.Scene.load(path)
    assert t.pbrt_info == s.pbrt_info
    kw = dict(camera=t.pbrt_info["camera"], rr_start_depth=5, env=(0.0, 0.0, 0.0))
    film, st = t.render(sptamd.make_params(48, 40, 8, 10, **kw))
    torch.cuda.synchronize()
    ref, casts = O.OracleScene(s.mesh, albedo=alb, emission=emi).render(O.reference_params(48, 40, 8, 10, **kw))
    np.testing.assert_array_equal(film.cpu().numpy(), ref)
    assert st["ray_casts"] == casts


def test_cache_damage_refused(tmp_path):
    s, _ = build("host6")
    path = str(tmp_path / "scene.sptc")
    s.save(path)
    raw = open(path, "rb").read()
    mid = len(raw) // 2                         # inside the node / triangle sections
    cases = {"flip": raw[:mid] + bytes([raw[mid] ^ 1]) + raw[mid + 1:],
             "truncated": raw[:-7], "magic": b"X" + raw[1:]}
    for name, data in cases.items():
        bad = str(tmp_path / f"{name}.sptc")
        with open(bad, "wb") as f:
            f.write(data)
        with pytest.raises(sptamd.SptError) as e:
            sptamd.Scene.load(bad)
        assert e.value.code == _lib.SPT_ERR_INVALID, name
    with pytest.raises(sptamd.SptError) as e:
        sptamd.Scene.load(str(tmp_path / "missing.sptc"))
    assert e.value.code == _lib.SPT_ERR_IO
    t = sptamd.Scene.load(path)                # the good file still loads
    assert t.backend.stats["ntri"] == s.backend.stats["ntri"]
    with pytest.raises(sptamd.SptError) as e:   # an unwritable path
        s.save(str(tmp_path / "no" / "such" / "dir.sptc"))
    assert e.value.code == _lib.SPT_ERR_IO


def test_cli_cache_roundtrip(tmp_path):
    """spt_render_cli --save-cache then the .sptc: same image; the cache (and
    its pbrt camera) reads back through the Python host too."""
    import subprocess
    from test_gpu_pbrt import read_pfm
    m = scenes.mitsuba_synth(detail=0.1)
    src = str(tmp_path / "m.pbrt")
    scenes.write_pbrt(src, m, width=40, height=30)
    cli = os.path.join(os.path.dirname(_lib.LIB_PATH), "spt_render_cli")
    cache = str(tmp_path / "m.sptc")
    outs = []
    for scene, extra in ((src, ["--save-cache", cache]), (cache, [])):
        out = str(tmp_path / f"out{len(outs)}.pfm")
        r = subprocess.run([cli, scene, "-s", "4", "-d", "4", "-o", out] + extra, capture_output=True, text=True,
                           timeout=120)
        assert r.returncode == 0, r.stderr
        outs.append(read_pfm(out))
    np.testing.assert_array_equal(outs[1], outs[0])
    assert outs[0].shape == (3, 30, 40)
    t = sptamd.Scene.load(cache)
    _, info = scenes.load_pbrt(src)
    assert t.pbrt_info == info
