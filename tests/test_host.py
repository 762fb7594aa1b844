"""Host-side checks without a GPU: the C ABI library loads and exports every
function include/spt.h declares (no compute calls), the reference defaults,
the OBJ reader's tinyobj index semantics (main.cpp:141-251), the PFM writer
(fimage.h:33-58) and error behaviour."""
import ctypes
import os
import re
import struct

import numpy as np
import pytest

import sptamd
from sptamd import _lib, scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "spt.h")


def declared_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(spt_[a-z_]+)\s*\(", txt)))


def test_header_symbols_exported():
    names = declared_functions()
    assert len(names) >= 15
    assert sorted(_lib.EXPORTED) == names
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for n in names:
        assert hasattr(lib, n), n


def test_version_and_errors_without_gpu():
    assert b"gfx950" in _lib.lib.spt_version()
    # invalid arguments are rejected before any device work
    st = _lib.lib.spt_scene_create(None, None, 0, 0, None, None, 0, None, None, 0, None, None)
    assert st == 1 and b"NULL" in _lib.lib.spt_last_error()
    with pytest.raises(sptamd.SptError):
        sptamd.check(_lib.lib.spt_render(None, None, None, None, None), "spt_render")


def test_default_params_are_the_reference_main():
    p = sptamd.default_params()
    assert (p.width, p.height, p.spp, p.max_depth) == (512, 512, 100, 2)          # main.cpp:357-361
    assert list(p.camera.look_from) == [0.0, np.float32(3.03), 5.0]              # main.cpp:383
    assert list(p.camera.look_at) == [0.0, np.float32(0.03), 0.0]
    assert p.camera.lens_radius == 0.0 and p.camera.focal_dist == 1.0
    assert p.camera.fov_y == np.float32(np.float32(40.0 / 180.0) * np.float32(np.pi))
    assert p.camera.film_size_y == np.float32(0.035)                              # pinhole.h:11
    assert p.rng_initstate == 0x853C49E6748FEA9B                                   # main.cpp:376
    assert list(p.env) == [1.0, 1.0, 1.0] and p.rng_order == 0


def _write(path, text):
    with open(path, "w") as f:
        f.write(text)


def test_obj_loader_semantics(tmp_path):
    _write(tmp_path / "m.mtl", "newmtl red\nKd 0.9 0.1 0.1\n\nnewmtl blue\nKd 0.1 0.1 0.9\nKe 4 5 6\n")
    _write(tmp_path / "a.obj", """# test
mtllib m.mtl
v 0 0 0
v 1 0 0
v 1 1 0
v 0 1 0
v 0 0 1
vn 0 0 1
vn 0 1 0
vt 0 0
vt 1 0
vt 1 1
f 1 2 3
usemtl blue
f 1//1 3//1 4//2
usemtl red
f 1/1/1 2/2/1 3/3/2 4/1/2
usemtl nope
f -1 -2 -3
""")
    m = scenes.load_obj(str(tmp_path / "a.obj"))
    np.testing.assert_array_equal(m["pos_tri"], [[0, 1, 2], [0, 2, 3], [0, 1, 2], [0, 2, 3], [4, 3, 2]])
    np.testing.assert_array_equal(m["nrm_tri"], [[-1, -1, -1], [0, 0, 1], [0, 0, 1], [0, 1, 1], [-1, -1, -1]])
    np.testing.assert_array_equal(m["tc_tri"], [[-1, -1, -1], [-1, -1, -1], [0, 1, 2], [0, 2, 0], [-1, -1, -1]])
    # obj material id + 1 (main.cpp:185): none -> 0, blue (index 1) -> 2, red (0) -> 1, unknown -> 0
    np.testing.assert_array_equal(m["mat_id"], [0, 2, 1, 1, 0])
    np.testing.assert_allclose(m["kd"], [[1, 1, 1], [0.9, 0.1, 0.1], [0.1, 0.1, 0.9]])
    np.testing.assert_allclose(m["ke"], [[0, 0, 0], [0, 0, 0], [4, 5, 6]])  # Ke: emission table
    assert m["pos"].shape == (5, 3) and m["nrm"].shape == (2, 3) and m["tc"].shape == (3, 2)


def test_obj_loader_errors(tmp_path):
    mesh = _lib.Mesh()
    assert _lib.lib.spt_obj_load(str(tmp_path / "missing.obj").encode(), ctypes.byref(mesh)) == 5
    _write(tmp_path / "bad.obj", "v 0 0 0\nv 1 0 0\nf 1 2 7\n")
    assert _lib.lib.spt_obj_load(str(tmp_path / "bad.obj").encode(), ctypes.byref(mesh)) == 1


def test_generated_scene_roundtrip(tmp_path):
    m = scenes.mitsuba_synth(detail=0.1)
    path = str(tmp_path / "s.obj")
    scenes.write_obj(path, m)
    l = scenes.load_obj(path)
    for k in ("pos_tri", "nrm_tri", "mat_id"):
        np.testing.assert_array_equal(l[k], m[k])
    for k in ("pos", "nrm", "kd"):
        np.testing.assert_array_equal(l[k], m[k].astype(np.float32))
    c = scenes.cornell_spheres(detail=0.25)
    scenes.write_obj(path, c)
    l = scenes.load_obj(path)
    np.testing.assert_array_equal(l["mat_id"], c["mat_id"])
    np.testing.assert_array_equal(l["ke"], c["ke"])
    assert l["ke"].max() == 12.0


def test_pfm_writer(tmp_path):
    h, w = 3, 4
    film = np.arange(3 * h * w, dtype=np.float32).reshape(3, h, w)
    path = str(tmp_path / "x.pfm")
    sptamd.write_pfm(path, film)
    data = open(path, "rb").read()
    header = b"PF\n%d %d\n-1\n" % (w, h)
    assert data.startswith(header)
    px = np.frombuffer(data[len(header):], dtype="<f4").reshape(h, w, 3)
    # rows bottom-up, interleaved RGB (fimage.h:46-55)
    np.testing.assert_array_equal(px, film.transpose(1, 2, 0)[::-1])
    assert struct.calcsize("<f") * 3 * h * w == len(data) - len(header)


def test_struct_layouts_match_header(tmp_path):
    """ctypes layouts == what a C compiler makes of include/spt.h."""
    import subprocess
    structs = {"spt_render_params": _lib.RenderParams, "spt_render_stats": _lib.RenderStats,
               "spt_scene_stats": _lib.SceneStats, "spt_rays": _lib.Rays, "spt_hits": _lib.Hits,
               "spt_hit_info": _lib.HitInfo, "spt_camera": _lib.Camera, "spt_mesh": _lib.Mesh,
               "spt_config": _lib.Config}
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void) {"]
    for cname, ct in structs.items():
        lines.append(f'printf("{cname} sizeof %zu\\n", sizeof({cname}));')
        for fname, _ in ct._fields_:
            lines.append(f'printf("{cname} {fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-o", str(exe), str(src)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    for line in filter(None, out):
        cname, field, val = line.split()
        ct = structs[cname]
        got = ctypes.sizeof(ct) if field == "sizeof" else getattr(ct, field).offset
        assert got == int(val), (cname, field, got, val)


def test_config_defaults_and_env_overrides():
    """spt_config carries every knob (the library reads no environment);
    the Python host maps SPT_* variables onto it as overrides."""
    c = sptamd.default_config()
    assert (c.build, c.bvh_width, c.collapse, c.ploc_radius) == (0, 6, 0, 16)
    assert (c.streams, c.isect_refill_idle, c.isect_static_share_q8, c.isect_chunk) == (4, 24, 128, 128)
    assert c.wavefront_paths == 1 << 25 and c.fused_max_paths == 1 << 20      # spt.h docs = code
    assert (c.drain_q8, c.drain_grid_q8, c.drain_casts) == (1024, 0, 1)
    assert (c.fit_streams, c.fit_paths, c.sub_queues) == (1, 1 << 28, 1)
    assert (c.drain_sort, c.lockstep_first, c.fit_chunks) == (0, 3, 1)
    assert sptamd.config_from_env(environ={"SPT_LOCKSTEP_FIRST": "0"}).lockstep_first == 0
    assert c.fit_bytes == 0 and sptamd.config_from_env(environ={"SPT_FIT_BYTES": "4096"}).fit_bytes == 4096
    assert c.drain_refill_idle == 0 and sptamd.config_from_env(environ={"SPT_DRAIN_IDLE": "40"}).drain_refill_idle == 40
    d = sptamd.config_from_env(environ={"SPT_DRAIN_Q8": "0", "SPT_DRAIN_CASTS": "4", "SPT_FIT_PATHS": "0"})
    assert (d.drain_q8, d.drain_casts, d.fit_paths) == (0, 4, 0)
    assert c.film_budget_bytes == 4 << 30 and c.public_refill_idle == 16
    assert c.pack_groups == 1
    assert (c.work_order, c.queue_cache) == (_lib.SPT_WORK_AUTO, _lib.SPT_QUEUE_CACHE_AUTO)
    assert sptamd.config_from_env(environ={"SPT_QUEUE_CACHE": "2"}).queue_cache == _lib.SPT_QUEUE_CACHE_STREAM
    e = sptamd.config_from_env(environ={"SPT_STREAMS": "2", "SPT_BUILD": "gpu", "SPT_FUSED": "0",
                                        "SPT_FILM_BUDGET": "1000", "SPT_COLLAPSE": "greedy", "SPT_BVH": "2"})
    assert (e.streams, e.build, e.pipeline, e.film_budget_bytes, e.collapse, e.bvh_width) == (2, 2, 1, 1000, 1, 2)
    with pytest.raises(ValueError):
        sptamd.config_from_env(environ={"SPT_BUILD": "cuda"})


@pytest.mark.parametrize("field,value", [("streams", 0), ("streams", 5), ("bvh_width", 4), ("ploc_radius", 12),
                                         ("isect_refill_idle", 65), ("film_budget_bytes", 0), ("pipeline", 3),
                                         ("bvh_width", 7), ("pack_groups", 3), ("work_order", 3),
                                         ("queue_cache", 3), ("drain_q8", 65536), ("drain_grid_q8", 4097),
                                         ("drain_casts", 65), ("fit_streams", 0), ("fit_streams", 5),
                                         ("fit_paths", (1 << 31) + 1), ("lockstep_first", 4), ("fit_chunks", 2),
                                         ("drain_refill_idle", 65)])
def test_config_validation_without_gpu(field, value):
    c = sptamd.default_config()
    setattr(c, field, value)
    pt = np.array([0, 1, 2], np.int32)
    pos = np.zeros(9, np.float32)
    out = ctypes.c_void_p()
    st = _lib.lib.spt_scene_create_cfg(pt.ctypes.data, pos.ctypes.data, 3, 1, None, None, 0, None, None, 0, None,
                                       ctypes.byref(c), ctypes.byref(out))
    assert st == 1 and field.encode() in _lib.lib.spt_last_error()
    assert _lib.lib.spt_scene_set_config(None, ctypes.byref(c)) == 1


def test_library_reads_no_environment():
    """the tuning knobs are C ABI fields, not getenv.
    (The .so still imports getenv: rocPRIM's headers, behind hipcub, read
    their own debug variables; no source of ours does.)"""
    import glob
    srcs = glob.glob(os.path.join(ROOT, "smallpt-enoki-optix_amd", "csrc", "*"))
    assert len(srcs) > 10
    for f in srcs:
        assert not re.search(r"\b(getenv|secure_getenv)\s*\(", open(f).read()), f


def test_tile_row_count_matches_library():
    """The Python host's closed-form row count (used on every render) equals spt_tile_rows."""
    from sptamd import _lib
    for h in (0, 1, 7, 40, 1000, 1024, 1080):
        for tc in (0, 1, 2, 3, 8):
            for rpg in (0, 1, 4, 8, 64):
                for ti in range(tc + 1):
                    assert _lib.tile_row_count(h, ti, tc, rpg) == _lib.lib.spt_tile_rows(h, ti, tc, rpg, None, 0), \
                        (h, ti, tc, rpg)


def test_env_snapshot_tracks_environment(monkeypatch):
    """sync_config's cheap env read sees every change made through os.environ."""
    from sptamd import _lib
    i = list(_lib._ENV_CONFIG).index("SPT_STREAMS")
    monkeypatch.delenv("SPT_STREAMS", raising=False)
    assert _lib.env_snapshot()[i] is None
    monkeypatch.setenv("SPT_STREAMS", "3")
    assert _lib.env_snapshot()[i] == "3" and _lib.config_from_env().streams == 3
    monkeypatch.setenv("SPT_STREAMS", "")
    assert _lib.config_from_env().streams == _lib.default_config().streams
    assert _lib.env_snapshot({"SPT_STREAMS": "2"})[i] == "2"


def test_shard_base_partitions_items(tmp_path):
    """The sharded camera cast's queue segments (spt_internal.h shard_base):
    for every item count and block size, segment j starts where shards 0..j-1's
    threads end, and the eight segments cover exactly the items (the drain's
    per-XCD pools read them by the same formula)."""
    import shutil
    import subprocess
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    src = os.path.join(os.path.dirname(__file__), "native", "shard_base_check.cpp")
    exe = tmp_path / "shard_base_check"
    csrc = os.path.join(os.path.dirname(os.path.dirname(__file__)), "smallpt-enoki-optix_amd", "csrc")
    subprocess.run([hipcc, "-std=c++17", "-I" + csrc, "-x", "hip", "--offload-arch=gfx950", "-o", str(exe), src],
                   check=True, capture_output=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    assert '"bad": 0' in out, out
