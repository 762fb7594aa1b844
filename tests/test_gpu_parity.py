"""GPU parity beyond the bitwise unit cases (VERDICT r1 "do this" 1):

  - BASELINE configs[0] (mitsuba stand-in, 256^2 x 4 spp, 4 casts) and the
    reference's own default run (512^2 x 100 spp x 2 casts, main.cpp:357-361)
    rendered WHOLE, bit-equal to the oracle, both pipelines;
  - the statistical leg of SURVEY §8c on the GPU: the GPU image against an
    independent float64 estimator (tests/independent.py) and against the
    oracle at another seed, per-pixel / block / whole-image z <= 5;
  - the analytic scenes (plane, closed box, emissive box 2 - 2^(1-D)) exactly;
  - the ABI edges ADVICE r1 named: partial spt_hit_info output planes, the
    sample-chunked film path (film_budget_bytes) under both pipelines and
    1-4 streams, and knobs set through spt_config instead of the environment.
"""
import ctypes
import os

import numpy as np
import pytest
import torch

import independent as I
import oracle as O
import sptamd
from sptamd import _lib, backend as B, scenes
from test_parity_tolerance import assert_within_tolerance
from test_statistical import Z_MAX, block_z

pytestmark = pytest.mark.gpu
THREADS = max(1, len(os.sched_getaffinity(0)))


@pytest.fixture(scope="module")
def mesh():
    return scenes.mitsuba_synth()  # the bench scene (231k triangles), configs[0..3]'s stand-in


@pytest.fixture(scope="module")
def gscene(mesh):
    s = sptamd.Scene()
    s.add_arrays(mesh)
    s.commit(0)
    return s


@pytest.fixture(scope="module")
def oscene(mesh):
    return O.OracleScene(mesh)


def render(scene, w, h, spp, depth, **kw):
    film, st = scene.render(sptamd.make_params(w, h, spp, depth, **kw))
    torch.cuda.synchronize()
    return film.cpu().numpy(), st


PIPELINES = ["wavefront", "fused", "percast"]  # percast: the wavefront with no drain (spt_config.drain_q8 = 0)


def pipeline_kw(pipeline, monkeypatch):
    if pipeline == "percast":
        monkeypatch.setenv("SPT_DRAIN_Q8", "0")
        return "wavefront"
    return pipeline


@pytest.mark.parametrize("pipeline", PIPELINES)
def test_config0_whole_image_bitexact(gscene, oscene, pipeline, monkeypatch):
    """BASELINE configs[0]: 256 x 256, 4 spp, max depth 4 — every pixel."""
    got, st = render(gscene, 256, 256, 4, 4, pipeline=pipeline_kw(pipeline, monkeypatch))
    if pipeline == "percast":
        assert st["drained_paths"] == 0 and st["drain_launches"] == 0
    elif pipeline == "wavefront":  # 262k paths: below the drain threshold from the start, all drained
        assert st["drained_paths"] == st["paths"] and st["drained_casts"] == st["ray_casts"]
    ref, casts = oscene.render(O.reference_params(256, 256, 4, 4), nthreads=THREADS)
    np.testing.assert_array_equal(got, ref)
    assert st["ray_casts"] == casts and st["paths"] == 256 * 256 * 4
    # and inside SURVEY §8c's tolerance of the oracle with every unpinned
    # arithmetic choice swapped at once (tests/test_parity_tolerance.py)
    alt, _ = O.OracleScene(gscene.mesh, lib=O.variant("all")).render(O.reference_params(256, 256, 4, 4),
                                                                      nthreads=THREADS)
    assert_within_tolerance(got, alt, 4, "gpu vs oracle(all variants)")


@pytest.mark.parametrize("pipeline", PIPELINES)
def test_reference_default_whole_image_bitexact(gscene, oscene, pipeline, monkeypatch):
    """The reference's hard-coded run, main.cpp:357-361: 512^2 x 100 spp x 2 casts."""
    p = sptamd.default_params()
    assert (p.width, p.height, p.spp, p.max_depth) == (512, 512, 100, 2)
    got, st = render(gscene, 512, 512, 100, 2, pipeline=pipeline_kw(pipeline, monkeypatch))
    ref, casts = oscene.render(O.reference_params(512, 512, 100, 2), nthreads=THREADS)
    np.testing.assert_array_equal(got, ref)
    assert st["ray_casts"] == casts


@pytest.fixture(scope="module")
def stat():
    m = I.stat_scene()
    s = sptamd.Scene()
    s.add_arrays(m)
    s.commit(0)
    return m, s


def test_statistical_gpu_vs_independent_estimator(stat):
    """Escape-fraction image (the reference's semantics): the GPU at 1024 spp
    against the float64 estimator at 256 spp and against the oracle at another
    seed; per-pixel and whole-image two-sample z <= 5."""
    m, s = stat
    cam = B.reference_camera()
    W = H = 32
    got, _ = render(s, W, H, 1024, 4)
    ref = I.render(m, W, H, 256, 4, cam, seed=21)
    assert 0.3 < got[0].mean() < 0.95
    z, zmean = I.bernoulli_z(got[0], ref[0], 1024, 256)
    assert z.max() <= Z_MAX and zmean <= Z_MAX, (z.max(), zmean)
    other, _ = O.OracleScene(m).render(O.reference_params(W, H, 256, 4, rng_initstate=0xC0FFEE), nthreads=THREADS)
    z2, zmean2 = I.bernoulli_z(got[0], other[0], 1024, 256)
    assert z2.max() <= Z_MAX and zmean2 <= Z_MAX, (z2.max(), zmean2)
    # a second GPU seed is a different image (the seed reaches the kernels)
    got2, _ = render(s, W, H, 1024, 4, rng_initstate=0xC0FFEE)
    assert not np.array_equal(got, got2)


def test_statistical_gpu_emitters(stat):
    """Albedo, an emitter, a coloured sky and roulette: block / image z <= 5."""
    m, s = stat
    albedo = np.array([[1, 1, 1], [0.7, 0.6, 0.5], [0.9, 0.2, 0.2], [0.3, 0.8, 0.3], [0.5, 0.5, 0.9]], np.float32)
    emission = np.zeros((5, 3), np.float32)
    emission[4] = (2.0, 1.5, 0.5)
    env = (0.2, 0.3, 0.4)
    s2 = sptamd.Scene()
    s2.add_arrays(m)
    s2.commit(0)
    s2.backend.set_albedo(albedo)
    s2.backend.set_emission(emission)
    W = H = 24
    got, _ = render(s2, W, H, 256, 6, rr_start_depth=2, env=env)
    mean_b, per_b = I.render(m, W, H, 256, 6, B.reference_camera(), env=env, albedo=albedo, emission=emission,
                             rr_start_depth=2, seed=5, samples=True)
    z, zimg = block_z(got.astype(np.float64), mean_b, per_b)
    assert z.max() <= Z_MAX and zimg.max() <= Z_MAX, (z.max(), zimg)


def _gpu_scene(mesh, albedo=None, emission=None):
    s = sptamd.Scene()
    s.add_arrays(mesh)
    s.commit(0)
    if albedo is not None:
        s.backend.set_albedo(albedo)
    if emission is not None:
        s.backend.set_emission(emission)
    return s


def _box():
    c = np.array([[x, y, z] for x in (-20, 20) for y in (-20, 20) for z in (-20, 20)], np.float32)
    quads = [(0, 1, 3, 2), (4, 6, 7, 5), (0, 4, 5, 1), (2, 3, 7, 6), (0, 2, 6, 4), (1, 5, 7, 3)]
    tris = np.array([t for a, b, cc, d in quads for t in ((a, b, cc), (a, cc, d))], np.int32)
    nrm = np.array([[1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1]], np.float32)
    nt = np.repeat(np.arange(6, dtype=np.int32), 2)[:, None].repeat(3, 1)
    return {"pos": c, "pos_tri": tris, "nrm": nrm, "nrm_tri": nt, "mat_id": np.ones(12, np.int32)}


@pytest.mark.parametrize("pipeline", ["wavefront", "fused"])
def test_analytic_scenes(pipeline):
    """tests/test_oracle.py's analytic cases, on the GPU, exactly."""
    plane = {"pos": np.array([[-100, -1, -100], [100, -1, -100], [100, -1, 100], [-100, -1, 100]], np.float32),
             "pos_tri": np.array([[0, 1, 2], [0, 2, 3]], np.int32), "nrm": np.array([[0, 1, 0]], np.float32),
             "nrm_tri": np.zeros((2, 3), np.int32)}
    s = _gpu_scene(plane)
    f1, st1 = render(s, 24, 24, 3, 1, pipeline=pipeline)
    assert np.all(f1 == 0.0) and st1["ray_casts"] == 24 * 24 * 3        # one cast: nothing escapes
    f3, st3 = render(s, 24, 24, 3, 3, pipeline=pipeline)
    assert np.all(f3 == 1.0) and st3["ray_casts"] == 2 * 24 * 24 * 3    # the bounce always escapes
    box = _box()
    f, st = render(_gpu_scene(box), 16, 16, 2, 5, pipeline=pipeline)
    assert np.all(f == 0.0) and st["ray_casts"] == 16 * 16 * 2 * 5      # closed: nothing escapes
    # every wall emits 1 with albedo 1/2: each sample gathers 1 + 1/2 + ... + 2^(1-D)
    e = _gpu_scene(box, albedo=[[1, 1, 1], [0.5, 0.5, 0.5]], emission=[[0, 0, 0], [1, 1, 1]])
    for depth in (1, 4, 7):
        f, st = render(e, 12, 10, 3, depth, rr_start_depth=depth, pipeline=pipeline)
        assert st["ray_casts"] == 12 * 10 * 3 * depth
        assert np.all(f == np.float32(2.0 - 2.0 ** (1 - depth))), depth


def test_hit_info_partial_output_planes():
    """each spt_hit_info plane may be NULL on its own."""
    m = scenes.mitsuba_synth(detail=0.25)
    b = sptamd.HipBackend()
    b.init(0)
    b.set_triangles_soup(m["pos_tri"], m["pos"], m["nrm_tri"], m["nrm"], None, None, m["mat_id"])
    rng = np.random.default_rng(4)
    n = 5000
    o = np.repeat(np.array([[0.0], [3.03], [5.0]], np.float32), n, 1)
    d = rng.normal(size=(3, n)).astype(np.float32)
    d[1] = -np.abs(d[1])
    rays = sptamd.Ray3.make(o, d)
    full, active = b.intersect(rays)
    torch.cuda.synchronize()
    hits = _lib.Hits(full.tri_id.data_ptr(), full.t.data_ptr(), full.barycentric[0].data_ptr(),
                     full.barycentric[1].data_ptr())
    names = [f for f, _ in _lib.HitInfo._fields_]
    planes = {"px": full.position[0], "py": full.position[1], "pz": full.position[2],
              "gnx": full.geometry_normal[0], "gny": full.geometry_normal[1], "gnz": full.geometry_normal[2],
              "snx": full.shading_normal[0], "sny": full.shading_normal[1], "snz": full.shading_normal[2],
              "tcu": full.texcoord[0], "tcv": full.texcoord[1], "mat_id": full.material_id}
    act = active.cpu().numpy()
    for subset in (["px"], ["pz", "gny"], ["snz", "mat_id"], ["tcv"], ["gnx", "sny", "py"]):
        outs = {k: torch.full_like(planes[k], -7) for k in subset}
        info = _lib.HitInfo(*[outs[k].data_ptr() if k in outs else None for k in names])
        rs = rays.c_struct()
        sptamd.check(_lib.lib.spt_hit_info_compute(b.handle, ctypes.byref(rs), ctypes.byref(hits), None, 0, n,
                                                   ctypes.byref(info), None), "spt_hit_info_compute")
        torch.cuda.synchronize()
        for k in subset:
            got = outs[k].cpu().numpy()
            np.testing.assert_array_equal(got[act], planes[k].cpu().numpy()[act])
            assert np.all(got[~act] == -7)          # inactive lanes untouched
    # the rays are needed only for the position: NULL ray planes with px is an error
    bad = _lib.Rays(None, None, None, None, None, None, None, None)
    info = _lib.HitInfo(*[planes["px"].data_ptr() if k == "px" else None for k in names])
    assert _lib.lib.spt_hit_info_compute(b.handle, ctypes.byref(bad), ctypes.byref(hits), None, 0, n,
                                         ctypes.byref(info), None) == 1
    info = _lib.HitInfo(*[planes["snx"].data_ptr() if k == "snx" else None for k in names])
    assert _lib.lib.spt_hit_info_compute(b.handle, ctypes.byref(bad), ctypes.byref(hits), None, 0, n,
                                         ctypes.byref(info), None) == 0
    nohits = _lib.Hits(None, None, None, None)
    assert _lib.lib.spt_hit_info_compute(b.handle, ctypes.byref(rays.c_struct()), ctypes.byref(nohits), None, 0, n,
                                         ctypes.byref(info), None) == 1


@pytest.fixture(scope="module")
def small():
    m = scenes.mitsuba_synth(detail=0.25)
    albedo = np.array([[1.0, 1.0, 1.0], [0.8, 0.6, 0.4], [0.9, 0.3, 0.2], [0.2, 0.2, 0.8], [0.9, 0.9, 0.3],
                       [0.4, 0.4, 0.4]], np.float32)[: len(m["kd"])]
    return m, albedo, O.OracleScene(m, albedo=albedo)


@pytest.mark.parametrize("pipeline", ["wavefront", "fused"])
@pytest.mark.parametrize("streams", [1, 2, 4])
@pytest.mark.parametrize("per_chunk", [1, 2, 3])
@pytest.mark.parametrize("mode", ["unit", "albedo", "emit"])
def test_film_chunking_bitexact(small, pipeline, streams, per_chunk, mode):
    """the sample-chunked path (per-sample film over budget; the
    running sum carried in acc across chunks) with 1-3 samples per chunk,
    both pipelines, 1-4 streams, in every path mode: unit (the reference's
    albedo 1: one escape byte per sample and pixel), albedo (roulette on) and
    emitters (RGB floats) — bit-equal to the oracle."""
    m, albedo, osc = small
    w, h, spp, depth = 40, 30, 7, 5
    film_unit = 1 if mode == "unit" else 12
    cfg = sptamd.default_config()
    cfg.film_budget_bytes = film_unit * w * h * per_chunk
    cfg.streams = streams
    s = sptamd.Scene(config=cfg)
    s.add_arrays(m)
    s.commit(0)
    kw = dict(rr_start_depth=2, env=(0.3, 0.7, 1.0))
    if mode == "unit":
        osc = O.OracleScene(m)
    elif mode == "albedo":
        s.backend.set_albedo(albedo)
    else:
        emi = np.zeros((len(albedo), 3), np.float32)
        emi[1] = (1.5, 0.5, 0.25)
        s.backend.set_albedo(albedo)
        s.backend.set_emission(emi)
        osc = O.OracleScene(m, albedo=albedo, emission=emi)
    assert s.backend.config["film_budget_bytes"] == film_unit * w * h * per_chunk
    got, st = render(s, w, h, spp, depth, pipeline=pipeline, wavefront_paths=1500, **kw)
    ref, casts = osc.render(O.reference_params(w, h, spp, depth, **kw))
    np.testing.assert_array_equal(got, ref)
    assert st["ray_casts"] == casts
    assert st["streams"] == (1 if pipeline == "fused" else streams)


@pytest.mark.parametrize("pipeline", ["wavefront", "fused"])
@pytest.mark.parametrize("block,order,per_chunk", [(0, 0, 0), (1, 1, 0), (3, 1, 0), (4, 0, 0), (8, 1, 0), (64, 0, 0),
                                                   (0, 2, 0), (3, 2, 0), (0, 2, 2), (4, 2, 2), (0, 1, 2), (0, 0, 2)])
def test_work_order_bitexact(small, pipeline, block, order, per_chunk):
    """spt_config.pixel_block (camera paths in B x B pixel blocks) and
    work_order (auto, sample- or pixel-major work items, with 2-sample film
    chunks too) change the order work starts in, never the image: bit-equal to the
    oracle on a tile whose sides are not multiples of B, and on an interleaved
    row tile."""
    m, albedo, osc = small
    w, h, spp, depth = 37, 29, 5, 4
    cfg = sptamd.default_config()
    cfg.pixel_block = block
    cfg.work_order = order
    if per_chunk:
        cfg.film_budget_bytes = 12 * w * h * per_chunk
    s = sptamd.Scene(config=cfg)
    s.add_arrays(m)
    s.commit(0)
    s.backend.set_albedo(albedo)
    got, st = render(s, w, h, spp, depth, pipeline=pipeline, wavefront_paths=1000, rr_start_depth=2)
    ref, casts = osc.render(O.reference_params(w, h, spp, depth, rr_start_depth=2))
    np.testing.assert_array_equal(got, ref)
    assert st["ray_casts"] == casts
    # rank 1 of 3 with 4-row groups: the tile's own (shorter) block rows
    tile, _ = render(s, w, h, spp, depth, pipeline=pipeline, wavefront_paths=1000, rr_start_depth=2,
                     tile_index=1, tile_count=3, rows_per_group=4)
    rows = [r for r in range(h) if (r // 4) % 3 == 1]
    np.testing.assert_array_equal(tile, ref[:, rows, :])
    # unit mode (albedo 1: one escape byte per film slot)
    u = sptamd.Scene(config=cfg)
    u.add_arrays(m)
    u.commit(0)
    got_u, _ = render(u, w, h, spp, depth, pipeline=pipeline, wavefront_paths=1000)
    ref_u, _ = O.OracleScene(m).render(O.reference_params(w, h, spp, depth))
    np.testing.assert_array_equal(got_u, ref_u)


@pytest.mark.parametrize("order", [1, 2])
def test_work_order_stream_shares(small, order):
    """Pixel-major work splits a chunk's samples over the streams (21 samples:
    5 / 5 / 5 / 6), so a stream's share no longer starts at k/K of the chunk's
    work items; the first isect / shade grids must cover the stream's whole
    first refill (a grid sized from k/K once dropped paths)."""
    m, albedo, osc = small
    w, h, spp, depth = 64, 48, 21, 3
    cfg = sptamd.default_config()
    cfg.work_order = order
    cfg.streams = 4
    s = sptamd.Scene(config=cfg)
    s.add_arrays(m)
    s.commit(0)
    s.backend.set_albedo(albedo)
    got, st = render(s, w, h, spp, depth, pipeline="wavefront", wavefront_paths=8000, rr_start_depth=2)
    ref, casts = osc.render(O.reference_params(w, h, spp, depth, rr_start_depth=2))
    np.testing.assert_array_equal(got, ref)
    assert st["ray_casts"] == casts


@pytest.mark.parametrize("cache", [1, 2])
def test_queue_cache_bitexact(small, cache):
    """spt_config.queue_cache (path-queue and hit records through the caches or
    non-temporal) changes cache policy only: every shade mode (albedo +
    roulette, emitters, unit) bit-equal to the oracle, and the stats name the
    policy that ran."""
    m, albedo, osc = small
    w, h, spp, depth = 40, 30, 6, 4
    cfg = sptamd.default_config()
    cfg.queue_cache = cache
    cfg.streams = 2
    s = sptamd.Scene(config=cfg)
    s.add_arrays(m)
    s.commit(0)
    s.backend.set_albedo(albedo)
    got, st = render(s, w, h, spp, depth, pipeline="wavefront", wavefront_paths=3000, rr_start_depth=2)
    ref, casts = osc.render(O.reference_params(w, h, spp, depth, rr_start_depth=2))
    np.testing.assert_array_equal(got, ref)
    assert st["ray_casts"] == casts
    assert st["queue_cache"] == cache
    emi = np.zeros_like(albedo)
    emi[1] = (0.5, 0.25, 0.125)
    s.backend.set_emission(emi)
    got_e, _ = render(s, w, h, spp, depth, pipeline="wavefront", wavefront_paths=3000)
    ref_e, _ = O.OracleScene(m, albedo=albedo, emission=emi).render(O.reference_params(w, h, spp, depth))
    np.testing.assert_array_equal(got_e, ref_e)
    u = sptamd.Scene(config=cfg)
    u.add_arrays(m)
    u.commit(0)
    got_u, st_u = render(u, w, h, spp, depth, pipeline="wavefront", wavefront_paths=3000)
    ref_u, _ = O.OracleScene(m).render(O.reference_params(w, h, spp, depth))
    np.testing.assert_array_equal(got_u, ref_u)
    assert st_u["queue_cache"] == cache
    # smallpt spheres with mirror / glass kinds: the kSpt shade instance honours the policy too
    sph = np.array([[0.0, 0.6, 0.0, 0.35]], np.float32)
    kinds = np.zeros(len(albedo), np.uint32)
    kinds[2] = 2
    s.backend.set_spheres(sph, np.array([2], np.int32))
    s.backend.set_material_kinds(kinds)
    got_s, st_s = render(s, w, h, spp, depth, pipeline="wavefront", wavefront_paths=3000)
    ref_s, _ = O.OracleScene(m, albedo=albedo, emission=emi, spheres=sph, sphere_mat=[2], kinds=kinds).render(
        O.reference_params(w, h, spp, depth))
    np.testing.assert_array_equal(got_s, ref_s)
    assert st_s["queue_cache"] == cache
    # AUTO on this small scene (< 256 MiB on the device): cached
    a = sptamd.Scene()
    a.add_arrays(m)
    a.commit(0)
    got_a, st_a = render(a, w, h, spp, depth, pipeline="wavefront", wavefront_paths=3000)
    np.testing.assert_array_equal(got_a, ref_u)
    assert st_a["queue_cache"] == _lib.SPT_QUEUE_CACHE_CACHED
    bad = sptamd.default_config()
    bad.queue_cache = 3
    assert _lib.lib.spt_scene_set_config(a.backend.handle, ctypes.byref(bad)) == 1
    assert b"queue_cache" in _lib.lib.spt_last_error()


def test_config_through_the_abi(small, monkeypatch):
    """Knobs set through spt_config (no environment variable anywhere) change
    scheduling only; invalid values are rejected by spt_scene_set_config."""
    for k in list(os.environ):
        if k.startswith("SPT_"):
            monkeypatch.delenv(k)
    m, albedo, osc = small
    ref, _ = osc.render(O.reference_params(48, 40, 7, 4, rr_start_depth=2))
    for knobs in ({"streams": 3, "isect_chunk": 7, "isect_refill_idle": 1, "xcd_remap": 0},
                  {"streams": 2, "isect_static_share_q8": 255, "isect_grid_q8": 16, "plane_pad": 77},
                  {"pipeline": _lib.SPT_PIPELINE_FUSED, "fused_refill_idle": 64, "fused_static_share_q8": 0},
                  {"pipeline": _lib.SPT_PIPELINE_WAVEFRONT, "wavefront_paths": 999}):
        cfg = sptamd.default_config()
        for k, v in knobs.items():
            setattr(cfg, k, v)
        s = sptamd.Scene(config=cfg)
        s.add_arrays(m)
        s.commit(0)
        s.backend.set_albedo(albedo)
        got, st = render(s, 48, 40, 7, 4, rr_start_depth=2)
        np.testing.assert_array_equal(got, ref)
        if "pipeline" in knobs:
            assert st["fused"] == (knobs["pipeline"] == _lib.SPT_PIPELINE_FUSED)
        if "wavefront_paths" in knobs:
            assert st["paths_in_flight"] == 999
    bad = sptamd.default_config()
    bad.streams = 9
    assert _lib.lib.spt_scene_set_config(s.backend.handle, ctypes.byref(bad)) == 1
    assert b"streams" in _lib.lib.spt_last_error()
    assert s.backend.config["wavefront_paths"] == 999      # the rejected config left the scene's as it was
