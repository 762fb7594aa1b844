"""GPU parity of spt_render (main.cpp:354-429 as a HIP wavefront) against the
CPU oracle.  The reference's image is an escape count per pixel (albedo 1,
sky radiance 1: SURVEY F6), so the film is an exact multiple of 1/spp and the
GPU result must equal the oracle bit for bit.  Non-unit albedo (Russian
roulette active) is bitwise too: every path writes one contribution per
(sample, pixel) and the resolve sums them in sample order, as the reference's
film += ... does (main.cpp:407)."""
import numpy as np
import pytest
import torch

import oracle as O
import sptamd
from conftest import assert_work_complete
from sptamd import scenes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mesh():
    return scenes.mitsuba_synth(detail=0.25)


@pytest.fixture(scope="module")
def gscene(mesh):
    s = sptamd.Scene()
    s.add_arrays(mesh)
    s.commit(0)
    return s


@pytest.fixture(scope="module")
def oscene(mesh):
    return O.OracleScene(mesh)


def gpu_render(gscene, w, h, spp, depth, **kw):
    """Without an explicit pipeline: render with both (wavefront and fused),
    require identical films, return the wavefront's."""
    if "pipeline" not in kw:
        got, st = gpu_render(gscene, w, h, spp, depth, pipeline="wavefront", **kw)
        fused, _ = gpu_render(gscene, w, h, spp, depth, pipeline="fused", **kw)
        np.testing.assert_array_equal(fused, got)
        return got, st
    p = sptamd.make_params(w, h, spp, depth, **kw)
    film, st = gscene.render(p)
    torch.cuda.synchronize()
    if st["paths"]:  # an empty tile returns before choosing a pipeline
        assert st["fused"] == (kw["pipeline"] == "fused")
    assert_work_complete(st, st["tile_rows"], w, spp)  # every render, on the device's own counts
    return film.cpu().numpy(), st


def oracle_render(oscene, w, h, spp, depth, rows=None, nthreads=8, **kw):
    film, casts = oscene.render(O.reference_params(w, h, spp, depth, **kw), rows=rows, nthreads=nthreads)
    return film, casts


@pytest.mark.parametrize("w,h,spp,depth", [(64, 48, 4, 4), (33, 17, 3, 1), (40, 40, 5, 2), (24, 20, 2, 8)])
def test_render_bitexact(gscene, oscene, w, h, spp, depth):
    got, st = gpu_render(gscene, w, h, spp, depth)
    ref, casts = oracle_render(oscene, w, h, spp, depth)
    np.testing.assert_array_equal(got, ref)
    assert st["ray_casts"] == casts            # same number of traced rays
    assert st["paths"] == w * h * spp


def test_render_rng_x_first(gscene, oscene):
    got, _ = gpu_render(gscene, 32, 32, 4, 3, rng_order=1)
    ref, _ = oracle_render(oscene, 32, 32, 4, 3, rng_order=1)
    np.testing.assert_array_equal(got, ref)
    other, _ = gpu_render(gscene, 32, 32, 4, 3, rng_order=0)
    assert not np.array_equal(got, other)


@pytest.mark.parametrize("wf", [1, 64, 1000, 48 * 40 * 7, 10**7])
def test_wavefront_size_invariance(gscene, oscene, wf):
    got, st = gpu_render(gscene, 48, 40, 7, 4, wavefront_paths=wf, pipeline="wavefront")
    ref, _ = oracle_render(oscene, 48, 40, 7, 4)
    np.testing.assert_array_equal(got, ref)
    assert st["paths_in_flight"] == min(wf, 48 * 40 * 7)


@pytest.mark.parametrize("tiles,rpg", [(2, 1), (3, 5), (8, 8), (5, 64)])
def test_tile_partition_invariance(gscene, tiles, rpg):
    w, h = 40, 37
    full, _ = gpu_render(gscene, w, h, 3, 4)
    img = np.zeros_like(full)
    covered = np.zeros(h, bool)
    for t in range(tiles):
        rows = sptamd.tile_rows(h, t, tiles, rpg)
        tile, st = gpu_render(gscene, w, h, 3, 4, tile_index=t, tile_count=tiles, rows_per_group=rpg)
        assert tile.shape == (3, len(rows), w)
        img[:, rows, :] = tile
        assert not covered[rows].any()
        covered[rows] = True
    assert covered.all()
    np.testing.assert_array_equal(img, full)


def test_albedo_and_russian_roulette(mesh):
    s = sptamd.Scene()
    s.add_arrays(mesh)
    s.commit(0)
    albedo = np.array([[1.0, 1.0, 1.0], [0.8, 0.6, 0.4], [0.9, 0.3, 0.2], [0.2, 0.2, 0.8], [0.9, 0.9, 0.3],
                       [0.4, 0.4, 0.4]], np.float32)
    s.backend.set_albedo(albedo)
    osc = O.OracleScene(mesh, albedo=albedo)
    got, st = gpu_render(s, 40, 30, 6, 6, rr_start_depth=2)
    ref, casts = oracle_render(osc, 40, 30, 6, 6, rr_start_depth=2)
    np.testing.assert_array_equal(got, ref)
    assert st["ray_casts"] == casts
    # a small wavefront: many refills, same per-sample summation order, same bits
    got3, _ = gpu_render(s, 40, 30, 6, 6, wavefront_paths=500, rr_start_depth=2)
    np.testing.assert_array_equal(got3, ref)
    # roulette disabled = the reference estimator (no RR): still exact
    got_norr, _ = gpu_render(s, 40, 30, 6, 6, rr_start_depth=99)
    ref_norr, _ = oracle_render(osc, 40, 30, 6, 6, rr_start_depth=99)
    np.testing.assert_array_equal(got_norr, ref_norr)


def test_env_radiance(gscene, oscene):
    got, _ = gpu_render(gscene, 20, 20, 2, 3, env=(0.5, 1.0, 2.0))
    ref, _ = oracle_render(oscene, 20, 20, 2, 3, env=(0.5, 1.0, 2.0))
    np.testing.assert_array_equal(got, ref)


# BASELINE configs[1] itself (the bench's 231k-triangle scene, whole image,
# both pipelines): tests/test_gpu_configs.py::test_config1_headline_whole_image


def test_gpu_matches_committed_golden():
    """GPU vs the committed oracle vectors (tests/golden/oracle_small.npz)."""
    import os
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "oracle_small.npz"))
    m = scenes.mitsuba_synth(detail=0.1)
    s = sptamd.Scene()
    s.add_arrays(m)
    s.commit(0)
    np.testing.assert_array_equal(gpu_render(s, 32, 24, 4, 4)[0], g["film_32x24_4spp_d4"])
    np.testing.assert_array_equal(gpu_render(s, 32, 24, 4, 4, rng_order=1)[0], g["film_32x24_4spp_d4_xfirst"])
    np.testing.assert_array_equal(gpu_render(s, 16, 16, 100, 2)[0], g["film_16x16_100spp_d2"])
    rays = sptamd.Ray3.make(g["isect_o"], g["isect_d"])
    tri, t, u, v = s.backend.intersect_raw(rays)
    torch.cuda.synchronize()
    tri = tri.cpu().numpy()
    np.testing.assert_array_equal(tri, g["isect_tri"])
    h = tri >= 0
    np.testing.assert_array_equal(t.cpu().numpy()[h], g["isect_t"][h])
    s.backend.set_albedo(g["albedo"])
    np.testing.assert_array_equal(gpu_render(s, 20, 16, 6, 6, rr_start_depth=2)[0], g["film_albedo_rr2"])


@pytest.fixture(scope="module")
def cornell():
    """smallpt's Cornell box (BASELINE config 3): Kd albedo, Ke = 12 light, black sky."""
    m = scenes.cornell_spheres(detail=0.25)
    alb, emi = scenes.smallpt_materials(m)
    s = sptamd.Scene()
    s.add_arrays(m)
    s.commit(0)
    s.backend.set_albedo(alb)
    s.backend.set_emission(emi)
    return s, O.OracleScene(m, albedo=alb, emission=emi)


@pytest.mark.parametrize("wavefront", [0, 777])
def test_cornell_emission_bitexact(cornell, wavefront):
    """Emitters: each path carries its gathered radiance and writes it once per
    (sample, pixel); the last cast is a closest hit (it must see the light)."""
    s, osc = cornell
    kw = dict(camera=scenes.cornell_camera(), rr_start_depth=5, env=(0.0, 0.0, 0.0))
    got, st = gpu_render(s, 48, 40, 8, 10, wavefront_paths=wavefront, **kw)
    ref, casts = oracle_render(osc, 48, 40, 8, 10, **kw)
    np.testing.assert_array_equal(got, ref)
    assert st["ray_casts"] == casts
    assert got.max() >= 12.0 / 8  # the light is in view


def test_emission_with_sky_and_albedo(mesh):
    """Emitters, non-unit albedo, roulette and a coloured sky together."""
    s = sptamd.Scene()
    s.add_arrays(mesh)
    s.commit(0)
    nm = len(mesh["kd"])
    albedo = np.full((nm, 3), 0.7, np.float32)
    emi = np.zeros((nm, 3), np.float32)
    emi[1] = (2.0, 1.0, 0.5)
    emi[nm - 1] = (0.0, 0.3, 3.0)
    s.backend.set_albedo(albedo)
    s.backend.set_emission(emi)
    osc = O.OracleScene(mesh, albedo=albedo, emission=emi)
    kw = dict(rr_start_depth=3, env=(0.5, 0.75, 1.0))
    got, st = gpu_render(s, 40, 30, 6, 7, **kw)
    ref, casts = oracle_render(osc, 40, 30, 6, 7, **kw)
    np.testing.assert_array_equal(got, ref)
    assert st["ray_casts"] == casts
    # clearing the emission table restores the any-hit last cast and the plain image
    s.backend.set_emission(np.zeros((nm, 3), np.float32))
    got0, _ = gpu_render(s, 40, 30, 6, 7, **kw)
    ref0, _ = oracle_render(O.OracleScene(mesh, albedo=albedo), 40, 30, 6, 7, **kw)
    np.testing.assert_array_equal(got0, ref0)


def test_city_scene_bitexact():
    """The config-5 generator (10M-triangle courtyard) at 300k triangles: a
    deeper, wider BVH8 than mitsuba_synth, same bits as the oracle."""
    m = scenes.city_synth(300_000)
    s = sptamd.Scene()
    s.add_arrays(m)
    s.commit(0)
    osc = O.OracleScene(m)
    cam = scenes.city_camera()
    got, st = gpu_render(s, 64, 36, 4, 8, camera=cam)
    ref, casts = oracle_render(osc, 64, 36, 4, 8, camera=cam)
    np.testing.assert_array_equal(got, ref)
    assert st["ray_casts"] == casts
    assert 0.0 < got.mean() < 1.0


@pytest.mark.parametrize("pipeline", ["fused", "wavefront"])
@pytest.mark.parametrize("w,h,spp,depth,rr", [(64, 48, 4, 4, 99), (40, 30, 6, 6, 2), (33, 17, 3, 1, 99)])
def test_pipelines_bitexact(mesh, pipeline, w, h, spp, depth, rr):
    """The fused persistent kernel (trace + shade + new paths in one launch)
    and the wavefront kernels give the oracle's image bit for bit."""
    s = sptamd.Scene()
    s.add_arrays(mesh)
    s.commit(0)
    albedo = np.array([[1.0, 1.0, 1.0], [0.8, 0.6, 0.4], [0.9, 0.3, 0.2], [0.2, 0.2, 0.8], [0.9, 0.9, 0.3],
                       [0.4, 0.4, 0.4]], np.float32)[: len(mesh["kd"])]
    s.backend.set_albedo(albedo)
    osc = O.OracleScene(mesh, albedo=albedo)
    got, st = gpu_render(s, w, h, spp, depth, rr_start_depth=rr, pipeline=pipeline)
    ref, casts = oracle_render(osc, w, h, spp, depth, rr_start_depth=rr)
    np.testing.assert_array_equal(got, ref)
    assert st["ray_casts"] == casts
    assert st["paths"] == w * h * spp


def test_fused_emission_and_tiles(cornell):
    s, osc = cornell
    kw = dict(camera=scenes.cornell_camera(), rr_start_depth=5, env=(0.0, 0.0, 0.0))
    got, _ = gpu_render(s, 48, 40, 8, 10, pipeline="fused", **kw)
    ref, _ = oracle_render(osc, 48, 40, 8, 10, **kw)
    np.testing.assert_array_equal(got, ref)
    # a 3-way tile split of the same image, fused
    img = np.zeros_like(ref)
    for t in range(3):
        rows = sptamd.tile_rows(40, t, 3, 4)
        tile, _ = gpu_render(s, 48, 40, 8, 10, tile_index=t, tile_count=3, rows_per_group=4, pipeline="fused", **kw)
        img[:, rows, :] = tile
    np.testing.assert_array_equal(img, ref)


@pytest.mark.parametrize("env", [
    {"SPT_STATIC_SHARE_Q8": "0", "SPT_REFILL_IDLE": "1"},
    {"SPT_STATIC_SHARE_Q8": "255", "SPT_REFILL_IDLE": "64", "SPT_CHUNK": "1"},
    {"SPT_STREAMS": "3", "SPT_ISECT_GRID_Q8": "16", "SPT_XCD": "0"},
    {"SPT_FUSED_STATIC_SHARE_Q8": "255", "SPT_FUSED_IDLE": "1"},
    {"SPT_FUSED_STATIC_SHARE_Q8": "0", "SPT_FUSED_IDLE": "64", "SPT_CHUNK": "7", "SPT_FUSED_GRID_Q8": "8"},
])
def test_scheduling_knobs_invariance(gscene, oscene, monkeypatch, env):
    """The work-distribution knobs (static/dynamic shares, refill thresholds,
    stream count, grid sizes) change only which lane traces which path: both
    pipelines must still produce the oracle's film bit for bit."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    got, st = gpu_render(gscene, 48, 40, 7, 4, wavefront_paths=3000)
    ref, casts = oracle_render(oscene, 48, 40, 7, 4)
    np.testing.assert_array_equal(got, ref)
    assert st["ray_casts"] == casts


def test_render_async_queue(gscene, oscene):
    """spt_render_async / spt_render_wait: renders queued back to back (both
    pipelines, different sizes, into different films) give the same images and
    work accounting as the synchronous call, in any collection order; a ticket
    is collected once; an empty tile queues nothing."""
    jobs = [(48, 40, 7, 4, "wavefront"), (32, 24, 4, 3, "fused"), (40, 40, 5, 2, "wavefront")]
    queued = []
    for w, h, spp, depth, pipe in jobs:
        film, ticket = gscene.render_async(sptamd.make_params(w, h, spp, depth, pipeline=pipe))
        queued.append((film, ticket))
    for (w, h, spp, depth, pipe), (film, ticket) in reversed(list(zip(jobs, queued))):
        st = gscene.render_wait(ticket)
        assert_work_complete(st, h, w, spp)
        assert st["fused"] == (pipe == "fused")
        ref, casts = oracle_render(oscene, w, h, spp, depth)
        np.testing.assert_array_equal(film.cpu().numpy(), ref)
        assert st["ray_casts"] == casts
        with pytest.raises(sptamd.SptError):
            gscene.render_wait(ticket)
    # an empty tile (tile 5 of 6 with 8-row groups of a 16-row image)
    _, t = gscene.render_async(sptamd.make_params(16, 16, 2, 2, tile_index=5, tile_count=6, rows_per_group=8))
    st = gscene.render_wait(t)
    assert st["tile_rows"] == 0 and st["paths"] == 0


def test_render_async_limit(gscene):
    """At most 64 renders queued without being collected: the 65th is refused
    (SPT_ERR_LIMIT) and nothing is lost — every queued one still collects."""
    p = sptamd.make_params(8, 8, 1, 1)
    film = torch.empty((3, 8, 8), dtype=torch.float32, device="cuda")
    tickets = [gscene.render_async(p, film=film)[1] for _ in range(64)]
    with pytest.raises(sptamd.SptError) as e:
        gscene.render_async(p, film=film)
    assert e.value.code == sptamd._lib.SPT_ERR_LIMIT
    for t in tickets:
        assert gscene.render_wait(t)["paths"] == 64


def test_render_async_two_streams(gscene, oscene):
    """Renders queued on two streams take the working set bound to their
    stream and may overlap on the GPU; each waits for the last render of its
    set, so back-to-back renders of different sizes and pipelines on two
    streams give the oracle's images bit for bit."""
    jobs = [(48, 40, 7, 4, "wavefront"), (32, 24, 4, 3, "fused"), (40, 40, 5, 2, "fused"), (24, 20, 2, 8, "wavefront"),
            (33, 17, 3, 1, "fused")]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    queued = []
    for i, (w, h, spp, depth, pipe) in enumerate(jobs):
        film, ticket = gscene.render_async(sptamd.make_params(w, h, spp, depth, pipeline=pipe),
                                           stream=streams[(i // 2) % 2])  # sets and streams out of phase
        queued.append((film, ticket))
    torch.cuda.synchronize()
    for (w, h, spp, depth, pipe), (film, ticket) in zip(jobs, queued):
        st = gscene.render_wait(ticket)
        assert_work_complete(st, h, w, spp)
        ref, _ = oracle_render(oscene, w, h, spp, depth)
        np.testing.assert_array_equal(film.cpu().numpy(), ref)


def test_render_async_three_streams(gscene, oscene):
    """A third caller stream takes over the least recently used working set
    (Workspace::pick_set): renders cycling over three streams, and the null
    stream between them, still give the oracle's images and complete work."""
    jobs = [(40, 32, 3, 4, "wavefront"), (24, 24, 2, 3, "wavefront"), (32, 16, 4, 2, "fused"), (40, 32, 3, 4, "wavefront"),
            (16, 40, 2, 5, "wavefront"), (24, 24, 2, 3, "fused"), (32, 16, 4, 2, "wavefront")]
    streams = [torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()]
    queued = []
    for i, (w, h, spp, depth, pipe) in enumerate(jobs):
        s = None if i == 4 else streams[i % 3]
        film, ticket = gscene.render_async(sptamd.make_params(w, h, spp, depth, pipeline=pipe), stream=s)
        queued.append((film, ticket))
    for (w, h, spp, depth, pipe), (film, ticket) in zip(jobs, queued):
        st = gscene.render_wait(ticket)
        assert_work_complete(st, h, w, spp)
        ref, _ = oracle_render(oscene, w, h, spp, depth)
        np.testing.assert_array_equal(film.cpu().numpy(), ref)
