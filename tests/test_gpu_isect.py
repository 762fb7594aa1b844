"""GPU parity of spt_intersect / spt_hit_info_compute (the OptiX raygen +
hit-reconstruction boundary, wavefront_isect.cu:80-112, optix_backend.h:422-487)
against the CPU oracle, bit-exact on tri id / t / u / v."""
import numpy as np
import pytest
import torch

import oracle as O
import sptamd
from sptamd import scenes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mesh():
    return scenes.mitsuba_synth(detail=0.25)


@pytest.fixture(scope="module")
def backend(mesh):
    b = sptamd.HipBackend()
    b.init(0)
    b.set_triangles_soup(mesh["pos_tri"], mesh["pos"], mesh["nrm_tri"], mesh["nrm"], None, None, mesh["mat_id"])
    return b


@pytest.fixture(scope="module")
def oracle_bvh(mesh):
    return O.OracleScene(mesh, use_bvh=True)


def random_rays(n, seed, scale_dirs=True):
    rng = np.random.default_rng(seed)
    o = rng.uniform(-2.5, 2.5, size=(3, n)).astype(np.float32)
    o[1] = rng.uniform(-0.9, 3.0, size=n)
    d = rng.normal(size=(3, n)).astype(np.float32)
    if scale_dirs:  # un-normalised directions (the reference's bounce rays are)
        d *= rng.uniform(0.2, 3.0, size=n).astype(np.float32)
    # a block of camera rays and rays starting exactly on vertices
    o[:, : n // 8] = np.array([[0.0], [3.03], [5.0]], np.float32)
    return o, d


def gpu_isect(backend, o, d, tmin=None, tmax=None, mask=None, closest=True):
    rays = sptamd.Ray3.make(o, d)
    if tmin is not None:
        rays.tmin.copy_(torch.as_tensor(tmin))
    if tmax is not None:
        rays.tmax.copy_(torch.as_tensor(tmax))
    tri, t, u, v = backend.intersect_raw(rays, mask=mask, do_closest=closest)
    torch.cuda.synchronize()
    return tri.cpu().numpy(), t.cpu().numpy(), u.cpu().numpy(), v.cpu().numpy()


def assert_hits_equal(got, ref):
    gt, gtt, gu, gv = got
    rt, rtt, ru, rv = ref
    np.testing.assert_array_equal(gt, rt)
    h = rt >= 0
    np.testing.assert_array_equal(gtt[h], rtt[h])
    np.testing.assert_array_equal(gu[h], ru[h])
    np.testing.assert_array_equal(gv[h], rv[h])


def test_closest_hit_matches_oracle_bvh(backend, oracle_bvh):
    o, d = random_rays(200_000, 1)
    assert_hits_equal(gpu_isect(backend, o, d), oracle_bvh.intersect(o, d))


def test_closest_hit_matches_bruteforce():
    m = scenes.mitsuba_synth(detail=0.08)
    b = sptamd.HipBackend()
    b.init(0)
    b.set_triangles_soup(m["pos_tri"], m["pos"], m["nrm_tri"], m["nrm"])
    brute = O.OracleScene(m, use_bvh=False)
    o, d = random_rays(3000, 2)
    ref = brute.intersect(o, d)
    assert (ref[0] >= 0).sum() > 500
    assert_hits_equal(gpu_isect(b, o, d), ref)


def test_interval_bounds(backend, oracle_bvh):
    o, d = random_rays(50_000, 3)
    rng = np.random.default_rng(3)
    tmin = rng.uniform(0.0, 1.0, size=o.shape[1]).astype(np.float32)
    tmax = (tmin + rng.uniform(0.0, 4.0, size=o.shape[1])).astype(np.float32)
    assert_hits_equal(gpu_isect(backend, o, d, tmin, tmax), oracle_bvh.intersect(o, d, tmin, tmax))


def test_anyhit_agrees_on_occlusion(backend, oracle_bvh):
    o, d = random_rays(100_000, 4)
    closest = gpu_isect(backend, o, d)
    anyh = gpu_isect(backend, o, d, closest=False)
    np.testing.assert_array_equal(anyh[0] >= 0, closest[0] >= 0)
    h = anyh[0] >= 0
    assert np.all(anyh[1][h] >= closest[1][h])
    assert np.all((anyh[1][h] >= 0.001) & (anyh[1][h] <= 1e20))


def test_mask_semantics(backend, oracle_bvh):
    o, d = random_rays(10_000, 5)
    n = o.shape[1]
    sentinel = (torch.full((n,), 77, dtype=torch.int32, device="cuda"),
                torch.full((n,), 5.0, device="cuda"), torch.full((n,), 6.0, device="cuda"),
                torch.full((n,), 7.0, device="cuda"))
    rays = sptamd.Ray3.make(o, d)
    backend.intersect_raw(rays, mask=np.zeros(1, np.uint8), out=sentinel)  # broadcast off: nothing written
    torch.cuda.synchronize()
    assert (sentinel[0].cpu().numpy() == 77).all() and (sentinel[1].cpu().numpy() == 5.0).all()
    mask = (np.arange(n) % 3 != 0).astype(np.uint8)
    backend.intersect_raw(rays, mask=mask, out=sentinel)
    torch.cuda.synchronize()
    tri = sentinel[0].cpu().numpy()
    assert (tri[mask == 0] == 77).all()
    ref = oracle_bvh.intersect(o, d, mask=mask, init=[np.full(n, 77, np.int32)] + [np.full(n, x, np.float32)
                                                                                    for x in (5.0, 6.0, 7.0)])
    np.testing.assert_array_equal(tri, ref[0])
    np.testing.assert_array_equal(sentinel[1].cpu().numpy(), ref[1])


def test_empty_scene_and_zero_rays():
    b = sptamd.HipBackend()
    b.init(0)
    b.set_triangles_soup(np.zeros((0, 3), np.int32), np.zeros((0, 3), np.float32))
    o, d = random_rays(1000, 6)
    tri, *_ = gpu_isect(b, o, d)
    assert (tri == -1).all()
    empty = sptamd.Ray3.make(np.zeros((3, 0), np.float32), np.zeros((3, 0), np.float32))
    out = b.intersect_raw(empty)
    assert out[0].numel() == 0


def test_single_triangle_root_leaf():
    pos = np.array([[-1, 0, -1], [1, 0, -1], [0, 0, 1]], np.float32)
    b = sptamd.HipBackend()
    b.init(0)
    b.set_triangles_soup(np.array([[0, 1, 2]], np.int32), pos)
    o = np.array([[0.0, 0.0, 5.0], [1.0, 1.0, 1.0], [0.0, 0.0, 0.0]], np.float32)
    d = np.array([[0.0, 0.0, 0.0], [-1.0, -1.0, -1.0], [0.0, 0.0, 0.0]], np.float32)
    tri, t, u, v = gpu_isect(b, o, d)
    ref = O.OracleScene({"pos_tri": np.array([[0, 1, 2]], np.int32), "pos": pos}, use_bvh=False).intersect(o, d)
    assert_hits_equal((tri, t, u, v), ref)
    assert tri[0] == 0 and tri[2] == -1


def test_hit_info(backend, mesh, oracle_bvh):
    o, d = random_rays(20_000, 7)
    rays = sptamd.Ray3.make(o, d)
    hit, active = backend.intersect(rays)
    torch.cuda.synchronize()
    tri = hit.tri_id.cpu().numpy()
    h = tri >= 0
    t, u, v = hit.t.cpu().numpy(), hit.barycentric[0].cpu().numpy(), hit.barycentric[1].cpu().numpy()
    np.testing.assert_array_equal(active.cpu().numpy(), h)
    p = hit.position.cpu().numpy()
    np.testing.assert_array_equal(p[:, h], (o + t * d)[:, h])  # optix_backend.h:469, float32 ops
    pt, nt, nrm, pos = mesh["pos_tri"], mesh["nrm_tri"], mesh["nrm"], mesh["pos"]
    ids = tri[h]
    w = (np.float32(1.0) - u[h]) - v[h]
    n0, n1, n2 = (nrm[nt[ids, k]].T for k in range(3))
    sn = (w * n0 + u[h] * n1) + v[h] * n2
    np.testing.assert_array_equal(hit.shading_normal.cpu().numpy()[:, h], sn)
    p0, p1, p2 = (pos[pt[ids, k]].T for k in range(3))
    gn = np.cross((p1 - p0).T, (p2 - p0).T).T
    gn = gn / np.linalg.norm(gn, axis=0)
    np.testing.assert_allclose(hit.geometry_normal.cpu().numpy()[:, h], gn, atol=2e-5)
    np.testing.assert_array_equal(hit.material_id.cpu().numpy()[h], mesh["mat_id"][ids])


def grid_mesh(n=16):
    """n x n quads in the plane y = 0, two triangles each, sharing edges."""
    xs = np.linspace(-1.0, 1.0, n + 1, dtype=np.float32)
    gx, gz = np.meshgrid(xs, xs, indexing="ij")
    pos = np.stack([gx.ravel(), np.zeros(gx.size, np.float32), gz.ravel()], 1)
    i = np.arange(n)[:, None] * (n + 1) + np.arange(n)[None, :]
    a, b, c, d = i, i + n + 1, i + n + 2, i + 1
    tris = np.concatenate([np.stack([a, b, c], -1).reshape(-1, 3), np.stack([a, c, d], -1).reshape(-1, 3)])
    return {"pos_tri": tris.astype(np.int32), "pos": pos}


def test_watertight_shared_edges_and_vertices():
    """Rays aimed exactly at shared edges and vertices of a triangle grid hit
    (no cracks: the watertight test, SURVEY §7 hard part 3), with the oracle's
    tie-broken triangle."""
    m = grid_mesh(16)
    b = sptamd.HipBackend()
    b.init(0)
    b.set_triangles_soup(m["pos_tri"], m["pos"])
    pts = m["pos"][np.abs(m["pos"][:, 0]) < 0.99]
    pts = pts[np.abs(pts[:, 2]) < 0.99]                              # interior vertices
    mids = (m["pos"][m["pos_tri"][:, 0]] + m["pos"][m["pos_tri"][:, 2]]) * np.float32(0.5)  # diagonal midpoints
    targets = np.concatenate([pts, mids]).astype(np.float32)
    rng = np.random.default_rng(11)
    o = (targets + rng.normal(size=targets.shape).astype(np.float32) * [0.3, 0.0, 0.3]).astype(np.float32)
    o[:, 1] = rng.uniform(0.5, 3.0, size=len(o))
    d = (targets - o).astype(np.float32).T.copy()
    o = o.T.copy()
    got = gpu_isect(b, o, d)
    ref = O.OracleScene(m, use_bvh=False).intersect(o, d)
    assert_hits_equal(got, ref)
    assert (got[0] >= 0).mean() > 0.99


def test_axis_aligned_and_degenerate_rays(backend, oracle_bvh):
    """Direction components of +0, -0 and tiny magnitude (1/d = inf or huge),
    zero-length and NaN directions: same answers as the oracle, no faults."""
    o, d = random_rays(6000, 12)
    n = o.shape[1]
    d[0, 0::6] = 0.0
    d[1, 1::6] = -0.0
    d[2, 2::6] = 1e-30
    d[:, 3::6] = 0.0                      # zero direction: misses
    d[0, 4::6] = 0.0
    d[2, 4::6] = 0.0                      # straight down/up the y axis
    d[0, 5::6] = np.nan                   # NaN direction: misses
    got = gpu_isect(backend, o, d)
    ref = oracle_bvh.intersect(o, d)
    assert_hits_equal(got, ref)
    assert (got[0][3::6] == -1).all() and (got[0][5::6] == -1).all()
    assert (got[0] >= 0).sum() > n // 10


@pytest.mark.parametrize("refill", ["1", "8", "64"])
def test_persistent_public_kernel(backend, oracle_bvh, monkeypatch, refill):
    """SPT_PUBLIC_PERSISTENT=1 swaps spt_intersect onto the lane-refill kernel;
    results must stay bit-identical to the oracle (closest, any-hit occlusion,
    interval bounds, per-ray and broadcast masks, a ragged ray count)."""
    monkeypatch.setenv("SPT_PUBLIC_PERSISTENT", "1")
    monkeypatch.setenv("SPT_PUBLIC_REFILL_IDLE", refill)
    o, d = random_rays(150_001, 11)
    ref = oracle_bvh.intersect(o, d)
    assert_hits_equal(gpu_isect(backend, o, d), ref)
    anyh = gpu_isect(backend, o, d, closest=False)
    np.testing.assert_array_equal(anyh[0] >= 0, ref[0] >= 0)
    rng = np.random.default_rng(12)
    n = o.shape[1]
    tmin = rng.uniform(0.0, 1.0, size=n).astype(np.float32)
    tmax = (tmin + rng.uniform(0.0, 4.0, size=n)).astype(np.float32)
    assert_hits_equal(gpu_isect(backend, o, d, tmin, tmax), oracle_bvh.intersect(o, d, tmin, tmax))
    rays = sptamd.Ray3.make(o, d)
    init = (77, 5.0, 6.0, 7.0)
    for mask in (np.zeros(1, np.uint8), np.ones(1, np.uint8), (np.arange(n) % 3 != 0).astype(np.uint8)):
        out = (torch.full((n,), 77, dtype=torch.int32, device="cuda"),) + tuple(
            torch.full((n,), x, device="cuda") for x in init[1:])
        backend.intersect_raw(rays, mask=mask, out=out)
        torch.cuda.synchronize()
        full = mask if mask.size == n else np.full(n, mask[0], np.uint8)
        r = oracle_bvh.intersect(o, d, mask=full, init=[np.full(n, 77, np.int32)] +
                                 [np.full(n, x, np.float32) for x in init[1:]])
        got = [g.cpu().numpy() for g in out]
        np.testing.assert_array_equal(got[0], r[0])
        np.testing.assert_array_equal(got[1], r[1])
        h = r[0] >= 0
        np.testing.assert_array_equal(got[2][h], r[2][h])
        np.testing.assert_array_equal(got[3][h], r[3][h])
