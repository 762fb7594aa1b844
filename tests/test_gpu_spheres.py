"""smallpt's analytic spheres and mirror / glass materials (SURVEY §8f row 3:
the smallpt semantics the reference's own scenes drop — smallpt.cpp's
Sphere::intersect and radiance() SPEC / REFR branches) on the GPU, bit-equal to
the oracle: whole images in both pipelines (with emitters, roulette, a diffuse
sphere seen from inside and outside, total internal reflection in the glass
ball), the public intersect / hit-info boundary (sphere ids -2 - k), and the
API's argument checks."""
import numpy as np
import pytest
import torch

import oracle as O
import sptamd
from sptamd import _lib, scenes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mesh():
    return scenes.smallpt_analytic(detail=0.5)


def gscene(mesh, config=None, **over):
    m = dict(mesh, **over)
    s = sptamd.Scene(config=config)
    s.add_arrays(m)
    s.commit(0)
    alb, emi = scenes.smallpt_materials(m)
    s.backend.set_albedo(alb)
    s.backend.set_emission(emi)
    return s


def render(s, w, h, spp, depth, **kw):
    film, st = s.render(sptamd.make_params(w, h, spp, depth, camera=scenes.cornell_camera(), **kw))
    torch.cuda.synchronize()
    return film.cpu().numpy(), st


def oracle_render(m, w, h, spp, depth, **kw):
    alb, emi = scenes.smallpt_materials(m)
    return O.OracleScene(m, albedo=alb, emission=emi).render(
        O.reference_params(w, h, spp, depth, camera=scenes.cornell_camera(), **kw))


@pytest.mark.parametrize("pipeline", ["wavefront", "fused"])
@pytest.mark.parametrize("rr", [3, 99])
def test_smallpt_scene_bitexact(mesh, pipeline, rr):
    kw = dict(rr_start_depth=rr, env=(0.0, 0.0, 0.0))
    s = gscene(mesh)
    got, st = render(s, 64, 48, 8, 8, pipeline=pipeline, **kw)
    ref, casts = oracle_render(mesh, 64, 48, 8, 8, **kw)
    np.testing.assert_array_equal(got, ref)
    assert st["ray_casts"] == casts
    assert ref.mean() > 0.05          # the light sphere is seen


@pytest.mark.parametrize("idle", [0, 1, 24, 64])
def test_smallpt_drain_refill_idle(mesh, idle, monkeypatch):
    """spt_config.drain_refill_idle on smallpt's scene (analytic spheres:
    AUTO picks 56): when a drain wave refills changes only the
    order of the work, not the bits."""
    monkeypatch.delenv("SPT_DRAIN_IDLE", raising=False)
    cfg = sptamd.default_config()
    cfg.drain_refill_idle = idle
    kw = dict(rr_start_depth=3, env=(0.0, 0.0, 0.0))
    got, st = render(gscene(mesh, config=cfg), 64, 48, 8, 8, pipeline="wavefront", **kw)
    ref, casts = oracle_render(mesh, 64, 48, 8, 8, **kw)
    np.testing.assert_array_equal(got, ref)
    assert st["ray_casts"] == casts and st["drained_paths"] > 0
    assert st["drain_refill_idle"] == (idle or 56)


def test_spheres_diffuse_and_sky_small_queue(mesh):
    """Every sphere diffuse (smallpt's nl flip; the light sphere is seen from
    inside by rays that leave through the box top), a coloured sky, a queue
    smaller than the image (chunked wavefront)."""
    kinds = np.zeros_like(mesh["kinds"])
    m = dict(mesh, kinds=kinds)
    kw = dict(rr_start_depth=2, env=(0.3, 0.2, 0.1))
    s = gscene(m)
    got, _ = render(s, 40, 30, 6, 7, pipeline="wavefront", wavefront_paths=700, **kw)
    ref, _ = oracle_render(m, 40, 30, 6, 7, **kw)
    np.testing.assert_array_equal(got, ref)
    ref_glass, _ = oracle_render(mesh, 40, 30, 6, 7, **kw)
    assert not np.array_equal(ref, ref_glass)   # the kinds matter


def test_glass_triangles_and_mirror_triangles(mesh):
    """Mirror / glass kinds on triangle materials (normalised interpolated
    shading normal) next to the analytic spheres."""
    kinds = mesh["kinds"].copy()
    kinds[1] = _lib.SPT_MAT_MIRROR        # left wall
    kinds[3] = _lib.SPT_MAT_GLASS         # back wall and floor
    m = dict(mesh, kinds=kinds)
    kw = dict(rr_start_depth=4, env=(0.1, 0.1, 0.1))
    for pipeline in ("wavefront", "fused"):
        s = gscene(m)
        got, _ = render(s, 48, 36, 4, 9, pipeline=pipeline, **kw)
        ref, _ = oracle_render(m, 48, 36, 4, 9, **kw)
        np.testing.assert_array_equal(got, ref)


def test_unit_albedo_with_spheres_uses_general_path(mesh):
    """No albedo table, no emission: the reference's unit-albedo case, but with
    spheres in the scene (not the unit fast path)."""
    s = sptamd.Scene()
    s.add_arrays(mesh)
    s.commit(0)
    got, _ = render(s, 32, 24, 4, 4)
    ref, _ = O.OracleScene(mesh).render(O.reference_params(32, 24, 4, 4, camera=scenes.cornell_camera()))
    np.testing.assert_array_equal(got, ref)
    s.backend.set_spheres(None)            # removing the spheres restores the triangle-only scene
    s.backend.set_material_kinds(np.zeros(len(mesh["kd"]), np.uint32))
    got0, _ = render(s, 32, 24, 4, 4)
    m0 = {k: v for k, v in mesh.items() if k not in ("spheres", "sphere_mat", "kinds")}
    ref0, _ = O.OracleScene(m0).render(O.reference_params(32, 24, 4, 4, camera=scenes.cornell_camera()))
    np.testing.assert_array_equal(got0, ref0)


def test_intersect_and_hit_info_with_spheres(mesh):
    s = gscene(mesh)
    rng = np.random.default_rng(5)
    n = 50_000
    o = np.stack([rng.uniform(0.05, 0.95, n), rng.uniform(0.02, 0.8, n), rng.uniform(0.05, 2.5, n)]).astype(np.float32)
    d = rng.normal(size=(3, n)).astype(np.float32)
    rays = sptamd.Ray3.make(o, d)
    tri, t, u, v = s.backend.intersect_raw(rays)
    torch.cuda.synchronize()
    ref = O.OracleScene(mesh).intersect(o, d)
    np.testing.assert_array_equal(tri.cpu().numpy(), ref[0])
    h = ref[0] != -1
    assert (ref[0] < -1).sum() > 1000
    for g, r in zip((t, u, v), ref[1:]):
        np.testing.assert_array_equal(g.cpu().numpy()[h], r[h])
    # any-hit: the same hit / miss answer
    tri_a, *_ = s.backend.intersect_raw(rays, do_closest=False)
    np.testing.assert_array_equal(tri_a.cpu().numpy() != -1, h)
    # hit info on sphere hits: p = o + t d, n = normalize(p - c), the sphere's material
    hit, active = s.backend.intersect(rays)
    torch.cuda.synchronize()
    ids = hit.tri_id.cpu().numpy()
    sel = ids < -1
    k = -2 - ids[sel]
    sph = mesh["spheres"][k]
    tt = ref[1][sel]
    p = np.stack([o[i][sel] + tt * d[i][sel] for i in range(3)]).astype(np.float32)
    np.testing.assert_array_equal(hit.position.cpu().numpy()[:, sel], p)
    q = (p - sph[:, :3].T).astype(np.float32)
    nn = q * (np.float32(1.0) / np.sqrt(((q[0] * q[0] + q[1] * q[1]) + q[2] * q[2]).astype(np.float32)))
    np.testing.assert_allclose(hit.shading_normal.cpu().numpy()[:, sel], nn, rtol=0, atol=2e-7)
    np.testing.assert_array_equal(hit.material_id.cpu().numpy()[sel], mesh["sphere_mat"][k])


def test_sphere_api_errors(mesh):
    s = gscene(mesh)
    b = s.backend
    with pytest.raises(sptamd.SptError):
        b.set_spheres(np.array([[0, 0, 0, 0.0]], np.float32))          # radius 0
    with pytest.raises(sptamd.SptError):
        b.set_spheres(np.array([[0, 0, np.nan, 1.0]], np.float32))     # non-finite
    with pytest.raises(sptamd.SptError):
        b.set_spheres(np.tile(np.array([[0, 0, 0, 1.0]], np.float32), (257, 1)))  # more than 256
    with pytest.raises(sptamd.SptError):
        b.set_material_kinds(np.array([0, 3], np.uint32))              # unknown kind
