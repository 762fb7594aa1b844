"""Scene mutators while renders are still queued: renders
queued with spt_render_async capture the scene's device arrays when they are
queued; spt_scene_set_albedo / set_emission / set_texture / set_spheres /
set_material_kinds free and replace those arrays.  The mutators wait for every
queued render of both working sets and for the last public call on every
stream (capi.cpp quiesce_scene) before they free anything, so each render
equals the oracle for the materials it was queued with, and a ray cast queued
before set_spheres still sees the old spheres."""
import numpy as np
import pytest
import torch

import oracle as O
import sptamd
from sptamd import scenes

pytestmark = pytest.mark.gpu

W, H, SPP, D = 48, 40, 4, 6


@pytest.fixture(scope="module")
def mesh():
    return scenes.with_planar_uv(scenes.mitsuba_synth(detail=0.25))


def test_mutators_wait_for_queued_renders(mesh):
    nm = len(mesh["kd"])
    rng = np.random.default_rng(11)
    alb = [rng.uniform(0.3, 0.95, size=(nm, 3)).astype(np.float32) for _ in range(3)]
    emi = np.zeros((nm, 3), np.float32)
    emi[4] = (2.0, 1.5, 1.0)
    tex = scenes.checker(8, 8, cell=1)
    sph = np.array([[0.0, 0.6, 0.0, 0.35], [0.7, 0.3, 0.4, 0.2]], np.float32)
    kw = dict(rr_start_depth=3, env=(1.0, 0.9, 0.8))
    p = sptamd.make_params(W, H, SPP, D, **kw)

    s = sptamd.Scene()
    s.add_arrays(mesh)
    s.commit(0)
    be = s.backend
    streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
    # each state: (albedo, emission, textures, spheres, kinds) as the render sees it
    states, tickets, films = [], [], []

    def queue(state):
        f = torch.empty((3, H, W), dtype=torch.float32, device="cuda")
        _, t = s.render_async(p, film=f, stream=streams[len(tickets) % 2])
        states.append(state)
        tickets.append(t)
        films.append(f)

    be.set_albedo(alb[0])
    queue((alb[0], None, {}, None, None))
    queue((alb[0], None, {}, None, None))
    be.set_albedo(alb[1])                          # renders 0 and 1 may still be running
    be.set_emission(emi)
    queue((alb[1], emi, {}, None, None))
    be.set_texture(1, tex)
    queue((alb[1], emi, {1: tex}, None, None))
    be.set_spheres(sph, np.array([2, 3], np.int32))
    kinds = np.zeros(nm, np.uint32)
    kinds[3] = 1                                   # mirror
    be.set_material_kinds(kinds)
    queue((alb[1], emi, {1: tex}, sph, kinds))
    be.set_albedo(alb[2])
    be.set_texture(1, None)
    be.set_spheres(None, None)
    queue((alb[2], emi, {}, None, kinds))
    stats = [s.render_wait(t) for t in tickets]
    torch.cuda.synchronize()
    for i, ((a, e, tx, sp, kd), f, st) in enumerate(zip(states, films, stats)):
        osc = O.OracleScene(mesh, albedo=a, emission=e, textures=tx, spheres=sp,
                            sphere_mat=None if sp is None else np.array([2, 3], np.int32), kinds=kd)
        ref, casts = osc.render(O.reference_params(W, H, SPP, D, **kw))
        np.testing.assert_array_equal(f.cpu().numpy(), ref, err_msg=f"render {i}")
        assert st["ray_casts"] == casts, i
    # the states differ, so the test would see a render that read a later state
    assert len({films[i].cpu().numpy().tobytes() for i in (0, 2, 3, 4, 5)}) == 5


def test_set_spheres_waits_for_queued_ray_casts(mesh):
    """A public ray cast queued on a side stream before set_spheres sees the
    spheres it was queued with."""
    s = sptamd.Scene()
    s.add_arrays(mesh)
    s.commit(0)
    sph = np.array([[0.0, 3.03, 3.0, 0.5]], np.float32)   # in front of the camera
    s.backend.set_spheres(sph, np.array([1], np.int32))
    n = 1 << 16
    o = np.tile(np.array([[0.0], [3.03], [5.0]], np.float32), (1, n))
    rng = np.random.default_rng(5)
    d = np.stack([rng.uniform(-0.05, 0.05, n), rng.uniform(-0.05, 0.05, n), -np.ones(n)]).astype(np.float32)
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        ray = sptamd.Ray3.make(o, d)
        hits = s.backend.intersect_raw(ray, stream=side)
    s.backend.set_spheres(None, None)            # must wait for the cast on `side`
    torch.cuda.synchronize()
    tri = hits[0].cpu().numpy()
    ref = O.OracleScene(mesh, spheres=sph, sphere_mat=[1]).intersect(o, d)[0]
    np.testing.assert_array_equal(tri, ref)
    assert np.any(tri == -2)
