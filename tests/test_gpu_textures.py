"""Sized-image reflectance textures (ImageTexture,
/root/reference/src/main.cpp:34-80, used by LambertBsdf::sample :109-117):
bilinear, clamped lookups at the hit's interpolated texcoord, with the
reference's texel index y * size.y + x (main.cpp:52), on the GPU bit-equal to
the oracle — square and non-square images, both pipelines, with roulette and
with emitters."""
import numpy as np
import pytest
import torch

import oracle as O
import sptamd
from sptamd import scenes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mesh():
    return scenes.with_planar_uv(scenes.mitsuba_synth(detail=0.25))


def textures():
    rng = np.random.default_rng(3)
    return {1: scenes.checker(8, 8, cell=1),                                # square
            2: rng.uniform(0.1, 0.95, size=(5, 3, 3)).astype(np.float32),   # 3 wide, 5 high: y * h + x runs past
            3: scenes.checker(16, 4, cell=2),                                # 16 wide, 4 high
            5: np.full((1, 1, 3), 0.7, np.float32)}                          # the reference's 1 x 1 image


def render(s, w, h, spp, depth, **kw):
    film, st = s.render(sptamd.make_params(w, h, spp, depth, **kw))
    torch.cuda.synchronize()
    return film.cpu().numpy(), st


def gscene(mesh, albedo, tex, emission=None):
    s = sptamd.Scene()
    s.add_arrays(mesh)
    s.commit(0)
    s.backend.set_albedo(albedo)
    if emission is not None:
        s.backend.set_emission(emission)
    for mat, img in tex.items():
        s.backend.set_texture(mat, img)
    return s


@pytest.mark.parametrize("pipeline", ["wavefront", "fused"])
@pytest.mark.parametrize("rr", [2, 99])
def test_textures_bitexact(mesh, pipeline, rr):
    nm = len(mesh["kd"])
    albedo = np.full((nm, 3), 0.8, np.float32)
    tex = textures()
    s = gscene(mesh, albedo, tex)
    kw = dict(rr_start_depth=rr, env=(1.0, 0.9, 0.8))
    got, st = render(s, 48, 40, 6, 6, pipeline=pipeline, **kw)
    ref, casts = O.OracleScene(mesh, albedo=albedo, textures=tex).render(O.reference_params(48, 40, 6, 6, **kw))
    np.testing.assert_array_equal(got, ref)
    assert st["ray_casts"] == casts
    # the images matter: without them the image differs
    plain, _ = O.OracleScene(mesh, albedo=albedo).render(O.reference_params(48, 40, 6, 6, **kw))
    assert not np.array_equal(ref, plain)


def test_textures_with_emitters_and_removal(mesh):
    nm = len(mesh["kd"])
    albedo = np.full((nm, 3), 0.9, np.float32)
    emi = np.zeros((nm, 3), np.float32)
    emi[4] = (3.0, 2.0, 1.0)
    tex = textures()
    s = gscene(mesh, albedo, tex, emission=emi)
    kw = dict(rr_start_depth=3, env=(0.2, 0.2, 0.3))
    got, _ = render(s, 40, 30, 5, 7, wavefront_paths=900, **kw)
    ref, _ = O.OracleScene(mesh, albedo=albedo, emission=emi, textures=tex).render(
        O.reference_params(40, 30, 5, 7, **kw))
    np.testing.assert_array_equal(got, ref)
    for mat in tex:                       # removing every image restores the constant albedo
        s.backend.set_texture(mat, None)
    got0, _ = render(s, 40, 30, 5, 7, **kw)
    ref0, _ = O.OracleScene(mesh, albedo=albedo, emission=emi).render(O.reference_params(40, 30, 5, 7, **kw))
    np.testing.assert_array_equal(got0, ref0)


def test_texture_without_texcoords():
    """No vt in the mesh: every lookup is at (0, 0) (the reference would gather
    at index -1)."""
    m = scenes.mitsuba_synth(detail=0.1)
    nm = len(m["kd"])
    albedo = np.full((nm, 3), 0.75, np.float32)
    tex = {1: scenes.checker(4, 4)}
    s = gscene(m, albedo, tex)
    got, _ = render(s, 32, 24, 4, 5)
    ref, _ = O.OracleScene(m, albedo=albedo, textures=tex).render(O.reference_params(32, 24, 4, 5))
    np.testing.assert_array_equal(got, ref)


def test_texture_api_errors(mesh):
    s = gscene(mesh, np.ones((len(mesh["kd"]), 3), np.float32), {})
    with pytest.raises(sptamd.SptError):
        s.backend.set_texture(1, np.zeros((0, 4, 3), np.float32))
    with pytest.raises(sptamd.SptError):
        s.backend.set_texture(1 << 21, np.ones((1, 1, 3), np.float32))
