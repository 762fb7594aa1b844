"""The statistical leg of SURVEY §8c on the CPU: the fp32 oracle (a bitwise
restatement sharing one op-order specification with the HIP kernels) against
an independent float64 estimator (tests/independent.py: numpy sin/cos/sqrt,
Moller-Trumbore without a BVH, Philox random numbers).  Agreement in
distribution shows the estimator is right independently of the
restatement's arithmetic choices (Cephes sincos mapping.h:9,25, 1/sqrt
normalise, unfused Frame3 coordframe.h:40-48, the watertight Woop test for
OptiX's optix_backend.h:314).  tests/test_gpu_parity.py repeats it on the GPU.

Tolerance: per-pixel two-sample z <= 5 (Bernoulli sigma^2 = p(1-p)/spp for the
reference's escape-fraction image) and whole-image z <= 5."""
import numpy as np

import independent as I
import oracle as O
from sptamd import backend

Z_MAX = 5.0


def test_oracle_matches_independent_estimator():
    m = I.stat_scene()
    cam = backend.reference_camera()
    W = H = 32
    spp, depth = 256, 4
    ref = I.render(m, W, H, spp, depth, cam, seed=7)
    got, _ = O.OracleScene(m).render(O.reference_params(W, H, spp, depth))
    assert 0.3 < got[0].mean() < 0.95          # escape fractions well inside (0, 1)
    z, zmean = I.bernoulli_z(got[0], ref[0], spp, spp)
    assert z.max() <= Z_MAX, (z.max(), np.unravel_index(z.argmax(), z.shape))
    assert zmean <= Z_MAX, zmean
    # and two oracle seeds against each other (a sanity check of the z statistic)
    got2, _ = O.OracleScene(m).render(O.reference_params(W, H, spp, depth, rng_initstate=0x1234567))
    z2, zmean2 = I.bernoulli_z(got[0], got2[0], spp, spp)
    assert 0 < z2.max() <= Z_MAX and zmean2 <= Z_MAX


def block_z(mean_a, mean_b, per_b, block=4):
    """z of block means (block x block pixels) per channel, with the variance
    estimated from the independent estimator's per-sample values (both sides
    assumed to share it: same estimator in distribution)."""
    C, H, W, n = per_b.shape
    hb, wb = H // block, W // block
    crop = lambda x: x[:, : hb * block, : wb * block]  # noqa: E731
    a = crop(mean_a).reshape(C, hb, block, wb, block).mean(axis=(2, 4))
    b = crop(mean_b).reshape(C, hb, block, wb, block).mean(axis=(2, 4))
    s = per_b[:, : hb * block, : wb * block].reshape(C, hb, block, wb, block, n)
    var = s.var(axis=(2, 4, 5), ddof=1) / (block * block * n)
    var = np.maximum(var, 1.0 / (block * block * n) ** 2)  # floor: a block with no spread
    z = np.abs(a - b) / np.sqrt(2.0 * var)
    zimg = np.abs(mean_a.mean(axis=(1, 2)) - mean_b.mean(axis=(1, 2))) / np.sqrt(
        2.0 * per_b.var(axis=3, ddof=1).sum(axis=(1, 2)) / n / (H * W) ** 2)
    return z, zimg


def test_oracle_matches_independent_estimator_emitters():
    """Albedo < 1, an emitter, a coloured sky and Russian roulette (the build's
    materials, §8f row 3): block and whole-image z per channel."""
    m = I.stat_scene()
    cam = backend.reference_camera()
    W = H = 24
    spp, depth = 256, 6
    albedo = np.array([[1, 1, 1], [0.7, 0.6, 0.5], [0.9, 0.2, 0.2], [0.3, 0.8, 0.3], [0.5, 0.5, 0.9]], np.float32)
    emission = np.zeros((5, 3), np.float32)
    emission[4] = (2.0, 1.5, 0.5)
    env = (0.2, 0.3, 0.4)
    mean_b, per_b = I.render(m, W, H, spp, depth, cam, env=env, albedo=albedo, emission=emission, rr_start_depth=2,
                             seed=11, samples=True)
    got, _ = O.OracleScene(m, albedo=albedo, emission=emission).render(
        O.reference_params(W, H, spp, depth, rr_start_depth=2, env=env))
    z, zimg = block_z(got.astype(np.float64), mean_b, per_b)
    assert z.max() <= Z_MAX, z.max()
    assert zimg.max() <= Z_MAX, zimg


def test_oracle_matches_independent_estimator_smallpt_spheres():
    """smallpt's own scene: analytic mirror and glass balls and the light
    sphere (smallpt.cpp radiance(): SPEC, REFR with Schlick's Fresnel term).
    The estimator picks reflection with probability Re at weight 1, the oracle
    with P = 1/4 + Re/2 at weight Re/P or Tr/(1-P): the same expectation.
    Swapping the two balls' kinds must fail the same test (sensitivity)."""
    from sptamd import scenes
    m = scenes.smallpt_analytic(detail=0.125)
    alb, emi = scenes.smallpt_materials(m)
    cam = scenes.cornell_camera()
    W = H = 32
    spp, depth = 512, 6
    kw = dict(env=(0.0, 0.0, 0.0), rr_start_depth=3)
    mean_b, per_b = I.render(m, W, H, spp, depth, cam, albedo=alb, emission=emi, seed=5, samples=True, **kw)
    got, _ = O.OracleScene(m, albedo=alb, emission=emi).render(O.reference_params(W, H, spp, depth, camera=cam, **kw))
    z, zimg = block_z(got.astype(np.float64), mean_b, per_b)
    assert z.max() <= Z_MAX, z.max()
    assert zimg.max() <= Z_MAX, zimg
    swapped = m["kinds"].copy()
    swapped[m["sphere_mat"][0]], swapped[m["sphere_mat"][1]] = m["kinds"][m["sphere_mat"][1]], m["kinds"][m["sphere_mat"][0]]
    bad, _ = O.OracleScene(m, albedo=alb, emission=emi, kinds=swapped).render(
        O.reference_params(W, H, spp, depth, camera=cam, **kw))
    zb, _ = block_z(bad.astype(np.float64), mean_b, per_b)
    assert zb.max() > Z_MAX, zb.max()
