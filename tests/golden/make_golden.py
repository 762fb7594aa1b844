"""Generate tests/golden/oracle_small.npz from the CPU oracle (committed data).

The reference ships no tests or fixtures and cannot be built here (no CUDA,
OptiX, Enoki, tinyobjloader), so these vectors are produced by the oracle in
this container and pin it against regressions; the independent pins are the
published PCG32 known answers and the analytic cases in tests/test_oracle.py.

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "smallpt-enoki-optix_amd"), os.path.join(ROOT, "oracle")]

import oracle as O  # noqa: E402
from sptamd import scenes  # noqa: E402


def rays(n, seed):
    rng = np.random.default_rng(seed)
    o = rng.uniform(-2.5, 2.5, size=(3, n)).astype(np.float32)
    o[1] = rng.uniform(-0.9, 3.0, size=n)
    o[:, : n // 8] = np.array([[0.0], [3.03], [5.0]], np.float32)
    d = (rng.normal(size=(3, n)) * rng.uniform(0.2, 3.0, size=n)).astype(np.float32)
    return o, d


def main():
    mesh = scenes.mitsuba_synth(detail=0.1)
    sc = O.OracleScene(mesh)
    out = {}
    out["pcg_seeds"] = np.array([0, 1, 1023, 262143, 1048575], np.uint64)
    out["pcg_u32"] = np.stack([O.pcg32_seq(O.PCG32_DEFAULT_STATE, int(s), 32) for s in out["pcg_seeds"]])
    o, d = rays(4096, 11)
    tri, t, u, v = sc.intersect(o, d)
    out.update(isect_o=o, isect_d=d, isect_tri=tri, isect_t=t, isect_u=u, isect_v=v)
    out["film_32x24_4spp_d4"], _ = sc.render(O.reference_params(32, 24, 4, 4))
    out["film_32x24_4spp_d4_xfirst"], _ = sc.render(O.reference_params(32, 24, 4, 4, rng_order=1))
    out["film_16x16_100spp_d2"], _ = sc.render(O.reference_params(16, 16, 100, 2))
    alb = np.array([[1, 1, 1], [.8, .6, .4], [.9, .3, .2], [.2, .2, .8], [.9, .9, .3], [.4, .4, .4]], np.float32)
    out["albedo"] = alb
    out["film_albedo_rr2"], _ = O.OracleScene(mesh, albedo=alb).render(
        O.reference_params(20, 16, 6, 6, rr_start_depth=2))
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "oracle_small.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
