import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "smallpt-enoki-optix_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libspt.so on cuda:0)")


def _has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


def assert_work_complete(st, rows, width, spp):
    """spt_render_stats' device-counted work (include/spt.h): every (sample,
    pixel) of the tile started, ended and wrote its film slot exactly once —
    the reference renders every pixel x sample (main.cpp:385-429)."""
    want = rows * width * spp
    assert st["paths_started"] == want, (st["paths_started"], want)
    assert st["paths_terminated"] == want, (st["paths_terminated"], want)
    assert st["film_slots_unwritten"] == 0, st["film_slots_unwritten"]
    assert st["paths"] == want
    assert want == 0 or st["work_order"] in (1, 2)


def spaced_rows(height, n):
    """n evenly spaced rows of [0, height) (first and last included)."""
    import numpy as np
    return np.unique(np.linspace(0, height - 1, n).round().astype(np.int32))


def surface_rays(intersect, lo, hi, n, seed):
    """Rays that leave surfaces, as a path's bounces do (the case where the
    closest hit could depend on the tree: an origin on or next to a
    triangle's plane).  Primary rays from random points of the
    box [lo, hi] in random directions are cast with `intersect(o, d) -> (tri,
    t, u, v)`; each hit point o + t d (float32, as shade computes it,
    optix_backend.h:469) starts a new ray in a random direction or toward a random point of the box.  Returns the
    secondary rays' (o, d), (3, m) float32 each."""
    import numpy as np
    rng = np.random.default_rng(seed)
    lo, hi = np.asarray(lo, np.float32), np.asarray(hi, np.float32)
    o = (lo[:, None] + (hi - lo)[:, None] * rng.random((3, n))).astype(np.float32)
    d = rng.normal(size=(3, n)).astype(np.float32)
    tri, t, _, _ = intersect(o, d)
    h = tri >= 0
    o, d, t = o[:, h], d[:, h], t[h]
    p = (o + t[None, :] * d).astype(np.float32)
    # half in uniform random directions, half toward random points of the box
    # (more of those meet geometry again)
    tgt = lo[:, None] + (hi - lo)[:, None] * rng.random(p.shape)
    d2 = np.where(np.arange(p.shape[1]) % 2 == 0, rng.normal(size=p.shape), tgt - p).astype(np.float32)
    return p, d2


def edge_leaving_rays(pos, pos_tri, n, seed):
    """Adversarial rays for the box-exit rule: each starts at a
    float32 point of a random triangle within 1e-6..1e-2 (barycentric) of one
    edge and leaves across that edge nearly in the triangle's plane (normal
    component 1e-8..1e-3, either side), so the triangle's own Woop t is
    rounding noise while the ray leaves its box within ~tmin.  Returns (o, d),
    (3, n) float32 each."""
    import numpy as np
    rng = np.random.default_rng(seed)
    pos = np.asarray(pos, np.float32)
    pt = np.asarray(pos_tri, np.int64).reshape(-1, 3)
    v = pos[pt[rng.integers(0, len(pt), n)]].astype(np.float64)
    b = rng.dirichlet([1, 1, 1], n)
    b[:, 0] = 10 ** rng.uniform(-6, -2, n)
    b[:, 1:] *= (1 - b[:, :1]) / b[:, 1:].sum(1, keepdims=True)
    p = (v[:, 0] * b[:, :1] + v[:, 1] * b[:, 1:2] + v[:, 2] * b[:, 2:3]).astype(np.float32)
    nrm = np.cross(v[:, 1] - v[:, 0], v[:, 2] - v[:, 0])
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True) + 1e-30
    e = v[:, 2] - v[:, 1]
    e /= np.linalg.norm(e, axis=1, keepdims=True) + 1e-30
    out = np.cross(e, nrm)                     # in-plane, across the edge v1 v2 ...
    out *= np.sign(np.einsum("ij,ij->i", out, v[:, 1] - v[:, 0]))[:, None]  # ... away from v0
    s = np.sign(rng.uniform(-1, 1, n)) * 10 ** rng.uniform(-8, -3, n)
    d = (out + rng.normal(size=(n, 1)) * 0.3 * e + s[:, None] * nrm).astype(np.float32)
    return np.ascontiguousarray(p.T), np.ascontiguousarray(d.T)
