"""Diagnose BVH2 (SPT_BVH=2) vs brute force on the watertight grid rays."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "smallpt-enoki-optix_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np
import oracle as O
import sptamd
from test_gpu_isect import grid_mesh, gpu_isect

m = grid_mesh(16)
b = sptamd.HipBackend(); b.init(0)
b.set_triangles_soup(m["pos_tri"], m["pos"])
print("bvh", b.stats)
pts = m["pos"][np.abs(m["pos"][:, 0]) < 0.99]
pts = pts[np.abs(pts[:, 2]) < 0.99]
mids = (m["pos"][m["pos_tri"][:, 0]] + m["pos"][m["pos_tri"][:, 2]]) * np.float32(0.5)
targets = np.concatenate([pts, mids]).astype(np.float32)
rng = np.random.default_rng(11)
o = (targets + rng.normal(size=targets.shape).astype(np.float32) * [0.3, 0.0, 0.3]).astype(np.float32)
o[:, 1] = rng.uniform(0.5, 3.0, size=len(o))
d = (targets - o).astype(np.float32).T.copy()
o = o.T.copy()
g = gpu_isect(b, o, d)
r = O.OracleScene(m, use_bvh=False).intersect(o, d)
bad = np.flatnonzero(g[0] != r[0])
print("mismatch", len(bad), "gpu misses", int((g[0][bad] < 0).sum()))
for i in bad[:6]:
    print(i, "o", o[:, i].tolist(), "d", d[:, i].tolist(), "target", targets[i].tolist(), "gpu", g[0][i], g[1][i], "ref", r[0][i], r[1][i])
