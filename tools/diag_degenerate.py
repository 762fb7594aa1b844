"""Diagnose GPU vs oracle (BVH and brute force) on degenerate-direction rays."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "smallpt-enoki-optix_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np
import torch
import oracle as O
import sptamd
from sptamd import scenes
from test_gpu_isect import random_rays, gpu_isect

m = scenes.mitsuba_synth(detail=0.25)
b = sptamd.HipBackend(); b.init(0)
b.set_triangles_soup(m["pos_tri"], m["pos"], m["nrm_tri"], m["nrm"], None, None, m["mat_id"])
o, d = random_rays(6000, 12)
d[0, 0::6] = 0.0; d[1, 1::6] = -0.0; d[2, 2::6] = 1e-30; d[:, 3::6] = 0.0; d[0, 4::6] = 0.0; d[2, 4::6] = 0.0; d[0, 5::6] = np.nan
g = gpu_isect(b, o, d)
rb = O.OracleScene(m, use_bvh=True).intersect(o, d)
rf = O.OracleScene(m, use_bvh=False).intersect(o, d)
for name, r in (("oracle-bvh", rb), ("brute", rf)):
    bad = np.flatnonzero(g[0] != r[0])
    print(name, "mismatches", len(bad), "by category", np.bincount(bad % 6, minlength=6).tolist())
    for i in bad[:5]:
        print("  ray", i, "o", o[:, i], "d", d[:, i], "gpu", g[0][i], g[1][i], name, r[0][i], r[1][i])
bad = np.flatnonzero(rb[0] != rf[0])
print("oracle bvh vs brute mismatches", len(bad), np.bincount(bad % 6, minlength=6).tolist())
