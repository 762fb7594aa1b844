"""Where do the GPU image and the oracle differ?  (Diagnostics; GPU box.)

Renders a bench config on the GPU and the same rows on the oracle (the rows
bench.py's cpu_baseline picks for --rows), lists the differing pixels, finds
for each the first sample whose outcome differs (renders at spp = 1..spp, by
bisection), then follows that sample's casts through the oracle
(oracle_trace_sample) and asks the GPU's public ray cast (spt_intersect) and a
brute-force oracle scene for the closest hit of each of those rays.

    python tools/diag_parity.py --config 4 --rows 86 [--brute]
"""
from __future__ import annotations

import argparse
import ctypes  # noqa: F401 (ctypes.byref)
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "smallpt-enoki-optix_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=4)
    ap.add_argument("--rows", type=int, default=86)
    ap.add_argument("--max-pixels", type=int, default=4)
    ap.add_argument("--brute", action="store_true", help="also a brute-force oracle scene (slow on 10M triangles)")
    ap.add_argument("--threads", type=int, default=16)
    a = ap.parse_args()

    import numpy as np
    import torch

    import bench
    import oracle as O
    import sptamd
    from sptamd import scenes

    sys.argv = ["bench.py", "--config", str(a.config)]
    args = bench.parse()
    src, kw, alb, emi = bench.workload(args, scenes)
    scene = sptamd.Scene()
    if isinstance(src, str):
        scene.add_triangle_mesh(src)
    else:
        scene.add_arrays(src)
    scene.commit(0)
    mesh = scene.mesh
    if scene.pbrt_info and scene.pbrt_info["camera"]:
        kw = dict(kw, camera=scene.pbrt_info["camera"])
    if alb:
        alb, emi = scenes.smallpt_materials(mesh)
        scene.backend.set_albedo(alb)
        scene.backend.set_emission(emi)
    else:
        alb = emi = None
    W, H, spp, D = args.width, args.height, args.spp, args.depth

    def gpu_film(k):
        film, t = scene.render_async(sptamd.make_params(W, H, k, D, **kw))
        st = scene.render_wait(t)
        assert st["film_slots_unwritten"] == 0 and st["paths_started"] == W * H * k
        return film.cpu().numpy()

    osc = O.OracleScene(mesh, albedo=alb, emission=emi)
    rows = np.unique(np.linspace(0, H - 1, a.rows).astype(np.int32))
    g = gpu_film(spp)[:, rows, :]
    ref, _ = osc.render(O.reference_params(W, H, spp, D, **kw), rows=rows, nthreads=a.threads)
    diff = np.argwhere(g != ref)
    pix = sorted({(int(rows[r]), int(x)) for _, r, x in diff})
    print(json.dumps({"config": a.config, "rows": int(rows.size), "values_differing": int(diff.shape[0]),
                      "pixels": pix[:32]}), flush=True)
    brute = O.OracleScene(mesh, use_bvh=False, albedo=alb, emission=emi) if a.brute else None
    lib = osc.lib
    for (y, x) in pix[:a.max_pixels]:
        # the first sample count whose film value differs (one changed sample
        # changes every later prefix)
        def differs(k):
            gg = gpu_film(k)[:, y, x]
            oo, _ = osc.render(O.reference_params(W, H, k, D, **kw), rows=np.array([y], np.int32), nthreads=a.threads)
            return not np.array_equal(gg, oo[:, 0, x]), gg, oo[:, 0, x]
        lo, hi = 1, spp
        while lo < hi:
            mid = (lo + hi) // 2
            if differs(mid)[0]:
                hi = mid
            else:
                lo = mid + 1
        s = lo - 1
        _, gg, oo = differs(lo)
        p = O.reference_params(W, H, spp, D, **kw)
        rays = np.zeros((D, 6), np.float32)
        ids = np.zeros(D, np.int32)
        tuv = np.zeros((D, 3), np.float32)
        L = np.zeros(3, np.float32)
        n = lib.oracle_trace_sample(osc.h, ctypes.byref(p), x, y, s, rays.ctypes.data, ids.ctypes.data,
                                    tuv.ctypes.data, L.ctypes.data)
        o = np.ascontiguousarray(rays[:n, :3].T)
        d = np.ascontiguousarray(rays[:n, 3:].T)
        rr = sptamd.Ray3.make(o, d)
        gt = [z.cpu().numpy() for z in scene.backend.intersect_raw(rr, do_closest=True)]
        ga = [z.cpu().numpy() for z in scene.backend.intersect_raw(rr, do_closest=False)]
        ob = osc.intersect(o, d)
        bf = brute.intersect(o, d) if brute else None
        casts = []
        for i in range(n):
            c = {"o": rays[i, :3].tolist(), "d": rays[i, 3:].tolist(),
                 "oracle_path": [int(ids[i])] + [float(v) for v in tuv[i]],
                 "oracle_isect": [int(ob[0][i]), float(ob[1][i]), float(ob[2][i]), float(ob[3][i])],
                 "gpu_closest": [int(gt[0][i]), float(gt[1][i]), float(gt[2][i]), float(gt[3][i])],
                 "gpu_anyhit_id": int(ga[0][i])}
            if bf is not None:
                c["brute"] = [int(bf[0][i]), float(bf[1][i]), float(bf[2][i]), float(bf[3][i])]
            c["same"] = c["gpu_closest"] == c["oracle_isect"]
            casts.append(c)
        print(json.dumps({"pixel": [x, y], "sample": s, "spp_first_diff": lo, "gpu": gg.tolist(), "oracle": oo.tolist(),
                          "oracle_L": L.tolist(), "casts": casts}), flush=True)


if __name__ == "__main__":
    main()
