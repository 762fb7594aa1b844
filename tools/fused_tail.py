"""Fixed per-frame cost of the fused kernel: frame time of tile 0 of 64 and of
8 (1/64 and 1/8 of config 1's paths) at several depths and refill thresholds;
the intercept a of t = a + b * paths is the time that does not scale with the
job (launch, ramp, the drain tail).

    python tools/fused_tail.py [--depths 1 2 4 8] [--idle 16 32] [--steps 5]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "smallpt-enoki-optix_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depths", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--idle", type=int, nargs="+", default=[32])
    ap.add_argument("--grid", type=int, nargs="+", default=[256])
    ap.add_argument("--share", type=int, nargs="+", default=[32])
    ap.add_argument("--tiles", type=int, nargs=2, default=[64, 8])
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    import torch

    import bench
    import sptamd
    from sptamd import scenes

    cfg = bench.CONFIGS[1]
    ns = argparse.Namespace(scene=cfg["scene"], smallpt=cfg["smallpt"])
    src, kw, alb, _ = bench.workload(ns, scenes)
    scene = sptamd.Scene()
    if isinstance(src, str):
        scene.add_triangle_mesh(src)
    else:
        scene.add_arrays(src)
    scene.commit(0)
    base = sptamd.default_config()
    W, H, spp = cfg["width"], cfg["height"], cfg["spp"]
    import itertools
    for idle, grid, share in itertools.product(a.idle, a.grid, a.share):
        c = sptamd.config_from_env(base)
        c.fused_refill_idle, c.fused_grid_q8, c.fused_static_share_q8 = idle, grid, share
        scene.backend.base_config = c
        for D in a.depths:
            t = {}
            for T in a.tiles:
                p = sptamd.make_params(W, H, spp, D, tile_index=0, tile_count=T, rows_per_group=8,
                                       pipeline="fused", **kw)
                film = None
                for _ in range(2):
                    film, st = scene.render(p, film)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.steps):
                    scene.render(p, film)
                torch.cuda.synchronize()
                t[T] = ((time.perf_counter() - t0) / a.steps * 1e3, st["paths"], st["ray_casts"])
            (ts, ns_, cs), (tl, nl, cl) = t[a.tiles[0]], t[a.tiles[1]]
            slope = (tl - ts) / (nl - ns_)
            rec = {"idle": idle, "grid_q8": grid, "share_q8": share, "depth": D,
                   "ms_small": round(ts, 3), "ms_large": round(tl, 3),
                   "paths_small": ns_, "paths_large": nl, "casts_per_path": round(cl / nl, 3),
                   "intercept_ms": round(ts - slope * ns_, 3), "ns_per_path": round(slope * 1e6, 4)}
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
