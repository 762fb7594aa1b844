"""Traversal statistics of the isect kernel at the headline workload (GPU).

    python tools/trav_stats.py [--spp 16] [--depths 1 2 8]
Prints per-ray node visits, triangle tests, loop steps and SIMD efficiency
(lane steps / (64 x wave steps)) next to the timed Grays/s of the normal build.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "smallpt-enoki-optix_amd"))

import torch  # noqa: E402

import sptamd  # noqa: E402
from sptamd import _lib, scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=16)
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--depths", type=int, nargs="+", default=[1, 2, 8])
    ap.add_argument("--scene", default="mitsuba_synth")
    ap.add_argument("--wavefront", type=int, default=0)
    ap.add_argument("--city", action="store_true", help="BASELINE config 4: the 10M-triangle pbrt city, 1920x1080")
    a = ap.parse_args()
    sc = sptamd.Scene()
    kw = {}
    W = H = a.size
    if a.city:
        sc.add_triangle_mesh(scenes.scene_pbrt("city_synth"))
        kw["camera"] = sc.pbrt_info["camera"]
        W, H = 1920, 1080
    elif a.scene == "smallpt_analytic":  # BASELINE config 2: smallpt's scene, Cornell camera, smallpt materials
        m = scenes.smallpt_analytic()
        m["albedo"], m["emission"] = scenes.smallpt_materials(m)
        sc.add_arrays(m)
        kw.update(camera=scenes.cornell_camera(), rr_start_depth=5, env=(0.0, 0.0, 0.0))
    else:
        sc.add_triangle_mesh(scenes.scene_obj(a.scene))
    sc.commit(0)
    print(json.dumps({"bvh": sc.backend.stats}))
    for D in a.depths:
        p = sptamd.make_params(W, H, a.spp, D, timing=True, wavefront_paths=a.wavefront, **kw)
        sc.render(p)
        _, st = sc.render(p)
        p.flags = _lib.SPT_FLAG_TRAVERSAL_STATS
        _, ss = sc.render(p)
        torch.cuda.synchronize()
        casts = ss["ray_casts"]
        rec = {"depth": D, "casts": casts, "casts_per_path": casts / st["paths"],
               "isect_ms": round(st["isect_ms"], 3), "shade_ms": round(st["shade_ms"], 3),
               "refill_ms": round(st["camera_ms"], 3), "iterations": st["iterations"],
               "grays_per_s": round(casts / (st["isect_ms"] * 1e-3) / 1e9, 3),
               "mpaths_per_s": round(st["paths"] / (st["total_ms"] * 1e-3) / 1e6, 1),
               "nodes_per_ray": round(ss["isect_nodes"] / casts, 2),
               "tris_per_ray": round(ss["isect_tris"] / casts, 2),
               "steps_per_ray": round(ss["isect_lane_steps"] / casts, 2),
               "simd_eff": round(ss["isect_lane_steps"] / (64.0 * ss["isect_wave_steps"]), 3),
               # the blocks the SIMD runs: fraction of wave steps, and lanes using them when run
               "tri_block_frac": round(ss["isect_tri_wave_steps"] / max(1, ss["isect_wave_steps"]), 3),
               "node_block_frac": round(ss["isect_node_wave_steps"] / max(1, ss["isect_wave_steps"]), 3),
               "tri_block_lanes": round(ss["isect_tris"] / max(1, ss["isect_tri_wave_steps"]), 2),
               "node_block_lanes": round(ss["isect_nodes"] / max(1, ss["isect_node_wave_steps"]), 2),
               "max_stack": ss["isect_max_stack"]}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
