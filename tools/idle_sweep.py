"""The drain's refill threshold (spt_config.drain_refill_idle) against scene
size: renders of the synthetic scenes at several detail levels (triangle
counts) at config 1's image, spp and depth (the reference's unit mode: albedo 1,
sky 1), one render at a time, for each threshold.  Evidence for the AUTO rule
(DESIGN.md §4); prints one JSON line per (scene, detail, threshold).

    python tools/idle_sweep.py [--scenes mitsuba_synth:0.1,0.25,1 cornell_spheres:0.25,1] [--idle 24 40 56]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "smallpt-enoki-optix_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenes", nargs="+", default=["mitsuba_synth:0.05,0.25,1", "cornell_spheres:0.25,1"])
    ap.add_argument("--idle", nargs="+", type=int, default=[24, 32, 40, 56])
    ap.add_argument("--renders", type=int, default=4)
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--spp", type=int, default=64)
    args = ap.parse_args()
    import torch

    import sptamd
    from sptamd import scenes

    for spec in args.scenes:
        name, details = spec.split(":")
        for detail in (float(x) for x in details.split(",")):
            mesh = getattr(scenes, name)(detail)
            kw = dict(camera=scenes.cornell_camera()) if name == "cornell_spheres" else {}
            for idle in args.idle:
                cfg = sptamd.default_config()
                cfg.drain_refill_idle = idle
                s = sptamd.Scene(config=cfg)
                s.add_arrays(mesh)
                s.commit(0)
                p = sptamd.make_params(args.size, args.size, args.spp, 8, **kw)
                film = torch.empty((3, args.size, args.size), dtype=torch.float32, device="cuda")
                s.render(p, film=film)  # warm-up: allocations
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(args.renders):
                    _, st = s.render(p, film=film)
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) / args.renders
                print(json.dumps({"scene": name, "detail": detail, "triangles": int(len(mesh["pos_tri"])),
                                  "refill_idle": st.get("drain_refill_idle"),
                                  "mpaths_s": round(args.size * args.size * args.spp / dt / 1e6, 1),
                                  "ms": round(dt * 1e3, 3)}), flush=True)
                del s


if __name__ == "__main__":
    main()
