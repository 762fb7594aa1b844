"""Host-side cost around spt_render on the bench workload (GPU).

    python tools/host_overhead.py [--config 1] [--steps 10]

Times K back-to-back renders of the bench's config with and without
SPT_FLAG_TIMING (the per-isect-launch HIP events the roofline uses), and the
bench's own step (render + tile gather + torch events), each as wall time per
render; the difference between them is host overhead the GPU waits on.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "smallpt-enoki-optix_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import sptamd  # noqa: E402
from sptamd import scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    cfg = bench.CONFIGS[a.config]
    src, kw, smallpt, _ = bench.workload(argparse.Namespace(scene=cfg["scene"], smallpt=cfg["smallpt"]), scenes)
    sc = sptamd.Scene()
    if isinstance(src, str):
        sc.add_triangle_mesh(src)
    else:
        sc.add_arrays(src)
    sc.commit(0)
    W, H, spp, D = cfg["width"], cfg["height"], cfg["spp"], cfg["depth"]
    film = torch.empty((3, H, W), dtype=torch.float32, device="cuda")
    out = {}
    for name, timing in (("no_timing", False), ("isect_events", True), ("no_timing_again", False)):
        p = sptamd.make_params(W, H, spp, D, timing=timing, **kw)
        sc.render(p, film=film)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tot = 0.0
        for _ in range(a.steps):
            _, st = sc.render(p, film=film)
            tot += st["total_ms"]
        torch.cuda.synchronize()
        out[name] = {"wall_ms_per_render": round((time.perf_counter() - t0) * 1e3 / a.steps, 3),
                     "spt_render_total_ms": round(tot / a.steps, 3)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
