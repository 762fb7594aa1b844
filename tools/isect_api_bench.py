"""Throughput of the public ray-cast entry point (spt_intersect, the drop-in for
OptixBackend::intersect, optix_backend.h:422) on config 1's scene (GPU).

    python tools/isect_api_bench.py [--n 4194304] [--reps 10]

Ray sets, n rays each, device-resident before timing (HIP events around the
calls): "camera" = the reference camera's pixel grid (coherent, like the
reference's first bounce), "random" = origins uniform in the scene's bounding
box and uniform random directions (incoherent, like later bounces); each
closest-hit and any-hit.  Prints one JSON line per case.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "smallpt-enoki-optix_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import sptamd  # noqa: E402
from sptamd import scenes  # noqa: E402


def camera_rays(n, dev):
    cam = sptamd.reference_camera()
    side = int(np.sqrt(n))
    o = torch.tensor(cam["look_from"], dtype=torch.float32, device=dev)
    z = torch.tensor(cam["look_at"], dtype=torch.float32, device=dev) - o
    z = z / z.norm()
    up = torch.tensor(cam["up"], dtype=torch.float32, device=dev)
    x = torch.linalg.cross(up, z)
    x = x / x.norm()
    y = torch.linalg.cross(z, x)
    s = torch.linspace(-0.36, 0.36, side, device=dev)
    gy, gx = torch.meshgrid(s, s, indexing="ij")
    d = z[:, None] + gx.reshape(1, -1) * x[:, None] + gy.reshape(1, -1) * y[:, None]
    d = d / d.norm(dim=0, keepdim=True)
    return o[:, None].expand(3, d.shape[1]).contiguous(), d.contiguous()


def random_rays(n, lo, hi, dev):
    g = torch.Generator(device=dev).manual_seed(7)
    o = torch.rand((3, n), generator=g, device=dev) * (hi - lo)[:, None] + lo[:, None]
    d = torch.randn((3, n), generator=g, device=dev)
    return o.contiguous(), (d / d.norm(dim=0, keepdim=True)).contiguous()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 22)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    sc = sptamd.Scene()
    mesh = scenes.mitsuba_synth()
    sc.add_arrays(mesh)
    sc.commit(0)
    pos = torch.as_tensor(np.asarray(mesh["pos"], np.float32).reshape(-1, 3), device=dev)
    lo, hi = pos.min(0).values, pos.max(0).values
    sets = {"camera": camera_rays(a.n, dev), "random": random_rays(a.n, lo, hi, dev)}
    for name, (o, d) in sets.items():
        rays = sptamd.Ray3.make(o, d, device=dev)
        n = len(rays)
        for closest in (True, False):
            out = sc.backend.intersect_raw(rays, do_closest=closest)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                sc.backend.intersect_raw(rays, do_closest=closest, out=out)
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1) / a.reps
            hit = float((out[0] >= 0).float().mean())
            print(json.dumps({"rays": name, "n": n, "query": "closest" if closest else "any",
                              "ms": round(ms, 3), "grays_per_s": round(n / ms / 1e6, 3),
                              "hit_fraction": round(hit, 4)}), flush=True)


if __name__ == "__main__":
    main()
