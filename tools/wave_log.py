"""Per-wave timeline of the lane-loop launches (drain, fused kernel) from the
diagnostic build (make BUILD=build_wlog EXTRA=-DSPT_WAVE_LOG=1): when each
wave of each launch started and ended, on which XCD / CU / hardware queue.
Answers "were all of a drain's waves resident from its start?" (VERDICT r5
item 1: a render's second drain ran 1.6x longer than its first on equal work).

    SPT_LIB=smallpt-enoki-optix_amd/build_wlog/libspt.so \
        python tools/wave_log.py [--config 1] [--renders 3] [--queued 4] [--json out.json]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "smallpt-enoki-optix_amd"))
sys.path.insert(0, ROOT)

TICK_US = 0.01  # s_memrealtime: 100 MHz


def read_log(lib, reset=True):
    n = lib.spt_debug_wave_log(None, 0, 0)
    if n < 0:
        raise RuntimeError("spt_debug_wave_log failed")
    buf = np.zeros((max(n, 1), 5), np.uint64)
    got = lib.spt_debug_wave_log(buf.ctypes.data, n, 1 if reset else 0)
    if got != n:
        raise RuntimeError(f"wave log changed under the read: {got} != {n}")
    return buf[:n]


def decode(rec):
    t0, t1 = rec[:, 0].astype(np.int64), rec[:, 1].astype(np.int64)
    hw = (rec[:, 2] & 0xffffffff).astype(np.int64)
    xcc = (rec[:, 2] >> 32).astype(np.int64)
    tag = (rec[:, 3] & 0xffffffff).astype(np.int64)
    casts = (rec[:, 3] >> 32).astype(np.int64)
    block = (rec[:, 4] & 0xffffffff).astype(np.int64)
    drain = (rec[:, 4] >> 32).astype(np.int64)
    return dict(t0=t0, t1=t1, hw=hw, xcc=xcc, tag=tag, casts=casts, block=block, drain=drain,
                simd=(hw >> 4) & 3, cu=(hw >> 8) & 15, sh=(hw >> 12) & 1, se=(hw >> 13) & 3, queue=(hw >> 24) & 7)


def summarise(d, origin=None):
    """One dict per launch (drain: by its queue-count tag; fused: tag 0)."""
    out = []
    org = int(d["t0"].min()) if origin is None else origin
    for tag in sorted(set(d["tag"].tolist()), key=lambda t: int(d["t0"][d["tag"] == t].min())):
        m = d["tag"] == tag
        t0, t1 = d["t0"][m], d["t1"][m]
        first = int(t0.min())
        s = (t0 - first) * TICK_US
        e = (t1 - first) * TICK_US
        cu_key = d["xcc"][m] * 64 + d["se"][m] * 32 + d["sh"][m] * 16 + d["cu"][m]
        ncu = len(set(cu_key.tolist()))
        per_cu = np.bincount(np.unique(cu_key, return_inverse=True)[1])
        # resident waves over time: how many of the launch's waves had started by t
        late = s > 20.0  # started more than 20 us after the launch's first wave
        out.append({
            "tag": hex(int(tag)), "drain": int(d["drain"][m][0]), "waves": int(m.sum()),
            "start_us": round((first - org) * TICK_US, 1),
            "end_us": round((int(t1.max()) - org) * TICK_US, 1),
            "dur_us": round(float(e.max()), 1),
            "start_spread_us": {q: round(float(np.percentile(s, p)), 1) for q, p in
                                (("p50", 50), ("p90", 90), ("p99", 99), ("max", 100))},
            "late_waves": int(late.sum()),
            "late_first_start_us": round(float(s[late].min()), 1) if late.any() else None,
            "wave_end_us": {q: round(float(np.percentile(e, p)), 1) for q, p in
                            (("p10", 10), ("p50", 50), ("p90", 90), ("max", 100))},
            "casts": int(d["casts"][m].sum()),
            "waves_per_xcc": np.bincount(d["xcc"][m], minlength=8).tolist(),
            "cus": ncu, "waves_per_cu": {"min": int(per_cu.min()), "max": int(per_cu.max())},
            "hw_queue_ids": sorted(set(d["queue"][m].tolist())),
        })
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=1)
    ap.add_argument("--renders", type=int, default=3, help="renders one at a time, each logged on its own")
    ap.add_argument("--queued", type=int, default=4, help="renders queued back to back on two streams (as bench.py)")
    ap.add_argument("--json", default="")
    args = ap.parse_args()
    import torch

    import bench
    import sptamd
    from sptamd import _lib, scenes

    lib = _lib.lib
    if not hasattr(lib, "spt_debug_wave_log"):
        raise SystemExit(f"{_lib.LIB_PATH} is not a wave-log build (make BUILD=build_wlog EXTRA=-DSPT_WAVE_LOG=1)")
    lib.spt_debug_wave_log.restype = ctypes.c_longlong
    lib.spt_debug_wave_log.argtypes = [ctypes.c_void_p, ctypes.c_ulonglong, ctypes.c_int]
    cfg = bench.CONFIGS[args.config]
    ns = argparse.Namespace(scene=cfg["scene"], smallpt=cfg["smallpt"])
    src, kw, alb, _ = bench.workload(ns, scenes)
    scene = sptamd.Scene()
    if isinstance(src, str):
        scene.add_triangle_mesh(src)
    else:
        scene.add_arrays(src)
    scene.commit(0)
    if alb:
        a, e = scenes.smallpt_materials(scene.mesh)
        scene.backend.set_albedo(a)
        scene.backend.set_emission(e)
    W, H, spp, D = cfg["width"], cfg["height"], cfg["spp"], cfg["depth"]
    p = sptamd.make_params(W, H, spp, D, **kw)
    films = [torch.empty((3, H, W), dtype=torch.float32, device="cuda") for _ in range(2)]
    streams = [sptamd.queue_stream(), sptamd.queue_stream()]
    for k in range(2):
        scene.render_wait(scene.render_async(p, film=films[k], stream=streams[k])[1])
    torch.cuda.synchronize()
    read_log(lib)
    result = {"config": args.config, "env": {k: v for k, v in sorted(os.environ.items()) if k.startswith("SPT_")},
              "single": [], "queued": None}
    for r in range(args.renders):
        st = scene.render_wait(scene.render_async(p, film=films[r % 2], stream=streams[r % 2])[1])
        torch.cuda.synchronize()
        d = decode(read_log(lib))
        launches = summarise(d)
        result["single"].append({"render": r, "streams": st["streams"], "drain_launches": st["drain_launches"],
                                 "launches": launches})
        print(f"== single render {r}: streams {st['streams']}", flush=True)
        for l in launches:
            print(json.dumps(l), flush=True)
    if args.queued:
        tickets = [scene.render_async(p, film=films[i % 2], stream=streams[i % 2])[1] for i in range(args.queued)]
        for t in tickets:
            scene.render_wait(t)
        torch.cuda.synchronize()
        d = decode(read_log(lib))
        # launches of the queued renders: split each tag's waves into launches by time gaps
        launches = []
        org = int(d["t0"].min())
        for tag in sorted(set(d["tag"].tolist())):
            idx = np.where(d["tag"] == tag)[0]
            idx = idx[np.argsort(d["t0"][idx])]
            t0 = d["t0"][idx]
            cuts = np.where(np.diff(t0) > 100_00)[0]  # > 100 us between consecutive wave starts
            for part in np.split(idx, cuts + 1):
                sub = {k: v[part] for k, v in d.items()}
                launches += summarise(sub, origin=org)
        launches.sort(key=lambda l: l["start_us"])
        result["queued"] = launches
        print(f"== {args.queued} queued renders", flush=True)
        for l in launches:
            print(json.dumps(l), flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(result, f, indent=1)


if __name__ == "__main__":
    main()
