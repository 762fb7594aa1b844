"""Where a lane-loop wave's time goes (drain, fused kernel), from the
diagnostic build (make BUILD=build_wlog EXTRA=-DSPT_WAVE_LOG=1): shader-clock
cycles in trace steps vs in shade + refill passes, summed over every wave, with
the lane occupancy of the trace steps and the lanes per pass.  Tells whether a
drain is bound by its traversal or by its per-pass shading / refill — what
spt_config.drain_refill_idle trades.

    SPT_LIB=smallpt-enoki-optix_amd/build_wlog/libspt.so \
        python tools/phase_log.py --config 1 [--renders 2]
(SPT_DRAIN_IDLE etc. in the environment pick the knob under study.)
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "smallpt-enoki-optix_amd"))
sys.path.insert(0, ROOT)

NAMES = ("trace_cycles", "pass_cycles", "trace_steps", "passes", "busy_lane_steps", "lanes_shaded",
         "lanes_refilled", "refill_cycles")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=1)
    ap.add_argument("--renders", type=int, default=2)
    args = ap.parse_args()
    import torch

    import bench
    import sptamd
    from sptamd import _lib, scenes

    lib = _lib.lib
    if not hasattr(lib, "spt_debug_phase_log"):
        raise SystemExit(f"{_lib.LIB_PATH} is not a wave-log build (make BUILD=build_wlog EXTRA=-DSPT_WAVE_LOG=1)")
    lib.spt_debug_phase_log.restype = ctypes.c_int
    lib.spt_debug_phase_log.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = (ctypes.c_ulonglong * 8)()

    def read(reset=True):
        if lib.spt_debug_phase_log(buf, 1 if reset else 0) != 0:
            raise RuntimeError("spt_debug_phase_log failed")
        return dict(zip(NAMES, [int(x) for x in buf]))

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
    film = torch.empty((3, H, W), dtype=torch.float32, device="cuda")
    scene.render(p, film=film)  # warm-up (builds, allocations)
    torch.cuda.synchronize()
    read()
    for r in range(args.renders):
        _, st = scene.render(p, film=film)
        torch.cuda.synchronize()
        c = read()
        tot = max(c["trace_cycles"] + c["pass_cycles"], 1)
        out = {"config": args.config, "render": r, "refill_idle": st.get("drain_refill_idle"),
               "env": {k: v for k, v in sorted(os.environ.items()) if k.startswith("SPT_") and k != "SPT_LIB"},
               "pass_frac": round(c["pass_cycles"] / tot, 4),
               "cycles_per_step": round(c["trace_cycles"] / max(c["trace_steps"], 1), 1),
               "cycles_per_pass": round(c["pass_cycles"] / max(c["passes"], 1), 1),
               "refill_cycles_per_pass": round(c["refill_cycles"] / max(c["passes"], 1), 1),
               "busy_lanes_per_step": round(c["busy_lane_steps"] / max(c["trace_steps"], 1), 2),
               "lanes_shaded_per_pass": round(c["lanes_shaded"] / max(c["passes"], 1), 2),
               "lanes_refilled_per_pass": round(c["lanes_refilled"] / max(c["passes"], 1), 2),
               "steps_per_pass": round(c["trace_steps"] / max(c["passes"], 1), 2),
               "counts": c}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
