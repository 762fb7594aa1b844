"""Strong-scaling projection on one GPU: render tile 0 of N (the share one
rank gets under `bench.py --gpus N`) and report the tile's Mpaths/s and the
projected whole-job rate N x that (ignores the gather, ~0.2 ms).

    python tools/tile_sim.py [--config 1] [--tiles 1 2 4 8] [--steps 5]
"""
from __future__ import annotations

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
    ap.add_argument("--config", type=int, default=1)
    ap.add_argument("--tiles", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--rows-per-group", type=int, default=8)
    ap.add_argument("--pipeline", default=None, help="wavefront | fused (default: the library's auto choice)")
    ap.add_argument("--timing", action="store_true", help="HIP events around every launch (as bench.py)")
    ap.add_argument("--wavefront", type=int, default=0, help="paths in flight (0 = the library default)")
    ap.add_argument("--sync", action="store_true", help="spt_render per step (no queued renders)")
    ap.add_argument("--sweep", nargs="*", default=[],
                    help="SPT_* knobs to sweep in this process, e.g. SPT_STREAMS=1,2,4 SPT_DRAIN_Q8=256,512 "
                         "(every combination, each tile count)")
    args = ap.parse_args()
    import itertools
    axes = [(kv.split("=", 1)[0], kv.split("=", 1)[1].split(",")) for kv in args.sweep]
    combos = list(itertools.product(*[v for _, v in axes])) or [()]
    import torch

    import bench
    import sptamd
    from sptamd import scenes

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
    for combo in combos:
        env = {name: val for (name, _), val in zip(axes, combo)}
        os.environ.update(env)
        run_tiles(args, scene, cfg, kw, W, H, spp, D, env)


_QUEUE_STREAMS = []


def run_tiles(args, scene, cfg, kw, W, H, spp, D, env):
    import torch

    import sptamd
    for n in args.tiles:
        p = sptamd.make_params(W, H, spp, D, tile_index=0, tile_count=n, rows_per_group=args.rows_per_group,
                               timing=args.timing, pipeline=None if args.pipeline in (None, "auto") else args.pipeline,
                               wavefront_paths=args.wavefront, **kw)
        rows = len(sptamd._lib.tile_rows(H, 0, n, args.rows_per_group))
        films = [torch.empty((3, rows, W), dtype=torch.float32, device="cuda") for _ in range(2)]
        # the two caller streams renders alternate on, as bench.py: two streams
        # with a hardware queue each (sptamd.queue_stream, made once);
        # SPT_SIM_POOL=1: two torch pool streams; SPT_SIM_POOL=0: the current
        # (legacy null) stream and one pool stream
        pool = os.environ.get("SPT_SIM_POOL", "2")
        if pool == "2":
            if not _QUEUE_STREAMS:
                _QUEUE_STREAMS.extend([sptamd.queue_stream(), sptamd.queue_stream()])
            streams = list(_QUEUE_STREAMS)
        elif pool == "3":  # a normal- and a high-priority pool stream (separate queue pools)
            streams = [torch.cuda.Stream(priority=0), torch.cuda.Stream(priority=-1)]
        else:
            streams = ([torch.cuda.Stream(), torch.cuda.Stream()] if pool == "1"
                       else [torch.cuda.current_stream(), torch.cuda.Stream()])
        for k in range(2):  # one setup render per stream (working set) before the timed steps, as bench.py
            scene.render_wait(scene.render_async(p, film=films[k], stream=streams[k])[1])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if args.sync:
            for _ in range(args.steps):
                _, st = scene.render(p, film=films[0])
        else:  # as bench.py: renders queued back to back on two alternating streams
            tickets = [scene.render_async(p, film=films[i % 2], stream=streams[i % 2])[1] for i in range(args.steps)]
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.steps
        if not args.sync:
            st = [scene.render_wait(t) for t in tickets][-1]
        paths = rows * W * spp
        rate = paths / dt / 1e6
        print(json.dumps({"tiles": n, "tile_rows": rows, "ms_per_step": round(dt * 1e3, 3),
                          "tile_mpaths_s": round(rate, 1), "projected_job_mpaths_s": round(rate * n, 1),
                          "iterations": st["iterations"], "fused": st["fused"], "streams": st["streams"],
                          "drained_paths": st["drained_paths"], "drain_launches": st["drain_launches"],
                          "paths": st["paths"], **env,
                          "env": {k: v for k, v in sorted(os.environ.items())
                                  if k.startswith("SPT_") or k == "GPU_MAX_HW_QUEUES"}}), flush=True)
        assert st["paths"] == paths and st["film_slots_unwritten"] == 0, st


if __name__ == "__main__":
    main()
