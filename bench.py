"""bench.py — Mpaths/s of the wavefront path tracer (BASELINE.json metric).

Workload (BASELINE.json configs[1]): mitsuba_synth (stand-in for the absent
mitsuba.obj), 1024 x 1024, 64 spp, 8 ray casts per path.  One step = one
full render of that image: every rank renders its interleaved row-group
tile, the fp32 tiles are gathered to rank 0 over RCCL and assembled.  With N
GPUs the same image is split N ways (strong scaling).  --config 0..4 selects
BASELINE.json configs[i] (0 = the 256^2 x 4 spp plumbing run).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...

Prints one JSON line (rank 0) with the metric, the isect kernel's roofline
(HIP events on the render stream) and the CPU-oracle baseline timed on this
host (N = 1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "smallpt-enoki-optix_amd"))

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
PMC_JSON = os.path.join(ROOT, "profiles", "isect_pmc.json")  # tools/pmc_isect.sh output
VALU_PEAK_G = 256 * 4 * 2.4 / 2  # wave64 VALU instr/s (G): 1024 SIMDs, 2 cycles each at 2.4 GHz (MI355X_MICROARCH.md)
ISECT_BYTES_PER_CAST = 52      # queue idx 4 + ray 32 (o, d, tmin, tmax) in, hit 16 out
KERNEL_BYTES_PER_CAST = 44     # what isect_queue_kernel moves: ray 24 + meta 4 in, hit 16 out
FUSED_BYTES_PER_PATH = 12      # per-sample film RGB write


# BASELINE.json configs (index = position in "configs"); 1 is the headline.
CONFIGS = {
    0: dict(scene="mitsuba_synth", width=256, height=256, spp=4, depth=4, smallpt=False),
    1: dict(scene="mitsuba_synth", width=1024, height=1024, spp=64, depth=8, smallpt=False),
    2: dict(scene="smallpt_analytic", width=1024, height=1024, spp=1024, depth=10, smallpt=True),
    3: dict(scene="mitsuba_synth", width=4096, height=4096, spp=256, depth=8, smallpt=False),
    4: dict(scene="city_synth", width=1920, height=1080, spp=64, depth=8, smallpt=False),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", type=int, default=1, choices=sorted(CONFIGS),
                    help="BASELINE.json configs[i]: 0 mitsuba 256^2x4 depth 4 (plumbing), 1 mitsuba 1024^2x64 "
                         "(headline), 2 smallpt's Cornell box 1024^2x1024 (analytic mirror / glass / light spheres, "
                         "emitters, albedo, roulette; --scene cornell_spheres: tessellated diffuse spheres), "
                         "3 mitsuba 4096^2x256, 4 10M-tri city 1920x1080x64")
    ap.add_argument("--width", type=int, default=0)
    ap.add_argument("--height", type=int, default=0)
    ap.add_argument("--spp", type=int, default=0)
    ap.add_argument("--depth", type=int, default=0)
    ap.add_argument("--scene", default="")
    ap.add_argument("--rows-per-group", type=int, default=8)
    ap.add_argument("--wavefront", type=int, default=0, help="paths in flight per launch (0 = auto)")
    ap.add_argument("--pipeline", choices=["auto", "wavefront", "fused"], default="auto",
                    help="isect/shade/refill kernels over path queues (north-star design), one fused "
                         "persistent trace+shade kernel, or auto (the library picks by per-GPU job size: "
                         "fused for at most two wavefronts of paths)")
    ap.add_argument("--timing-all", action="store_true",
                    help="HIP events around every launch (shade/refill/resolve ms too; costs ~5%% host time)")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU-baseline threads (0 = the CPUs this process may use: affinity mask and cgroup quota)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--save", default="", help="write the rank-0 image (.npy) here")
    args = ap.parse_args()
    cfg = CONFIGS[args.config]
    for k in ("scene", "width", "height", "spp", "depth"):
        if not getattr(args, k):
            setattr(args, k, cfg[k])
    args.smallpt = cfg["smallpt"]
    return args


def workload(args, scenes):
    """(mesh dict or OBJ path, render kwargs, albedo, emission) for the config.
    smallpt mode (config 2): Kd albedo, Ke emitters, black sky, roulette from
    cast 5, smallpt's camera; otherwise the reference's semantics (albedo 1,
    sky 1, main.cpp:383 camera)."""
    if args.scene == "city_synth":  # 10M triangles through the pbrt-v3 reader (San Miguel's format), PLY meshes
        return scenes.scene_pbrt("city_synth"), {}, None, None
    if args.scene == "smallpt_analytic":  # smallpt's own scene: quads for the walls, analytic mirror / glass / light spheres
        src = scenes.smallpt_analytic()
    else:
        src = scenes.scene_obj(args.scene)
    if not args.smallpt:
        return src, {}, None, None
    kw = dict(camera=scenes.cornell_camera(), rr_start_depth=5, env=(0.0, 0.0, 0.0))
    return src, kw, True, True


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_share():
    """CPUs this process may run on: the affinity mask, bounded by a cgroup
    CPU quota when one is set (cpu.max), and where each figure came from."""
    import math
    aff = len(os.sched_getaffinity(0))
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(path).read().split()[:2]
            if q != "max":
                quota = float(q) / float(per)
        except (OSError, ValueError):
            pass
    if quota is None:
        try:  # cgroup v1
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    n = aff if quota is None else max(1, min(aff, int(math.floor(quota + 1e-9))))
    return n, {"affinity_cpus": aff, "cgroup_quota_cpus": quota, "os_cpu_count": os.cpu_count()}


def stream_copy_gbs(torch, dev, nbytes=1 << 30, reps=5):
    """Measured HBM peak for the roofline (BASELINE.md plan): a device-to-device
    copy of nbytes, read + write bytes over the best of reps (HIP events)."""
    a = torch.empty(nbytes // 4, dtype=torch.float32, device=dev)
    b = torch.empty_like(a)
    a.fill_(1.0)
    b.copy_(a)
    best = None
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        b.copy_(a)
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1)
        best = ms if best is None else min(best, ms)
    del a, b
    return 2.0 * nbytes / (best * 1e-3) / 1e9


def cpu_baseline(mesh, args, threads, kw, albedo, emission):
    """Oracle (oracle/, a C restatement of main.cpp:354-446, binned-SAH BVH2,
    one pthread per CPU this process may use) on a bounded row sample of the
    same workload, on this host's cores."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle as O

    share, share_src = cpu_share()
    if not threads:
        threads = share
    sc = O.OracleScene(mesh, albedo=albedo, emission=emission)
    p = O.reference_params(args.width, args.height, args.spp, args.depth, **kw)
    # calibrate on 8 rows spread over the image (sky rows at the top are cheap)
    rows = np.unique(np.linspace(0, args.height - 1, 8).astype(np.int32))
    t0 = time.perf_counter()
    sc.render(p, rows=rows, nthreads=threads)
    dt = time.perf_counter() - t0
    # scale the sample to ~cpu_baseline_seconds of work, rows spread over the image
    want = int(max(1, min(args.height, len(rows) * args.cpu_baseline_seconds / max(dt, 1e-3))))
    rows = np.unique(np.linspace(0, args.height - 1, want).astype(np.int32))
    t0 = time.perf_counter()
    _, casts = sc.render(p, rows=rows, nthreads=threads)
    dt = time.perf_counter() - t0
    paths = rows.size * args.width * args.spp
    return {"value": paths / dt / 1e6, "unit": "Mpaths/s", "cores": threads, "kind": "port",
            "cpu": _cpu_model(), "cpus": share_src,
            "sample": f"{rows.size} of {args.height} rows (evenly spaced) x {args.width} px x {args.spp} spp, "
                      f"depth {args.depth}: {paths} paths, {casts} casts in {dt:.2f} s "
                      f"(oracle: C restatement, binned-SAH BVH2, {threads} threads)"}


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    import sptamd
    from sptamd import scenes
    from sptamd.distributed import TileGather

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    # One process per GPU.  SPT_REHEARSE_SHARED_GPU=1 (with SPT_DIST_BACKEND=gloo)
    # lets N ranks share the GPUs there are, to rehearse the N-rank flow on a
    # one-GPU box; the default is strict one-rank-per-device over RCCL.
    if os.environ.get("SPT_REHEARSE_SHARED_GPU") == "1":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        backend = os.environ.get("SPT_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    # scene: generated stand-in, loaded through the OBJ reader like main.cpp:365
    # (rank 0 writes the cached OBJ first)
    if rank == 0 or world == 1:
        src, kw, alb, emi = workload(args, scenes)
    if world > 1:
        dist.barrier()
        if rank != 0:
            src, kw, alb, emi = workload(args, scenes)
    scene = sptamd.Scene()
    if isinstance(src, str):
        scene.add_triangle_mesh(src)
    else:
        scene.add_arrays(src)
    t_commit = time.perf_counter()
    scene.commit(local)
    t_commit = time.perf_counter() - t_commit
    mesh = scene.mesh
    if scene.pbrt_info and scene.pbrt_info["camera"]:  # the .pbrt file's camera
        kw = dict(kw, camera=scene.pbrt_info["camera"])
    if alb:
        alb, emi = scenes.smallpt_materials(mesh)
        scene.backend.set_albedo(alb)
        scene.backend.set_emission(emi)
    else:
        alb = emi = None
    sstats = scene.backend.stats

    W, H = args.width, args.height
    R = args.rows_per_group
    params = sptamd.make_params(W, H, args.spp, args.depth, tile_index=rank, tile_count=world, rows_per_group=R,
                                wavefront_paths=args.wavefront,
                                timing="all" if args.timing_all else True,
                                pipeline=None if args.pipeline == "auto" else args.pipeline, **kw)
    dev = torch.device("cuda", local)
    tg = TileGather(H, W, rank, world, R, dev)
    film = tg.tile_view()
    stream = torch.cuda.current_stream()

    gather_ev = []

    def step(timed=False):
        _, st = scene.render(params, film=film, stream=stream)
        if timed:  # the tile gather (RCCL over xGMI at N > 1) on the render stream's clock
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
        tg.gather()
        if timed:
            e1.record(stream)
            gather_ev.append((e0, e1))
        return st

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    agg = {"ray_casts": 0, "iterations": 0, "isect_ms": 0.0, "shade_ms": 0.0, "continuations": 0,
           "regenerations": 0, "camera_ms": 0.0, "resolve_ms": 0.0, "isect_launches": 0, "isect_busy_ms": 0.0}
    st = {}
    for _ in range(args.steps):
        st = step(timed=True)
        for k in agg:
            agg[k] += st[k]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        rdev = dev if dist.get_backend() == "nccl" else torch.device("cpu")
        t = torch.tensor([elapsed], dtype=torch.float64, device=rdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        tot = torch.tensor([agg["ray_casts"], agg["isect_ms"], agg["iterations"], agg["continuations"]],
                           dtype=torch.float64, device=rdev)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        agg_casts_all = float(tot[0].item())
        agg_cont_all = float(tot[3].item())
    else:
        agg_casts_all = float(agg["ray_casts"])
        agg_cont_all = float(agg["continuations"])

    paths = W * H * args.spp * args.steps
    value = paths / elapsed / 1e6
    gather_ms = sum(e0.elapsed_time(e1) for e0, e1 in gather_ev) / max(1, len(gather_ev))
    if rank == 0:
        # Roofline of the dominant kernel.  Wavefront:
        # isect_queue_kernel, SURVEY §8(d)'s 52 B per ray cast.  The K
        # sub-wavefront streams' isect launches overlap, so the headline
        # divides the bytes of ALL isect launches by the union of their
        # intervals (HIP events on each launch's own stream): the time the
        # kernel occupies the chip, <= ms_per_step.  `per_launch` keeps the
        # per-launch figure (a 1/K-chip rate when K > 1).  Fused:
        # render_fused_kernel, whose only HBM stream is the per-sample film
        # write (12 B per path; rays stay in registers).
        fused = bool(st.get("fused"))
        wo = scene.backend.config["work_order"]
        work_order = {1: "sample-major", 2: "pixel-major"}.get(wo) or (
            ("pixel-major" if sstats["device_bytes"] >= 256 << 20 or (fused and W * H * args.spp // world >= 16 << 20)
             or (not fused and sstats["device_bytes"] >= 4 << 20 and W * H // world <= 4 << 20)
             else "sample-major") + " (auto)")
        launches = max(agg["isect_launches"], 1)
        avg_ms = agg["isect_ms"] / launches
        casts_per_launch = agg["ray_casts"] / launches
        if fused:
            bytes_per_unit, kernel_bytes_per_unit = FUSED_BYTES_PER_PATH, FUSED_BYTES_PER_PATH
            total_bytes = st["paths"] * args.steps * FUSED_BYTES_PER_PATH
        else:
            bytes_per_unit, kernel_bytes_per_unit = ISECT_BYTES_PER_CAST, KERNEL_BYTES_PER_CAST
            total_bytes = agg["ray_casts"] * ISECT_BYTES_PER_CAST
        bytes_per_launch = total_bytes / launches
        busy_ms = agg["isect_busy_ms"]
        achieved = total_bytes / (busy_ms * 1e-3) / 1e9 if busy_ms > 0 else 0.0
        per_launch = bytes_per_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
        # whole-path bytes: B_path = 84 + 120 S + 60 C, S = casts and
        # C = continuations per path, over the whole frame time, against the spec
        # peak and a stream-copy peak measured here (BASELINE.md plan)
        s_bar = agg_casts_all / paths
        c_bar = agg_cont_all / paths
        b_path = 84.0 + 120.0 * s_bar + 60.0 * c_bar
        path_gbs = b_path * paths / elapsed / 1e9
        copy_gbs = stream_copy_gbs(torch, dev)
        pmc = None
        if os.path.exists(PMC_JSON) and not fused and world == 1:  # PMC passes (profiles/, tools/pmc_isect.py)
            pmc = json.load(open(PMC_JSON)).get(f"config{args.config}")
        traffic = traffic_per_cast = None
        if pmc and pmc.get("traffic_bytes_per_cast"):
            traffic_per_cast = pmc["traffic_bytes_per_cast"]
            traffic = round(traffic_per_cast * casts_per_launch)
        valu = None
        if pmc and pmc.get("valu_insts_per_cast") and busy_ms > 0:
            rate = pmc["valu_insts_per_cast"] * agg["ray_casts"] / (busy_ms * 1e-3) / 1e9
            valu = {"insts_per_cast": round(pmc["valu_insts_per_cast"], 2), "achieved": round(rate, 1),
                    "peak": VALU_PEAK_G, "unit": "G wave64 VALU instr/s over isect busy time",
                    "frac": round(rate / VALU_PEAK_G, 4)}
        rec = {
            "metric": "Mpaths/sec (pixels x spp / s), mitsuba.obj-standin 1024^2 x 64spp, depth 8"
                      if args.config == 1 else f"Mpaths/sec (pixels x spp / s), BASELINE config {args.config}",
            "value": round(value, 3),
            "unit": "Mpaths/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic ({args.scene} stand-in generated in-run; reference asset absent)",
            "work_order_rule": "auto: pixel-major for scenes of >= 256 MiB, fused tiles of >= 16M paths and "
                               "wavefront tiles of <= 4M px over scenes of >= 4 MiB (24M paths in flight), "
                               "else sample-major (DESIGN.md §4)",
            "pipeline_rule": "auto: fused for tiles of <= 32M paths, else wavefront (DESIGN.md §6)"
                             if args.pipeline == "auto" else f"--pipeline {args.pipeline}",
            "config": {"pipeline": "fused" if fused else "wavefront", "streams": st.get("streams"),
                       "workload": f"{args.scene} {W}x{H} {args.spp}spp depth {args.depth}"
                                   + (" (smallpt materials: Kd albedo, Ke light, black sky, RR from cast 5)"
                                      if args.smallpt else ""),
                       "triangles": int(sstats["ntri"]), "tiles": f"{world} x interleaved {R}-row groups",
                       "paths_in_flight": st.get("paths_in_flight"), "rays_per_path": round(agg_casts_all / paths, 4),
                       "work_order": work_order},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                         "kernel": "render_fused_kernel" if fused else "isect_queue_kernel",
                         "basis": "algorithmic bytes of all launches / union of their intervals (isect busy)",
                         "bytes_per_unit": bytes_per_unit, "kernel_bytes_per_unit": kernel_bytes_per_unit,
                         "unit_of_work": "path" if fused else "ray cast",
                         "algorithmic_bytes_per_launch": round(bytes_per_launch),
                         "traffic_per_unit": traffic_per_cast,
                         "traffic_ratio": round(traffic / bytes_per_launch, 3) if traffic else None,
                         "busy_ms_per_step": round(busy_ms / args.steps, 4),
                         "launches_per_step": round(launches / args.steps, 2),
                         "avg_launch_ms": round(avg_ms, 4),
                         "grays_per_s": round(agg["ray_casts"] / (busy_ms * 1e-3) / 1e9, 4) if busy_ms else None,
                         "per_launch": {"achieved": round(per_launch, 2), "frac": round(per_launch / HBM_PEAK_GBS, 5),
                                        "note": f"per-launch duration; {st.get('streams')} streams overlap"},
                         "pmc_source": os.path.relpath(PMC_JSON, ROOT) + f"#config{args.config}" if pmc else None,
                         "valu": valu,
                         "stream_copy_peak": round(copy_gbs, 1),
                         "path": {"bytes_per_path": round(b_path, 1),
                                  "formula": "84 + 120*S + 60*C (SURVEY 8d), S=%.4f C=%.4f" % (s_bar, c_bar),
                                  "achieved": round(path_gbs, 1), "frac": round(path_gbs / HBM_PEAK_GBS, 4),
                                  "frac_of_stream_copy": round(path_gbs / copy_gbs, 4)}},
            "gather_ms": round(gather_ms, 4),
            "kernel_ms_per_step": {k: round(agg[k] / args.steps, 3) for k in
                                   (("isect_ms", "shade_ms", "camera_ms", "resolve_ms") if args.timing_all
                                    else ("isect_ms",))},
            "bvh": dict({k: sstats[k] for k in ("builder", "nodes", "max_depth", "build_ms", "sah_cost", "device_bytes")},
                        commit_s=round(t_commit, 3)),
        }
        if args.save:
            np.save(args.save, tg.image.cpu().numpy())
        if world == 1 and not args.no_cpu_baseline:
            rec["cpu_baseline"] = cpu_baseline(mesh, args, args.cpu_threads, kw, alb, emi)
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
