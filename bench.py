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
(HIP events on the render stream), the CPU-oracle baseline timed on this
host, and the parity of the (assembled) image against that oracle render.
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "smallpt-enoki-optix_amd"))

# Hardware queues per process: the environment's GPU_MAX_HW_QUEUES (HIP's
# default and the GPU box's setting: 4) is what a library caller gets, so the
# bench keeps it.  The library's default wavefront (two
# sub-wavefront streams per working set, two sets: four streams, DESIGN.md
# §6b) fits four queues.  SPT_HW_QUEUES overrides it for an experiment; the
# HIP runtime reads it when it starts, so that happens before torch is
# imported.  The line records the value in effect.
HW_QUEUES_ENV = os.environ.get("GPU_MAX_HW_QUEUES")
if os.environ.get("SPT_HW_QUEUES"):
    os.environ["GPU_MAX_HW_QUEUES"] = os.environ["SPT_HW_QUEUES"]

PG_TIMEOUT = datetime.timedelta(minutes=20)  # torch.distributed collectives (CPU baseline on rank 0)
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
PMC_JSON = os.path.join(ROOT, "profiles", "isect_pmc.json")  # tools/pmc_isect.sh output
VALU_PEAK_G = 256 * 4 * 2.4 / 2  # wave64 VALU instr/s (G): 1024 SIMDs, 2 cycles each at 2.4 GHz (MI355X_MICROARCH.md)
ISECT_BYTES_PER_CAST = 52      # queue idx 4 + ray 32 (o, d, tmin, tmax) in, hit 16 out
KERNEL_BYTES_PER_CAST = 44     # what isect_queue_kernel moves: ray 24 + meta 4 in, hit 16 out
# what render_fused_kernel itself moves per path: its per-sample
# film write, one escape byte (the reference's unit mode) or an RGB float triple
FUSED_BYTES_PER_PATH = {True: 1, False: 12}


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
    # 20 timed steps by default (0.26 s on config 1): the first and last renders of the timed
    # region overlap nothing, which costs a 3-step run ~1 % (5096 vs 5159 Mpaths/s, r04_final)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
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
    ap.add_argument("--no-fused-leg", action="store_true",
                    help="at N > 1, skip timing the fused pipeline beside the wavefront on the same tiles")
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
    copy of nbytes through torch's vectorised elementwise kernel (b = a * 1),
    read + write bytes over the best of reps (HIP events).  That kernel reads
    6.24 TB/s on the box, the float4-copy rate MI355X_MICROARCH.md quotes
    (6.29); `copy_` goes through the runtime's blit kernel at 5.2
    (profiles/r05_exp/c4_knobs_copy/copy_peak.log, tools/copy_peak.py)."""
    a = torch.empty(nbytes // 4, dtype=torch.float32, device=dev)
    b = torch.empty_like(a)
    a.fill_(1.0)
    torch.mul(a, 1.0, out=b)
    best = None
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        torch.mul(a, 1.0, out=b)
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1)
        best = ms if best is None else min(best, ms)
    del a, b
    return 2.0 * nbytes / (best * 1e-3) / 1e9


def cpu_baseline(mesh, args, threads, kw, albedo, emission):
    """Oracle (oracle/, a C restatement of main.cpp:354-446, binned-SAH BVH2,
    one pthread per CPU this process may use) on a bounded row sample of the
    same workload, on this host's cores.  Returns the record and the oracle's
    (rows, film) so the caller can check the GPU image against it."""
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
    # the whole image when that costs at most ~3x the budget: the GPU image is
    # then checked against the oracle row for row (the "parity" field)
    if args.height * dt / len(rows) <= 3.0 * args.cpu_baseline_seconds:
        want = args.height
    rows = np.unique(np.linspace(0, args.height - 1, want).astype(np.int32))
    t0 = time.perf_counter()
    film, casts = sc.render(p, rows=rows, nthreads=threads)
    dt = time.perf_counter() - t0
    paths = rows.size * args.width * args.spp
    return (rows, film), {"value": paths / dt / 1e6, "unit": "Mpaths/s", "cores": threads, "kind": "port",
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
    from sptamd import _lib, scenes
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
        ndev = max(1, torch.cuda.device_count())
        local = local % ndev
        # the ranks on one device split its memory: each rank's two working
        # sets get an equal share of 3/4 of it for a fitting job (spt_config.fit_bytes;
        # the library's own free-memory check races when all ranks start at once)
        if "SPT_FIT_BYTES" not in os.environ:
            share = (world + ndev - 1) // ndev
            total = torch.cuda.get_device_properties(local).total_memory
            os.environ["SPT_FIT_BYTES"] = str(total * 3 // 4 // (2 * share))
    torch.cuda.set_device(local)
    if world > 1:
        backend = os.environ.get("SPT_DIST_BACKEND", "nccl")
        if backend == "nccl":
            # rank 0 times the CPU baseline (up to ~40 s on config 4) while the
            # others wait at a barrier: a timeout well past that
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=PG_TIMEOUT)
        else:
            dist.init_process_group(backend, timeout=PG_TIMEOUT)

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

    def check_work(st):
        """Device-counted work of one render against the job (main.cpp:385-429
        renders every pixel x sample): paths started == paths ended == tile
        pixels x spp, and no per-sample film slot left unwritten."""
        want = st["tile_rows"] * W * args.spp
        bad = (st["paths_started"] != want or st["paths_terminated"] != want or st["film_slots_unwritten"] != 0)
        if bad:
            raise RuntimeError(f"rank {rank}: lost work: started {st['paths_started']}, terminated "
                               f"{st['paths_terminated']}, unwritten film slots {st['film_slots_unwritten']}, "
                               f"expected {want} paths")
        return want

    # one setup render per stream: the library binds a working set to each
    # caller stream (spt.h spt_render_async); SPT_BENCH_SETUP / SPT_BENCH_SYNC
    # (experiment knobs, tools/ov.sh): setup renders, one render at a time
    SETUP_RENDERS = int(os.environ.get("SPT_BENCH_SETUP", "2"))
    SYNC_STEPS = os.environ.get("SPT_BENCH_SYNC", "0") == "1"
    # Consecutive steps alternate between two streams and two film buffers
    # (the library alternates two working sets), so a step's render can start
    # while the previous one drains; the gathers stay in step order.
    # two side streams with a hardware queue each (sptamd.queue_stream, as
    # INTEGRATION.md tells a caller queueing renders): on two ordinary streams
    # that HIP happened to map onto one hardware queue, the caller-side wait
    # that ends one render blocked the next render's start, and about one run
    # in ten lost the overlap (~30 % slower).  SPT_BENCH_STREAMS
    # =pool: two torch pool streams instead (the earlier behaviour, A/B only).
    if os.environ.get("SPT_BENCH_STREAMS", "queue") == "pool":
        streams = [torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)]
    elif os.environ.get("SPT_BENCH_STREAMS") == "prio":  # experiment: normal + high priority pool streams
        streams = [torch.cuda.Stream(device=dev, priority=0), torch.cuda.Stream(device=dev, priority=-1)]
    else:
        streams = [sptamd.queue_stream(dev.index if dev.index is not None else 0) for _ in range(2)]
    films = [film, tg.tile_view(1)]
    last_gather = [None]

    def step(p, ev=None, k=0):
        """One step: the render of this rank's tile, queued (spt_render_async:
        the GPU runs from one step's render into the next without waiting for
        the host), then the tile gather behind it on the same stream, after the
        previous step's gather (timed by the event pair ev, if given).  Returns
        the render's ticket; its device counters are collected after the loop."""
        s = streams[k % 2]
        with torch.cuda.stream(s):
            _, ticket = scene.render_async(p, film=films[k % 2], stream=s)
            if last_gather[0] is not None:
                s.wait_event(last_gather[0])
            if ev is not None:  # the tile gather (RCCL over xGMI at N > 1) on the render stream's clock
                ev[0].record(s)
            tg.gather(k % 2)
            done = torch.cuda.Event()
            done.record(s)
            last_gather[0] = done
            if ev is not None:
                ev[1].record(s)
        return ticket

    def timed_loop(p):
        """W untimed steps, then exactly K timed steps between barriers +
        synchronize; returns (max-over-ranks seconds, summed stats, last stats,
        device-counted [casts, continuations, paths] of all ranks, this loop's
        mean gather ms).  Every step's work accounting is checked once the
        timed region has ended.  Before the warmup, one setup render per
        working set and stream (SETUP_RENDERS): their buffers are allocated on
        first use, which W = 1 warmup step would leave to the first timed step."""
        # this loop's own gather timing events (recorded on the step's stream)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(args.steps)]
        for k in range(SETUP_RENDERS):
            check_work(scene.render_wait(step(p, k=k)))
        for w in range(args.warmup):
            check_work(scene.render_wait(step(p, k=w)))
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        # the isect (fused) kernel's busy time: the union of every timed
        # launch interval of the K renders, which overlap on two streams
        scene.isect_busy_begin()
        t0 = time.perf_counter()
        tickets, sts = [], []
        for i in range(args.steps):
            tickets.append(step(p, evs[i], k=i))
            if SYNC_STEPS:
                sts.append(scene.render_wait(tickets.pop(0)))
            if len(tickets) > 32:  # the library holds at most 64 uncollected renders
                sts.append(scene.render_wait(tickets.pop(0)))
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        agg = {"ray_casts": 0, "iterations": 0, "isect_ms": 0.0, "shade_ms": 0.0, "continuations": 0,
               "regenerations": 0, "camera_ms": 0.0, "resolve_ms": 0.0, "isect_launches": 0, "isect_busy_ms": 0.0,
               "paths": 0, "drained_paths": 0, "drained_casts": 0, "drain_launches": 0, "drain_ms": 0.0,
               "lockstep_casts": 0}
        sts += [scene.render_wait(t) for t in tickets]
        for st in sts:
            check_work(st)
            for k in agg:
                agg[k] += st[k]
        # consecutive renders overlap on the GPU (two streams, two working
        # sets): the kernel's busy time is the union of all their launch
        # intervals on the scene's clock (spt_scene_kernel_busy / _isect_busy_end)
        agg["drain_busy_ms"], agg["drain_launches_timed"] = scene.kernel_busy(_lib.SPT_KERNEL_DRAIN)
        agg["trace_busy_ms"], _ = scene.kernel_busy(_lib.SPT_KERNEL_ISECT | _lib.SPT_KERNEL_DRAIN)
        agg["isect_busy_ms"], nl = scene.isect_busy_end()
        if nl != agg["isect_launches"]:
            raise RuntimeError(f"isect intervals {nl} != timed launches {agg['isect_launches']}")
        gather_ms = sum(e0.elapsed_time(e1) for e0, e1 in evs) / max(1, len(evs))
        tot = [agg["ray_casts"], agg["continuations"], agg["paths"]]
        if world > 1:
            rdev = dev if dist.get_backend() == "nccl" else torch.device("cpu")
            t = torch.tensor([elapsed], dtype=torch.float64, device=rdev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
            tt = torch.tensor(tot, dtype=torch.float64, device=rdev)
            dist.all_reduce(tt, op=dist.ReduceOp.SUM)
            tot = [float(x) for x in tt.tolist()]
        return elapsed, agg, sts[-1], tot, gather_ms

    elapsed, agg, st, (agg_casts_all, agg_cont_all, paths), gather_ms = timed_loop(params)
    if paths != W * H * args.spp * args.steps:
        raise RuntimeError(f"device-counted paths {paths} != {W * H * args.spp * args.steps} (W x H x spp x steps)")
    image_main = tg.image.clone() if rank == 0 else None
    # At N > 1 the fused pipeline is timed beside the wavefront on the same
    # tiles (a second loop after the first), so the N-GPU line says how the
    # north-star pipeline compares per tile (>= 0.9x).
    other_leg = None
    if world > 1 and args.pipeline == "auto" and not args.no_fused_leg:
        other = "wavefront" if st.get("fused") else "fused"
        pw = sptamd.make_params(W, H, args.spp, args.depth, tile_index=rank, tile_count=world, rows_per_group=R,
                                wavefront_paths=args.wavefront, timing=True, pipeline=other, **kw)
        w_el, w_agg, w_st, w_tot, w_gather_ms = timed_loop(pw)
        w_paths = w_tot[2]
        other_leg = {"pipeline": other, "value": round(w_paths / w_el / 1e6, 3),
                     "ms_per_step": round(w_el / args.steps * 1e3, 3), "streams": w_st.get("streams"),
                     "paths_device_counted": int(w_paths), "gather_ms": round(w_gather_ms, 4)}
        if rank == 0 and image_main is not None:
            other_leg["image_equal"] = bool(torch.equal(image_main, tg.image))
    value = paths / elapsed / 1e6
    if rank == 0:
        # Roofline of the dominant kernel.  Wavefront:
        # isect_queue_kernel, SURVEY §8(d)'s 52 B per ray cast.  The K
        # sub-wavefront streams' isect launches overlap, so the headline
        # divides the bytes of ALL isect launches by the union of their
        # intervals (HIP events on each launch's own stream): the time the
        # kernel occupies the chip, <= ms_per_step.  `per_launch` keeps the
        # per-launch figure (a 1/K-chip rate when K > 1).  Fused:
        # render_fused_kernel runs the whole path (trace + shade + bounce) in
        # registers; its unit is the ray cast at SURVEY §8(d)'s 52 B, like the
        # isect kernel and the drain, while what it moves is the per-sample
        # film write (1 B in the reference's unit mode, 12 B of RGB
        # otherwise: kernel_bytes_per_unit); §8(d)'s whole-path model B_path =
        # 84 + 120 S + 60 C over its busy time is reported beside it as
        # `equivalent_wavefront`.
        fused = bool(st.get("fused"))
        work_order = {1: "sample-major", 2: "pixel-major"}.get(st.get("work_order"), "?")
        if scene.backend.config["work_order"] == 0:
            work_order += " (auto)"
        queue_cache = {0: None, 1: "cached", 2: "stream"}.get(st.get("queue_cache"), "?")
        if queue_cache and scene.backend.config["queue_cache"] == 0:
            queue_cache += " (auto)"
        # The wavefront's two tracing kernels: isect_queue_kernel (the casts
        # of the per-cast launches, SURVEY §8(d)'s 52 B per cast) and the drain
        # (render_fused_kernel's lane loop over a queue: it reads each queued
        # path once and writes its film slot; the casts after that stay in
        # registers).  The roofline names the one with the longer busy time
        # (the union of its launch intervals over the timed renders).
        isect_launches = max(agg["isect_launches"], 1)
        s_bar = agg_casts_all / paths
        c_bar = agg_cont_all / paths
        b_path = 84.0 + 120.0 * s_bar + 60.0 * c_bar
        unit_mode = not args.smallpt  # albedo 1, no emitters: the reference's case (one escape byte per path)
        film_b = FUSED_BYTES_PER_PATH[unit_mode]
        queue_b = 32 if unit_mode else 56  # PathQueue planes a queued path carries (q1, q2 [, q0, rad])
        isect_casts = agg["ray_casts"] - agg["drained_casts"]
        kernels = {}
        if fused:
            # the same per-cast basis as the drain (the same lane loop): SURVEY
            # §8(d)'s 52 B per cast; the kernel itself moves only its film writes
            # (kernel_bytes_per_unit per cast), so the HBM fraction is low and
            # `limiter` names what bounds it
            kernels["render_fused_kernel"] = dict(
                units=agg["ray_casts"], unit="ray cast", bytes_per_unit=ISECT_BYTES_PER_CAST,
                kernel_bytes_per_unit=round(agg["paths"] * film_b / max(agg["ray_casts"], 1), 3),
                bytes=agg["ray_casts"] * ISECT_BYTES_PER_CAST, busy_ms=agg["isect_busy_ms"], launches=isect_launches,
                sum_ms=agg["isect_ms"], casts=agg["ray_casts"],
                basis="SURVEY 8(d) 52 B per ray cast of all fused launches / union of their intervals (the fused "
                      "kernel keeps a path in registers: it moves kernel_bytes_per_unit per cast, its film write)")
        else:
            # the isect launches: a fitting job's first cast runs in the
            # one-lane-per-ray kernel (spt_config.lockstep_first), later casts
            # and other jobs in the persistent one; the name says which ran
            lock = agg["lockstep_casts"]
            # (lockstep_first >= 2 on a wide-BVH scene: the camera-cast kernel makes,
            # traces and shades the first cast; it moves its survivors' queue
            # entries and the others' film writes)
            cam = scene.backend.config["lockstep_first"] >= 2 and int(sstats["bvh_width"]) != 2
            first = "camera_cast_kernel" if cam else "isect_lockstep_kernel"
            isect_name = (first if lock == isect_casts else
                          "isect_queue_kernel" if lock == 0 else first + "+isect_queue_kernel")
            kb = KERNEL_BYTES_PER_CAST
            if cam and lock == isect_casts and isect_casts:
                kb = round((agg["drained_paths"] * queue_b + (isect_casts - agg["drained_paths"]) * film_b)
                           / isect_casts, 3)
            kernels[isect_name] = dict(
                units=isect_casts, unit="ray cast", bytes_per_unit=ISECT_BYTES_PER_CAST,
                kernel_bytes_per_unit=kb, bytes=isect_casts * ISECT_BYTES_PER_CAST,
                busy_ms=agg["isect_busy_ms"], launches=isect_launches, sum_ms=agg["isect_ms"], casts=isect_casts,
                basis="algorithmic bytes of all isect launches / union of their intervals (isect busy)")
            if agg["drain_launches"]:
                # SURVEY §8(d)'s per-cast figure, as for the isect kernel: the drain
                # traces (and shades) ray casts; what it moves per cast — the queued
                # path read once, its film write — is kernel_bytes_per_unit
                moved = agg["drained_paths"] * (queue_b + film_b) / max(agg["drained_casts"], 1)
                kernels["render_fused_kernel<drain>"] = dict(
                    units=agg["drained_casts"], unit="ray cast", bytes_per_unit=ISECT_BYTES_PER_CAST,
                    kernel_bytes_per_unit=round(moved, 2), bytes=agg["drained_casts"] * ISECT_BYTES_PER_CAST,
                    busy_ms=agg["drain_busy_ms"], launches=max(agg["drain_launches_timed"], 1),
                    sum_ms=agg["drain_ms"], casts=agg["drained_casts"],
                    basis="SURVEY 8(d) 52 B per ray cast of all drain launches / union of their intervals (the "
                          "drain keeps a path in registers between casts: it moves kernel_bytes_per_unit per cast)")
        dom_name = max(kernels, key=lambda k: kernels[k]["busy_ms"])
        dom = kernels[dom_name]
        launches = dom["launches"]
        avg_ms = dom["sum_ms"] / launches
        busy_ms = dom["busy_ms"]
        bytes_per_unit, kernel_bytes_per_unit = dom["bytes_per_unit"], dom["kernel_bytes_per_unit"]
        total_bytes = dom["bytes"]
        bytes_per_launch = total_bytes / launches
        achieved = total_bytes / (busy_ms * 1e-3) / 1e9 if busy_ms > 0 else 0.0
        per_launch = bytes_per_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
        kernel_table = {
            k: {"busy_ms_per_step": round(v["busy_ms"] / args.steps, 4), "launches_per_step": round(v["launches"] / args.steps, 2),
                "casts_per_step": round(v["casts"] / args.steps), "units_per_step": round(v["units"] / args.steps),
                "unit": v["unit"], "bytes_per_unit": v["bytes_per_unit"],
                "achieved_gbs": round(v["bytes"] / (v["busy_ms"] * 1e-3) / 1e9, 2) if v["busy_ms"] > 0 else None,
                "grays_per_s": round(v["casts"] / (v["busy_ms"] * 1e-3) / 1e9, 4) if v["busy_ms"] > 0 else None}
            for k, v in kernels.items()}
        equiv = None
        if fused:
            eq_gbs = paths / world * b_path / (busy_ms * 1e-3) / 1e9 if busy_ms > 0 else 0.0
            equiv = {"bytes_per_path": round(b_path, 1), "achieved": round(eq_gbs, 2),
                     "frac": round(eq_gbs / HBM_PEAK_GBS, 5),
                     "note": "SURVEY 8(d) whole-path bytes the per-cast launches would move for these paths, over the "
                             "kernel's busy time; the lane loop keeps them in registers"}
        # whole-path bytes over the whole frame time, against the
        # spec peak and a stream-copy peak measured here (BASELINE.md plan)
        path_gbs = b_path * paths / elapsed / 1e9
        copy_gbs = stream_copy_gbs(torch, dev)
        build_id = _lib.lib.spt_build_id().decode()
        pmc = pmc_note = None
        key = f"config{args.config}" + ("_fused" if fused else "_drain" if dom_name.endswith("<drain>") else "")
        if os.path.exists(PMC_JSON) and world == 1:  # PMC passes (profiles/, tools/pmc_isect.sh)
            pmc = json.load(open(PMC_JSON)).get(key)
            if pmc and pmc.get("build_id") != build_id:
                pmc_note = (f"{key} was measured on build {pmc.get('build_id')}, this library is {build_id}: "
                            "not used")
                pmc = None
        # PMC figures are per ray cast for every kernel (the drain and the
        # fused kernel also per path), so the same basis serves any of them
        traffic = traffic_per_unit = None
        if pmc and pmc.get("traffic_bytes_per_cast"):
            traffic_per_unit = pmc["traffic_bytes_per_cast"]
            traffic = round(traffic_per_unit * dom["casts"] / launches)
        valu = None
        if pmc and pmc.get("valu_insts_per_cast") and busy_ms > 0:
            rate = pmc["valu_insts_per_cast"] * dom["casts"] / (busy_ms * 1e-3) / 1e9
            valu = {"insts_per_cast": round(pmc["valu_insts_per_cast"], 2), "achieved": round(rate, 1),
                    "peak": VALU_PEAK_G, "unit": "G wave64 VALU instr/s over kernel busy time",
                    "frac": round(rate / VALU_PEAK_G, 4)}
        rec = {
            "metric": "Mpaths/sec (pixels x spp / s), mitsuba.obj-standin 1024^2 x 64spp, depth 8"
                      if args.config == 1 else f"Mpaths/sec (pixels x spp / s), BASELINE config {args.config}",
            "value": round(value, 3),
            "unit": "Mpaths/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "setup_renders": SETUP_RENDERS,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic ({args.scene} stand-in generated in-run; reference asset absent)",
            "work_check": {"paths_device_counted": int(paths), "expected": W * H * args.spp * args.steps,
                           "rule": "every step, every rank: paths started == paths ended == tile px x spp, "
                                   "0 film slots unwritten (spt_render_stats)"},
            "dist": {"backend": dist.get_backend() if world > 1 else None, "world_size": world},
            "work_order_rule": "auto: pixel-major for scenes of >= 256 MiB, fused tiles of >= 16M paths, and "
                               "wavefront tiles of <= 4M px or jobs started at once (fit) over scenes of >= 4 MiB, "
                               "else sample-major (DESIGN.md §4)",
            "queue_cache_rule": "auto: non-temporal path-queue / hit accesses for scenes of >= 256 MiB, else "
                                "cached (DESIGN.md §4)",
            "pipeline_rule": "auto: the wavefront (isect + ballot-compaction shade per cast; a job of <= 2^28 "
                             "paths starts every path at once on one sub-wavefront, a larger one in sample chunks "
                             "that each do; the first cast in the camera-cast kernel (camera ray, lockstep trace and "
                             "shade in one launch, survivors compacted per XCD shard); the drain finishes the paths "
                             "still in flight after drain_casts casts; DESIGN.md §4, §6)"
                             if args.pipeline == "auto" else f"--pipeline {args.pipeline}",
            "config": {"pipeline": "fused" if fused else "wavefront", "streams": st.get("streams"),
                       "drain": None if fused else {
                           "drained_paths_per_step": round(agg["drained_paths"] / args.steps),
                           "drained_casts_per_step": round(agg["drained_casts"] / args.steps),
                           "wavefront_casts_per_step": round((agg["ray_casts"] - agg["drained_casts"]) / args.steps),
                           "drain_launches_per_step": round(agg["drain_launches"] / args.steps, 2),
                           "refill_idle": st.get("drain_refill_idle"),
                           "refill_idle_rule": "auto (drain_refill_idle 0): 56 for scenes with analytic spheres, "
                                               "40 when the queue is streamed, else 24 (DESIGN.md §4)"
                                               if scene.backend.config["drain_refill_idle"] == 0 else "set"},
                       "hw_queues": {"in_effect": os.environ.get("GPU_MAX_HW_QUEUES", "unset (HIP default 4)"),
                                     "environment": HW_QUEUES_ENV,
                                     "note": "the environment's GPU_MAX_HW_QUEUES (SPT_HW_QUEUES overrides it for "
                                             "an experiment); the library sets none (DESIGN.md §6b)"},
                       "workload": f"{args.scene} {W}x{H} {args.spp}spp depth {args.depth}"
                                   + (" (smallpt materials: Kd albedo, Ke light, black sky, RR from cast 5)"
                                      if args.smallpt else ""),
                       "triangles": int(sstats["ntri"]), "tiles": f"{world} x interleaved {R}-row groups",
                       "paths_in_flight": st.get("paths_in_flight"), "rays_per_path": round(s_bar, 4),
                       "work_order": work_order, "queue_cache": queue_cache},
            # the roof that binds: the larger of the HBM fraction (achieved / peak,
            # kept as the headline frac so rounds stay comparable) and the VALU
            # issue fraction of this build's PMC pass
            "roofline": {"bound": "valu" if valu and valu["frac"] > achieved / HBM_PEAK_GBS else "hbm",
                         "bound_rule": "the larger of frac (HBM bytes) and valu.frac (VALU issue, this build's PMC)",
                         "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                         "kernel": dom_name,
                         "basis": dom["basis"],
                         "limiter": "latency of dependent node / triangle gathers and VALU issue (DESIGN.md §4)",
                         "bytes_per_unit": bytes_per_unit, "kernel_bytes_per_unit": kernel_bytes_per_unit,
                         "unit_of_work": dom["unit"],
                         "algorithmic_bytes_per_launch": round(bytes_per_launch),
                         "traffic_per_cast": traffic_per_unit,
                         "traffic_ratio": round(traffic / bytes_per_launch, 3) if traffic else None,
                         "traffic_note": "L2 memory-side bytes per launch from the PMC passes of this build "
                                         "(FETCH_SIZE + WRITE_SIZE; FETCH_SIZE counts the traversal's random 64-B "
                                         "node / triangle gathers exactly, profiles/r06_fetch_calibration/; "
                                         "traffic_hi_per_cast doubles the reads, the bound for coalesced 128-B "
                                         "requests): node and triangle gathers the caches miss, besides the "
                                         "algorithmic bytes",
                         "traffic_hi_per_cast": pmc.get("traffic_hi_bytes_per_cast") if pmc else None,
                         "busy_ms_per_step": round(busy_ms / args.steps, 4),
                         "busy_note": "union over the step's launch intervals and over consecutive steps' renders, "
                                      "which overlap on two streams",
                         "launches_per_step": round(launches / args.steps, 2),
                         "avg_launch_ms": round(avg_ms, 4),
                         "grays_per_s": round(dom["casts"] / (busy_ms * 1e-3) / 1e9, 4) if busy_ms else None,
                         "per_launch": {"achieved": round(per_launch, 2), "frac": round(per_launch / HBM_PEAK_GBS, 5),
                                        "note": f"per-launch duration; {st.get('streams')} stream(s) per render, "
                                                "two renders overlap"},
                         "kernels": kernel_table,
                         "trace_busy_ms_per_step": round(agg["trace_busy_ms"] / args.steps, 4),
                         "pmc_source": os.path.relpath(PMC_JSON, ROOT) + "#" + key if pmc else None,
                         "pmc_note": pmc_note,
                         "build_id": build_id,
                         "valu": valu,
                         "equivalent_wavefront": equiv,
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
        if other_leg:
            rec[other_leg["pipeline"] + "_leg"] = other_leg
        if args.save:
            np.save(args.save, image_main.cpu().numpy())
        if not args.no_cpu_baseline:
            # rank 0 only, at any world size: the oracle on this host's cores,
            # and the parity of the assembled image (every rank's tile,
            # gathered) against that oracle render; the other ranks wait at
            # the barrier below
            (orows, ofilm), rec["cpu_baseline"] = cpu_baseline(mesh, args, args.cpu_threads, kw, alb, emi)
            got = image_main[:, torch.as_tensor(orows, dtype=torch.long, device=dev), :].cpu().numpy()
            diff = got != ofilm
            rec["parity"] = {"rows": int(orows.size), "of_rows": H, "bitexact": bool(not diff.any()),
                             "values_differing": int(diff.sum()),
                             "max_abs_diff": float(np.abs(got - ofilm).max()) if got.size else 0.0,
                             "image": "assembled from %d rank tile(s) by the gather" % world,
                             "against": "oracle/ (C restatement of main.cpp:354-446), the cpu_baseline render"}
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
