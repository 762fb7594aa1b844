"""The wavefront's drain (kernels.hip render_fused_kernel<kDrain>, capi.cpp
spt_render_async): once a sub-wavefront's last work item has started, a queue
shorter than drain_q8/256 of its isect lanes — or any queue drain_casts casts
later — is finished by one launch whose lanes continue each path in registers.
Every combination must give the oracle's bits and the device-counted work:
threshold only, forced only, both; 1 and 3 sub-wavefronts; jobs that fit in
flight (fit_paths) and jobs that refill (wavefront_paths set); a fitting
job's first cast in the one-lane-per-ray isect kernel or not; the
reference's unit mode, albedo + roulette, emitters + smallpt spheres with
mirror / glass; sample chunks (film_budget_bytes)."""
import numpy as np
import pytest
import torch

import oracle as O
import sptamd
from conftest import assert_work_complete
from sptamd import scenes

pytestmark = pytest.mark.gpu
W, H, SPP, D = 40, 32, 6, 6


@pytest.fixture(scope="module")
def mesh():
    return scenes.mitsuba_synth(detail=0.25)


def materials(mesh, mode):
    nm = len(mesh["kd"])
    rng = np.random.default_rng(4)
    if mode == "unit":
        return {}
    alb = rng.uniform(0.3, 0.95, size=(nm, 3)).astype(np.float32)
    if mode == "albedo":
        return {"albedo": alb}
    emi = np.zeros((nm, 3), np.float32)
    emi[4] = (2.0, 1.5, 1.0)
    kinds = np.zeros(nm, np.uint32)
    kinds[2], kinds[3] = 1, 2  # mirror, glass
    return {"albedo": alb, "emission": emi, "kinds": kinds,
            "spheres": np.array([[0.0, 0.6, 0.0, 0.35], [0.7, 0.3, 0.4, 0.2]], np.float32),
            "sphere_mat": np.array([2, 3], np.int32)}


def gpu_scene(mesh, mat, **knobs):
    cfg = sptamd.default_config()
    for k, v in knobs.items():
        setattr(cfg, k, v)
    s = sptamd.Scene(config=cfg)
    s.add_arrays(mesh)
    s.commit(0)
    if "albedo" in mat:
        s.backend.set_albedo(mat["albedo"])
    if "emission" in mat:
        s.backend.set_emission(mat["emission"])
    if "spheres" in mat:
        s.backend.set_spheres(mat["spheres"], mat["sphere_mat"])
        s.backend.set_material_kinds(mat["kinds"])
    return s


@pytest.mark.parametrize("mode", ["unit", "albedo", "emit_spheres"])
@pytest.mark.parametrize("q8,casts", [(0, 0), (1, 0), (1024, 0), (65535, 0), (1024, 1), (0, 3), (1024, 2)])
@pytest.mark.parametrize("streams,wf", [(1, 0), (3, 0), (1, 700), (3, 1500)])
def test_drain_bitexact(mesh, mode, q8, casts, streams, wf, monkeypatch):
    for k in [k for k in list(__import__("os").environ) if k.startswith("SPT_")]:
        monkeypatch.delenv(k)
    mat = materials(mesh, mode)
    knobs = dict(drain_q8=q8, drain_casts=casts, streams=streams, fit_streams=streams)
    s = gpu_scene(mesh, mat, **knobs)
    kw = dict(rr_start_depth=3, env=(1.0, 0.9, 0.8))
    # on a side stream: the set's own (CU-masked) streams, fit_streams sub-wavefronts
    # (a caller's null stream gets plain streams and one sub-wavefront for a fitting job)
    side = torch.cuda.Stream()
    film, st = s.render(sptamd.make_params(W, H, SPP, D, wavefront_paths=wf, pipeline="wavefront", **kw),
                        stream=side)
    torch.cuda.synchronize()
    osc = O.OracleScene(mesh, albedo=mat.get("albedo"), emission=mat.get("emission"), spheres=mat.get("spheres"),
                        sphere_mat=mat.get("sphere_mat"), kinds=mat.get("kinds"))
    ref, casts_ref = osc.render(O.reference_params(W, H, SPP, D, **kw))
    np.testing.assert_array_equal(film.cpu().numpy(), ref)
    assert st["ray_casts"] == casts_ref
    assert_work_complete(st, H, W, SPP)
    assert st["drained_casts"] <= st["ray_casts"] and st["drained_paths"] <= st["paths"]
    if q8 == 0:
        assert st["drained_paths"] == 0 and st["drain_launches"] == 0
    if q8 == 65535:  # every short queue drains at once: nothing after the first drained cast
        assert st["drained_paths"] > 0
    if q8 and casts and not wf:  # the job fits: the drain runs `casts` casts after the start
        assert st["drained_paths"] > 0 and st["streams"] == streams
    # the same render from the null stream: plain streams, one sub-wavefront when it fits
    if q8 == 1024 and casts == 1 and not wf:
        film0, st0 = s.render(sptamd.make_params(W, H, SPP, D, wavefront_paths=wf, pipeline="wavefront", **kw))
        torch.cuda.synchronize()
        np.testing.assert_array_equal(film0.cpu().numpy(), ref)
        assert st0["streams"] == 1


@pytest.mark.parametrize("mode", ["unit", "emit_spheres"])
def test_drain_sorted_bitexact(mesh, mode, monkeypatch):
    """spt_config.drain_sort: the forced drain takes its queue sorted by
    direction octant and origin (launch_drain_sort); order only, same bits."""
    for k in [k for k in list(__import__("os").environ) if k.startswith("SPT_")]:
        monkeypatch.delenv(k)
    mat = materials(mesh, mode)
    s = gpu_scene(mesh, mat, drain_sort=1)
    kw = dict(rr_start_depth=3)
    side = torch.cuda.Stream()
    film, st = s.render(sptamd.make_params(W, H, SPP, D, pipeline="wavefront", **kw), stream=side)
    torch.cuda.synchronize()
    osc = O.OracleScene(mesh, albedo=mat.get("albedo"), emission=mat.get("emission"), spheres=mat.get("spheres"),
                        sphere_mat=mat.get("sphere_mat"), kinds=mat.get("kinds"))
    ref, casts = osc.render(O.reference_params(W, H, SPP, D, **kw))
    np.testing.assert_array_equal(film.cpu().numpy(), ref)
    assert st["ray_casts"] == casts and st["drained_paths"] > 0


def test_drain_sample_chunks(mesh, monkeypatch):
    """Several film chunks (film_budget_bytes): each chunk's queue drains."""
    for k in [k for k in list(__import__("os").environ) if k.startswith("SPT_")]:
        monkeypatch.delenv(k)
    mat = materials(mesh, "albedo")
    s = gpu_scene(mesh, mat, film_budget_bytes=12 * W * H * 2)
    kw = dict(rr_start_depth=2)
    film, st = s.render(sptamd.make_params(W, H, 7, D, pipeline="wavefront", **kw))
    torch.cuda.synchronize()
    ref, casts = O.OracleScene(mesh, albedo=mat["albedo"]).render(O.reference_params(W, H, 7, D, **kw))
    np.testing.assert_array_equal(film.cpu().numpy(), ref)
    assert st["ray_casts"] == casts and st["drained_paths"] > 0


def test_queued_renders_on_queue_streams(mesh, monkeypatch):
    """sptamd.queue_stream (the caller streams bench.py queues renders on):
    renders queued back to back, alternating over two such streams and two
    films, each equal to the oracle, with a read of each film queued on its
    stream behind the render (the caller-side join)."""
    for k in [k for k in list(__import__("os").environ) if k.startswith("SPT_")]:
        monkeypatch.delenv(k)
    s = gpu_scene(mesh, {})
    streams = [sptamd.queue_stream(), sptamd.queue_stream()]
    assert streams[0].cuda_stream != streams[1].cuda_stream
    seeds = [0x853C49E6748FEA9B + i for i in range(6)]
    films = [torch.empty((3, H, W), dtype=torch.float32, device="cuda") for _ in range(2)]
    copies, tickets = [], []
    for i, seed in enumerate(seeds):
        st_ = streams[i % 2]
        _, t = s.render_async(sptamd.make_params(W, H, SPP, D, rng_initstate=seed), film=films[i % 2], stream=st_)
        tickets.append(t)
        with torch.cuda.stream(st_):
            copies.append(films[i % 2].clone())
    stats = [s.render_wait(t) for t in tickets]
    torch.cuda.synchronize()
    osc = O.OracleScene(mesh)
    for seed, img, st in zip(seeds, copies, stats):
        ref, casts = osc.render(O.reference_params(W, H, SPP, D, rng_initstate=seed))
        np.testing.assert_array_equal(img.cpu().numpy(), ref)
        assert st["ray_casts"] == casts
        assert_work_complete(st, H, W, SPP)


@pytest.mark.parametrize("mode", ["unit", "albedo", "emit_spheres"])
@pytest.mark.parametrize("lockstep", [3, 2, 1, 0])
def test_lockstep_first_cast_bitexact(mesh, mode, lockstep, monkeypatch):
    """spt_config.lockstep_first: a fitting job's first cast in the
    one-lane-per-ray isect kernel (1: isect_lockstep_kernel, then the shade
    kernel; 2: camera_cast_kernel, which also makes the camera rays and shades
    the hits in the same launch; 3, the default: the same with its survivors
    compacted per XCD shard and the drain's pools over those segments);
    drain_q8 = 1 makes the drain threshold small enough for this image to take
    that path."""
    for k in [k for k in list(__import__("os").environ) if k.startswith("SPT_")]:
        monkeypatch.delenv(k)
    mat = materials(mesh, mode)
    s = gpu_scene(mesh, mat, drain_q8=1, drain_casts=1, lockstep_first=lockstep)
    kw = dict(rr_start_depth=3, env=(1.0, 0.9, 0.8))
    film, st = s.render(sptamd.make_params(W, H, SPP, D, pipeline="wavefront", **kw), stream=torch.cuda.Stream())
    torch.cuda.synchronize()
    osc = O.OracleScene(mesh, albedo=mat.get("albedo"), emission=mat.get("emission"), spheres=mat.get("spheres"),
                        sphere_mat=mat.get("sphere_mat"), kinds=mat.get("kinds"))
    ref, casts = osc.render(O.reference_params(W, H, SPP, D, **kw))
    np.testing.assert_array_equal(film.cpu().numpy(), ref)
    assert st["ray_casts"] == casts
    assert_work_complete(st, H, W, SPP)
    assert st["lockstep_casts"] == (W * H * SPP if lockstep else 0)


@pytest.mark.parametrize("mode", ["unit", "albedo", "emit_spheres"])
@pytest.mark.parametrize("chunks", [1, 0])
def test_fit_chunks_bitexact(mesh, mode, chunks, monkeypatch):
    """spt_config.fit_chunks: a job of more than fit_paths paths runs as sample
    chunks that each start every path at once (2 samples per chunk here, the
    last chunk short), with the first cast in lockstep; 0: the per-cast
    wavefront.  Same bits either way."""
    for k in [k for k in list(__import__("os").environ) if k.startswith("SPT_")]:
        monkeypatch.delenv(k)
    mat = materials(mesh, mode)
    s = gpu_scene(mesh, mat, drain_q8=1, drain_casts=1, fit_paths=W * H * 2, fit_chunks=chunks)
    kw = dict(rr_start_depth=3, env=(1.0, 0.9, 0.8))
    spp = 7
    film, st = s.render(sptamd.make_params(W, H, spp, D, pipeline="wavefront", **kw), stream=torch.cuda.Stream())
    torch.cuda.synchronize()
    osc = O.OracleScene(mesh, albedo=mat.get("albedo"), emission=mat.get("emission"), spheres=mat.get("spheres"),
                        sphere_mat=mat.get("sphere_mat"), kinds=mat.get("kinds"))
    ref, casts = osc.render(O.reference_params(W, H, spp, D, **kw))
    np.testing.assert_array_equal(film.cpu().numpy(), ref)
    assert st["ray_casts"] == casts
    assert_work_complete(st, H, W, spp)
    if chunks:
        # every chunk whose queue is not already short goes through the lockstep
        # first cast (the 1-sample last chunk may be shorter than the drain's
        # threshold, which depends on the chip's lane count)
        assert st["paths_in_flight"] == W * H * 2 and W * H * 2 <= st["lockstep_casts"] <= W * H * spp
        assert st["drained_paths"] > 0
    else:
        assert st["lockstep_casts"] == 0


@pytest.mark.parametrize("mode", ["unit", "emit_spheres"])
def test_fit_bytes_shrinks_fit(mesh, mode, monkeypatch):
    """spt_config.fit_bytes: a fitting job whose queues, hit records and film
    would exceed it runs with fit_paths cut to what fits (here 2 of 5 samples' paths
    per chunk), and with less than one chunk of the tile's pixels on the
    per-cast wavefront.  fit_bytes 0 asks the device for its free memory (the
    default, a full fit here).  Same bits every way."""
    for k in [k for k in list(__import__("os").environ) if k.startswith("SPT_")]:
        monkeypatch.delenv(k)
    mat = materials(mesh, mode)
    planes, film = (2, 1) if mode == "unit" else (4, 12)
    per_path = 2 * 16 * planes + 16 + film  # two queues of `planes` 16-B planes, the hit record, the film slot
    kw = dict(rr_start_depth=3, env=(1.0, 0.9, 0.8))
    spp = 5
    osc = O.OracleScene(mesh, albedo=mat.get("albedo"), emission=mat.get("emission"), spheres=mat.get("spheres"),
                        sphere_mat=mat.get("sphere_mat"), kinds=mat.get("kinds"))
    ref, casts = osc.render(O.reference_params(W, H, spp, D, **kw))
    for fit_bytes, fit_paths, in_flight in [(0, 1 << 28, W * H * spp),
                                            (W * H * 2 * per_path + 10, W * H * 2, W * H * 2),
                                            (W * H * per_path // 2, W * H // 2, None)]:
        s = gpu_scene(mesh, mat, drain_q8=1, drain_casts=1, fit_bytes=fit_bytes)
        film, st = s.render(sptamd.make_params(W, H, spp, D, pipeline="wavefront", **kw), stream=torch.cuda.Stream())
        torch.cuda.synchronize()
        np.testing.assert_array_equal(film.cpu().numpy(), ref)
        assert st["ray_casts"] == casts
        assert_work_complete(st, H, W, spp)
        assert st["fit_paths"] == fit_paths, (fit_bytes, st["fit_paths"])
        if in_flight is not None:  # fitting (chunks): every chunk's paths in flight, first cast in lockstep
            assert st["paths_in_flight"] == in_flight and st["lockstep_casts"] > 0
        else:  # below one chunk of the tile's pixels: the per-cast wavefront, as many paths in flight
            assert st["lockstep_casts"] == 0 and st["paths_in_flight"] == fit_paths


@pytest.mark.parametrize("mode", ["unit", "emit_spheres"])
@pytest.mark.parametrize("nth", [1, 5, 8])
def test_oom_retry_frees_and_halves(mesh, mode, nth, monkeypatch):
    """The fit whose working-set allocation fails anyway (capi.cpp retry_fit,
    ADVICE / VERDICT r5): spt_debug_fail_workspace_alloc makes the nth device
    allocation of a fresh working set fail once — inside sub-wavefront 0's
    queues, inside sub-wavefront 1's, the film chunk (two sub-wavefronts: qa,
    qb, hits, counters each, then film and running sum).  The render frees
    what the attempt allocated, halves its paths in flight (2 sample chunks
    instead of 1), retries once and gives the oracle's bits.  (A real
    out-of-memory on a device the earlier tests have used can leave the HIP
    runtime waiting inside hipMalloc — tools/probe_oom.py — so the failure is
    injected.)"""
    for k in [k for k in list(__import__("os").environ) if k.startswith("SPT_")]:
        monkeypatch.delenv(k)
    w, h, spp = 64, 48, 32  # 98304 paths: above the retry floor of 65536
    mat = materials(mesh, mode)
    kw = dict(rr_start_depth=3, env=(1.0, 0.9, 0.8))
    osc = O.OracleScene(mesh, albedo=mat.get("albedo"), emission=mat.get("emission"), spheres=mat.get("spheres"),
                        sphere_mat=mat.get("sphere_mat"), kinds=mat.get("kinds"))
    ref, casts = osc.render(O.reference_params(w, h, spp, D, **kw))
    s = gpu_scene(mesh, mat, drain_q8=1, drain_casts=1, fit_streams=2)
    sptamd._lib.lib.spt_debug_fail_workspace_alloc(nth)
    try:
        film, st = s.render(sptamd.make_params(w, h, spp, D, pipeline="wavefront", **kw),
                            stream=torch.cuda.Stream())
        torch.cuda.synchronize()
    finally:
        sptamd._lib.lib.spt_debug_fail_workspace_alloc(-1)
    assert st["fit_retries"] == 1 and st["fit_paths"] == w * h * spp // 2, (st["fit_retries"], st["fit_paths"])
    assert st["paths_in_flight"] == w * h * spp // 2 and st["streams"] == 2
    np.testing.assert_array_equal(film.cpu().numpy(), ref)
    assert st["ray_casts"] == casts
    assert_work_complete(st, h, w, spp)
    # the next render on the same set: no failure, the halved buffers grown back
    film2, st2 = s.render(sptamd.make_params(w, h, spp, D, pipeline="wavefront", **kw), stream=torch.cuda.Stream())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(film2.cpu().numpy(), ref)
    assert st2["fit_retries"] == 0 and st2["paths_in_flight"] == w * h * spp


@pytest.mark.parametrize("mode", ["unit", "emit_spheres"])
@pytest.mark.parametrize("lockstep", [3, 1])
@pytest.mark.parametrize("w,h", [(40, 32), (37, 29)])
def test_xcd_pools_bitexact(mesh, mode, lockstep, w, h, monkeypatch):
    """spt_config.xcd_remap bit 2 (per-XCD work pools with stealing in the
    drain and fused lane loops) on both pipelines, with a sharded
    or a plain first cast, on an image whose block count is not a multiple of
    eight: film bits and ray casts equal the oracle's."""
    for k in [k for k in list(__import__("os").environ) if k.startswith("SPT_")]:
        monkeypatch.delenv(k)
    mat = materials(mesh, mode)
    kw = dict(rr_start_depth=3, env=(1.0, 0.9, 0.8))
    osc = O.OracleScene(mesh, albedo=mat.get("albedo"), emission=mat.get("emission"), spheres=mat.get("spheres"),
                        sphere_mat=mat.get("sphere_mat"), kinds=mat.get("kinds"))
    ref, casts = osc.render(O.reference_params(w, h, SPP, D, **kw))
    for pipeline in ("wavefront", "fused"):
        s = gpu_scene(mesh, mat, xcd_remap=7, drain_q8=1, drain_casts=1, lockstep_first=lockstep)
        film, st = s.render(sptamd.make_params(w, h, SPP, D, pipeline=pipeline, **kw), stream=torch.cuda.Stream())
        torch.cuda.synchronize()
        np.testing.assert_array_equal(film.cpu().numpy(), ref)
        assert st["ray_casts"] == casts
        assert_work_complete(st, h, w, SPP)


@pytest.mark.parametrize("mode", ["unit", "emit_spheres"])
@pytest.mark.parametrize("idle", [0, 1, 40, 64])
def test_drain_refill_idle_bitexact(mesh, mode, idle, monkeypatch):
    """spt_config.drain_refill_idle: the drain's refill threshold (AUTO: 24 for
    this cache-resident mesh, 40 with the queue streamed, 56 with analytic
    spheres) only reorders the drain's work — same bits, same casts."""
    for k in [k for k in list(__import__("os").environ) if k.startswith("SPT_")]:
        monkeypatch.delenv(k)
    mat = materials(mesh, mode)
    kw = dict(rr_start_depth=3, env=(1.0, 0.9, 0.8))
    osc = O.OracleScene(mesh, albedo=mat.get("albedo"), emission=mat.get("emission"), spheres=mat.get("spheres"),
                        sphere_mat=mat.get("sphere_mat"), kinds=mat.get("kinds"))
    ref, casts = osc.render(O.reference_params(W, H, SPP, D, **kw))
    for cache in (sptamd._lib.SPT_QUEUE_CACHE_AUTO, sptamd._lib.SPT_QUEUE_CACHE_STREAM):
        s = gpu_scene(mesh, mat, drain_refill_idle=idle, queue_cache=cache)
        film, st = s.render(sptamd.make_params(W, H, SPP, D, pipeline="wavefront", **kw), stream=torch.cuda.Stream())
        torch.cuda.synchronize()
        np.testing.assert_array_equal(film.cpu().numpy(), ref)
        assert st["ray_casts"] == casts and st["drained_paths"] > 0
        auto = 56 if "spheres" in mat else 40 if cache == sptamd._lib.SPT_QUEUE_CACHE_STREAM else 24
        assert st["drain_refill_idle"] == (idle or auto)
