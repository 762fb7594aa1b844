"""Probe: how much device memory hipMalloc hands out before it fails (in
16 GiB blocks), and how the library's OOM retry behaves on a job whose
working set exceeds the card (tests/test_gpu_drain.py::test_oom_retry_*).
    python tools/probe_oom.py [--render]"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "smallpt-enoki-optix_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    hip = ctypes.CDLL("libamdhip64.so")
    free, tot = ctypes.c_size_t(), ctypes.c_size_t()
    torch.cuda.init()
    hip.hipMemGetInfo(ctypes.byref(free), ctypes.byref(tot))
    print(f"free {free.value / 2**30:.1f} GiB of {tot.value / 2**30:.1f}", flush=True)
    ptrs, blk = [], 16 << 30
    t0 = time.time()
    while True:
        p = ctypes.c_void_p()
        e = hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(blk))
        if e != 0:
            print(f"hipMalloc #{len(ptrs)} failed with {e} after {len(ptrs) * 16} GiB ({time.time() - t0:.2f} s)", flush=True)
            hip.hipGetLastError()
            break
        ptrs.append(p)
        if len(ptrs) > 40:
            print("more than 640 GiB handed out: stopping", flush=True)
            break
    for p in ptrs:
        hip.hipFree(p)
    if "--render" in sys.argv:
        import numpy as np
        import sptamd
        from sptamd import scenes
        import test_gpu_drain as T
        mesh = scenes.mitsuba_synth(detail=0.25)
        mat = T.materials(mesh, "emit_spheres")
        w, h, spp = 256, 1024, 8188
        s = T.gpu_scene(mesh, mat, fit_paths=w * h * spp, fit_bytes=1 << 42)
        t0 = time.time()
        film, st = s.render(sptamd.make_params(w, h, spp, 4, pipeline="wavefront", rr_start_depth=2,
                                               env=(1.0, 0.9, 0.8)), stream=torch.cuda.Stream())
        torch.cuda.synchronize()
        print(f"render {time.time() - t0:.2f} s: fit_retries {st['fit_retries']} fit_paths {st['fit_paths']} "
              f"in flight {st['paths_in_flight']} paths {st['paths']} casts {st['ray_casts']}", flush=True)


if __name__ == "__main__":
    main()
