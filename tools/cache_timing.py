"""Scene-cache timing on the GPU: parse + build vs spt_scene_load, and the
renders of the built and the loaded scene compared bit for bit.

    python tools/cache_timing.py [--city] [--out gpurun_out/cache]
Prints one JSON line per scene: parse_ms (pbrt + PLY read), build_ms (BVH build
+ layout + upload, spt_scene_stats.build_ms), save_ms, file bytes, load_ms
(spt_scene_load wall time: read, checksums, upload), equal (frames match).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "smallpt-enoki-optix_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import sptamd  # noqa: E402
from sptamd import scenes  # noqa: E402


def frame(s, W, H, cam):
    film, _ = s.render(sptamd.make_params(W, H, 2, 4, camera=cam))
    torch.cuda.synchronize()
    return film.cpu().numpy()


def one(name, path, out, W, H):
    t0 = time.perf_counter()
    s = sptamd.Scene()
    s.add_triangle_mesh(path)
    t1 = time.perf_counter()
    s.commit(0)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    cam = s.pbrt_info["camera"] if s.pbrt_info else None
    a = frame(s, W, H, cam)
    cache = os.path.join(out, name + ".sptc")
    t3 = time.perf_counter()
    s.save(cache)
    t4 = time.perf_counter()
    del s
    torch.cuda.synchronize()
    t5 = time.perf_counter()
    t = sptamd.Scene.load(cache)
    torch.cuda.synchronize()
    t6 = time.perf_counter()
    b = frame(t, W, H, t.pbrt_info["camera"] if t.pbrt_info else None)
    rec = {"scene": name, "ntri": t.backend.stats["ntri"], "parse_ms": round((t1 - t0) * 1e3, 1),
           "commit_ms": round((t2 - t1) * 1e3, 1), "save_ms": round((t4 - t3) * 1e3, 1),
           "file_bytes": os.path.getsize(cache), "load_ms": round((t6 - t5) * 1e3, 1),
           "load_stats_ms": round(t.backend.stats["build_ms"], 1), "equal": bool(np.array_equal(a, b))}
    os.remove(cache)
    print(json.dumps(rec), flush=True)
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--city", action="store_true", help="also BASELINE config 4's 10M-triangle pbrt city")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "cache"))
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    m = scenes.mitsuba_synth()
    src = os.path.join(a.out, "mitsuba.pbrt")
    scenes.write_pbrt(src, m, width=512, height=512)
    recs = [one("mitsuba_synth", src, a.out, 256, 256)]
    if a.city:
        recs.append(one("city_synth", scenes.scene_pbrt("city_synth"), a.out, 480, 270))
    assert all(r["equal"] for r in recs)


if __name__ == "__main__":
    main()
