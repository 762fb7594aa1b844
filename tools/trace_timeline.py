"""Per-stream timeline of one render from a rocprofv3 kernel trace
(run_kernel_trace.csv): every launch's start, duration and the gap before it
on its queue, plus a summary of where the render's wall time goes (isect /
shade / refill / resolve busy, gaps, and the chip-level union of isect time).

    python tools/trace_timeline.py gpurun_out/proftile8/run_kernel_trace.csv [--render -1] [--quiet]

A render is the span from the first launch after the previous render's
resolve up to and including its own resolve (resolve_kernel /
resolve_flags_kernel / render_fused_kernel's resolve).
"""
from __future__ import annotations

import argparse
import csv
from collections import defaultdict


def short(name: str) -> str:
    for k in ("isect_queue_kernel", "isect_lockstep_kernel", "shade_kernel", "refill_kernel", "resolve_flags_kernel", "resolve_kernel",
              "render_fused_kernel", "drain_kernel", "fillBuffer", "copyBuffer"):
        if k in name:
            return k
    return name.split("(")[0][-40:]


def union(iv):
    iv = sorted(iv)
    tot, lo, hi = 0.0, None, None
    for a, b in iv:
        if hi is None or a > hi:
            if hi is not None:
                tot += hi - lo
            lo, hi = a, b
        else:
            hi = max(hi, b)
    if hi is not None:
        tot += hi - lo
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--render", type=int, default=-1, help="which render (python index; default the last)")
    ap.add_argument("--quiet", action="store_true", help="summary only")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]), short(r["Kernel_Name"]),
                         int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))))
    rows.sort()
    # render boundaries: each resolve ends a render; the first render starts after setup
    ends = [i for i, r in enumerate(rows) if r[3].startswith("resolve")]
    if not ends:
        raise SystemExit("no resolve launch in the trace")
    k = a.render if a.render >= 0 else len(ends) + a.render
    lo_i = ends[k - 1] + 1 if k > 0 else 0
    hi_i = ends[k]
    sel = [r for r in rows[lo_i:hi_i + 1] if r[3] not in ("fillBuffer", "copyBuffer") or True]
    # the render's own launches may interleave with the neighbouring renders'
    # (two working sets overlap); keep everything between the boundaries
    t0 = min(r[0] for r in sel)
    t1 = max(r[1] for r in sel)
    by_q = defaultdict(list)
    for r in sel:
        by_q[r[2]].append(r)
    busy = defaultdict(float)
    for r in sel:
        busy[r[3]] += (r[1] - r[0]) / 1e3
    print(f"render {k} of {len(ends)}: {len(sel)} launches, wall {(t1 - t0) / 1e3:.1f} us")
    for q, lst in sorted(by_q.items()):
        prev = None
        gaps = 0.0
        if not a.quiet:
            print(f"-- queue {q}")
        for s, e, _, n, g in lst:
            gap = (s - prev) / 1e3 if prev is not None else (s - t0) / 1e3
            gaps += max(0.0, gap) if prev is not None else 0.0
            if not a.quiet:
                print(f"   {n:22s} start {(s - t0) / 1e3:9.1f}  dur {(e - s) / 1e3:8.1f}  gap {gap:7.1f}  blocks {g}")
            prev = e
        print(f"   queue {q}: {len(lst)} launches, busy {sum(e - s for s, e, *_ in lst) / 1e3:.1f} us, "
              f"gaps {gaps:.1f} us, span {(lst[-1][1] - lst[0][0]) / 1e3:.1f} us")
    print("busy per kernel (summed over queues, us):", {k2: round(v, 1) for k2, v in sorted(busy.items())})
    iv = [(r[0], r[1]) for r in sel if r[3] in ("isect_queue_kernel", "isect_lockstep_kernel")]
    print(f"isect union {union(iv) / 1e3:.1f} us; any-kernel union {union([(r[0], r[1]) for r in sel]) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
