"""Do consecutive queued renders overlap?  From a rocprofv3 kernel trace
(run_kernel_trace.csv) of renders alternating over two working sets.

A working set's render starts on its stream 0 and ends with its resolve there
(resolve_flags_kernel / resolve_kernel), so each resolve's queue names a set.
A render's span is [its first kernel on that queue after the set's previous
resolve, its own resolve's end].  Renders sorted by start: a render that
starts only after the previous one ended ran serialised.  With --runs R
--per-run N the renders are split into R consecutive runs of N (tile_sim: two
synchronous setup renders, then the timed steps) and each run's timed renders
get a line.

    python tools/render_overlap.py gpurun_out/tr/run_kernel_trace.csv --runs 16 --per-run 42
"""
from __future__ import annotations

import argparse
import csv
from collections import defaultdict


def spans(trace):
    rows = list(csv.DictReader(open(trace)))
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    rows.sort(key=lambda r: r["s"])
    by_q = defaultdict(list)
    for r in rows:
        by_q[r["Queue_Id"]].append(r)
    out = []
    for q, rs in by_q.items():
        prev_end = None
        for r in rs:
            if "resolve" not in r["Kernel_Name"]:
                continue
            if prev_end is not None:
                first = next(x for x in rs if x["s"] > prev_end)
                out.append((first["s"], r["e"], q))
            prev_end = r["e"]
    out.sort()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--runs", type=int, default=1)
    ap.add_argument("--per-run", type=int, default=0, help="renders per run (0: all in one run)")
    a = ap.parse_args()
    sp = spans(a.trace)
    # the first render of each set has no predecessor on its queue, so span i
    # is render i + 2; with --per-run N, run k's renders are [kN, kN + N), the
    # first two of them its synchronous setup renders: spans [kN, kN + N - 2)
    # are its timed renders
    for k in range(a.runs):
        run = sp[k * a.per_run:(k + 1) * a.per_run - 2] if a.per_run else sp
        if len(run) < 2:
            break
        serial = sum(1 for p, n in zip(run, run[1:]) if n[0] >= p[1])
        ms = (run[-1][1] - run[0][0]) / 1e6
        print(f"run {k}: {len(run)} renders over {ms:.2f} ms ({ms / len(run):.3f} ms each), "
              f"{serial} of {len(run) - 1} started after the previous one ended")


if __name__ == "__main__":
    main()
