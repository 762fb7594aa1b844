"""Average duration of a kernel's launches inside bench.py's timed region, from a
rocprofv3 kernel trace (run_kernel_trace.csv).

rocprofv3 --stats averages over every launch of the command, which includes
bench.py's setup and warmup renders; the roofline line's avg_launch_ms covers
only the timed steps. The timed region is the last `--launches` launches of
the kernel (bench's `launches_per_step` x steps), so this prints both averages
side by side.

    python tools/trace_window_avg.py gpurun_out/prof/run_kernel_trace.csv --kernel render_fused --launches 4
"""
from __future__ import annotations

import argparse
import csv


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", required=True, help="substring of the kernel name")
    ap.add_argument("--launches", type=int, required=True, help="launches in the timed region")
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace)) if a.kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    if not dur:
        raise SystemExit(f"no launch of {a.kernel!r} in {a.trace}")
    last = dur[-a.launches:]
    print(f"{a.kernel}: {len(dur)} launches, all {sum(dur) / len(dur):.4f} ms avg; "
          f"last {len(last)} (timed region) {sum(last) / len(last):.4f} ms avg: "
          + " ".join(f"{d:.3f}" for d in last))


if __name__ == "__main__":
    main()
