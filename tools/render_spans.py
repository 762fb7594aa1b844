"""Per-render spans from a rocprofv3 kernel trace (run_kernel_trace.csv): a
render ends with its resolve launch; prints each render's span from the
previous resolve's end to its own, so outlier renders stand out.

    python tools/render_spans.py gpurun_out/proftile8/run_kernel_trace.csv
"""
import csv
import sys

rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
ends = [e for s, e, n in rows if "resolve" in n]
print("renders:", len(ends))
print("spans (us):", [round((b - a) / 1e3, 1) for a, b in zip(ends, ends[1:])])
