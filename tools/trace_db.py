"""Kernel timeline from a rocprofv3 database (rocpd SQLite, the default output
when --output-format csv is not given): one line per dispatch with its queue,
start / end (ms from the first dispatch), duration, grid, scratch, VGPRs.
    python tools/trace_db.py DIR_OR_DB [--last N] [--csv out.csv]"""
import argparse
import glob
import os
import sqlite3


def short(n):
    if "render_fused_kernel" in n:
        return "drain" if "Lb1ELb" in n or ", true" in n.split("render_fused_kernel")[1][:80] else "fused"
    n = n.split("(")[0].replace("void ", "").replace("spt::", "")
    return n.split("<")[0][:30]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--last", type=int, default=0, help="only the last N dispatches")
    ap.add_argument("--csv", default="")
    a = ap.parse_args()
    db = a.path if a.path.endswith(".db") else glob.glob(os.path.join(a.path, "**", "*.db"), recursive=True)[0]
    cur = sqlite3.connect(db).cursor()
    cols = [r[1] for r in cur.execute("pragma table_info(kernels)")]
    rows = cur.execute("select * from kernels order by start").fetchall()
    K = {c: i for i, c in enumerate(cols)}
    t0 = rows[0][K["start"]]
    out = []
    for r in rows[-a.last:] if a.last else rows:
        name = r[K["name"]]
        s, e = (r[K["start"]] - t0) / 1e6, (r[K["end"]] - t0) / 1e6
        out.append((r[K["queue_id"]], short(name), s, e, r[K["grid_x"]], r[K["scratch_size"]], name))
    for q, n, s, e, g, scr, _ in out:
        print(f"q{q:>3} {n:30s} {s:10.3f} {e:10.3f} {e - s:8.3f} grid={g} scr={scr}")
    if a.csv:
        with open(a.csv, "w") as f:
            f.write("queue,kernel,start_ms,end_ms,dur_ms,grid,scratch,name\n")
            for q, n, s, e, g, scr, name in out:
                f.write(f'{q},{n},{s:.4f},{e:.4f},{e - s:.4f},{g},{scr},"{name}"\n')


if __name__ == "__main__":
    main()
