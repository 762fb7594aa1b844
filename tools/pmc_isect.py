"""Per-launch and per-cast PMC figures of the isect launches (isect_queue_kernel,
isect_lockstep_kernel) or another kernel from rocprofv3 --pmc passes over one
bench config.

    python tools/pmc_isect.py OUT_JSON KEY BENCH_LOG COUNTER_CSV [COUNTER_CSV ...] [--kernel REGEX]

Each CSV is one pass (run_counter_collection.csv).  Every counter is averaged
over the isect dispatches of its pass.  BENCH_LOG holds the bench JSON line of
one pass (casts per launch = algorithmic bytes per launch / bytes per cast).
Derived, per launch and per ray cast:
  traffic = FETCH_SIZE + WRITE_SIZE (KiB -> B).  Calibrated for this access
      pattern (profiles/r06_fetch_calibration/, tools/micro_fetch.hip):
      FETCH_SIZE = memory-side read requests x 64 B; a random 64-B gather —
      a node visit (4 x 16 B of one 64-B node) or a triangle record (3 x 12 B
      of one 64-B record) — is one 64-B request, counted exactly (factor
      1.00 / 0.94 against the true bytes), while a 128-B line or a coalesced
      stream is one 128-B request counted at 64 B (factor 2, the
      MI355X_MICROARCH.md correction).  The traversal's misses are the 64-B
      gathers, so reads count x1; traffic_hi (reads x2) bounds the share of
      coalesced queue reads.  FETCH_SIZE also counts Infinity-Cache hits.
  valu_insts = SQ_INSTS_VALU (wave64 VALU instructions, all waves).
  l2_hit_rate = TCC_HIT / (TCC_HIT + TCC_MISS).
The result is merged into OUT_JSON under KEY (e.g. "config1"); bench.py reads
profiles/isect_pmc.json#config<N> for roofline.traffic and roofline.valu.
"""
import csv
import gzip
import json
import os
import re
import sys
from collections import defaultdict


def passes(paths, kernel=r"isect_(queue|lockstep)|camera_cast"):
    per = defaultdict(dict)  # counter -> {dispatch: value}
    for path in paths:
        fh = gzip.open(path, "rt") if path.endswith(".gz") else open(path)  # committed passes are gzipped
        for r in csv.DictReader(fh):
            if not re.search(kernel, r["Kernel_Name"]):
                continue
            d = per[r["Counter_Name"]]
            d[(path, r["Dispatch_Id"])] = d.get((path, r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"])
    return per


def bench_line(log):
    for line in open(log):
        line = line.strip()
        if line.startswith("{") and '"metric"' in line:
            return json.loads(line)
    raise SystemExit(f"no bench JSON line in {log}")


def main(out, key, log, *paths):
    kernel = r"isect_(queue|lockstep)|camera_cast"
    paths = list(paths)
    if "--kernel" in paths:
        i = paths.index("--kernel")
        kernel = paths[i + 1]
        del paths[i:i + 2]
    per = passes(paths, kernel)
    mean = {c: sum(v.values()) / max(len(v), 1) for c, v in per.items()}
    b = bench_line(log)
    roof = b["roofline"]
    # units per launch (ray casts for isect_queue_kernel, paths for the fused
    # kernel and the drain): from the bench line's per-kernel table when it
    # names this kernel (the drain: ray casts and drained paths per launch),
    # else its algorithmic bytes per launch / bytes per unit
    kt = {k: v for k, v in roof.get("kernels", {}).items() if re.search(kernel, k)}
    cast_per_launch = None
    if kt:
        (kname, kv), = kt.items()
        cast_per_launch = kv["casts_per_step"] / max(kv["launches_per_step"], 1e-9)
        unit = "cast" if kv["unit"] == "ray cast" else "path"
        casts = kv["units_per_step"] / max(kv["launches_per_step"], 1e-9)
    else:
        unit = "cast" if roof.get("unit_of_work") == "ray cast" else "path"
        casts = roof["algorithmic_bytes_per_launch"] / roof["bytes_per_unit"]
    rec = {"kernel": kernel, "workload": b["config"]["workload"], "streams": b["config"]["streams"],
           "pipeline": b["config"].get("pipeline"), "work_order": b["config"].get("work_order"),
           # the library build the passes measured (spt_build_id): bench.py uses
           # this entry only while the loaded libspt.so reports the same id
           "build_id": roof.get("build_id"),
           # hardware queues the profiled process ran with (bench.py requests 8;
           # under rocprofv3 the runtime may start first, so both are recorded)
           "hw_queues": b["config"].get("hw_queues"),
           f"{unit}s_per_launch": casts, "dispatches": {c: len(v) for c, v in per.items()}, "per_launch": mean,
           "source": [os.path.relpath(p) for p in paths]}
    if cast_per_launch:
        rec["casts_per_launch"] = cast_per_launch
    if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
        t = (mean["FETCH_SIZE"] + mean["WRITE_SIZE"]) * 1024.0
        t_hi = (2.0 * mean["FETCH_SIZE"] + mean["WRITE_SIZE"]) * 1024.0
        rec["traffic_bytes_per_launch"] = t
        rec[f"traffic_bytes_per_{unit}"] = t / casts
        rec[f"traffic_hi_bytes_per_{unit}"] = t_hi / casts
        if cast_per_launch and unit != "cast":
            rec["traffic_bytes_per_cast"] = t / cast_per_launch
            rec["traffic_hi_bytes_per_cast"] = t_hi / cast_per_launch
        rec[f"read_bytes_per_{unit}"] = mean["FETCH_SIZE"] * 1024.0 / casts
        rec[f"write_bytes_per_{unit}"] = mean["WRITE_SIZE"] * 1024.0 / casts
        rec["traffic_correction"] = ("reads x1: FETCH_SIZE counts a random 64-B gather (node, triangle record) "
                                     "exactly, profiles/r06_fetch_calibration/; traffic_hi: reads x2 (coalesced "
                                     "128-B requests, MI355X_MICROARCH.md)")
    if "SQ_INSTS_VALU" in mean:
        rec["valu_insts_per_launch"] = mean["SQ_INSTS_VALU"]
        rec[f"valu_insts_per_{unit}"] = mean["SQ_INSTS_VALU"] / casts
        if cast_per_launch and unit != "cast":
            rec["valu_insts_per_cast"] = mean["SQ_INSTS_VALU"] / cast_per_launch
    if "TCC_HIT_sum" in mean:
        rec["l2_hit_rate"] = mean["TCC_HIT_sum"] / max(1.0, mean["TCC_HIT_sum"] + mean.get("TCC_MISS_sum", 0.0))
    if "SQ_WAVE_CYCLES" in mean:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if c in mean:
                rec[c.lower() + "_frac"] = mean[c] / mean["SQ_WAVE_CYCLES"]
    if "GRBM_GUI_ACTIVE" in mean:
        for c in ("TA_TA_BUSY_sum", "TD_TD_BUSY_sum"):
            if c in mean:  # summed over the 256 CUs' units
                rec[c.lower().replace("_sum", "") + "_frac"] = mean[c] / (256.0 * mean["GRBM_GUI_ACTIVE"])
    allrec = json.load(open(out)) if os.path.exists(out) else {}
    if "kernel" in allrec and "per_launch" in allrec:  # the round-1 single-config layout
        allrec = {}
    allrec[key] = rec
    json.dump(allrec, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main(*sys.argv[1:])
