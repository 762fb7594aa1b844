"""Per-launch PMC figures of isect_queue_kernel from rocprofv3 --pmc passes.

    python tools/pmc_isect.py OUT_JSON COUNTER_CSV [COUNTER_CSV ...]

Each CSV is one pass (run_counter_collection.csv).  Every counter is averaged
over the isect dispatches of its pass.  Derived:
  traffic_bytes_per_launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> B).  gfx950
      correction from MI355X_MICROARCH.md §HBM: FETCH_SIZE reads half the bytes
      of a wide coalesced stream, so reads are doubled; it also counts
      Infinity-Cache hits, and the correction is calibrated for 16 B/lane
      streams only, so the figure is an estimate (upper bound on HBM bytes).
  valu_insts_per_launch = SQ_INSTS_VALU (wave64 VALU instructions, all waves).
bench.py reads this file (profiles/isect_pmc.json) for roofline.traffic and
roofline.valu.
"""
import csv
import json
import sys
from collections import defaultdict


def passes(paths, kernel="isect_queue"):
    per = defaultdict(dict)  # counter -> {dispatch: value}
    for path in paths:
        for r in csv.DictReader(open(path)):
            if kernel not in r["Kernel_Name"]:
                continue
            d = per[r["Counter_Name"]]
            d[(path, r["Dispatch_Id"])] = d.get((path, r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"])
    return per


def main(out, *args):
    # trailing argument without ".csv": the kernel-name substring (default isect_queue)
    kernel = "isect_queue"
    paths = list(args)
    if paths and not paths[-1].endswith(".csv"):
        kernel = paths.pop()
    per = passes(paths, kernel)
    mean = {c: sum(v.values()) / max(len(v), 1) for c, v in per.items()}
    rec = {"kernel": kernel,
           "dispatches": {c: len(v) for c, v in per.items()},
           "per_launch": mean,
           "source": list(paths)}
    if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
        rec["traffic_bytes_per_launch"] = (2.0 * mean["FETCH_SIZE"] + mean["WRITE_SIZE"]) * 1024.0
        rec["traffic_correction"] = "reads x2 (gfx950 FETCH_SIZE half-count, MI355X_MICROARCH.md HBM); estimate"
    if "SQ_INSTS_VALU" in mean:
        rec["valu_insts_per_launch"] = mean["SQ_INSTS_VALU"]
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main(*sys.argv[1:])
