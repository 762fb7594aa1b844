"""Summarise rocprofv3 --pmc counter_collection.csv: per-counter sums over
dispatches of each kernel, plus the dispatch-weighted duration."""
import csv
import sys
from collections import defaultdict


def main(paths):
    for path in paths:
        sums = defaultdict(lambda: defaultdict(float))
        durs = defaultdict(dict)
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"][:60]
            sums[k][r["Counter_Name"]] += float(r["Counter_Value"])
            durs[k][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        for k, c in sums.items():
            ns = sum(durs[k].values())
            print(f"{path}: {k}  dispatches={len(durs[k])} total_ns={ns}")
            for name, v in sorted(c.items()):
                print(f"   {name:32s} {v:18.0f}   per_us={v / max(ns, 1) * 1e3:14.1f}")


if __name__ == "__main__":
    main(sys.argv[1:])
