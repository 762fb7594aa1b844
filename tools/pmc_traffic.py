"""HBM traffic per isect launch from rocprofv3 FETCH_SIZE / WRITE_SIZE passes.

    python tools/pmc_traffic.py FETCH_CSV WRITE_CSV OUT_JSON

FETCH_SIZE and WRITE_SIZE are in KiB per dispatch (collected in separate
passes: they do not fit one TCC pass).  gfx950 correction from
MI355X_MICROARCH.md §HBM: FETCH_SIZE reads exactly half the bytes of a wide
coalesced stream, so reads are doubled; WRITE_SIZE is taken as is.  The
correction is calibrated for 16 B/lane streams only (our ray/hit planes are
4 B/lane and the node gathers 16 B/lane random), so the result is an estimate.
"""
import csv
import json
import sys


def per_dispatch(path, counter, kernel="isect_queue"):
    vals = {}
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return vals


def main(fetch_csv, write_csv, out):
    f = per_dispatch(fetch_csv, "FETCH_SIZE")
    w = per_dispatch(write_csv, "WRITE_SIZE")
    nf, nw = max(len(f), 1), max(len(w), 1)
    fkb = sum(f.values()) / nf
    wkb = sum(w.values()) / nw
    rec = {"kernel": "isect_queue_kernel", "dispatches_fetch": len(f), "dispatches_write": len(w),
           "fetch_kib_per_launch_raw": fkb, "write_kib_per_launch": wkb,
           "traffic_bytes_per_launch": (2.0 * fkb + wkb) * 1024.0,
           "correction": "reads x2 (gfx950 FETCH_SIZE half-count, MI355X_MICROARCH.md HBM); estimate",
           "source": [fetch_csv, write_csv]}
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main(*sys.argv[1:4])
