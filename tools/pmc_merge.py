"""Merge PMC entries (tools/pmc_isect.sh output) into profiles/isect_pmc.json.

    python tools/pmc_merge.py gpurun_out/pmc/isect_pmc.json [--keep-suffix _r04]
An entry replaced by one of another build is kept under key + suffix (once)."""
import argparse
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--dst", default=os.path.join(ROOT, "profiles", "isect_pmc.json"))
    ap.add_argument("--keep-suffix", default="")
    a = ap.parse_args()
    new = json.load(open(a.src))
    old = json.load(open(a.dst)) if os.path.exists(a.dst) else {}
    for k, v in new.items():
        prev = old.get(k)
        if a.keep_suffix and prev and prev.get("build_id") != v.get("build_id") and k + a.keep_suffix not in old:
            old[k + a.keep_suffix] = prev
        old[k] = v
    json.dump(old, open(a.dst, "w"), indent=1)
    print("merged", sorted(new), "into", a.dst)


if __name__ == "__main__":
    main()
