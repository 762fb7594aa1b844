"""Tabulate gpu_run.sh `matrix` logs: one row per configuration (fresh process
each), Mpaths/s per tile count over the repetitions.
    python tools/matrix_table.py gpurun_out/matrix*.log"""
import json
import sys
from collections import defaultdict

for f in sys.argv[1:]:
    lines = open(f).read().splitlines()
    rows = [json.loads(l) for l in lines if l.startswith("{")]
    if not rows:
        print(f, "no result")
        continue
    tab = defaultdict(list)
    for r in rows:
        tab[r["tiles"]].append(r["tile_mpaths_s"])
    head = lines[0] if lines and not lines[0].startswith("{") else ""
    env = {k: v for k, v in rows[0].items() if k.startswith(("SPT_", "GPU_"))}
    print(f.split("/")[-1], rows[0].get("env"), {t: v for t, v in sorted(tab.items())})
