"""One line per bench.py log: value, pipeline, streams, dominant kernel and the
tracing kernels' busy time per step.
    python tools/bench_table.py gpurun_out/benchm*.log"""
import json
import sys

for f in sys.argv[1:]:
    rec = None
    env = ""
    for line in open(f):
        if line.startswith("{"):
            rec = json.loads(line)
    if rec is None:
        print(f, "no result")
        continue
    rf = rec["roofline"]
    ks = {k.split("<")[-1].rstrip(">") if "<" in k else k.split("_")[0]: (v["busy_ms_per_step"], v["grays_per_s"])
          for k, v in rf.get("kernels", {}).items()}
    print(f"{f.split('/')[-1]:14s} {rec['value']:9.1f}  {rec['config']['pipeline']:9s} K={rec['config']['streams']} "
          f"ms/step {rec['ms_per_step']:8.3f}  dom {rf['kernel']:28s} {ks}")
