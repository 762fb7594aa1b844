"""One driver for the measured experiments (A/B runs, knob sweeps, PMC passes).

    python tools/exp.py list                      every experiment of tools/experiments.yaml
    python tools/exp.py show NAME                 its description, script and results
    python tools/exp.py build NAME                build the variant libraries it names (CPU, here)
    python tools/exp.py run NAME                  run its script (on the GPU box: gpurun -- python tools/exp.py run NAME)
    python tools/exp.py ab [--variants ...]       alternate bench runs of library / environment variants

`ab` is the A/B primitive the experiments use: each variant is "name=LIB"
(LIB empty: smallpt-enoki-optix_amd/build/libspt.so, else a variant build),
with optional per-variant environment "name:VAR=val,VAR=val"; it runs
`bench.py --steps 5 --warmup 1 --no-cpu-baseline` ROUNDS times per variant,
alternating, each run under its own time limit, and appends one line per run
(variant, Mpaths/s, isect ms) to gpurun_out/ab.log.  The same settings may come
from the environment (VARIANTS, ENVS, ROUNDS, BENCH_ARGS), as the scripts in the
manifest pass them.

Manifest entries (tools/experiments.yaml): what (the question), round, build
(variant name -> make EXTRA flags, built into build_<name>/), script (the bash
the GPU box runs, each GPU step under a time limit, stopping at the first one
that faults or times out), results (profiles/ paths) and outcome (kept / not
kept, with the numbers).  DESIGN.md cites entries by name.
"""
from __future__ import annotations

import argparse
import json
import os
import shlex
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "smallpt-enoki-optix_amd")
MANIFEST = os.path.join(ROOT, "tools", "experiments.yaml")
OUT = os.path.join(ROOT, "gpurun_out")


def manifest() -> dict:
    import yaml
    with open(MANIFEST) as f:
        return yaml.safe_load(f)


def cmd_list(_):
    for name, e in sorted(manifest().items()):
        print(f"{name:24s} r{e.get('round', '?')}  {e.get('outcome', '')[:90]}")


def cmd_show(a):
    e = manifest()[a.name]
    for k in ("what", "round", "build", "results", "outcome"):
        if k in e:
            print(f"{k}: {e[k]}")
    print("script:\n" + e.get("script", ""))


def cmd_build(a):
    """make BUILD=build_<variant> EXTRA=<flags> for each variant the entry names."""
    e = manifest()[a.name]
    jobs = str(min(16, os.cpu_count() or 4))
    for var, extra in (e.get("build") or {}).items():
        print(f"== build_{var}: EXTRA={extra}", flush=True)
        subprocess.run(["make", "-s", "-j", jobs, "-C", PKG, f"BUILD=build_{var}", f"EXTRA={extra}", "ARCH=gfx950"],
                       check=True)


def cmd_run(a):
    e = manifest()[a.name]
    os.makedirs(OUT, exist_ok=True)
    script = "set -u\ncd " + shlex.quote(os.environ.get("GRAFT_REPO_ROOT", ROOT)) + "\nexport TMPDIR=/tmp\n" + e["script"]
    r = subprocess.run(["bash", "-o", "pipefail", "-c", script])
    sys.exit(r.returncode)


def _variants(spec: str):
    out = []
    for v in spec.split():
        name, _, lib = v.partition("=")
        out.append((name, os.path.join(ROOT, lib) if lib else ""))
    return out


def _envs(spec: str):
    env = {}
    for item in spec.split():
        name, _, kv = item.partition(":")
        env[name] = dict(x.split("=", 1) for x in kv.split(",") if x)
    return env


def cmd_ab(a):
    """Alternating bench runs; stops at the first run that fails or times out."""
    variants = _variants(a.variants or os.environ.get("VARIANTS", "base="))
    envs = _envs(a.envs or os.environ.get("ENVS", ""))
    rounds = a.rounds or int(os.environ.get("ROUNDS", "3"))
    bench_args = shlex.split(a.bench_args if a.bench_args is not None else os.environ.get("BENCH_ARGS", ""))
    os.makedirs(OUT, exist_ok=True)
    log = os.path.join(OUT, "ab.log")
    for _ in range(rounds):
        for name, lib in variants:
            env = dict(os.environ)
            env.pop("SPT_LIB", None)
            if lib:
                env["SPT_LIB"] = lib
            env.update(envs.get(name, {}))
            cmd = [sys.executable, "bench.py", "--steps", "5", "--warmup", "1", "--no-cpu-baseline", *bench_args]
            try:
                r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=a.timeout)
            except subprocess.TimeoutExpired:
                print(f"{name}: timed out after {a.timeout} s", file=sys.stderr)
                sys.exit(124)
            if r.returncode != 0:
                print(r.stderr[-2000:], file=sys.stderr)
                sys.exit(r.returncode if r.returncode > 0 else 1)
            rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
            line = f"{name} {rec['value']} {rec['kernel_ms_per_step']}"
            print(line, flush=True)
            with open(log, "a") as f:
                f.write(line + "\n")


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = ap.add_subparsers(dest="cmd", required=True)
    sub.add_parser("list").set_defaults(fn=cmd_list)
    for c, fn in (("show", cmd_show), ("build", cmd_build), ("run", cmd_run)):
        p = sub.add_parser(c)
        p.add_argument("name")
        p.set_defaults(fn=fn)
    p = sub.add_parser("ab")
    p.add_argument("--variants", default=None, help='"name=LIB name2=LIB2" (LIB empty = the default build)')
    p.add_argument("--envs", default=None, help='"name:VAR=val,VAR2=val name2:..."')
    p.add_argument("--rounds", type=int, default=0)
    p.add_argument("--bench-args", default=None)
    p.add_argument("--timeout", type=int, default=200)
    p.set_defaults(fn=cmd_ab)
    a = ap.parse_args()
    a.fn(a)


if __name__ == "__main__":
    main()
