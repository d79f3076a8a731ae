"""A/B of libgolhip builds on one box: every round runs every case once per
library, in alternating order, each in its own process (GOLHIP_LIB), through
scripts/sweep_opts.py (wall clock, no per-launch events).  Prints one JSON
line per run and the best / median GCUPS per (case, library).

    python scripts/ab_builds.py --libs a.so,b.so --cases 65536x65536,16384x16384,65536x8192r [--rounds 3] [--turns 1000]
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ap = argparse.ArgumentParser()
ap.add_argument("--libs", required=True)
ap.add_argument("--cases", default="65536x65536,16384x16384,65536x8192r")
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--turns", type=int, default=1000)
ap.add_argument("--sets", default="")
a = ap.parse_args()
libs = [os.path.abspath(l) for l in a.libs.split(",")]
res = {}
for rnd in range(a.rounds):
    order = libs if rnd % 2 == 0 else libs[::-1]
    for lib in order:
        env = dict(os.environ, GOLHIP_LIB=lib)
        p = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "sweep_opts.py"), "--no-timing", "--reps", "1",
                            "--cases", a.cases, "--sets", a.sets, "--turns", str(a.turns)], env=env,
                           capture_output=True, text=True, timeout=600)
        if p.returncode:
            print(p.stdout[-2000:], p.stderr[-2000:], file=sys.stderr)
            sys.exit(1)
        for line in p.stdout.splitlines():
            if line.startswith("{"):
                d = json.loads(line)
                d["lib"] = os.path.basename(lib)
                d["round"] = rnd
                print(json.dumps(d), flush=True)
                res.setdefault((d["case"], json.dumps(d["opts"]), d["lib"]), []).append(d["gcups"])
print("# case opts lib: best median (GCUPS)")
for (case, opts, lib), v in sorted(res.items()):
    print(f"{case:14s} {opts:28s} {lib:28s} {max(v):10.1f} {statistics.median(v):10.1f}")
