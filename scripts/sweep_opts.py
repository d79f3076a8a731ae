"""A/B sweep of engine options on whole boards (torus) and one-rank-ring strips.

    python scripts/sweep_opts.py --cases "65536x65536,65536x8192r" --sets "skew=1;skew=0;skew_young=80" [--turns 1000] [--reps 3]

A case WxR is a W-wide board of R rows (suffix r: a one-rank RCCL ring strip,
force_halo).  Each option set (k=v,k=v) runs every case `reps` times
(interleaved, so box drift hits every set alike); prints one JSON line per
run and a summary (best GCUPS per set and case).
"""
import argparse
import json
import os

os.environ.setdefault("GOLHIP_TUNING", "1")  # A/B knobs of the kernel plans (golhip.h)
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "game-of-life-distributed_amd")]
import golhip  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--cases", default="65536x65536,65536x8192r")
ap.add_argument("--sets", default="skew=1;skew=0")
ap.add_argument("--turns", type=int, default=1000)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--depth", type=int, default=20)
ap.add_argument("--no-timing", action="store_true", help="no per-launch HIP timing events (wall clock only)")
a = ap.parse_args()
sets = [dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in s.split(",") if kv) for s in a.sets.split(";")]
if any("halo_skip" in o or "flip_debug" in o for o in sets):  # wrong results by design: measurement only
    os.environ["GOLHIP_MEASUREMENT"] = "1"
best = {}
for rep in range(a.reps):
    for case in a.cases.split(","):
        ring = case.endswith("r")
        W, R = (int(x) for x in case.rstrip("r").split("x"))
        for opts in sets:
            with golhip.Board(W, R, timing=not a.no_timing) as b:
                if ring:
                    b.comm_init(golhip.unique_id(), 1, 0)
                    b.set_option("force_halo", 1)
                b.set_tb_depth(a.depth)
                for k, v in opts.items():
                    if k == "tb_depth":
                        b.set_tb_depth(v)
                    else:
                        b.set_option(k, v)
                b.fill_random(0x5EED0002)
                b.step(min(a.turns, 200))
                b.sync()
                b.perf_reset()
                t0 = time.perf_counter()
                b.step(a.turns)
                b.sync()
                dt = time.perf_counter() - t0
                p = b.perf()
                g = W * R * a.turns / dt / 1e9
                key = (case, json.dumps(opts))
                best[key] = max(best.get(key, 0), g)
                print(json.dumps({"case": case, "opts": opts, "lib": os.path.basename(golhip.LIB_PATH), "rep": rep, "gcups": round(g, 1),
                                  "launch_ms": round(p["step_kernel_ms"] / max(1, p["step_launches"]), 5),
                                  "skew": p["skew_launches"],
                                  "launches": p["step_launches"], "persist": p["persist_launches"],
                                  "exchanges": p["halo_exchanges"],
                                  "exchange_ms": round(p["halo_ms"] / max(1, p["halo_exchanges"]), 5)}), flush=True)
print("# best GCUPS per (case, options)")
for (case, opts), g in sorted(best.items()):
    print(f"{case:16s} {opts:50s} {g:10.1f}")
