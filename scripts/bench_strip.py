"""One rank's share of the strong-scaled multi-GPU bench, on one GPU.

At N GPUs, bench.py gives each rank a W x (H/N) strip whose halo rows come over
the RCCL ring.  This runs that strip as a one-rank ring (option force_halo: the
same deep-halo exchanges and kernels, the neighbours being the strip itself)
and reports GCUPS for the resident kernel between exchanges (the default for
strips of <= 64 MiB) and for per-launch kernels, so the N > 1 default can be
chosen on measurements.  Prints one JSON line per (strip, persistent).

    python scripts/bench_strip.py [--turns 1000] [--strips 65536x8192,262144x32768]
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
ap.add_argument("--turns", type=int, default=1000)
ap.add_argument("--strips", default="65536x8192,65536x16384,65536x32768,262144x32768")
ap.add_argument("--persistent", default="-1,0")
ap.add_argument("--depths", default="16")
ap.add_argument("--torus", action="store_true", help="whole-board torus instead of a one-rank ring")
ap.add_argument("--option", action="append", default=[], help="engine option key=value (every run)")
a = ap.parse_args()
for spec in a.strips.split(","):
    W, R = (int(x) for x in spec.split("x"))
    for pers, depth in [(int(x), int(d)) for x in a.persistent.split(",") for d in a.depths.split(",")]:
        with golhip.Board(W, R, timing=True) as b:
            if not a.torus:
                b.comm_init(golhip.unique_id(), 1, 0)
                b.set_option("force_halo", 1)
            b.set_option("persistent", pers)
            for kv in a.option:
                k, v = kv.split("=")
                b.set_option(k, int(v))
            b.set_tb_depth(depth)
            b.fill_random(0x5EED0002)
            b.step(min(a.turns, 200))
            b.sync()
            b.perf_reset()
            t0 = time.perf_counter()
            b.step(a.turns)
            b.sync()
            dt = time.perf_counter() - t0
            p = b.perf()
            print(json.dumps({"strip": [R, W], "torus": a.torus, "persistent": pers, "depth": depth, "turns": a.turns, "seconds": dt,
                              "gcups": W * R * a.turns / dt / 1e9, "persist_launches": p["persist_launches"],
                              "step_launches": p["step_launches"], "words_per_lane": p["words_per_lane"],
                              "tb_depth": p["tb_depth"], "halo_MB": p["halo_bytes"] / 1e6,
                              "skew_launches": p["skew_launches"], "options": a.option}), flush=True)
