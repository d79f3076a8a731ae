"""Tuning sweep (one process, one device): GCUPS of the step kernel per
(board, depth, rows_per_wave, engine options).  Variants are interleaved over
--repeats rounds so device clock drift hits them alike; the best round is kept."""
import argparse
import json
import os

os.environ.setdefault("GOLHIP_TUNING", "1")  # A/B knobs of the kernel plans (golhip.h)
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "game-of-life-distributed_amd"))
import golhip  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--sizes", default="16384,65536")
ap.add_argument("--depths", default="8,16,32")
ap.add_argument("--rpw", default="0,32,64,128,256,512,1024")
ap.add_argument("--variants", default="", help="semicolon-separated option sets, e.g. 'fill_skip=0;fill_skip=1'")
ap.add_argument("--turns", type=int, default=256)
ap.add_argument("--repeats", type=int, default=1)
ap.add_argument("--rows", type=int, default=0, help="board height (0 = square)")
a = ap.parse_args()
variants = [v for v in a.variants.split(";") if v] or [""]
# engine options are sticky on a handle: every variant starts from the defaults
DEFAULTS = {"wpl": 0, "persistent": -1, "persist_depth": 0, "persist_waves": 0, "persist_wg_tx": 0, "dummy_rows": 0, "paired_bands": 1,
            "fill_skip": 1}
for N in map(int, a.sizes.split(",")):
    H = a.rows or N
    b = golhip.Board(N, H, timing=True)
    b.fill_random(0x5EED0001)
    for d in map(int, a.depths.split(",")):
        for s in map(int, a.rpw.split(",")):
            best = {}
            for _ in range(a.repeats):
                for v in variants:
                    opts = dict(DEFAULTS)
                    opts.update(kv.split("=") for kv in v.split(",") if kv)
                    for k, val in opts.items():
                        b.set_option(k, int(val))
                    b.set_tb_depth(d)
                    b.set_rows_per_wave(s)
                    b.step(2 * d)
                    b.sync()
                    b.perf_reset()
                    t0 = time.perf_counter()
                    b.step(a.turns)
                    b.sync()
                    dt = time.perf_counter() - t0
                    p = b.perf()
                    kms = p["step_kernel_ms"] + p["persist_kernel_ms"]
                    kern = kms / max(1, p["step_launches"] + p["persist_launches"])
                    rec = dict(N=N, H=H, depth=d, rpw=s, variant=v, rpw_used=p["rows_per_wave"], persist=p["persist_launches"],
                               wall_gcups=N * H * a.turns / dt / 1e9,
                               kernel_gcups=N * H * a.turns / (kms * 1e-3) / 1e9, launch_ms=kern)
                    if rec["wall_gcups"] > best.get(v, {"wall_gcups": 0})["wall_gcups"]:
                        best[v] = rec
            for v in variants:
                print(json.dumps(best[v]), flush=True)
    b.close()
