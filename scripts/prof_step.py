"""Fixed workload for rocprofv3 passes: fill a board, run warmup turns, then
`--launches` fused step launches of `--depth` turns (automatic rows/wave)."""
import argparse
import json
import os

os.environ.setdefault("GOLHIP_TUNING", "1")  # A/B knobs of the kernel plans (golhip.h)
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "game-of-life-distributed_amd"))
import golhip  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--size", type=int, default=16384)
ap.add_argument("--depth", type=int, default=16)
ap.add_argument("--launches", type=int, default=20)
ap.add_argument("--persistent", type=int, default=1)
a = ap.parse_args()
with golhip.Board(a.size, a.size, timing=True) as b:
    b.set_tb_depth(a.depth)
    b.set_option("persistent", a.persistent)
    b.fill_random(0x5EED0001 if a.size == 16384 else 0x5EED0002)
    b.step(2 * a.depth)
    b.sync()
    b.perf_reset()
    # persistent: `launches` separate step calls of 4 super-steps each;
    # per-launch: `launches` launches of `depth` turns
    for _ in range(a.launches):
        b.step(4 * a.depth if a.persistent else a.depth)
    b.sync()
    p = b.perf()
    n = p["persist_launches"] + p["step_launches"]
    print(json.dumps({"turns_per_launch": (p["persist_turns"] + p["step_turns"]) / max(1, n), "launches": n,
                      "words_per_lane": p["words_per_lane"], "tb_depth": p["tb_depth"]}), flush=True)
