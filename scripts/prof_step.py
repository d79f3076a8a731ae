"""Fixed workload for rocprofv3 passes: fill a board, run warmup turns, then
`--launches` fused step launches of `--depth` turns (automatic rows/wave)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "game-of-life-distributed_amd"))
import golhip  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--size", type=int, default=16384)
ap.add_argument("--depth", type=int, default=16)
ap.add_argument("--launches", type=int, default=20)
a = ap.parse_args()
with golhip.Board(a.size, a.size, timing=True) as b:
    b.set_tb_depth(a.depth)
    b.fill_random(0x5EED0001 if a.size == 16384 else 0x5EED0002)
    b.step(2 * a.depth)
    b.sync()
    b.perf_reset()
    b.step(a.launches * a.depth)
    b.sync()
    p = b.perf()
    print({"size": a.size, "depth": a.depth, "launches": p["step_launches"],
           "avg_launch_ms": p["step_kernel_ms"] / max(1, p["step_launches"]), "rows_per_wave": p["rows_per_wave"]})
