"""Diagnostic: wall time of 100-turn steps with and without per-launch HIP
timing events (GOLHIP_FLAG_TIMING), alternating, on one board size."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "game-of-life-distributed_amd"))
import golhip  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
turns = int(sys.argv[2]) if len(sys.argv) > 2 else 100
for rnd in range(2):
    for timing in (True, False):
        with golhip.Board(N, N, timing=timing) as b:
            b.fill_random(0x5EED0002)
            b.step(turns)
            b.sync()
            t0 = time.perf_counter()
            for _ in range(5):
                b.step(turns)
            b.sync()
            dt = time.perf_counter() - t0
            print(json.dumps({"round": rnd, "N": N, "timing": timing, "gcups": N * N * turns * 5 / dt / 1e9,
                              "ms_per_step": dt / 5 * 1e3}), flush=True)
