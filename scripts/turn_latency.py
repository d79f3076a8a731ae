"""1-turn launches at 5120^2 under different host patterns (kernel-trace them):
  A  step(1) + sync, 200 times         (host round trip per turn)
  B  step(1) x 200, one sync           (back-to-back)
  C  step(1, want_flips) + flips(), 200 times (the per-turn event path)
Prints wall time per turn of each phase."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "game-of-life-distributed_amd")]
import golhip  # noqa: E402

N, T = 5120, 200
out = {}
with golhip.Board(N, N) as b:
    b.fill_random(0x5EED0005)
    b.step(64)
    b.sync()
    for name in "ABCAB":
        t0 = time.perf_counter()
        for _ in range(T):
            if name == "A":
                b.step(1)
                b.sync()
            elif name == "B":
                b.step(1)
            else:
                b.step(1, want_flips=True)
                b.flips()
        b.sync()
        out.setdefault(name, []).append((time.perf_counter() - t0) / T * 1e6)
print(json.dumps({"us_per_turn": out}))
