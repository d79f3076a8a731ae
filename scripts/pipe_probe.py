"""K1t (resident LDS turn pipeline) against K1r / K1p on small tori: GCUPS of
long steps (HIP events on the engine stream), plus K1t's wait breakdown
(option "trace": wave ticks waiting for ring rows, ring room, imports, edge
room, of all wave ticks).  Usage: python scripts/pipe_probe.py [turns]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "game-of-life-distributed_amd")]
import golhip  # noqa: E402


def measure(W, H, turns, opts, reps=3):
    with golhip.Board(W, H) as b:
        for k, v in opts.items():
            b.set_option(k, v)
        b.fill_random(0x5EED0077)
        b.step(turns)  # warm
        b.sync()
        best = 1e9
        for _ in range(reps):
            b.perf_reset()
            t0 = time.perf_counter()
            b.step(turns)
            b.sync()
            best = min(best, time.perf_counter() - t0)
        p = b.perf()
        tr = None
        if opts.get("trace"):
            tr = b.persist_trace()
    return {"W": W, "H": H, "turns": turns, "opts": opts, "gcups": round(W * H * turns / best / 1e9, 1),
            "ms": round(best * 1e3, 3), "pipe": p["pipe_launches"], "lds": p["lds_launches"],
            "persist": p["persist_launches"], "wpl": p["words_per_lane"], "trace": tr}


if __name__ == "__main__":
    turns = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    for W, H in [(8192, 8192), (4096, 4096), (2048, 2048), (8192, 4096)]:
        for opts in ({"lds_pipe": 1}, {"lds_pipe": 0}, {"lds_pipe": 1, "trace": 1}):
            print(json.dumps(measure(W, H, turns, opts)), flush=True)
