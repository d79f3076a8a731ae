"""Diagnostic: repeat 65536^2 fill + 32 turns through the per-launch kernel on
fresh handles and report every digest that differs from the first."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "game-of-life-distributed_amd"))
import golhip  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
N, turns = 65536, 32
first = None
bad = 0
t0 = time.time()
for rep in range(reps):
    for d in (32, 16):
        with golhip.Board(N, N) as b:
            b.set_tb_depth(d)
            b.fill_random(0x5EED0002)
            b.step(turns)
            r = (b.board_hash(), b.alive_count()[0])
        first = first or r
        if r != first:
            bad += 1
            print(json.dumps({"rep": rep, "depth": d, "hash": r[0], "alive": r[1], "want": first}), flush=True)
    if rep % 10 == 0:
        print(json.dumps({"rep": rep, "bad": bad, "s": round(time.time() - t0, 1)}), flush=True)
print(json.dumps({"reps": reps, "bad": bad, "want": first}), flush=True)
