"""Diagnostic: repeat the sequence of tests/test_gpu_parity.py::
test_persistent_full_size_matches_per_launch and report any digest that
differs from the first run of the same path (nondeterminism hunt)."""
import json
import os

os.environ.setdefault("GOLHIP_TUNING", "1")  # A/B knobs of the kernel plans (golhip.h)
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "game-of-life-distributed_amd"))
import golhip  # noqa: E402

seen = {}
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
for rep in range(reps):
    for N, turns in ((16384, 512), (65536, 64)):
        for persistent in (1, 0):
            with golhip.Board(N, N) as b:
                b.set_option("persistent", persistent)
                b.fill_random(0x5EED0001)
                b.step(turns)
                r = (b.board_hash(), b.alive_count()[0])
            key = (N, persistent)
            ok = seen.setdefault(key, r) == r and seen.get((N, 1 - persistent), r) == r
            print(json.dumps({"rep": rep, "N": N, "persistent": persistent, "hash": r[0], "alive": r[1], "ok": ok}),
                  flush=True)
