"""K1w diagnosis, second pass: for every wrong row of one skew launch, the
(generation, row shift) of the oracle board it equals, if any (a wrong
generation or a shifted store shows up as such a match).

    python scripts/skew_debug2.py W H depth wpl launches [k=v ...]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "game-of-life-distributed_amd")]
import golhip  # noqa: E402
from oracle.oracle import COracle  # noqa: E402

W, H, depth, wpl, nl = (int(x) for x in sys.argv[1:6])  # nl: launches of depth turns
opts = dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in sys.argv[6:])
co = COracle()
board = co.fill_random(W, H, 0x5EED0031 + W + H)
gens = [board]
for g in range(nl * depth + 4):
    gens.append(co.run(gens[-1], 1))
want = gens[nl * depth]
with golhip.Board(W, H) as b:
    b.set_option("persistent", 0)
    b.set_option("skew", 2)
    b.set_option("wpl", wpl)
    for k, v in opts.items():
        b.set_option(k, v)
    b.set_tb_depth(depth)
    b.load_bytes(board)
    for _ in range(nl):
        b.step(depth)
    got = b.snapshot_bytes()
bad = np.nonzero((got != want).any(axis=1))[0].tolist()
for r in bad[:40]:
    hits = []
    for g in list(range(0, 3)) + list(range(max(3, nl * depth - 4), nl * depth + 4)):
        for sh in range(-4, 5):
            if np.array_equal(got[r], gens[g][(r + sh) % H]):
                hits.append((g, sh))
    nb = int((got[r] != want[r]).sum())
    print(json.dumps({"row": r, "ncells_bad": nb, "all_zero": bool((got[r] == 0).all()), "matches": hits}), flush=True)
