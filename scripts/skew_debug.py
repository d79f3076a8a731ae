"""K1w diagnosis: one skew launch (turns = depth) per case against the C
oracle, with and without the cross-stack hand-off; prints the rows that
differ (as ranges) so a wrong band or stack boundary shows up by position.

    python scripts/skew_debug.py [--cases 2048x1024,4096x777] [--depths 8:2,20:2,9:4]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "game-of-life-distributed_amd")]
import golhip  # noqa: E402
from oracle.oracle import COracle  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--cases", default="2048x1024,4096x777,8192x331,16384x1600")
ap.add_argument("--depths", default="8:2,12:2,16:2,20:2,8:4,9:4,16:1,32:1")
ap.add_argument("--sets", default="skew_xstack=0;skew_xstack=1")
a = ap.parse_args()
co = COracle()


def ranges(rows):
    out, start, prev = [], None, None
    for r in rows:
        if start is None:
            start = prev = r
        elif r == prev + 1:
            prev = r
        else:
            out.append((start, prev))
            start = prev = r
    if start is not None:
        out.append((start, prev))
    return out


for case in a.cases.split(","):
    W, H = (int(x) for x in case.split("x"))
    for dw in a.depths.split(","):
        depth, wpl = (int(x) for x in dw.split(":"))
        if W % (32 * wpl):
            continue
        board = co.fill_random(W, H, 0x5EED0031 + W + H)
        want = co.run(board, depth)
        for s in a.sets.split(";"):
            opts = dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in s.split(",") if kv)
            with golhip.Board(W, H) as b:
                b.set_option("persistent", 0)
                b.set_option("skew", 2)
                b.set_option("wpl", wpl)
                for k, v in opts.items():
                    b.set_option(k, v)
                b.set_tb_depth(depth)
                b.load_bytes(board)
                b.step(depth)
                p = b.perf()
                got = b.snapshot_bytes()
            bad = np.nonzero((got != want).any(axis=1))[0].tolist()
            cols = np.nonzero((got != want).any(axis=0))[0].tolist()
            print(json.dumps({"W": W, "H": H, "depth": depth, "wpl": wpl, "opts": opts,
                              "skew": p["skew_launches"], "rpw": p["rows_per_wave"], "nbad_rows": len(bad),
                              "bad_rows": ranges(bad)[:12], "bad_cols": ranges(cols)[:6]}), flush=True)
