"""Diagnostic: repeat the 65536^2 fill + step on fresh handles and compare the
board digest / alive count (after fill and after the steps)."""
import argparse
import json
import os

os.environ.setdefault("GOLHIP_TUNING", "1")  # A/B knobs of the kernel plans (golhip.h)
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "game-of-life-distributed_amd"))
import golhip  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--size", type=int, default=65536)
ap.add_argument("--turns", type=int, default=32)
ap.add_argument("--depths", default="32,16,16,32")
ap.add_argument("--options", default="")
a = ap.parse_args()
for d in map(int, a.depths.split(",")):
    with golhip.Board(a.size, a.size) as b:
        for kv in filter(None, a.options.split(",")):
            k, v = kv.split("=")
            b.set_option(k, int(v))
        b.set_tb_depth(d)
        b.fill_random(0x5EED0002)
        h0 = b.board_hash()
        b.step(a.turns)
        print(json.dumps(dict(lib=os.path.basename(os.path.dirname(golhip.LIB_PATH)), depth=d, fill_hash=h0,
                              hash=b.board_hash(), alive=b.alive_count())), flush=True)
