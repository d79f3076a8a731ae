"""Diagnostic: 65536^2 board digests after `turns` through the persistent
kernel, the per-launch kernel (depth 16) and the per-launch kernel at depth 1
(the referee), for both words-per-lane layouts."""
import json
import os

os.environ.setdefault("GOLHIP_TUNING", "1")  # A/B knobs of the kernel plans (golhip.h)
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "game-of-life-distributed_amd"))
import golhip  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
for turns in (16, 32, 48, 64):
    for wpl in (2, 1):
        out = {}
        for name, opts, depth in (("persist", {"persistent": 1}, 16), ("launch16", {"persistent": 0}, 16),
                                  ("launch1", {"persistent": 0}, 1)):
            with golhip.Board(N, N) as b:
                b.set_option("wpl", wpl)
                for k, v in opts.items():
                    b.set_option(k, v)
                b.set_tb_depth(depth)
                b.fill_random(0x5EED0001)
                b.step(turns)
                out[name] = (b.board_hash(), b.alive_count()[0], b.perf()["persist_launches"])
        ok = out["persist"][:2] == out["launch1"][:2] and out["launch16"][:2] == out["launch1"][:2]
        print(json.dumps({"turns": turns, "wpl": wpl, "ok": ok, **{k: list(v) for k, v in out.items()}}), flush=True)
