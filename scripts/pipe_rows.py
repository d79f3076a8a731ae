"""K1t per-row cost: bands whose height leaves the circular pipeline no
bubble (h >= 3 x 8 stages), steady-state row loop ticks per row with and
without its ring waits (option "trace": golhip_persist_trace_waves words 0..2)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "game-of-life-distributed_amd")]
import golhip  # noqa: E402

for W, H, cus, turns in [(8192, 60, 1, 800), (8192, 240, 4, 800), (8192, 8192, 0, 800), (4096, 4096, 0, 800),
                         (2048, 500, 1, 800), (2048, 2048, 0, 800), (4096, 120 * 256, 0, 400)]:
    with golhip.Board(W, H) as b:
        b.set_option("lds_pipe", 1)
        b.set_option("persistent", 1)
        b.set_option("trace", 1)
        if cus:
            b.set_option("cu_count", cus)
        b.fill_random(5)
        b.step(turns)
        b.sync()
        ex = b.persist_trace_waves(1).reshape(-1)[:3]
        tr = b.persist_trace()
        p = b.perf()
        b.set_option("trace", 0)
    rows = int(ex[1]) or 1
    print(json.dumps({"W": W, "H": H, "cus": cus, "turns": turns, "pipe": p["pipe_launches"], "trace": tr,
                      "fast_ticks_per_row": round(int(ex[0]) / rows, 2),
                      "fast_wait_ticks_per_row": round(int(ex[2]) / rows, 2), "fast_rows": rows}), flush=True)
