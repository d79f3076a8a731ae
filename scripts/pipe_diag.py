"""K1t diagnostics: which configurations launch K1t, fall back (timeout) or do
not fit; prints the perf counters of one step each."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "game-of-life-distributed_amd")]
import golhip  # noqa: E402

for W, H, cus, turns in [(2048, 303, 1, 70), (2048, 305, 2, 70), (2048, 307, 3, 70), (2048, 512, 0, 100),
                         (2048, 512, 0, 9), (8192, 8192, 0, 100)]:
    with golhip.Board(W, H) as b:
        b.set_option("lds_pipe", 1)
        b.set_option("trace", 1)
        if cus:
            b.set_option("cu_count", cus)
        b.fill_random(5)
        err = None
        try:
            b.step(turns)
            b.sync()
        except golhip.GolHipError as e:
            err = str(e)
        p = b.perf()
        tr = b.persist_trace()
    print(json.dumps({"W": W, "H": H, "cus": cus, "turns": turns, "err": err,
                      **{k: p[k] for k in ("pipe_launches", "lds_launches", "persist_launches", "persist_fallbacks",
                                           "step_launches", "kernel_variant", "words_per_lane")}, "trace": tr}), flush=True)
