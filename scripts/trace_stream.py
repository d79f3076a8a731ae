"""K5 (fused turn + flip list) per-launch time at 5120^2, by phase (A/B only).

flip_debug 1 skips the look-back, 2 the entry writes, 3 both (results wrong;
measurement only).  Each leg: 60 launches from the configs[4] board at turn
2064, every launch a real turn (cap large enough), kernel time from HIP events.
"""
import json
import os

os.environ.setdefault("GOLHIP_TUNING", "1")  # A/B knobs of the kernel plans (golhip.h)
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "game-of-life-distributed_amd")]
os.environ["GOLHIP_MEASUREMENT"] = "1"  # flip_debug 1-3: wrong lists by design
import golhip  # noqa: E402

N, SEED, T = 5120, 0x5EED0005, 60
res = {}
with golhip.Board(N, N, timing=True) as b:
    for fmt, name in ((golhip.FLIPS_XY, "xy"), (golhip.FLIPS_INDEX, "index")):
        buf = golhip.host_array((T * 600000,) + ((2,) if fmt == golhip.FLIPS_XY else ()),
                                np.int32 if fmt == golhip.FLIPS_XY else np.uint32)
        for dbg in (0, 1, 2, 3):
            for pinned in (False, True):
                out = buf if pinned else np.empty_like(np.asarray(buf))
                b.set_option("flip_debug", 0)
                b.fill_random(SEED)
                b.step(2064)
                b.sync()
                b.set_option("flip_debug", dbg)
                b.perf_reset()
                ent, counts, done = b.flip_stream(T, cap=out.shape[0], fmt=fmt, out=out)
                p = b.perf()
                res[f"{name}_dbg{dbg}_{'pinned' if pinned else 'dev'}"] = {
                    "done": done, "launches": p["flip_launches"],
                    "us_per_launch": p["flip_kernel_ms"] * 1e3 / max(1, p["flip_launches"])}
print(json.dumps(res))
