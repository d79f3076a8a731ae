"""Flip-stream timeline at 5120^2 for rocprofv3 --kernel-trace --memory-copy-trace:
200 turns from the configs[4] board at turn 2064 per leg (no HIP timing events):
  index into a golhip_host_alloc buffer, index into pageable memory, pairs into
  pageable memory.  Prints each leg's wall time."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "game-of-life-distributed_amd")]
import golhip  # noqa: E402

N, SEED, T = 5120, 0x5EED0005, 200
res = {}
with golhip.Board(N, N) as b:
    cap = 32 << 20
    for name, fmt, pinned in (("index_pinned", golhip.FLIPS_INDEX, True), ("index_pageable", golhip.FLIPS_INDEX, False),
                              ("xy_pageable", golhip.FLIPS_XY, False), ("xy_pinned", golhip.FLIPS_XY, True)):
        shape, dty = ((cap, 2), np.int32) if fmt == golhip.FLIPS_XY else ((cap,), np.uint32)
        buf = golhip.host_array(shape, dty) if pinned else np.empty(shape, dtype=dty)
        buf.fill(0)
        b.fill_random(SEED)
        b.step(2064)
        b.sync()
        done, calls = 0, 0
        t0 = time.perf_counter()
        while done < T:
            ent, counts, k = b.flip_stream(T - done, cap=cap, fmt=fmt, out=buf)
            done += k
            calls += 1
        res[name] = {"turns_per_s": T / (time.perf_counter() - t0), "calls": calls}
print(json.dumps(res))
