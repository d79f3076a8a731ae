"""K5 (fused turn + flip list) into golhip_host_alloc memory, per-launch device
time with flip_overlap 0 / 1 and without entries (flip_debug 2, measurement),
beside the host-link probe at the list's own size (one launch per list).
    python scripts/k5_overlap_probe.py > gpurun_out/k5_overlap.jsonl"""
import json
import os
import sys

os.environ.setdefault("GOLHIP_TUNING", "1")
os.environ.setdefault("GOLHIP_MEASUREMENT", "1")  # flip_debug 2: no entries (wrong lists by design)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "game-of-life-distributed_amd")]
import numpy as np  # noqa: E402

import golhip  # noqa: E402

N, T0, TURNS = 5120, 2064, 200
cap = 32 << 20
idx = golhip.host_array((cap,), np.uint32)
for mode in ("overlap", "direct", "no_entries"):
    with golhip.Board(N, N, timing=True) as b:
        b.set_option("flip_overlap", 1 if mode == "overlap" else 0)
        if mode == "no_entries":
            b.set_option("flip_debug", 2)
        b.fill_random(0x5EED0005)
        b.step(T0)
        b.sync()
        done = 0
        while done < 50:
            _, _, k = b.flip_stream(50 - done, cap=cap, fmt=golhip.FLIPS_INDEX, out=idx)
            done += k
        b.perf_reset()
        done, ent = 0, 0
        while done < TURNS:
            e, _, k = b.flip_stream(TURNS - done, cap=cap, fmt=golhip.FLIPS_INDEX, out=idx)
            done += k
            ent += len(e)
        p = b.perf()
        print(json.dumps({"mode": mode, "turns": TURNS, "launches": p["flip_launches"],
                          "us_per_launch": round(p["flip_kernel_ms"] * 1e3 / p["flip_launches"], 2),
                          "entries_per_turn": ent / TURNS}), flush=True)
for nbytes in (1 << 20, 1388544, 4 << 20, 64 << 20):
    r = golhip.host_link_probe(0, nbytes, 50)
    print(json.dumps({"probe_bytes": nbytes, **r, "us_per_pass": round(nbytes / r["kernel_write_GBps"] / 1e3, 2)}),
          flush=True)
