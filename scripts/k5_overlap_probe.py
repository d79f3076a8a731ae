"""K5 (fused turn + flip list) into golhip_host_alloc memory, per-launch device
time with flip_overlap 0 / 1 / 2 and without entries (flip_debug 2, measurement),
beside the host-link probe at the list's own size (one launch per list).
Optional: the host buffer sizes to try, in entries (default 32M: the bench's).
    python scripts/k5_overlap_probe.py [cap ...] > gpurun_out/k5_overlap.jsonl"""
import json
import os
import sys
import time

os.environ.setdefault("GOLHIP_TUNING", "1")
os.environ.setdefault("GOLHIP_MEASUREMENT", "1")  # flip_debug 2: no entries (wrong lists by design)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "game-of-life-distributed_amd")]
import numpy as np  # noqa: E402

import golhip  # noqa: E402

N, T0, TURNS = 5120, 2064, 200
caps = [int(x) for x in sys.argv[1:]] or [32 << 20]
MODES = {"resident": 2, "overlap": 1, "direct": 0, "no_entries": 0, "resident_no_entries": 2}
if os.environ.get("K5_MODES"):  # e.g. K5_MODES=overlap for a counter pass over one mode
    MODES = {m: MODES[m] for m in os.environ["K5_MODES"].split(",")}
for cap, mode in [(c, m) for c in caps for m in MODES]:
    idx = golhip.host_array((cap,), np.uint32)
    with golhip.Board(N, N, timing=not os.environ.get("K5_UNTIMED")) as b:
        b.set_option("flip_overlap", MODES[mode])
        if mode.endswith("no_entries"):
            b.set_option("flip_debug", 2)
        b.fill_random(0x5EED0005)
        b.step(T0)
        b.sync()
        done = 0
        while done < 50:
            _, _, k = b.flip_stream(50 - done, cap=cap, fmt=golhip.FLIPS_INDEX, out=idx)
            done += k
        b.sync()
        b.perf_reset()
        t0 = time.perf_counter()
        done, ent = 0, 0
        while done < TURNS:
            e, _, k = b.flip_stream(TURNS - done, cap=cap, fmt=golhip.FLIPS_INDEX, out=idx)
            done += k
            ent += len(e)
        b.sync()
        wall = time.perf_counter() - t0
        p = b.perf()
        print(json.dumps({"mode": mode, "cap": cap, "turns": TURNS, "wall_turns_per_s": round(TURNS / wall, 1),
                          "launches": p["flip_launches"],
                          "us_per_launch": round(p["flip_kernel_ms"] * 1e3 / max(1, p["flip_launches"]), 2),
                          "resident_launches": p["flip_resident_launches"],
                          "entries_per_turn": ent / TURNS}), flush=True)
for nbytes in () if os.environ.get("K5_MODES") else (1 << 20, 1388544, 4 << 20, 64 << 20):
    r = golhip.host_link_probe(0, nbytes, 50)
    print(json.dumps({"probe_bytes": nbytes, **r, "us_per_pass": round(nbytes / r["kernel_write_GBps"] / 1e3, 2)}),
          flush=True)
