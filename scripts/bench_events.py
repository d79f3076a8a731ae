"""BASELINE configs[4]: 5120 x 5120 board with the full event stream.

Prints one JSON object with:
  events_off      fused turns (no per-turn side channels), GCUPS
  events_on       one turn per call + that turn's CellFlipped list copied to
                  the host (golhip_step(1, want_flips) + golhip_flips) +
                  AliveCellsCount every 2 s: turns/s, flips/s
  events_batched  golhip_step_flips, batches of 50 turns (int32 pairs)
  stream_xy /     golhip_flip_stream (fused turn + flip list, K5), as many
  stream_index    turns per call as a 32 M-entry caller buffer holds, pairs
  (_pinned)       (8 B) / cell indices (4 B), in a pageable numpy buffer
                  (device list + one copy) or a golhip_host_alloc buffer
                  (the kernel writes the host memory): turns/s, flips/s (no
                  HIP timing events), the K5 kernel alone (HIP events on a
                  second run): us per launch, algorithmic bytes
                  per turn (board read + board written + entries) and their
                  rate against the 8 TB/s HBM peak
  snapshot_s      one 's' snapshot (golhip_snapshot_bytes + PGM write), ms
Every leg starts from the same state (seed 0x5EED0005 + 2064 turns: ~0.4 M
flips a turn; the first turns of the random board flip 3-7 M) and runs the
same 200 turns, so the flip totals must agree (checked).
"""
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "game-of-life-distributed_amd")]
import golhip  # noqa: E402
from oracle.oracle import pgm_bytes  # noqa: E402  (PGM header format only)

N = 5120
SEED = 0x5EED0005
TURNS = 200
HBM_PEAK = 8.0e12
out = {"workload": "configs[4]: 5120^2 random 25%, seed 0x5EED0005, turns 2065..2264", "board": [N, N]}


# the host link itself: one 64 MiB device -> host copy, pageable vs page-locked
# (torch first: its HIP runtime must initialise before libgolhip's does)
import torch
src = torch.empty(16 << 20, dtype=torch.int32, device="cuda")
for label, dst in (("pageable", torch.empty(16 << 20, dtype=torch.int32)),
                   ("pinned", torch.empty(16 << 20, dtype=torch.int32, pin_memory=True))):
    dst.copy_(src)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        dst.copy_(src)
    torch.cuda.synchronize()
    out[f"d2h_{label}_GBps"] = 5 * (64 << 20) / (time.perf_counter() - t0) / 1e9



def reset(b):
    b.fill_random(SEED)
    b.step(64)
    b.step(2000)
    b.sync()


with golhip.Board(N, N, timing=True) as b:
    b.fill_random(SEED)
    b.step(64)
    b.sync()
    t0 = time.perf_counter()
    b.step(2000)
    b.sync()
    dt = time.perf_counter() - t0
    out["events_off"] = {"turns": 2000, "seconds": dt, "gcups": N * N * 2000 / dt / 1e9}

    flips_total = 0
    last_tick = time.perf_counter()
    ticks = 0
    t0 = time.perf_counter()
    for _ in range(TURNS):
        b.step(1, want_flips=True)
        flips_total += len(b.flips())
        if time.perf_counter() - last_tick >= 2.0:
            b.alive_count()
            ticks += 1
            last_tick = time.perf_counter()
    dt = time.perf_counter() - t0
    out["events_on"] = {"turns": TURNS, "seconds": dt, "turns_per_s": TURNS / dt, "flips": flips_total,
                        "flips_per_s": flips_total / dt, "gcups": N * N * TURNS / dt / 1e9, "ticks": ticks}

    reset(b)
    BATCH = 50
    xy = np.empty((BATCH * 1_500_000, 2), dtype=np.int32)
    xy.fill(0)  # touch the pages outside the timed region
    flips_b = 0
    t0 = time.perf_counter()
    for _ in range(TURNS // BATCH):
        got, counts = b.step_flips(BATCH, cap=xy.shape[0], xy=xy)
        flips_b += len(got)
    dt = time.perf_counter() - t0
    out["events_batched"] = {"turns": TURNS, "batch": BATCH, "seconds": dt, "turns_per_s": TURNS / dt,
                             "flips": flips_b, "flips_per_s": flips_b / dt, "gcups": N * N * TURNS / dt / 1e9,
                             "same_flips_as_events_on": flips_b == flips_total}

    legs = (("stream_xy", golhip.FLIPS_XY, 8, False), ("stream_index", golhip.FLIPS_INDEX, 4, False),
            ("stream_xy_pinned", golhip.FLIPS_XY, 8, True), ("stream_index_pinned", golhip.FLIPS_INDEX, 4, True))
    # turns/s on a board without per-launch HIP timing events (they cost the
    # pinned legs ~2x in host time), the K5 kernel time on the timed board
    plain = golhip.Board(N, N)
    for name, fmt, esz, pinned in legs:
        cap = 32 << 20
        shape, dty = ((cap, 2), np.int32) if esz == 8 else ((cap,), np.uint32)
        buf = golhip.host_array(shape, dty) if pinned else np.empty(shape, dtype=dty)
        buf.fill(0)
        rec = {"turns": TURNS}
        for bb, timed in ((plain, False), (b, True)):
            reset(bb)
            bb.perf_reset()
            done, flips_s, calls = 0, 0, 0
            t0 = time.perf_counter()
            while done < TURNS:
                ent, counts, k = bb.flip_stream(TURNS - done, cap=cap, fmt=fmt, out=buf)
                done += k
                flips_s += len(ent)
                calls += 1
            dt = time.perf_counter() - t0
            if not timed:
                rec.update({"calls": calls, "seconds": dt, "turns_per_s": TURNS / dt, "flips": flips_s,
                            "flips_per_s": flips_s / dt, "gcups": N * N * TURNS / dt / 1e9,
                            "same_flips_as_events_on": flips_s == flips_total})
            else:
                p = bb.perf()
                kus = p["flip_kernel_ms"] * 1e3 / max(1, p["flip_launches"])
                alg = 2 * N * N / 8 + flips_s / TURNS * esz  # board in + board out + entries, per turn
                rec.update({"kernel_us_per_launch": kus, "launches": p["flip_launches"], "alg_bytes_per_turn": alg,
                            "kernel_GBps": alg / (kus * 1e-6) / 1e9 if kus > 0 else None,
                            "kernel_hbm_frac": alg / (kus * 1e-6) / HBM_PEAK if kus > 0 else None})
        out[name] = rec
    plain.close()

    t0 = time.perf_counter()
    snap = b.snapshot_bytes()
    with tempfile.NamedTemporaryFile(suffix=".pgm") as f:
        f.write(pgm_bytes(snap))
        f.flush()
    out["snapshot_s_ms"] = (time.perf_counter() - t0) * 1e3

print(json.dumps(out))
