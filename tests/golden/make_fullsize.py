"""Generate the full-size BASELINE fixtures (tests/golden/fullsize.json + .npz).

Run in the build container (8 cores, ~17 GB of RAM for configs[3]):

    python tests/golden/make_fullsize.py [--only c1,c2,c3,c4] [--threads 8]

Every BASELINE.json config that the GPU runs gets an oracle answer here, made
by the bit-packed CPU comparator oracle/gol_fastcpu.c (B3/S23 torus, the rule
and wrap of gol/distributor.go:350-417), which tests/test_oracle_golden.py pins
to the reference's own fixtures (all 9 check/images boards and the 30,000
check/alive counts) and to the per-cell restatement oracle/gol_oracle.c:

  c1  configs[1]  16384^2,  seed 0x5EED0001, turns 0/1/16/100/1000/10000
  c2  configs[2]  65536^2,  seed 0x5EED0002, turns 0/1/100/1000
  c3  configs[3]  262144^2, seed 0x5EED0003, turns 0/1/100
  c4  configs[4]  5120^2,   seed 0x5EED0005, the CellFlipped stream of turns
                  1..50: per-turn flip counts and the SHA-256 of the
                  concatenated (x = col, y = row) int32 pairs, row-major within
                  a turn (initializeAliveCells, distributor.go:212-220), and
                  per turn an order-dependent digest (ordered_digest) that the
                  host mirror's C++ drain can recompute

For each checkpoint: the board digest of golhip_board_hash (include/golhip.h,
restated by fastcpu_hash) and the alive count; for the last checkpoint also
four whole rows (0, 1, H/2, H-1) as canonical uint32 words in fullsize.npz.
Synthetic boards follow fill_random's rule:
cell (y, x) alive <=> (splitmix64(seed ^ (y*W + x)) & 3) == 0.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from oracle.oracle import COracle  # noqa: E402

CONFIGS = {
    "c1": dict(config="configs[1]", N=16384, seed=0x5EED0001, turns=[0, 1, 16, 100, 1000, 10000]),
    "c2": dict(config="configs[2]", N=65536, seed=0x5EED0002, turns=[0, 1, 100, 1000]),
    "c3": dict(config="configs[3]", N=262144, seed=0x5EED0003, turns=[0, 1, 100]),
}
EVENTS = dict(config="configs[4]", N=5120, seed=0x5EED0005, turns=50)
SAMPLE_ROWS = lambda N: [0, 1, N // 2, N - 1]  # noqa: E731


def canon_rows(words64: np.ndarray, rows: list[int]) -> np.ndarray:
    """Packed uint64 rows -> canonical uint32 words (word 2k = low half of uint64 k)."""
    return np.ascontiguousarray(words64[rows]).view(np.uint32).copy()


def flips_xy(old: np.ndarray, new: np.ndarray, W: int) -> np.ndarray:
    """Row-major (x, y) int32 pairs of the cells that differ (packed uint64 boards)."""
    d = np.bitwise_xor(old, new)
    bits = np.unpackbits(d.view(np.uint8), axis=1, bitorder="little")[:, :W]
    ys, xs = np.nonzero(bits)
    return np.stack([xs, ys], axis=1).astype(np.int32)


def make_board(o: COracle, key: str, c: dict, th: int, arrays: dict) -> dict:
    N, seed = c["N"], c["seed"]
    t0 = time.time()
    w = o.fill_random64(N, N, seed, th)
    print(f"{key}: {N}^2 filled in {time.time() - t0:.1f} s", flush=True)
    done, rec = 0, {"config": c["config"], "width": N, "height": N, "seed": seed, "checkpoints": {}}
    for t in c["turns"]:
        t1 = time.time()
        if t > done:
            o.run_fast_words(w, N, t - done, th)
            done = t
        h, a = o.hash64(w, N, th), o.popcount64(w, N, th)
        rec["checkpoints"][str(t)] = {"hash": f"{h:016x}", "alive": a}
        print(f"{key}: turn {t}: hash {h:016x} alive {a} ({time.time() - t1:.1f} s)", flush=True)
    rec["sample_turn"] = done
    rec["sample_rows"] = SAMPLE_ROWS(N)
    arrays[f"{key}_rows"] = canon_rows(w, rec["sample_rows"])
    return rec


def ordered_digest(xy: np.ndarray, W: int) -> int:
    """Order-dependent digest of one turn's list, cheap in C++ too (the host
    mirror's golrun_drain): sum over positions i of
    splitmix64(i + 1) * (y * W + x + 1) mod 2^64."""
    i = np.arange(1, len(xy) + 1, dtype=np.uint64)
    e = xy[:, 1].astype(np.uint64) * np.uint64(W) + xy[:, 0].astype(np.uint64) + np.uint64(1)
    with np.errstate(over="ignore"):
        z = i + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
        return int((z * e).sum(dtype=np.uint64))


def make_events(o: COracle, th: int) -> dict:
    N, seed, T = EVENTS["N"], EVENTS["seed"], EVENTS["turns"]
    w = o.fill_random64(N, N, seed, th)
    init = flips_xy(np.zeros_like(w), w, N)  # the CellFlipped of every alive cell at load (:72-80)
    sha, counts, digests = hashlib.sha256(), [], []
    for _ in range(T):
        nxt = w.copy()
        o.run_fast_words(nxt, N, 1, th)
        xy = flips_xy(w, nxt, N)
        sha.update(xy.tobytes())
        counts.append(int(len(xy)))
        digests.append(f"{ordered_digest(xy, N):016x}")
        w = nxt
    rec = {"config": EVENTS["config"], "width": N, "height": N, "seed": seed, "turns": T,
           "initial_alive": int(len(init)), "initial_sha256": hashlib.sha256(init.tobytes()).hexdigest(),
           "flip_counts": counts, "flips_sha256": sha.hexdigest(), "flip_digests": digests,
           "final": {"hash": f"{o.hash64(w, N, th):016x}", "alive": o.popcount64(w, N, th)}}
    print(f"c4: {T} turns, {sum(counts)} flips, sha {rec['flips_sha256'][:16]}", flush=True)
    return rec


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="c1,c2,c3,c4")
    ap.add_argument("--threads", type=int, default=min(8, os.cpu_count() or 1))
    a = ap.parse_args()
    keys = a.only.split(",")
    o = COracle()
    jpath, npath = os.path.join(HERE, "fullsize.json"), os.path.join(HERE, "fullsize.npz")
    out, arrays = {}, {}
    if os.path.exists(jpath):  # regenerate a subset, keep the rest
        with open(jpath) as f:
            out = json.load(f)
        with np.load(npath, allow_pickle=False) as z:
            arrays = {k: z[k] for k in z.files}
    for k in keys:
        if k in CONFIGS:
            out[k] = make_board(o, k, CONFIGS[k], a.threads, arrays)
        elif k == "c4":
            out[k] = make_events(o, a.threads)
    out["generator"] = ("tests/golden/make_fullsize.py: oracle/gol_fastcpu.c (fastcpu_fill_random, fastcpu_run, "
                        "fastcpu_hash, fastcpu_popcount)")
    with open(jpath, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    np.savez_compressed(npath, **arrays)
    print("wrote", jpath, npath)


if __name__ == "__main__":
    main()
