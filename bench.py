"""bench.py — cell-updates/s of the MI355X Game of Life engine (libgolhip.so).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload 65536|16384|262144|5120]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

A "step" is one run of the workload's BASELINE config over the whole board:
its turns (configs[2]: 1,000) of the synthetic torus, run as fused launches.
Timed region: exactly K steps, bracketed by a barrier and
torch.cuda.synchronize() on both sides, max over ranks.

Workloads (BASELINE.json configs; synthetic boards, data="synthetic"), all
strong-scaled: ONE board of the config, rank r of N owns rows
[r*N_rows/N, (r+1)*N_rows/N) and exchanges halo rows with its ring neighbours
over RCCL (the only collective on the path):
  65536  (default, configs[2]) 65536^2,  seed 0x5EED0002, 1,000 turns a step
  16384  (configs[1])          16384^2,  seed 0x5EED0001, 10,000 turns a step
  262144 (configs[3])          262144^2, seed 0x5EED0003, 100 turns a step
  5120   (configs[4])          5120^2, seed 0x5EED0005, the full event stream: every
                               turn's CellFlipped list (fused turn + list kernel K5,
                               4-byte cell indices into page-locked host memory),
                               200 turns a step from turn 2064 on; one GPU

Parity: the first untimed step starts from the freshly filled board, so after
it the board is at exactly the config's turns; its digest (golhip_board_hash,
summed over ranks) and alive count must equal tests/golden/fullsize.json (the
oracle's answer, tests/golden/make_fullsize.py).  The JSON line carries
"parity": true/false and the run exits 1 after printing on a mismatch.

Warmup: W untimed steps (at least 1, the parity step), then more untimed steps
until --warmup-seconds have passed.  Rank 0 prints ONE JSON line; `roofline`
is measured live on the step kernels with HIP events on the engine's stream
(see roofline_block); `cpu_baseline` times the oracle's port of the reference
worker pool on a bounded sample (rank 0, N = 1 only), with the bit-packed
OpenMP CPU comparator beside it (`cpu_baseline.fast_cpu`).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "game-of-life-distributed_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import golhip  # noqa: E402

METRIC = "cell-updates/sec (GCUPS) at 1/2/4/8 MI355X; % of HBM roofline"
HBM_PEAK_GBS = 8000.0         # MI355X_MICROARCH.md: 8.0 TB/s spec
ALG_BYTES_PER_UPDATE = 0.25   # 1 bit read + 1 bit written per cell-update
# VALU issue peak (MI355X_MICROARCH.md, chip table + "Wave scheduling"): 256 CUs x
# 4 SIMD-32 x one wave64 VALU instruction per 2 cycles x 2.4 GHz max clock.
# A "slot" is one full-rate wave64 instruction; DPP moves and v_alignbit_b32
# issue at half rate on gfx950 (scripts/ubench) and cost 2.
VALU_PEAK_GSLOTS = 256 * 4 * 0.5 * 2.4
WORKLOADS = {
    65536: dict(key="c2", seed=0x5EED0002, turns=1000, desc="configs[2]: 65536^2 random 25%, 1000 turns a step"),
    16384: dict(key="c1", seed=0x5EED0001, turns=10000, desc="configs[1]: 16384^2 random 25%, 10000 turns a step"),
    262144: dict(key="c3", seed=0x5EED0003, turns=100, desc="configs[3]: 262144^2 random 25%, 100 turns a step"),
    5120: dict(key="c4", seed=0x5EED0005, turns=200,
               desc="configs[4]: 5120^2 random 25%, full CellFlipped stream, 200 turns a step from turn 2064"),
    512: dict(key=None, seed=None, turns=100,
              desc="configs[0]: images/512x512.pgm, 100 turns, Threads=8, end to end through gol.Run (host mirror): "
                   "PGM in, every event drained, PGM out"),
}
FULLSIZE = os.path.join(ROOT, "tests", "golden", "fullsize.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--warmup-seconds", type=float, default=3.0,
                    help="keep warming up (untimed) until this much wall time has passed: a first run on an idle "
                         "GPU is ~4 %% slower for its first second (clock ramp, first touch of the buffers); 3 s "
                         "also keeps the GPU visibly busy for an outside utilisation sampler (BENCH_r01: 0/3 "
                         "samples saw the 0.6 s of GPU work beside the 10 s CPU baseline)")
    ap.add_argument("--workload", type=int, default=65536, choices=sorted(WORKLOADS))
    ap.add_argument("--turns-per-step", type=int, default=None,
                    help="default: the config's turns (parity is only checked then)")
    ap.add_argument("--tb-depth", type=int, default=20)
    ap.add_argument("--rows-per-wave", type=int, default=0, help="0 = automatic")
    ap.add_argument("--option", action="append", default=[], help="engine option key=value (A/B runs)")
    ap.add_argument("--e2e-turns", type=int, default=20,
                    help="--workload 5120: turns of the end_to_end block through gol.Run (0 = skip)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample length")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--launch-timeout", type=float, default=1500.0,
                    help="--gpus N > 1 without a launcher: end the ranks after this long (s)")
    ap.add_argument("--stage-timeout", type=float, default=300.0,
                    help="multi-rank runs: the longest one stage (comm init, parity step, warmup, timed "
                         "steps) may take before the watchdog ends the rank with a JSON error line")
    ap.add_argument("--ring", action="store_true",
                    help="one GPU: run the board as a one-rank RCCL ring (force_halo) through the multi-rank path "
                         "(gloo control plane, golhip_comm_init, halo exchanges, the library's allreduce)")
    ap.add_argument("--no-configs3", dest="configs3", action="store_false",
                    help="default workload: skip the configs[3] block (262144^2 x 100 turns over the same ranks)")
    ap.add_argument("--configs3-warmup-seconds", type=float, default=1.0)
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_bench.json"),
                    help="rocprofv3 --pmc summary of this bench command (scripts/pmc_bench.py)")
    return ap.parse_args()


def host_info() -> dict:
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"cpu_model": model, "nproc": os.cpu_count(), "share": cpu_share()}


def cgroup_cpu_quota() -> float | None:
    """CPUs the cgroup's CFS quota allows (cgroup v2 cpu.max, else v1
    cpu.cfs_quota_us / cpu.cfs_period_us); None when unlimited or unreadable."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        return None if q == "max" else int(q) / int(period)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            period = int(f.read())
        return None if q <= 0 else q / period
    except (OSError, ValueError):
        return None


def cpu_share() -> dict:
    """The CPUs this process may actually use, measured: the scheduler
    affinity mask and the cgroup quota.  `threads` (what the CPU baselines
    run on) is the smaller of the two; Go's GOMAXPROCS defaults to the same
    (the affinity count, capped by the cgroup quota since Go 1.25)."""
    aff = len(os.sched_getaffinity(0))
    quota = cgroup_cpu_quota()
    threads = max(1, min(aff, int(quota + 0.5)) if quota else aff)
    return {"affinity": aff, "cgroup_quota_cpus": round(quota, 2) if quota else None, "threads": threads,
            "gomaxprocs_equiv": threads, "nproc": os.cpu_count()}


def cpu_threads() -> int:
    return cpu_share()["threads"]


def cpu_baseline(W: int, seed: int, target_s: float) -> dict:
    """Oracle port of the reference worker pool (distributor.go:116-173) on a
    bounded sample of the same synthetic board: a band of up to 4096 rows,
    as many turns as fit in ~target_s.  Beside it (`fast_cpu`), the bit-packed
    OpenMP comparator (oracle/gol_fastcpu.c) on up to 16384 rows, ~target_s / 2."""
    from oracle.oracle import COracle

    o = COracle()
    rows = min(4096, W)
    board = o.fill_random(W, rows, seed)
    threads = max(1, cpu_threads() - 1)  # Threads; the pool runs Threads+1 workers
    t0 = time.perf_counter()
    o.run_workerpool(board, 1, threads)
    one = time.perf_counter() - t0
    turns = max(1, int(target_s / max(one, 1e-6)))
    t0 = time.perf_counter()
    o.run_workerpool(board, turns, threads)
    dt = time.perf_counter() - t0
    out = {
        "value": W * rows * turns / dt / 1e9,
        "unit": "GCUPS",
        "cores": threads + 1,
        "kind": "port",
        "sample": f"{rows}x{W} band of the workload board (torus), {turns} turns, oracle/gol_oracle.c "
                  f"worker-pool port (Threads={threads}, Threads+1 workers), {dt:.1f} s",
        "host": host_info(),
    }
    nth = cpu_threads()
    fast_rows = min(W, 16384)
    words = o.fill_random64(W, fast_rows, seed, nth)
    t0 = time.perf_counter()
    o.run_fast_words(words, W, 2, nth)
    one = (time.perf_counter() - t0) / 2
    fturns = max(1, int(target_s / 2 / max(one, 1e-6)))
    t0 = time.perf_counter()
    o.run_fast_words(words, W, fturns, nth)
    fdt = time.perf_counter() - t0
    out["fast_cpu"] = {
        "value": W * fast_rows * fturns / fdt / 1e9,
        "unit": "GCUPS",
        "cores": nth,
        "kind": "bit-packed OpenMP comparator (not the reference algorithm)",
        "sample": f"{fast_rows}x{W} torus, {fturns} turns, oracle/gol_fastcpu.c (64 cells/uint64, "
                  f"{nth} OpenMP threads), {fdt:.1f} s",
    }
    return out


def cpu_config0() -> dict:
    """BASELINE configs[0]: images/512x512.pgm, 100 turns, Threads = 8, on the
    oracle's port of the reference worker pool (distributor.go:116-173:
    Threads + 1 workers, row queue, per-row alive lists, per-turn allocation,
    flip diff), checked against check/images/512x512x100.pgm (the reference's
    golden board, tests/golden/fixtures.npz).

    `value` is the port as gol.Run runs it, the same workload as the GPU
    line's `--workload 512` value: every event (the load-time CellFlipped of
    :72-80, each turn's CellFlipped of :212-220 and TurnComplete, the final
    ImageOutputComplete / FinalTurnComplete / StateChange) through an
    unbuffered events channel of the host mirror's type, drained by main.go's
    loop on another thread, the final PGM written (oracle/gol_port_events.cpp).
    `buffered_1000` is the same through main.go:53's capacity-1000 channel
    (the GPU line's `buffered_1000`); `engine_only` counts the flips without
    delivering them (oracle_run_workerpool)."""
    import tempfile

    from oracle.oracle import COracle, unpack_bits

    o = COracle()
    with np.load(os.path.join(ROOT, "tests", "golden", "fixtures.npz"), allow_pickle=False) as z:
        board = unpack_bits(z["image_512"], 512)
        golden = unpack_bits(z["check_512x100"], 512)
        alive = int(z["alive_512"][100])
    cells = 512 * 512 * 100

    def timed(run):
        run()  # warm
        reps, t0 = 0, time.perf_counter()
        while True:
            res = run()
            reps += 1
            if time.perf_counter() - t0 > 1.0:
                break
        return (time.perf_counter() - t0) / reps, reps, res

    dt, reps, (b, _) = timed(lambda: o.run_workerpool(board, 100, 8))
    engine = {"gcups": round(cells / dt / 1e9, 4), "seconds_per_run": round(dt, 5), "runs": reps,
              "parity": bool(np.array_equal(b, golden)),
              "note": "flips counted, not delivered (oracle_run_workerpool)"}
    out = {}
    with tempfile.TemporaryDirectory() as d:
        pgm = os.path.join(d, "512x512x100.pgm")
        for cap in (0, 1000):
            dt, reps, (b, counts, last, fin) = timed(lambda: o.run_workerpool_events(board, 100, 8, cap, pgm))
            out[cap] = {"gcups": round(cells / dt / 1e9, 4), "seconds_per_run": round(dt, 5), "runs": reps,
                        "events": counts, "parity": bool(np.array_equal(b, golden) and last == 100 and fin == alive)}
    ev = out[0]
    return {"value": ev["gcups"], "unit": "GCUPS", "cores": 9, "kind": "port",
            "seconds_per_run": ev["seconds_per_run"], "runs": ev["runs"], "events": ev["events"],
            "parity": ev["parity"] and out[1000]["parity"] and engine["parity"],
            "buffered_1000": out[1000], "engine_only": engine,
            "sample": "configs[0]: images/512x512.pgm, 100 turns, Threads=8 (9 workers), oracle/gol_oracle.c "
                      "worker-pool port with every event through an unbuffered channel (gol_test.go's) drained on "
                      "another thread, final PGM written (oracle/gol_port_events.cpp); parity vs "
                      "check/images/512x512x100.pgm and check/alive"}


def roofline_block(perf: dict, W: int, rows: int, workload: int, pmc_path: str, region_ms: float) -> dict:
    """Roofline of the dominant step kernel, from two HIP events on the
    engine's stream around the whole timed region (region_ms): the average
    launch = region / launches, kernel boundaries included (per-launch events
    cost ~5 us a launch themselves: 16384^2 ran 66 vs 74 TCUPS with and
    without them in an earlier round-3 A/B), so rocprofv3's per-kernel
    average is that minus the small gap between dependent launches
    (profiles/r3final: 65536^2 671.9 us rocprof vs 670.9 us here).

    The kernels are VALU-issue-bound: a launch fuses 8-16
    turns per board pass, so HBM moves ~1/D of the single-pass bytes.  `frac`
    is therefore the VALU issue fraction: algorithmic issue slots per launch
    (output words x turns / 64 lanes x slots per word-turn: 9 bitop3 LUTs, 8
    on the pair rule's launches, + 2 half-rate shifts per `words_per_lane`
    words, i.e. 9 + 8/wpl or 8 + 8/wpl; tile-halo lanes and pipeline fill are
    overhead, not counted) / launch time / peak.
    The HBM side comes from the rocprofv3 PMC passes of this same bench
    command (scripts/pmc_bench.sh -> profiles/pmc_bench.json): measured bytes
    (2 x FETCH_SIZE + WRITE_SIZE, gfx950 correction) per launch of the same
    kernel / the live launch time / 8 TB/s."""
    if perf["persist_turns"] >= perf["step_turns"]:
        kname, launches, kms, kturns = "gol_persist_kernel", perf["persist_launches"], region_ms, \
            perf["persist_turns"]
        depth = perf["persist_depth"]
    else:
        # named after the family that ran most of the step launches
        kname = ("gol_skew_kernel" if 2 * perf.get("skew_launches", 0) > perf["step_launches"] else
                 "gol_tb_pair_kernel")
        launches, kms, kturns = perf["step_launches"], region_ms, perf["step_turns"]
        depth = None  # the turns a launch fused (the plan may cap tb_depth)
    launches = max(1, launches)
    avg_s = kms / launches * 1e-3
    wpl = max(1, perf["words_per_lane"])
    # 9 LUTs a word-turn, 8 on the pair rule's launches (round 6, DESIGN.md
    # §5.13), + the two half-rate shifts per wpl words; weighted by turns
    pt = min(perf.get("pair_turns", 0), kturns) if kname == "gol_skew_kernel" else 0
    spw = 9.0 + 8.0 / wpl - (pt / kturns if kturns else 0.0)
    words = rows * ((W + 31) // 32)
    tpl = kturns / launches
    if depth is None and abs(tpl - round(tpl)) < 1e-9:
        depth = int(round(tpl))  # every launch fused the same turns
    slots = words * tpl / 64.0 * spw
    achieved = slots / avg_s / 1e9 if avg_s > 0 else None
    alg_bytes = W * rows * tpl * ALG_BYTES_PER_UPDATE
    out = {
        "bound": "valu",
        "achieved": round(achieved, 1) if achieved else None,
        "peak": VALU_PEAK_GSLOTS,
        "unit": "Gslot/s (wave64 VALU issue slots)",
        "frac": round(achieved / VALU_PEAK_GSLOTS, 4) if achieved else None,
        "traffic": None,
        # the instantiation when every launch fused the same turns, else the
        # family (turns_per_launch holds the average)
        "kernel": f"{kname}<{depth}, {wpl}>" if depth is not None else kname,
        "words_per_lane": wpl,
        "launch_time": "HIP events on the engine stream around the timed region / launches (boundaries included)",
        "avg_launch_ms": round(avg_s * 1e3, 5),
        "launches": launches,
        "skew_launches": perf.get("skew_launches", 0),
        "turns_per_launch": tpl,
        "slots_per_word_turn": round(spw, 4),
        "pair_rule_turns": pt,
        "alg_bytes_per_launch": alg_bytes,
        "temporal_blocking": {"alg_bytes_GBps": round(alg_bytes / avg_s / 1e9, 1) if avg_s > 0 else None,
                              "note": "0.25 B/cell-update (SURVEY 8d) over the launch time: the single-pass "
                                      "HBM-equivalent rate, > 8 TB/s because one pass fuses many turns"},
    }
    try:
        with open(pmc_path) as f:
            rec = json.load(f).get(f"{workload}:{kname}")
    except (OSError, ValueError):
        rec = None
    if rec and kname != "gol_persist_kernel" and abs(rec.get("turns_per_launch", 0) - tpl) > 1e-6:
        # counters of another launch plan (an older tree): not this line's kernel
        out["pmc_stale"] = {"source": os.path.relpath(pmc_path, ROOT), "bench_kernel": rec.get("bench_kernel"),
                            "turns_per_launch": rec.get("turns_per_launch")}
        rec = None
    if rec:
        traffic = rec["hbm_bytes_per_launch"] * (tpl / rec["turns_per_launch"] if kname == "gol_persist_kernel" else 1)
        out["traffic"] = traffic
        out["hbm"] = {"achieved_GBps": round(traffic / avg_s / 1e9, 1), "peak_GBps": HBM_PEAK_GBS,
                      "frac": round(traffic / avg_s / 1e9 / HBM_PEAK_GBS, 4), "source": os.path.relpath(pmc_path, ROOT)}
        if rec.get("sq_insts_valu"):
            inst = rec["sq_insts_valu"] * (tpl / rec["turns_per_launch"] if kname == "gol_persist_kernel" else 1)
            out["valu_measured"] = {"sq_insts_valu_per_launch": inst,
                                    "issue_frac_vs_peak": round(inst / avg_s / 1e9 / VALU_PEAK_GSLOTS, 4),
                                    "valu_active_frac": rec.get("valu_active_frac"),
                                    "clock_ghz": rec.get("clock_ghz_est"),
                                    "note": "SQ_INSTS_VALU counts instructions (half-rate ones once)"}
    return out


def events_main(a) -> None:
    """configs[4]: 5120^2 with the full event stream ("GCUPS with
    events on vs off").  Parity first: the CellFlipped lists of turns 1..50
    from the fresh board (int32 (x, y) pairs, row-major per turn) must equal
    tests/golden/fullsize.json c4 (per-turn counts + SHA-256 of the pairs).
    Then the board runs untimed to turn 2064 (past the random board's first
    turns of 3-7 M flips, ~0.4 M a turn on), and each timed step is 200 turns
    through golhip_flip_stream with 4-byte cell indices written by the kernel
    into page-locked host memory (golhip_host_alloc), every turn's list
    complete on the host: `value` = W x H x turns / s with events on.
    `events_off` times the same turns on fused launches (no lists)."""
    import hashlib

    import torch
    torch.cuda.set_device(0)
    wl = WORKLOADS[5120]
    N, tps = 5120, a.turns_per_step or wl["turns"]
    with open(FULLSIZE) as f:
        rec = c4 = json.load(f)["c4"]
    cap = 32 << 20
    # parity: turns 1..T of the fixture, pairs
    T = len(rec["flip_counts"])
    xy = np.empty((cap, 2), dtype=np.int32)
    sha, counts = hashlib.sha256(), []
    with golhip.Board(N, N) as b:
        b.fill_random(wl["seed"])
        done = 0
        while done < T:
            ent, cnt, k = b.flip_stream(T - done, cap=cap, fmt=golhip.FLIPS_XY, out=xy)
            sha.update(ent.tobytes())
            counts += [int(c) for c in cnt]
            done += k
    parity = {"turns": T, "flips": sum(counts), "sha256": sha.hexdigest()[:16],
              "ok": sha.hexdigest() == rec["flips_sha256"] and counts == rec["flip_counts"][:T],
              "fixture": "tests/golden/fullsize.json c4 turns 1..%d" % T}
    idx = golhip.host_array((cap,), np.uint32)
    idx.fill(0)

    def stream(b, turns):
        done, flips = 0, 0
        while done < turns:
            ent, cnt, k = b.flip_stream(turns - done, cap=cap, fmt=golhip.FLIPS_INDEX, out=idx)
            done += k
            flips += len(ent)
        return flips

    res = {}
    for timed in (False, True):  # turns/s without per-launch HIP events; the K5 kernel time with them
        with golhip.Board(N, N, timing=timed) as b:
            for kv in a.option:  # A/B runs (the plan's knobs need GOLHIP_TUNING=1)
                k, v = kv.split("=", 1)
                b.set_option(k, int(v))
            b.fill_random(wl["seed"])
            b.step(2064)
            b.sync()
            stream(b, max(1, a.warmup) * tps)  # warmup steps (untimed)
            b.sync()
            b.perf_reset()
            t0 = time.perf_counter()
            flips = sum(stream(b, tps) for _ in range(a.steps))
            b.sync()
            dt = time.perf_counter() - t0
            if not timed:
                res.update(dt=dt, flips=flips)
                # events off: the same turns on fused launches, from the same turn
                b.fill_random(wl["seed"])
                b.step(2064 + max(1, a.warmup) * tps)
                b.sync()
                t1 = time.perf_counter()
                for _ in range(a.steps):
                    b.step(tps)
                b.sync()
                res["dt_off"] = time.perf_counter() - t1
            else:
                res["perf"] = b.perf()
                res["flips_timed"] = flips
    p = res["perf"]
    turns = tps * a.steps
    kus = p["flip_kernel_ms"] * 1e3 / max(1, p["flip_launches"])
    host_b = res["flips_timed"] / max(1, turns) * 4  # K5's entries per launch (4-byte indices, host memory)
    alg = 2 * N * N / 8 + host_b  # board in + out + entries, per launch
    link = golhip.host_link_probe(0)  # the link's ceiling for those stores, measured here
    # ... and at the size of one turn's list, one launch a list (K5's own shape)
    link_turn = golhip.host_link_probe(0, max(4096, int(host_b) // 16 * 16), 50)
    out = {
        "metric": METRIC, "value": round(N * N * turns / res["dt"] / 1e9, 3), "unit": "GCUPS", "n_gpus": 1,
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(res["dt"] / a.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
        "dtype": "u32 bit-sliced (1 bit/cell) + u32 cell-index lists",
        "data": "synthetic (splitmix64 counter-hash board, 25% alive)",
        "parity": parity["ok"], "parity_check": parity,
        "config": {"workload": wl["desc"], "board": [N, N], "turns_per_step": tps,
                   "events": "every turn's CellFlipped list (4-byte y*W+x) into golhip_host_alloc memory",
                   "parallelism": "single GPU torus"},
        "events_on": {"turns_per_s": round(turns / res["dt"], 1), "flips_per_s": round(res["flips"] / res["dt"], 1),
                      "flips": res["flips"]},
        "events_off": {"gcups": round(N * N * turns / res["dt_off"] / 1e9, 3),
                       "turns_per_s": round(turns / res["dt_off"], 1)},
        "roofline": {"bound": "host-link", "achieved": round(host_b / (kus * 1e-6) / 1e9, 2) if kus > 0 else None,
                     "peak": link["kernel_write_GBps"], "unit": "GB/s",
                     "frac": round(host_b / (kus * 1e-6) / 1e9 / link["kernel_write_GBps"], 4)
                     if kus > 0 and link["kernel_write_GBps"] > 0 else None,
                     "traffic": None,
                     "kernel": "gol_flip_stream_kernel (K5r, one resident launch a batch)"
                     if p.get("flip_resident_launches") else "gol_flip_turn_kernel (K5)",
                     "avg_launch_ms": round(kus / 1e3, 5), "launches": p["flip_launches"],
                     "resident_launches": p.get("flip_resident_launches"),
                     "host_bytes_per_launch": host_b,
                     "peak_source": "golhip_host_link_probe on this box, this run: a kernel's coalesced 16-byte "
                                    "stores into golhip_host_alloc memory (K5's store path)",
                     "link_probe": link,
                     "link_probe_list_size": link_turn,
                     "frac_vs_list_size_probe": round(host_b / (kus * 1e-6) / 1e9 / link_turn["kernel_write_GBps"], 4)
                     if kus > 0 and link_turn["kernel_write_GBps"] > 0 else None,
                     "stream_GBps": round(host_b * turns / res["dt"] / 1e9, 2),
                     "hbm_side": {"alg_bytes_per_launch": alg,
                                  "achieved_GBps": round(alg / (kus * 1e-6) / 1e9, 1) if kus > 0 else None,
                                  "peak_GBps": HBM_PEAK_GBS,
                                  "note": "board in + board out + entries; the 5120^2 board is cache-resident"},
                     "note": "one turn + its list a turn (K5r: a batch of turns in one launch, `launches` and "
                             "`avg_launch_ms` count turns): the entries cross the host link into page-locked "
                             "memory; achieved = entry bytes per turn / the turn's device time (HIP events), "
                             "stream_GBps the same bytes over the timed wall clock (host syncs included)"},
    }
    try:  # HBM bytes of K5 from the PMC passes of this command (scripts/pmc_bench.sh ... 5120)
        with open(a.pmc) as f:
            rec = json.load(f).get(f"{N}:gol_flip_turn_kernel")
    except (OSError, ValueError):
        rec = None
    if p.get("flip_resident_launches"):
        # (the entry is of per-turn K5 launches; a K5r dispatch carries a whole
        # batch of turns, the parity check's and the timed ones alike)
        rec = None
        out["roofline"]["hbm_side"]["pmc_note"] = ("no PMC entry for K5r: profiles/pmc_bench.json holds the per-turn "
                                                   "K5 launches' (flip_overlap 1)")
    if rec and rec.get("hbm_bytes_per_launch") and kus > 0:
        out["roofline"]["hbm_side"].update(
            pmc_bytes_per_launch=rec["hbm_bytes_per_launch"],
            pmc_GBps=round(rec["hbm_bytes_per_launch"] / (kus * 1e-6) / 1e9, 1), source=os.path.relpath(a.pmc, ROOT),
            pmc_note="FETCH_SIZE x2 + WRITE_SIZE; the entries go to page-locked host memory")
    if a.e2e_turns > 0:
        out["end_to_end"] = events_end_to_end(c4, a.e2e_turns)
        parity["ok"] = parity["ok"] and out["end_to_end"]["parity"]
        out["parity"] = parity["ok"]
    if not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(N, wl["seed"], a.cpu_seconds)
        out["cpu_baseline"]["config0"] = cpu_config0()
    print(json.dumps(out), flush=True)
    if parity["ok"] is False:
        sys.exit(1)


def events_end_to_end(rec: dict, T: int) -> dict:
    """configs[4] through the whole gol.Run mirror (SURVEY 8d end to end):
    images/5120x5120.pgm of the fixture board, T turns, every CellFlipped
    event (the initial alive cells, then each turn's flips) delivered through
    an events channel of capacity 1000 (main.go:53) into main.go's headless
    drain loop (golrun_drain, C++), then the final PGM and FinalTurnComplete.
    Parity: per-turn CellFlipped counts and order-dependent digests equal
    tests/golden/fullsize.json c4 (turns 1..T)."""
    import tempfile

    from oracle.oracle import COracle

    N = rec["width"]
    T = min(T, len(rec["flip_counts"]))
    board = COracle().fill_random(N, N, rec["seed"])
    with tempfile.TemporaryDirectory() as root:
        write_images(root, {f"{N}x{N}": board})
        del board
        with StdoutToStderr():
            t0 = time.perf_counter()
            r = golhip.Run(T, 8, N, N, root, events_cap=1000)
            counts, last, final_alive, flips, digests = r.drain(T, N)
            err = r.wait()
            r.close()
            dt = time.perf_counter() - t0
    ok = (not err and last == T and [int(x) for x in flips] == rec["flip_counts"][:T]
          and [f"{int(x):016x}" for x in digests] == rec["flip_digests"][:T]
          and counts["CellFlipped"] == rec["initial_alive"] + sum(rec["flip_counts"][:T]))
    return {"turns": T, "seconds": round(dt, 3), "turns_per_s": round(T / dt, 2),
            "events_per_s": round(sum(counts.values()) / dt, 1), "events": counts, "parity": ok,
            "fixture": f"tests/golden/fullsize.json c4 turns 1..{T}: per-turn counts + ordered digests",
            "timed": "one whole gol.Run: PGM read, handle create + load, T turns with every CellFlipped through a "
                     "capacity-1000 channel drained by main.go's loop (C++), PGM write, close",
            "note": "the first turns of the random board flip 2.6-7.2 M cells each: the channel hand-off of "
                    "every event (one at a time, as the reference's consumer) bounds this rate, not the GPU"}


def error_line(a, msg: str, **extra) -> None:
    """The one JSON line of a run that could not measure: value null, the
    reason in `error`, exit status non-zero (the caller exits)."""
    out = {"metric": METRIC, "value": None, "unit": "GCUPS", "n_gpus": a.gpus, "steps": a.steps,
           "warmup": a.warmup, "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
           "error": msg, "config": {"workload": WORKLOADS[a.workload]["desc"]}}
    out.update(extra)
    print(json.dumps(out), flush=True)


class Watchdog:
    """Bounds every multi-rank stage (RCCL comm init, parity step, warmup,
    timed steps): a stage that does not finish in time prints a JSON error
    line naming the rank and the stage and ends the process with status 3,
    instead of hanging until an outside timeout (a lost peer blocks
    ncclCommInitRank and every exchange forever)."""

    def __init__(self, a, rank: int):
        import threading
        self.a, self.rank = a, rank
        self.stage, self.deadline = None, None
        self._lock = threading.Lock()
        t = threading.Thread(target=self._run, daemon=True)
        t.start()

    def arm(self, stage: str, seconds: float) -> None:
        with self._lock:
            self.stage, self.deadline = stage, time.monotonic() + seconds

    def disarm(self) -> None:
        with self._lock:
            self.stage, self.deadline = None, None

    def _run(self) -> None:
        while True:
            time.sleep(0.5)
            with self._lock:
                late = self.deadline is not None and time.monotonic() > self.deadline
                stage = self.stage
            if late:
                msg = f"rank {self.rank}: stage '{stage}' did not finish in time (watchdog)"
                print(msg, file=sys.stderr, flush=True)
                if self.rank == 0:
                    error_line(self.a, msg, rank=self.rank, stage=stage)
                os._exit(3)


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def count_gpus() -> tuple[int | None, str]:
    """GPUs the ranks would see, counted without touching HIP (a process that
    has initialised the GPU must not start the rank processes): the KFD
    topology's GPU nodes (simd_count > 0; CPU nodes have 0), restricted by
    HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES when set.
    Returns (count, how) or (None, why) when the topology is unreadable."""
    import glob
    nodes = 0
    paths = glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties")
    for path in paths:
        try:
            with open(path) as f:
                for line in f:
                    k, _, v = line.partition(" ")
                    if k == "simd_count" and int(v) > 0:
                        nodes += 1
                        break
        except (OSError, ValueError):
            continue
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            listed = [x for x in v.split(",") if x.strip()]
            if not listed:
                return 0, f"{var} is empty"
            nodes = min(nodes, len(listed)) if paths else len(listed)
    if not paths and nodes == 0:
        return None, "no /sys/class/kfd/kfd/topology/nodes (no amdgpu KFD visible)"
    return nodes, "kfd topology"


def launch_ranks(a, cmd: list | None = None, n_devices: int | None = None) -> int:
    """`--gpus N > 1` without a launcher (no WORLD_SIZE): start the N rank
    processes here, torchrun-style (RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_ADDR=127.0.0.1 / MASTER_PORT in each child's environment), before
    this process touches the GPU (count_gpus reads the KFD topology, no HIP
    call).  Rank 0's stdout is relayed line by line;
    the first rank to fail ends the others and the launcher prints a JSON
    error line if rank 0 printed none.  Returns the exit status.  (`cmd` /
    `n_devices` replace the child command and the device count in the CPU
    tests of the launcher.)"""
    import subprocess
    import threading

    if n_devices is None:
        n_devices, how = count_gpus()
        if n_devices is None:
            error_line(a, f"cannot count the GPUs without initialising HIP: {how}")
            return 2
    n = n_devices
    if n < a.gpus:
        error_line(a, f"{n} devices < {a.gpus} ranks: --gpus {a.gpus} needs {a.gpus} visible GPUs", devices=n)
        return 2
    port = free_port()
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, GOL_BENCH_SELF_LAUNCH="1", RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus),
                   LOCAL_WORLD_SIZE=str(a.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(cmd or [sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL, text=True,
                                      start_new_session=True))
    printed = []

    def relay():
        for line in procs[0].stdout:
            print(line, end="", flush=True)
            if line.lstrip().startswith("{") and '"metric"' in line:
                printed.append(line)

    th = threading.Thread(target=relay, daemon=True)
    th.start()
    deadline = time.monotonic() + a.launch_timeout
    failed = None
    while True:
        codes = [p.poll() for p in procs]
        bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
        if bad:
            failed = f"rank {bad[0][0]} exited with status {bad[0][1]}"
            break
        if all(c == 0 for c in codes):
            break
        if time.monotonic() > deadline:
            failed = f"ranks still running after --launch-timeout {a.launch_timeout:.0f} s"
            break
        time.sleep(0.2)
    if failed:
        import signal
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except OSError:
                    pass
        t_kill = time.monotonic() + 10
        for p in procs:
            try:
                p.wait(timeout=max(0.1, t_kill - time.monotonic()))
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except OSError:
                    pass
                p.wait()
    th.join(timeout=5)
    if failed:
        if not printed:
            error_line(a, failed, rank_status=[p.returncode for p in procs])
        return max(1, max(abs(p.returncode or 0) for p in procs))
    return 0


class StdoutToStderr:
    """The host mirror prints the io goroutine's "File ... done!" lines
    (io.go:86, :125) on the C stdout; during the timed runs they go to stderr
    so the bench's stdout holds only its JSON line."""

    def __enter__(self):
        import ctypes
        self.libc = ctypes.CDLL(None)
        sys.stdout.flush()
        self.libc.fflush(None)
        self.saved = os.dup(1)
        os.dup2(2, 1)
        return self

    def __exit__(self, *exc):
        self.libc.fflush(None)
        os.dup2(self.saved, 1)
        os.close(self.saved)


def write_images(root: str, names: dict) -> None:
    """images/<name>.pgm under `root` (the reference's io.go reads them from images/)."""
    from oracle.oracle import pgm_bytes
    os.makedirs(os.path.join(root, "images"), exist_ok=True)
    for name, board in names.items():
        with open(os.path.join(root, "images", f"{name}.pgm"), "wb") as f:
            f.write(pgm_bytes(board))


def run_main(a) -> None:
    """configs[0] end to end ("... and end-to-end through gol.Run";
    gol_test.go:15-47's shape): one step = one whole gol.Run(Params{Turns: 100,
    Threads: 8, 512, 512}) through the C++ mirror (libgolhost.so over
    libgolhip.so) -- images/512x512.pgm read, a GPU handle created and loaded,
    100 turns with every CellFlipped and TurnComplete event delivered through
    the events channel and drained (main.go's headless loop, golrun_drain),
    out/512x512x100.pgm written, FinalTurnComplete, close.  Parity: the PGM's
    SHA-256 equals check/images/512x512x100.pgm (tests/golden/manifest.json)
    and the alive count equals check/alive.  `value` = cells x turns / wall
    seconds of a whole Run; the CPU port of the reference's worker pool on the
    same config sits beside it (cpu_baseline.config0)."""
    import hashlib
    import tempfile

    from oracle.oracle import unpack_bits

    with np.load(os.path.join(ROOT, "tests", "golden", "fixtures.npz"), allow_pickle=False) as z:
        board = unpack_bits(z["image_512"], 512)
        alive = z["alive_512"]
    with open(os.path.join(ROOT, "tests", "golden", "manifest.json")) as f:
        want_sha = json.load(f)["check_512x100"]["sha256"]
    N, T = 512, a.turns_per_step or 100
    with tempfile.TemporaryDirectory() as root:
        write_images(root, {"512x512": board})

        def one(cap):
            r = golhip.Run(T, 8, N, N, root, events_cap=cap)
            counts, last, final_alive, _, _ = r.drain(0, 0)
            err = r.wait()
            r.close()
            if err:
                raise RuntimeError(err)
            return counts, last, final_alive

        with StdoutToStderr():
            for _ in range(max(1, a.warmup)):
                one(0)
            times, res = [], None
            for _ in range(a.steps):
                t0 = time.perf_counter()
                res = one(0)
                times.append(time.perf_counter() - t0)
            btimes = []  # main.go's capacity-1000 events channel (main.go:53)
            for _ in range(a.steps):
                t0 = time.perf_counter()
                bres = one(1000)
                btimes.append(time.perf_counter() - t0)
        counts, last, final_alive = res
        if bres != res:
            raise RuntimeError(f"buffered run differs: {bres} vs {res}")
        with open(os.path.join(root, "out", f"{N}x{N}x{T}.pgm"), "rb") as f:
            sha = hashlib.sha256(f.read()).hexdigest()
    dt = sum(times)
    if T == 100:  # the reference's own golden board
        fixture = "check/images/512x512x100.pgm (manifest sha256), check/alive/512x512.csv"
    else:  # no golden board for T: the C oracle's board after T turns (and check/alive when it has row T)
        from oracle.oracle import COracle, pgm_bytes
        want_sha = hashlib.sha256(pgm_bytes(COracle().run(board, T))).hexdigest()
        fixture = f"oracle/gol_oracle.c board after {T} turns" + (", check/alive/512x512.csv" if T < len(alive) else "")
    ok = sha == want_sha and last == T and (T >= len(alive) or final_alive == int(alive[T]))
    out = {
        "metric": METRIC, "value": round(N * N * T * a.steps / dt / 1e9, 4), "unit": "GCUPS", "n_gpus": 1,
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(dt / a.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
        "dtype": "u32 bit-sliced (1 bit/cell) on the GPU; 0/255 bytes at the PGM boundary",
        "data": "images/512x512.pgm (the reference's own input, tests/golden/fixtures.npz)",
        "parity": ok,
        "parity_check": {"pgm_sha256": sha[:16], "final_alive": final_alive, "last_turn": last,
                         "fixture": fixture},
        "config": {"workload": WORKLOADS[512]["desc"], "board": [N, N], "turns_per_step": T, "threads": 8,
                   "events": {k: v for k, v in counts.items()}, "parallelism": "single GPU torus",
                   "timed": "whole gol.Run calls, wall clock: PGM read, handle create + load, turns, every event, "
                            "PGM write, close"},
        "runs_per_s": round(a.steps / dt, 2),
        "ms_per_run_min": round(min(times) * 1e3, 3),
        "events_channel": "unbuffered (gol_test.go:15-47's make(chan gol.Event)): every send waits for the receive",
        "buffered_1000": {"gcups": round(N * N * T * a.steps / sum(btimes) / 1e9, 4),
                          "ms_per_run": round(sum(btimes) / a.steps * 1e3, 3),
                          "note": "main.go:53's make(chan gol.Event, 1000), same events, same parity"},
    }
    if not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_config0()
    print(json.dumps(out), flush=True)
    if not ok:
        sys.exit(1)


class RankEnv:
    """One rank's view of the job: its rank, device and host control plane,
    and the few collectives bench.py needs around the timed region.

    The control plane is a **gloo** process group on CPU tensors (rank 0's
    RCCL unique id, the parity digest sum, the max-over-ranks time, the
    warmup count, the per-rank rows, barriers): none of it is on the data
    path, and with gloo the library's own RCCL communicator (golhip_comm_init:
    the halo ring and golhip_alive_count_global's allreduce) is the only GPU
    communication of the job -- no second communicator per device.  The
    one-GPU ring tests (tests/test_gpu_bench_ring.py) subclass this class and
    override ring_init alone, so every other line here is what the driver's
    multi-GPU run executes."""

    def __init__(self, a, world: int, rank: int, local: int):
        self.a, self.world, self.rank, self.local = a, world, rank, local
        self.ringed = world > 1 or bool(getattr(a, "ring", False))
        self.wd = Watchdog(a, rank) if self.ringed else None
        import torch
        self.torch = torch
        torch.cuda.set_device(local)
        self.dist = None
        if self.ringed:
            # RCCL's own warnings on stderr: a failed comm init or exchange is
            # diagnosable from the run's log (the driver keeps stderr)
            os.environ.setdefault("NCCL_DEBUG", "WARN")
            self.init_control()

    def init_control(self) -> None:
        """The gloo process group (host control plane).  A launcher's
        MASTER_ADDR / MASTER_PORT when present, else (one rank, --ring) a
        local port on 127.0.0.1."""
        import torch.distributed as dist
        self.stage("control plane init (gloo process group)")
        if "MASTER_ADDR" in os.environ and "MASTER_PORT" in os.environ:
            dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
        else:
            dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{free_port()}", rank=self.rank,
                                    world_size=self.world)
        self.dist = dist

    def stage(self, name: str) -> None:  # bound the next multi-rank stage
        if self.wd is not None:
            self.wd.arm(name, self.a.stage_timeout)
            print(f"[rank {self.rank}/{self.world}] {name}", file=sys.stderr, flush=True)

    def board(self, W: int, H: int, row0: int, rows: int):
        if self.world > 1:
            return golhip.Board(W, H, device=self.local, row0=row0, rows=rows)
        return golhip.Board(W, H, device=self.local)

    def unique_id(self) -> bytes:  # rank 0's RCCL id, on every rank
        uid = [golhip.unique_id() if self.rank == 0 else None]
        self.dist.broadcast_object_list(uid, src=0)
        return uid[0]

    def ring_init(self, board, tag: str = "") -> None:
        """This rank's strip joins the halo ring: the library's own RCCL
        communicator (rank 0's unique id broadcast over the control plane).
        One rank (--ring): the whole board as a one-rank RCCL ring
        (force_halo), the exchanges and the allreduce of the N-rank run."""
        self.stage(tag + "golhip_comm_init (ncclCommInitRank + strip-row allreduce)")
        if self.world == 1:
            board.set_option("force_halo", 1)
        board.comm_init(self.unique_id(), self.world, self.rank)

    def barrier(self, board) -> None:
        if self.dist is not None:
            self.dist.barrier()
        board.sync()
        self.torch.cuda.synchronize()

    def _cpu(self, x, dtype):
        return self.torch.tensor([x], dtype=dtype)  # gloo: CPU tensors

    def gsum(self, x: int) -> int:  # mod 2^64 over ranks
        if self.dist is None:
            return x % (1 << 64)
        t = self._cpu(x - (1 << 64) if x >= (1 << 63) else x, self.torch.int64)
        self.dist.all_reduce(t)
        return int(t.item()) % (1 << 64)

    def gmax(self, x: float) -> float:
        if self.dist is None:
            return x
        t = self._cpu(x, self.torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def bcast(self, x: int) -> int:  # rank 0's value
        if self.dist is None:
            return x
        t = self._cpu(x, self.torch.int64)
        self.dist.broadcast(t, src=0)
        return int(t.item())

    def gather(self, obj):
        if self.dist is None:
            return None
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def region_timer(self, board):
        """HIP events on the engine's own stream (torch.cuda.Event sees only
        torch's current stream otherwise): start(), stop() -> ms."""
        torch = self.torch
        st = torch.cuda.ExternalStream(board.stream())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

        class T:
            def start(self):
                e0.record(st)

            def stop(self):
                e1.record(st)
                board.sync()
                torch.cuda.synchronize()
                return e0.elapsed_time(e1)
        return T()

    def close(self) -> None:
        if self.wd is not None:
            self.wd.arm("shutdown", 120.0)
        if self.dist is not None:
            self.dist.destroy_process_group()


def measure(a, env, workload: int, steps: int, warmup: int, warmup_seconds: float, tps: int | None = None) -> dict:
    """One strong-scaled board of `workload` over the job's ranks: rank r
    owns rows [r H / N, (r + 1) H / N) and steps them with its RCCL halo ring.
    Parity: the first untimed step starts from the freshly filled board, so
    its digest and alive count (summed over ranks) must equal the config's
    tests/golden/fullsize.json checkpoint at `tps` turns.  Then untimed
    warmup steps, then exactly `steps` timed steps between a barrier +
    synchronize on both sides, the time the max over ranks."""
    wl = WORKLOADS[workload]
    world, rank = env.world, env.rank
    N = workload
    if N % world:
        raise SystemExit(f"{N} rows do not split over {world} ranks")
    W = H = N
    rows = H // world
    row0 = rank * rows
    tps = tps or wl["turns"]
    tag = f"{wl['key']}: "
    board = env.board(W, H, row0, rows)
    try:
        board.set_tb_depth(a.tb_depth)
        board.set_rows_per_wave(a.rows_per_wave)
        if a.option:  # A/B runs: the plan's tuning knobs need the library's consent
            os.environ.setdefault("GOLHIP_TUNING", "1")
        for kv in a.option:
            k, v = kv.split("=")
            board.set_option(k, int(v))
        comm = None
        ringed = getattr(env, "ringed", world > 1)
        if ringed:
            env.ring_init(board, tag)
            comm = board.comm_info()
            if comm["nranks"] != world or comm["rank"] != rank:
                raise SystemExit(f"RCCL ring reports rank {comm['rank']} of {comm['nranks']}, "
                                 f"expected {rank} of {world}")
        board.fill_random(wl["seed"])
        # warmup step 1 from the fresh board = the parity run
        env.stage(tag + "parity step (first warmup step, halo exchanges)")
        t_w = time.perf_counter()
        board.step(tps)
        board.sync()
        digest = env.gsum(board.board_hash())
        # the ring's own allreduce (golhip_alive_count_global: ncclAllReduce on
        # the library's communicator), checked against the fixture every run
        alive = board.alive_count(global_sum=ringed)[0]
        parity = {"turns": tps, "digest": f"{digest:016x}", "alive": alive}
        try:
            with open(FULLSIZE) as f:
                cp = json.load(f)[wl["key"]]["checkpoints"].get(str(tps))
        except (OSError, ValueError, KeyError):
            cp = None
        parity["ok"] = None if cp is None else (cp["hash"] == parity["digest"] and cp["alive"] == alive)
        parity["fixture"] = "tests/golden/fullsize.json " + (f"{wl['key']} turn {tps}" if cp else "(no checkpoint)")
        for _ in range(max(0, warmup - 1)):
            board.step(tps)
        board.sync()
        # every rank runs the same number of extra warmup steps (decided by rank 0's clock)
        extra = 0
        done_w = max(1, warmup)
        if warmup_seconds > 0:
            per = max(1e-6, (time.perf_counter() - t_w) / done_w)
            extra = env.bcast(min(1000, int(max(0.0, warmup_seconds - (time.perf_counter() - t_w)) / per)))
        env.stage(tag + "warmup steps")
        for _ in range(extra):
            board.step(tps)
        env.barrier(board)
        env.stage(tag + "timed steps")
        board.perf_reset()
        timer = env.region_timer(board)
        t0 = time.perf_counter()
        timer.start()
        for _ in range(steps):
            board.step(tps)
        region_ms = timer.stop()
        dt_rank = time.perf_counter() - t0
        dt = env.gmax(dt_rank)
        if env.dist is not None:
            env.dist.barrier()
        perf = board.perf()
        alive_end, at_turn = board.alive_count(global_sum=ringed)
        me = {"rank": rank, "row0": row0, "rows": rows, "comm": comm, "seconds": round(dt_rank, 6),
              "region_ms": round(region_ms, 3), "launches": perf["step_launches"] + perf["persist_launches"],
              "words_per_lane": perf["words_per_lane"], "halo_exchanges": perf.get("halo_exchanges", 0),
              "halo_bytes": perf["halo_bytes"]}
        ranks = env.gather(me) if world > 1 else None
        return {
            "value": round(W * H * tps * steps / dt / 1e9, 3), "unit": "GCUPS", "n_gpus": world, "steps": steps,
            "warmup": warmup, "warmup_extra_steps": extra, "ms_per_step": round(dt / steps * 1e3, 4),
            "parity": parity["ok"], "parity_check": parity,
            "config": {"workload": wl["desc"], "board": [H, W], "rows_per_rank": rows, "turns_per_step": tps,
                       "tb_depth": a.tb_depth,  # the cap asked for; the plan's launches: roofline.turns_per_launch
                       "rows_per_wave": perf["rows_per_wave"],
                       "words_per_lane": perf["words_per_lane"],
                       "parallelism": f"row strips x{world} (RCCL halo ring)" if world > 1 else
                       "one-rank RCCL ring (force_halo)" if ringed else "single GPU torus",
                       "control_plane": "gloo process group (CPU tensors)" if ringed else None,
                       # halo traffic of this rank over the timed steps (deep halos: one
                       # exchange of k x depth rows feeds k launches)
                       "halo_exchanges": perf.get("halo_exchanges", 0),
                       "halo_bytes_per_step": perf["halo_bytes"] // max(1, steps),
                       "comm": comm, "ranks": ranks},
            "roofline": roofline_block(perf, W, rows, N, a.pmc, region_ms),
            "final_alive": alive_end, "final_turn": at_turn,
        }
    finally:
        board.close()


def main(env_factory=RankEnv):
    a = parse()
    if a.workload == 512:
        if int(os.environ.get("WORLD_SIZE", "1")) != 1 or a.gpus != 1:
            raise SystemExit("--workload 512 (configs[0] through gol.Run) runs on one GPU")
        return run_main(a)
    if a.workload == 5120:
        if int(os.environ.get("WORLD_SIZE", "1")) != 1 or a.gpus != 1:
            raise SystemExit("--workload 5120 (the event stream) runs on one GPU")
        return events_main(a)
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        error_line(a, f"--gpus {a.gpus} but WORLD_SIZE={world}")
        sys.exit(2)
    env = env_factory(a, world, rank, local)
    m = measure(a, env, a.workload, a.steps, a.warmup, a.warmup_seconds, a.turns_per_step)
    out = {"metric": METRIC, **{k: m[k] for k in ("value", "unit", "n_gpus", "steps", "warmup",
                                                    "warmup_extra_steps", "ms_per_step")},
           "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
           "dtype": "u32 bit-sliced (1 bit/cell)", "data": "synthetic (splitmix64 counter-hash board, 25% alive)",
           "parity": m["parity"], "parity_check": m["parity_check"], "config": m["config"]}
    out["config"]["launcher"] = ("self (bench.py --gpus N)" if os.environ.get("GOL_BENCH_SELF_LAUNCH") else
                                 "torch.distributed.run" if world > 1 else None)
    out["roofline"] = m["roofline"]
    out["final_alive"], out["final_turn"] = m["final_alive"], m["final_turn"]
    if a.workload == 65536 and a.configs3:
        # north_star's strong-scaling target is configs[3] (262144^2, >= 80 % at 8
        # GPUs): every default line also measures it over the same ranks, so the
        # driver's one-shot N = 1/2/4/8 runs record both curves.  `value` stays
        # configs[2]'s (BENCH and SCALE lines stay comparable across rounds).
        c3 = measure(a, env, 262144, a.steps, 1, a.configs3_warmup_seconds)
        c3["metric"] = METRIC
        c3["scaling"] = "strong"
        out["configs3"] = c3
        ps = (out["parity"], c3["parity"])  # the line's parity covers both boards
        out["parity"] = False if False in ps else None if None in ps else True
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(a.workload, WORKLOADS[a.workload]["seed"], a.cpu_seconds)
        out["cpu_baseline"]["config0"] = cpu_config0()
    if rank == 0:
        print(json.dumps(out), flush=True)
    env.close()
    if out["parity"] is False:
        sys.exit(1)


if __name__ == "__main__":
    main()
