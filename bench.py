"""bench.py — cell-updates/s of the MI355X Game of Life engine (libgolhip.so).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload 16384|65536|262144]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

A "step" is one pass of the hot path over the whole board: `--turns-per-step`
B3/S23 turns (default 1000) of the synthetic torus, run as fused launches of
`--tb-depth` turns.  Timed region: exactly K steps, bracketed by a barrier and
torch.cuda.synchronize() on both sides, max over ranks.

Workloads (BASELINE.json configs; synthetic boards, data="synthetic"):
  16384  (default, configs[1]) 16384 x 16384 per GPU, seed 0x5EED0001, 10 steps = 10k turns
  65536  (configs[2])          65536 x 65536 per GPU, seed 0x5EED0002
  262144 (configs[3])          262144 x 262144 total, strong-scaled over N GPUs, seed 0x5EED0003
For N > 1 the 16384/65536 workloads are weak-scaled: the torus is N boards
tall, rank r owns rows [r*S, (r+1)*S) and exchanges halo rows with its ring
neighbours over RCCL every fused launch (the only collective on the path).

Warmup: W untimed steps, then more untimed steps until --warmup-seconds
(default 0.5 s) have passed, so the timed steps do not see the clock ramp of
an idle GPU.  Rank 0 prints ONE JSON line; `roofline` is measured on the step kernel with
HIP events on the engine's stream; `cpu_baseline` times the oracle's port of
the reference worker pool on a bounded sample (rank 0, N = 1 only), with the
bit-packed OpenMP CPU comparator beside it (`cpu_baseline.fast_cpu`).
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
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: 8.0 TB/s spec
ALG_BYTES_PER_UPDATE = 0.25  # 1 bit read + 1 bit written per cell-update
WORKLOADS = {
    16384: dict(seed=0x5EED0001, scaling="weak", desc="configs[1]: 16384^2 random 25% per GPU"),
    65536: dict(seed=0x5EED0002, scaling="weak", desc="configs[2]: 65536^2 random 25% per GPU"),
    262144: dict(seed=0x5EED0003, scaling="strong", desc="configs[3]: 262144^2 random 25%, strong-scaled"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--warmup-seconds", type=float, default=0.5,
                    help="keep warming up (untimed) until this much wall time has passed: a first run on an idle "
                         "GPU is ~4 %% slower for its first second (clock ramp, first touch of the buffers)")
    ap.add_argument("--workload", type=int, default=16384, choices=sorted(WORKLOADS))
    ap.add_argument("--turns-per-step", type=int, default=None)
    ap.add_argument("--tb-depth", type=int, default=16)
    ap.add_argument("--rows-per-wave", type=int, default=0, help="0 = automatic")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample length")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                    help="measured HBM traffic per launch (from rocprofv3 --pmc), keyed by workload")
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
    return {"cpu_model": model, "nproc": os.cpu_count()}


def cpu_threads() -> int:
    # the box's CPU share is 16 threads (nproc shows the whole machine)
    return max(1, min(16, os.cpu_count() or 1))


def cpu_baseline(W: int, target_s: float) -> dict:
    """Oracle port of the reference worker pool (distributor.go:116-173) on a
    bounded sample of the same synthetic board: a 4096-row band of the board,
    as many turns as fit in ~target_s.  Beside it (`fast_cpu`), the bit-packed
    OpenMP comparator (oracle/gol_fastcpu.c) on the whole board, ~target_s / 2."""
    from oracle.oracle import COracle

    o = COracle()
    seed = WORKLOADS.get(W, WORKLOADS[16384])["seed"]
    rows = min(4096, W)
    board = o.fill_random(W, rows, seed)
    threads = cpu_threads() - 1  # Threads; the pool runs Threads+1 workers
    threads = max(1, threads)
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
    # fast comparator: whole board if it fits in a few GB of host memory, else a band
    fast_rows = W if W <= 65536 else 16384
    words = o.pack64(o.fill_random(W, fast_rows, seed)) if W <= 16384 else \
        np.ascontiguousarray(np.random.default_rng(seed).integers(0, 2**64, (fast_rows, W // 64), dtype=np.uint64))
    nth = cpu_threads()
    t0 = time.perf_counter()
    o.run_fast_words(words, W, 4, nth)
    one = (time.perf_counter() - t0) / 4
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


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    wl = WORKLOADS[a.workload]
    N = a.workload
    if wl["scaling"] == "weak":
        W, H, rows = N, N * world, N
    else:
        W = H = N
        rows = H // world
    row0 = rank * rows
    turns_per_step = a.turns_per_step or (1000 if N <= 16384 else 100)

    import torch
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    board = golhip.Board(W, H, device=local, row0=row0, rows=rows, timing=True) if world > 1 \
        else golhip.Board(W, H, device=local, timing=True)
    board.set_tb_depth(a.tb_depth)
    board.set_rows_per_wave(a.rows_per_wave)
    if world > 1:
        uid = [golhip.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        board.comm_init(uid[0], world, rank)
    board.fill_random(wl["seed"])

    def barrier():
        if dist is not None:
            dist.barrier()
        board.sync()
        torch.cuda.synchronize()

    t_w = time.perf_counter()
    for _ in range(a.warmup):
        board.step(turns_per_step)
    board.sync()
    # every rank runs the same number of extra warmup steps (decided by rank 0's clock)
    extra = 0
    if a.warmup > 0 and a.warmup_seconds > 0:
        per = max(1e-6, (time.perf_counter() - t_w) / a.warmup)
        extra = min(1000, int(max(0.0, a.warmup_seconds - (time.perf_counter() - t_w)) / per))
        if dist is not None:
            x = torch.tensor([extra], dtype=torch.int64, device="cuda")
            dist.broadcast(x, src=0)
            extra = int(x.item())
    for _ in range(extra):
        board.step(turns_per_step)
    barrier()
    board.perf_reset()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        board.step(turns_per_step)
    board.sync()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        dist.barrier()
    perf = board.perf()
    alive, at_turn = board.alive_count(global_sum=world > 1)

    total_updates = W * H * turns_per_step * a.steps if wl["scaling"] == "weak" or world == 1 \
        else W * H * turns_per_step * a.steps
    gcups = total_updates / dt / 1e9
    # dominant kernel (by device time): the persistent or the per-launch step
    # kernel, each timed with HIP events on the engine stream around every launch
    if perf["persist_kernel_ms"] >= perf["step_kernel_ms"]:
        kname, launches, kms, kturns = "gol_persist_kernel", perf["persist_launches"], perf["persist_kernel_ms"], \
            perf["persist_turns"]
    else:
        # per-launch K1: the paired-band kernel (engine default, paired_bands = fill_skip = 1)
        kname, launches, kms, kturns = "gol_tb_pair_kernel", perf["step_launches"], perf["step_kernel_ms"], \
            perf["step_turns"]
    launches = max(1, launches)
    avg_ms = kms / launches
    alg_bytes_per_launch = W * rows * (kturns / launches) * ALG_BYTES_PER_UPDATE
    achieved = alg_bytes_per_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else None
    traffic = None
    try:
        with open(a.pmc) as f:
            rec = json.load(f).get(f"{N}:{kname}")
        if rec:
            # measured per profiled launch.  A per-launch kernel makes one pass over
            # the board whatever its depth (read + write once), so its bytes carry
            # over as they are; a resident launch makes one pass per super-step, so
            # its bytes scale with this run's turns per launch.
            traffic = rec["hbm_bytes_per_launch"]
            if kname == "gol_persist_kernel":
                traffic *= (kturns / launches) / rec.get("turns_per_launch", kturns / launches)
    except (OSError, ValueError):
        pass

    out = {
        "metric": METRIC,
        "value": round(gcups, 3),
        "unit": "GCUPS",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "warmup_extra_steps": extra,
        "ms_per_step": round(dt / a.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": wl["scaling"],
        "vs_baseline": None,
        "dtype": "u32 bit-sliced (1 bit/cell)",
        "data": "synthetic (splitmix64 counter-hash board, 25% alive)",
        "config": {
            "workload": wl["desc"],
            "board": [H, W],
            "rows_per_rank": rows,
            "turns_per_step": turns_per_step,
            "tb_depth": a.tb_depth,
            "rows_per_wave": perf["rows_per_wave"],
            "parallelism": f"row-strips x{world} (RCCL halo ring)" if world > 1 else "single GPU torus",
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1) if achieved else None,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
            "traffic": traffic,
            "kernel": f"{kname}<{perf['tb_depth']}, {perf['words_per_lane']}>",
            "avg_launch_ms": round(avg_ms, 5),
            "launches": launches,
            "turns_per_launch": kturns / launches,
            "alg_bytes_per_launch": alg_bytes_per_launch,
            "note": "achieved = 0.25 B/cell-update (SURVEY 8d) x cell-updates per launch / avg launch time; "
                    "a launch fuses many turns, so frac > 1 means temporal blocking beat the single-pass "
                    "HBM roofline (the kernel is VALU-bound, see DESIGN.md 5); traffic = measured HBM bytes "
                    "per launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, profiles/pmc_traffic.json; one board pass "
                    "for a per-launch kernel, scaled by super-steps for the resident kernel)",
        },
        "final_alive": alive,
        "final_turn": at_turn,
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(W, a.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    board.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
