"""Cost of the multi-GPU step path on one GPU: the board stepped as a one-rank
RCCL ring (option force_halo: per-launch kernels, RCCL send/recv of the halo
rows to itself once per deep-halo exchange), next to the persistent torus
kernel the single-GPU bench uses and the per-launch torus kernel.
usage: python scripts/bench_halo.py [--size 16384] [--turns 1024] [--depths 16,32]"""
import argparse
import json
import os

os.environ.setdefault("GOLHIP_TUNING", "1")  # A/B knobs of the kernel plans (golhip.h)
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "game-of-life-distributed_amd"))
import golhip  # noqa: E402

VARIANTS = (("persistent_torus", {}), ("per_launch_torus", {"persistent": 0}), ("rccl_ring", {"force_halo": 1}),
            ("rccl_ring_launch", {"force_halo": 1, "persistent": 0}),
            ("rccl_ring_wpl1", {"force_halo": 1, "wpl": 1}), ("rccl_ring_wpl2", {"force_halo": 1, "wpl": 2}))


def run(N: int, depth: int, turns: int, opts: dict) -> dict:
    with golhip.Board(N, N, timing=True) as b:
        if opts.get("force_halo"):
            b.comm_init(golhip.unique_id(), 1, 0)
        for k, v in opts.items():
            b.set_option(k, v)
        b.set_tb_depth(depth)
        b.fill_random(0x5EED0001)
        b.step(2 * depth)
        b.sync()
        b.perf_reset()
        t0 = time.perf_counter()
        b.step(turns)
        b.sync()
        dt = time.perf_counter() - t0
        p = b.perf()
        kms = p["step_kernel_ms"] + p["persist_kernel_ms"]
        return {"wall_gcups": N * N * turns / dt / 1e9, "kernel_gcups": N * N * turns / max(kms * 1e-3, 1e-12) / 1e9,
                "launches": p["step_launches"] + p["persist_launches"], "halo_bytes": p["halo_bytes"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=16384)
    ap.add_argument("--turns", type=int, default=1024)
    ap.add_argument("--depths", default="16,32")
    a = ap.parse_args()
    for depth in map(int, a.depths.split(",")):
        for name, opts in VARIANTS:
            rec = {"variant": name, "N": a.size, "depth": depth, "turns": a.turns}
            rec.update(run(a.size, depth, a.turns, opts))
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
