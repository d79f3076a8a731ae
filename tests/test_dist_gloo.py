"""Row-strip decomposition over torch.distributed (gloo, CPU): the N > 1 path.

Each rank owns a strip of the 64x64 fixture torus and follows libgolhip's
RCCL path (golhip.hip golhip_step / exchange_rccl): the library's own
golhip_halo_schedule (the same helper golhip_step calls, for both the
per-launch and the resident kernel's schedule) says how deep the next exchange is (k launches of
`depth` turns per exchange of k * depth rows), golhip_halo_plan which rows to
send / receive, and the four p2p operations are posted in the same order
(send up, recv bottom, send down, recv top), which is what makes 2 ranks
(prev == next) pair correctly.  Launch i of an exchange steps the strip
extended by (k - 1 - i) * depth rows on each side, rebuilding the next
launch's halos from the deeper exchanged ones.  The
turn computation uses the numpy oracle (test infrastructure), so the test
checks the decomposition protocol, not the kernel; the GPU kernel's halo mode
is covered by tests/test_gpu_parity.py::test_group_strips_*.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

golhip = pytest.importorskip("golhip")

HALO = golhip.HALO_ROWS  # golk::kHalo


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, splits, turns, tb, resident, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "game-of-life-distributed_amd")]
    import golhip as g
    from oracle.oracle import step_np, unpack_bits

    with np.load(os.path.join(root, "tests", "golden", "fixtures.npz"), allow_pickle=False) as z:
        board = unpack_bits(z["image_64"], 64)
    row0 = sum(splits[:rank])
    rows = splits[rank]
    # physical strip buffer with HALO rows above and below, like the device buffer
    buf = np.zeros((rows + 2 * HALO, 64), dtype=np.uint8)
    buf[HALO:HALO + rows] = board[row0:row0 + rows]
    left = turns
    while left > 0:
        # every rank derives the same schedule from the smallest strip
        d, k = g.halo_schedule(min(splits), tb, left, resident)
        x = k * d
        p = g.halo_plan(64, rows, world, rank, x)
        up = torch.from_numpy(buf[p["send_up_row"]:p["send_up_row"] + x].copy())
        down = torch.from_numpy(buf[p["send_down_row"]:p["send_down_row"] + x].copy())
        bot = torch.empty_like(up)
        top = torch.empty_like(up)
        ops = [dist.P2POp(dist.isend, up, p["prev_rank"]), dist.P2POp(dist.irecv, bot, p["next_rank"]),
               dist.P2POp(dist.isend, down, p["next_rank"]), dist.P2POp(dist.irecv, top, p["prev_rank"])]
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        buf[p["recv_bottom_row"]:p["recv_bottom_row"] + x] = bot.numpy()
        buf[p["recv_top_row"]:p["recv_top_row"] + x] = top.numpy()
        for i in range(k):
            e = (k - 1 - i) * d
            # d turns on the strip extended by e rows, from input extended by
            # e + d rows: rows within d of the input's edge become garbage,
            # the kernel's cone argument
            ext = buf[HALO - e - d:HALO + rows + e + d].copy()
            for _ in range(d):
                ext = step_np(ext)
            buf[HALO - e:HALO + rows + e] = ext[d:d + rows + 2 * e]
            left -= d
    gathered = [None] * world
    dist.all_gather_object(gathered, (row0, buf[HALO:HALO + rows]))
    if rank == 0:
        q.put(np.concatenate([s for _, s in sorted(gathered, key=lambda t: t[0])]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("splits,tb", [([32, 32], 16), ([10, 54], 8), ([20, 20, 24], 32), ([16, 16, 16, 16], 4),
                                       ([1, 63], 32)])
@pytest.mark.parametrize("resident", [False, True])
def test_gloo_strips_match_golden(fixtures, splits, tb, resident):
    from oracle.oracle import unpack_bits
    world = len(splits)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, splits, 100, tb, resident, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert np.array_equal(got, unpack_bits(fixtures["check_64x100"], 64))


def _rankenv_worker(rank, world, port, q):
    """bench.RankEnv's control plane as the driver's ranks run it (gloo, CPU
    tensors), without the device half of __init__ (no GPU here)."""
    import argparse
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "game-of-life-distributed_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import bench
    import golhip as g
    g.unique_id = lambda: b"rccl-id-of-rank-0"  # ncclGetUniqueId needs no peer, but keep RCCL out of the CPU suite
    env = bench.RankEnv.__new__(bench.RankEnv)
    env.a = argparse.Namespace(stage_timeout=60.0)
    env.world, env.rank, env.local, env.wd, env.torch = world, rank, rank, None, torch
    env.init_control()
    res = {
        "backend": dist.get_backend(),
        # digests are uint64: the sum wraps mod 2^64 over ranks
        "gsum": env.gsum((1 << 64) - 1 - rank if rank % 2 else (1 << 63) + rank),
        "gmax": env.gmax(0.5 + rank),
        "bcast": env.bcast(1000 + rank),
        "gather": env.gather({"rank": rank}),
        "uid": env.unique_id(),
    }
    dist.barrier()
    q.put((rank, res))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_bench_rankenv_control_plane_is_gloo_on_cpu(world):
    """the production RankEnv's collectives (the unique-id
    broadcast, digest sum mod 2^64, max-over-ranks time, warmup broadcast,
    per-rank rows) run on a gloo process group over CPU tensors, so the
    library's RCCL communicator is the job's only GPU communication."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rankenv_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    vals = [(1 << 64) - 1 - r if r % 2 else (1 << 63) + r for r in range(world)]
    for r in range(world):
        res = got[r]
        assert res["backend"] == "gloo"
        assert res["gsum"] == sum(vals) % (1 << 64)
        assert res["gmax"] == world - 0.5 and res["bcast"] == 1000
        assert res["gather"] == [{"rank": i} for i in range(world)]
        assert res["uid"] == b"rccl-id-of-rank-0"
