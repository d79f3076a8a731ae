"""A two-process ring on one GPU: the cross-process strip
logic of golhip_step's RCCL path, everything but RCCL's own transport.

Two (or three) processes, spawned before either touches the GPU, each hold
one strip handle of the same board on device 0 and join a ring through the
test hook golhip_test_ring_init (GOLHIP_TEST_HOOKS=1): the library runs its
own ring schedule (golhip_halo_schedule's rounds of k launches of d turns,
the deep-halo extension, golhip_halo_plan's rows, the kernels a ring share
of that size plans) and, at the exact point where it would post the RCCL
group (exchange_rccl), stages its two send blocks in pinned memory and hands
them to a host callback; here that callback trades them with the
neighbours over multiprocessing queues (send up -> prev's bottom halo, send
down -> next's top halo, as the RCCL group pairs them).  The strips'
results are checked against the reference's own fixture
(check/images/64x64x100.pgm via tests/golden/fixtures.npz) and against the
configs[2] full-size fixture at turn 1000 (65536^2 in two strips: summed
board digests and alive counts, sample rows bit for bit), as
distributor.go:116-173's turn loop over a partitioned board would produce.
"""
import multiprocessing as mp
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

golhip = pytest.importorskip("golhip")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def _rank_main(rank, nranks, W, H, turns, board_key, seed, sample_rows, inboxes, out_q, opts):
    """One ring rank: its strip, the host transport, the run; results to out_q."""
    os.environ["GOLHIP_TEST_HOOKS"] = "1"
    sys.path[:0] = [ROOT, os.path.join(ROOT, "game-of-life-distributed_amd")]
    try:
        import golhip as g
        bounds = [H * i // nranks for i in range(nranks + 1)]
        row0, rows = bounds[rank], bounds[rank + 1] - bounds[rank]
        ring_rows = min(bounds[i + 1] - bounds[i] for i in range(nranks))

        def exchange(prev, nxt, up, down):
            # as the RCCL group: our first rows go up (prev's bottom halo), our
            # last rows down (next's top halo); theirs come back the same way.
            # One queue per directed edge: inboxes[2 r] holds what
            # r's next rank sent up, inboxes[2 r + 1] what its prev sent down,
            # each in exchange order, so a neighbour that runs a round ahead
            # can never pair its halo with another neighbour's older one
            inboxes[2 * prev].put(up)
            inboxes[2 * nxt + 1].put(down)
            return inboxes[2 * rank + 1].get(timeout=60), inboxes[2 * rank].get(timeout=60)

        with g.Board(W, H, row0=row0, rows=rows) as b:
            for k, v in opts.items():
                b.set_option(k, v)
            b.test_ring_init(nranks, rank, ring_rows, exchange)
            info = b.comm_info()
            assert info == {"nranks": nranks, "rank": rank, "ring_rows": ring_rows}, info
            if board_key:
                from oracle.oracle import unpack_bits
                with np.load(os.path.join(GOLDEN, "fixtures.npz"), allow_pickle=False) as z:
                    board = unpack_bits(z[board_key], W)
                b.load_bytes(board[row0:row0 + rows])
            else:
                b.fill_random(seed)
            b.step(turns)
            cnt, at = b.alive_count()
            p = b.perf()
            res = {"rank": rank, "row0": row0, "rows": rows, "alive": cnt, "at": at, "hash": b.board_hash(),
                   "halo_exchanges": p["halo_exchanges"], "halo_bytes": p["halo_bytes"],
                   "step_turns": p["step_turns"], "persist_launches": p["persist_launches"]}
            if board_key:
                res["cells"] = b.snapshot_bytes()
            res["sample"] = {r: b.snapshot_rows(r - row0, 1)[0] for r in sample_rows if row0 <= r < row0 + rows}
            out_q.put(res)
    except BaseException as e:  # noqa: BLE001 - the parent reports it
        out_q.put({"rank": rank, "error": repr(e)})


def run_ring(nranks, W, H, turns, board_key=None, seed=0, sample_rows=(), timeout=300, **opts):
    ctx = mp.get_context("spawn")
    inboxes = [ctx.Queue() for _ in range(2 * nranks)]  # per directed edge: [2 r] from below, [2 r + 1] from above
    out_q = ctx.Queue()
    procs = [ctx.Process(target=_rank_main, args=(r, nranks, W, H, turns, board_key, seed, list(sample_rows), inboxes,
                                                        out_q, opts))
             for r in range(nranks)]
    for p in procs:
        p.start()
    try:
        res = [out_q.get(timeout=timeout) for _ in range(nranks)]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    errs = [r["error"] for r in res if "error" in r]
    assert not errs, errs
    return sorted(res, key=lambda r: r["rank"])


@pytest.mark.parametrize("nranks", [2, 3])
def test_ring_64x64_fixture(nranks):
    """The reference's 64x64 image after 100 turns (check/images/64x64x100.pgm),
    as 2 and 3 strips in 2 and 3 processes."""
    from oracle.oracle import unpack_bits
    res = run_ring(nranks, 64, 64, 100, board_key="image_64")
    with np.load(os.path.join(GOLDEN, "fixtures.npz"), allow_pickle=False) as z:
        want = unpack_bits(z["check_64x100"], 64)
        alive = int(z["alive_64"][100])
    got = np.concatenate([r["cells"] for r in res])
    assert np.array_equal(got, want)
    assert sum(r["alive"] for r in res) == alive and all(r["at"] == 100 for r in res)
    assert all(r["halo_exchanges"] >= 1 and r["step_turns"] == 100 for r in res), res


def test_ring_config2_two_processes():
    """configs[2]: 65536^2 x 1,000 turns as two 32768-row strips in two
    processes (the 2-GPU plan's shares), against the full-size fixture."""
    import json
    with open(os.path.join(GOLDEN, "fullsize.json")) as f:
        rec = json.load(f)["c2"]
    with np.load(os.path.join(GOLDEN, "fullsize.npz"), allow_pickle=False) as z:
        rows = z["c2_rows"]
    N = rec["width"]
    res = run_ring(2, N, N, 1000, seed=rec["seed"], sample_rows=rec["sample_rows"])
    cp = rec["checkpoints"]["1000"]
    digest = sum(r["hash"] for r in res) % (1 << 64)
    assert f"{digest:016x}" == cp["hash"]
    assert sum(r["alive"] for r in res) == cp["alive"]
    assert all(r["halo_bytes"] > 0 and r["step_turns"] == 1000 for r in res), res
    assert rec["sample_turn"] == 1000
    sample = {r: v for x in res for r, v in x["sample"].items()}
    for i, r in enumerate(rec["sample_rows"]):
        assert np.array_equal(sample[r], rows[i]), ("row", r)


def test_ring_hook_needs_consent(monkeypatch):
    """Without GOLHIP_TEST_HOOKS=1 the hook is refused (product builds never
    run a ring without RCCL by accident)."""
    monkeypatch.delenv("GOLHIP_TEST_HOOKS", raising=False)
    with golhip.Board(64, 64, row0=0, rows=32) as b:
        with pytest.raises(golhip.GolHipError):
            b.test_ring_init(2, 0, 32, lambda *a: (b"", b""))
