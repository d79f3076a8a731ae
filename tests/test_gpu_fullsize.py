"""Every BASELINE.json config at full size against the oracle's own answer.

The fixtures (tests/golden/fullsize.json + .npz) come from
tests/golden/make_fullsize.py: the bit-packed CPU comparator
oracle/gol_fastcpu.c, pinned to the reference's check/images and check/alive
by tests/test_oracle_golden.py, run on the same synthetic boards.  Each check
compares the HIP engine's board digest (golhip_board_hash) and alive count
at every checkpoint turn, plus four whole rows bit for bit at the last one:

  configs[1]  16384^2  x 10,000 turns   (gol_test.go:15-47 shape: final board)
  configs[2]  65536^2  x  1,000 turns   (also as 8 in-process strips and
                                          through the one-rank RCCL ring)
  configs[3]  262144^2 x    100 turns   (one GPU holds the whole board)
  configs[4]  5120^2 CellFlipped stream, turns 1..50 (sdl_test.go:93-128
              shape: every flip list of every turn, batched and per turn)

The engine options varied here (resident vs per-launch kernel, words per
lane, fused depth) must never change a result.
"""
import hashlib
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

golhip = pytest.importorskip("golhip")

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def full():
    path = os.path.join(GOLDEN, "fullsize.json")
    if not os.path.exists(path):
        pytest.fail("tests/golden/fullsize.json missing: run tests/golden/make_fullsize.py")
    with open(path) as f:
        js = json.load(f)
    with np.load(os.path.join(GOLDEN, "fullsize.npz"), allow_pickle=False) as z:
        rows = {k: z[k] for k in z.files}
    return js, rows


def check_board(b, rec, rows, key, turn):
    cp = rec["checkpoints"][str(turn)]
    cnt, at = b.alive_count()
    assert at == turn
    assert (f"{b.board_hash():016x}", cnt) == (cp["hash"], cp["alive"]), (key, turn)
    if turn == rec["sample_turn"]:
        for i, r in enumerate(rec["sample_rows"]):
            assert np.array_equal(b.snapshot_rows(r, 1)[0], rows[f"{key}_rows"][i]), (key, "row", r)


def run_checkpoints(full, key, **options):
    js, rows = full
    rec = js[key]
    N = rec["width"]
    with golhip.Board(N, N) as b:
        for k, v in options.items():
            if k == "tb_depth":
                b.set_tb_depth(v)
            else:
                b.set_option(k, v)
        b.fill_random(rec["seed"])
        done = 0
        for t in sorted(int(x) for x in rec["checkpoints"]):
            b.step(t - done)
            done = t
            check_board(b, rec, rows, key, t)
        return b.perf()


# ---------------------------------------------------------------- configs[1]
@pytest.mark.parametrize("opts", [{}, {"persistent": 1}, {"skew": 0, "persistent": 0}, {"wpl": 2},
                                  {"persistent": 0, "skew_pairs": 1, "skew_half": -1}, {"skew_pairs": 1},
                                  {"persistent": 0, "wpl": 4}, {"tb_depth": 32, "wpl": 1},
                                  {"persistent": 0, "tb_depth": 6}, {"tb_depth": 16}])
def test_config1_16384_10k_turns(full, opts):
    """configs[1]: 16384^2, 10,000 turns (default: skewed band stacks, K1w, on
    half-wave tiles and the pair rule at 18 turns a launch; skew_pairs 1: the
    same tiles at 16 on the 9-LUT stages; persistent 1: the resident kernel
    K1p; skew 0: the overlapped K1)."""
    run_checkpoints(full, "c1", **opts)


# ---------------------------------------------------------------- configs[2]
@pytest.mark.parametrize("opts", [{}, {"skew": 0}, {"tb_depth": 16}, {"wpl": 4},
                                  {"persistent": 1}, {"wpl": 1, "tb_depth": 32}, {"skew_tx": 2},
                                  {"skew_young": 70, "skew_prio": 1}, {"skew_pairs": 1}])
def test_config2_65536_1k_turns(full, opts):
    """configs[2]: 65536^2, 1,000 turns (default: skewed band stacks, 20-turn launches;
    skew 0: the overlapped paired-band kernel)."""
    run_checkpoints(full, "c2", **opts)


@pytest.mark.parametrize("nstrips", [8, 3])
def test_config2_strips_in_process(full, nstrips):
    """configs[2] decomposed into row strips (the multi-GPU layout, halos by
    device copies): the strip digests add up to the fixture."""
    js, _ = full
    rec = js["c2"]
    N = rec["width"]
    bounds = [N * i // nstrips for i in range(nstrips + 1)]
    strips = [golhip.Board(N, N, row0=bounds[i], rows=bounds[i + 1] - bounds[i]) for i in range(nstrips)]
    try:
        for s in strips:
            s.fill_random(rec["seed"])
        done = 0
        for t in (100, 1000):
            golhip.group_step(strips, t - done)
            done = t
            cp = rec["checkpoints"][str(t)]
            digest = sum(s.board_hash() for s in strips) % (1 << 64)
            assert f"{digest:016x}" == cp["hash"]
            assert sum(s.alive_count()[0] for s in strips) == cp["alive"]
    finally:
        for s in strips:
            s.close()


@pytest.mark.parametrize("persistent", [-1, 1, 0])
def test_config2_rccl_ring_one_rank(full, persistent):
    """configs[2] through the RCCL halo path (a one-rank ring, deep halos)."""
    js, rows = full
    rec = js["c2"]
    N = rec["width"]
    with golhip.Board(N, N) as b:
        b.comm_init(golhip.unique_id(), 1, 0)
        b.set_option("force_halo", 1)
        b.set_option("persistent", persistent)
        if persistent == 0:
            b.set_option("skew", 0)
        b.fill_random(rec["seed"])
        b.step(1000)
        assert b.perf()["halo_bytes"] > 0
        check_board(b, rec, rows, "c2", 1000)


# ---------------------------------------------------------------- configs[3]
@pytest.mark.parametrize("opts", [{}, {"wpl": 2}, {"skew": 0}])
def test_config3_262144_100_turns(full, opts):  # default: skewed band stacks
    """configs[3]: the whole 262144^2 board on one GPU, 100 turns (default:
    four words per lane, 8-turn launches)."""
    run_checkpoints(full, "c3", **opts)


@pytest.mark.parametrize("nstrips", [8, 2])
def test_config3_strips_in_process(full, nstrips):
    """configs[3] as the row strips of its 8- and 2-GPU strong-scaling plan
    (distributor.go:116-173's turn loop over a partitioned board; the README's
    halo extension): 262144^2 in `nstrips` strips of 262144 / nstrips rows,
    100 turns with deep halos moved by device copies, the strips' digests and
    alive counts summed against the c3 fixture, the fixture's sample rows
    compared bit for bit.  Every strip must have run the plan a ring share
    of that size runs: K1w (skewed band stacks) on four words per lane, on
    its extended rows."""
    js, rows = full
    rec = js["c3"]
    N = rec["width"]
    bounds = [N * i // nstrips for i in range(nstrips + 1)]
    strips = [golhip.Board(N, N, row0=bounds[i], rows=bounds[i + 1] - bounds[i]) for i in range(nstrips)]
    try:
        for s in strips:
            s.fill_random(rec["seed"])
        golhip.group_step(strips, 100)
        cp = rec["checkpoints"]["100"]
        digest = sum(s.board_hash() for s in strips) % (1 << 64)
        assert f"{digest:016x}" == cp["hash"]
        assert sum(s.alive_count()[0] for s in strips) == cp["alive"]
        assert rec["sample_turn"] == 100
        for i, r in enumerate(rec["sample_rows"]):
            k = max(j for j in range(nstrips) if bounds[j] <= r)
            assert np.array_equal(strips[k].snapshot_rows(r - bounds[k], 1)[0], rows["c3_rows"][i]), ("row", r)
        for s in strips:
            p = s.perf()
            assert p["words_per_lane"] == 4, p
            assert p["step_launches"] > 0 and p["skew_launches"] == p["step_launches"], p
            assert p["step_turns"] == 100 and p["halo_bytes"] > 0, p
    finally:
        for s in strips:
            s.close()


# ---------------------------------------------------------------- configs[4]
def test_config4_5120_event_stream_batched(full):
    """configs[4]: the initial CellFlipped list (alive cells at load,
    distributor.go:72-80) and the flip lists of turns 1..50
    (initializeAliveCells :212-220) through golhip_step_flips in uneven batches."""
    js, _ = full
    rec = js["c4"]
    N = rec["width"]
    counts_all, sha = [], hashlib.sha256()
    with golhip.Board(N, N) as b:
        b.fill_random(rec["seed"])
        init = b.alive_cells()
        assert len(init) == rec["initial_alive"]
        assert hashlib.sha256(init.tobytes()).hexdigest() == rec["initial_sha256"]
        cap = 6 * N * N
        xy = np.empty((cap, 2), dtype=np.int32)
        for k in (1, 7, 16, 20, 6):
            got, counts = b.step_flips(k, cap=cap, xy=xy)
            sha.update(got.tobytes())
            counts_all += [int(c) for c in counts]
        assert counts_all == rec["flip_counts"]
        assert sha.hexdigest() == rec["flips_sha256"]
        assert (f"{b.board_hash():016x}", b.alive_count()) == (rec["final"]["hash"], (rec["final"]["alive"], 50))


def test_config4_5120_event_stream_per_turn(full):
    """The same stream one turn per call (golhip_step(1, want_flips) + golhip_flips)."""
    js, _ = full
    rec = js["c4"]
    N = rec["width"]
    sha = hashlib.sha256()
    with golhip.Board(N, N) as b:
        b.fill_random(rec["seed"])
        for t in range(rec["turns"]):
            b.step(1, want_flips=True)
            fl = b.flips()
            assert len(fl) == rec["flip_counts"][t], t
            sha.update(fl.tobytes())
        assert sha.hexdigest() == rec["flips_sha256"]


def test_config4_5120_flip_stream_index(full):
    """configs[4] through golhip_flip_stream (fused K5 kernel, 4-byte cell
    indices, a 16 M-entry buffer so calls stop early and resume): decoded to
    (x, y) pairs the stream hashes to the fixture."""
    js, _ = full
    rec = js["c4"]
    N = rec["width"]
    sha, counts_all = hashlib.sha256(), []
    cap = 16 << 20  # turns 1..50 flip 2.6-7.2 M cells each
    out = np.empty(cap, dtype=np.uint32)
    with golhip.Board(N, N) as b:
        b.fill_random(rec["seed"])
        while len(counts_all) < rec["turns"]:
            ent, counts, done = b.flip_stream(rec["turns"] - len(counts_all), cap=cap, fmt=golhip.FLIPS_INDEX,
                                              out=out)
            assert done >= 1
            idx = ent.astype(np.int64)
            sha.update(np.stack([idx % N, idx // N], axis=1).astype(np.int32).tobytes())
            counts_all += [int(c) for c in counts]
        assert counts_all == rec["flip_counts"]
        assert sha.hexdigest() == rec["flips_sha256"]
        assert (f"{b.board_hash():016x}", b.alive_count()) == (rec["final"]["hash"], (rec["final"]["alive"], 50))


@pytest.mark.parametrize("overlap", [2, 1, 0])
def test_config4_5120_flip_stream_pinned(full, overlap):
    """configs[4] as bench.py streams it: 4-byte indices into golhip_host_alloc
    memory, the host lists written by the copy blocks of the batch's one
    resident launch (K5r, flip_overlap 2, round 6), by the copy blocks of the
    next launch (1) or by the turn's own blocks (0); a 12 M-entry buffer makes
    calls stop before a turn that would not fit and resume.  The stream hashes
    to the fixture."""
    js, _ = full
    rec = js["c4"]
    N = rec["width"]
    sha, counts_all = hashlib.sha256(), []
    cap = 12 << 20
    out = golhip.host_array((cap,), np.uint32)
    with golhip.Board(N, N) as b:
        b.set_option("flip_overlap", overlap)
        b.fill_random(rec["seed"])
        calls = 0
        while len(counts_all) < rec["turns"]:
            ent, counts, done = b.flip_stream(rec["turns"] - len(counts_all), cap=cap, fmt=golhip.FLIPS_INDEX,
                                              out=out)
            assert done >= 1
            idx = ent.astype(np.int64)
            sha.update(np.stack([idx % N, idx // N], axis=1).astype(np.int32).tobytes())
            counts_all += [int(c) for c in counts]
            calls += 1
        assert calls > 10
        assert (b.perf()["flip_resident_launches"] >= 1) == (overlap == 2)
        assert counts_all == rec["flip_counts"]
        assert sha.hexdigest() == rec["flips_sha256"]
        assert (f"{b.board_hash():016x}", b.alive_count()) == (rec["final"]["hash"], (rec["final"]["alive"], 50))
    del out
