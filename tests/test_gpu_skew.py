"""GPU parity of skewed band stacks (option "skew", gol_kernels.hip K1w) against the C oracle.

K1w runs a launch as stacks of bands, one workgroup per stack: band [a, e)
of input rows owns generation g of the rows [a + g, e + g), takes the
bottom rows it needs from the band below through LDS (exported during that
band's pipeline fill) and the stack's bottom band computes its drain from
the board.  Bit-exact against oracle/gol_fastcpu.c (the C restatement pinned
to the reference's fixtures in tests/test_oracle_golden.py) for every
instantiated (depth, words per lane), stacks of 8 and of 4 bands, unequal
band heights, the torus seam inside a band, row strips (one-rank RCCL ring
and in-process strips, where the launches step extended row ranges) and
the fused alive count.  The full-size BASELINE fixtures run on K1w by
default (tests/test_gpu_fullsize.py).
"""
import numpy as np
import pytest

from oracle.oracle import COracle

pytestmark = pytest.mark.gpu

golhip = pytest.importorskip("golhip")

SKEW = [(8, 2), (12, 2), (16, 2), (20, 2), (6, 4), (8, 4), (9, 4), (16, 1), (32, 1)]


@pytest.fixture(scope="module")
def coracle():
    return COracle()


def run_skew(board, turns, depth, wpl, **opts):
    H, W = board.shape
    with golhip.Board(W, H) as b:
        b.set_option("persistent", 0)
        b.set_option("skew", 2)  # whenever a plan exists (the default also wants the CUs filled)
        b.set_option("wpl", wpl)
        b.set_option("skew_pairs", 0)  # the instantiation under test, not the pair rule's 18 (opts may set it)
        for k, v in opts.items():
            b.set_option(k, v)
        b.set_tb_depth(depth)
        b.load_bytes(board)
        b.step(turns)
        p = b.perf()
        out = b.snapshot_bytes()
        cnt, at = b.alive_count()
        assert at == turns
        assert cnt == int((out == 255).sum())
        return out, p


@pytest.mark.parametrize("depth,wpl", SKEW)
@pytest.mark.parametrize("W,H", [(2048, 1024), (4096, 777), (8192, 331), (3968, 2500), (16384, 1600)])
def test_skew_matches_oracle(coracle, depth, wpl, W, H):
    if W % (32 * wpl):
        pytest.skip("width not a multiple of the lane chunk")
    board = coracle.fill_random(W, H, 0x5EED0031 + W + H)
    turns = 2 * depth + 3  # two skew launches and a remainder on the other kernels
    want = coracle.run(board, turns)
    got, p = run_skew(board, turns, depth, wpl)
    assert p["skew_launches"] >= 1
    assert np.array_equal(got, want)


@pytest.mark.parametrize("depth,wpl", SKEW)
@pytest.mark.parametrize("tx", [1, 2])
def test_skew_single_stack(coracle, depth, wpl, tx):
    """One stack per tile column (a narrow board, few rows): the torus seam
    runs through the top band's first rows and the bottom band's drain."""
    W = 62 * 32 * wpl  # one tile
    sy = 8 // tx
    H = sy * (2 * depth + 3) + 5
    board = coracle.fill_random(W, H, 0x5EED0032 + depth * 8 + wpl)
    turns = 2 * depth
    want = coracle.run(board, turns)
    got, p = run_skew(board, turns, depth, wpl, skew_tx=tx)
    assert p["skew_launches"] == 2 and p["kernel_variant"] == 3
    assert np.array_equal(got, want)


@pytest.mark.parametrize("depth,wpl", [(20, 2), (16, 2), (9, 4), (32, 1)])
@pytest.mark.parametrize("opts", [{"skew_young": 60}, {"skew_young": 150}, {"skew_hcap": 0}, {"skew_hcap": 40},
                                  {"skew_prio": 1}, {"skew_tx": 2, "skew_young": 80}])
def test_skew_band_heights(coracle, depth, wpl, opts):
    """Unequal bands (taller or shorter younger waves, bottom-band handicap,
    static priority) change only the schedule, never the result."""
    W, H = 4096, 2000 + depth
    board = coracle.fill_random(W, H, 0x5EED0033 + depth)
    turns = 3 * depth
    want = coracle.run(board, turns)
    got, p = run_skew(board, turns, depth, wpl, **opts)
    assert p["skew_launches"] == 3
    assert np.array_equal(got, want)


@pytest.mark.parametrize("depth,wpl", [(20, 2), (16, 2), (8, 4), (9, 4), (16, 1), (32, 1), (18, 2)])
@pytest.mark.parametrize("W,H", [(4096, 1500), (8192, 700), (2048, 4096)])
def test_skew_rccl_ring_one_rank(coracle, depth, wpl, W, H):
    """The multi-GPU path on K1w: deep-halo exchange, then launches over the
    extended row ranges [-e, rows + e) (one-rank RCCL ring, force_halo)."""
    board = coracle.fill_random(W, H, 0x5EED0034 + W)
    # (the pair rule: 7 launches of 18; 128 turns would plan as 8 x 16)
    turns = 7 * depth + (0 if depth == 18 else 2)
    want = coracle.run(board, turns)
    with golhip.Board(W, H) as b:
        b.comm_init(golhip.unique_id(), 1, 0)
        b.set_option("force_halo", 1)
        b.set_option("persistent", 0)
        b.set_option("skew", 2)
        b.set_option("wpl", wpl)
        b.set_option("skew_pairs", 3 if depth == 18 else 0)
        if depth == 18:
            b.set_option("skew_half", -1)  # (the pair rule plans on full-width tiles)
        b.set_tb_depth(20 if depth == 18 else depth)
        b.load_bytes(board)
        b.step(turns)
        p = b.perf()
        assert p["halo_bytes"] > 0 and p["skew_launches"] >= 3
        assert (p["pair_launches"] >= 3) == (depth == 18), p
        assert np.array_equal(b.snapshot_bytes(), want)
        assert b.alive_count() == (int((want == 255).sum()), turns)


@pytest.mark.parametrize("nstrips", [2, 3, 5])
@pytest.mark.parametrize("depth,wpl,pairs", [(20, 2, 0), (9, 4, 0), (20, 2, 1), (9, 4, 2)])
def test_skew_group_strips(coracle, nstrips, depth, wpl, pairs):
    """In-process row strips (halos by device copies) stepped on K1w."""
    W, H = 4096, 3001
    board = coracle.fill_random(W, H, 0x5EED0035 + nstrips)
    turns = 5 * depth + 1
    want = coracle.run(board, turns)
    bounds = [H * i // nstrips for i in range(nstrips + 1)]
    strips = [golhip.Board(W, H, row0=bounds[i], rows=bounds[i + 1] - bounds[i]) for i in range(nstrips)]
    try:
        for i, s in enumerate(strips):
            s.set_option("wpl", wpl)
            s.set_option("skew", 2)
            s.set_option("skew_pairs", pairs)
            s.set_option("skew_half", -1 if pairs else 0)
            s.set_tb_depth(depth)
            s.load_bytes(board[bounds[i]:bounds[i + 1]])
        golhip.group_step(strips, turns)
        got = np.concatenate([s.snapshot_bytes() for s in strips])
        assert sum(s.perf()["skew_launches"] for s in strips) > 0
        assert np.array_equal(got, want)
        assert sum(s.alive_count()[0] for s in strips) == int((want == 255).sum())
    finally:
        for s in strips:
            s.close()


def test_skew_off_uses_other_kernels(coracle):
    board = coracle.fill_random(4096, 1000, 0x5EED0036)
    want = coracle.run(board, 40)
    got, p = run_skew(board, 40, 20, 2, skew=0)
    assert p["skew_launches"] == 0 and p["kernel_variant"] in (1, 2)
    assert np.array_equal(got, want)


def test_skew_every_launch_counts(coracle):
    """Steps of one launch each: the fused popcount of every K1w launch."""
    board = coracle.fill_random(8192, 1200, 0x5EED0037)
    with golhip.Board(8192, 1200) as b:
        b.set_option("persistent", 0)
        b.set_option("skew", 2)
        b.set_option("skew_pairs", 0)
        b.set_tb_depth(20)
        b.load_bytes(board)
        cur = board
        for t in range(5):
            b.step(20)
            cur = coracle.run(cur, 20)
            assert b.alive_count() == (int((cur == 255).sum()), 20 * (t + 1))
        assert b.perf()["skew_launches"] == 5
        assert np.array_equal(b.snapshot_bytes(), cur)


# ------------------------------------------------- half-wave tiles (option "skew_half")
@pytest.mark.parametrize("depth", [20, 16, 18])
@pytest.mark.parametrize("W,H", [(16384, 1000), (5120, 2222), (3072, 1502), (4160, 3000), (2048, 818)])
@pytest.mark.parametrize("tx", [0, 2])
def test_skew_half_tiles_match_oracle(coracle, depth, W, H, tx):
    """Half-wave tiles: lanes 0-31 and 32-63 of a wave are two 30-lane tiles
    of one tile column, the upper one H / 2 rows further down (the same band
    of a second stack); torus seam, narrow and ragged tile columns.  Depth 18
    is the pair rule on half tiles (skew_pairs 5, the 16384^2 default)."""
    board = coracle.fill_random(W, H, 0x5EED0041 + W + H + depth)
    turns = 2 * depth + 5
    want = coracle.run(board, turns)
    if depth == 18:
        got, p = run_skew(board, turns, 20, 2, skew_half=1, skew_tx=tx, skew_pairs=5)
        assert p["pair_launches"] >= 2 and p["tb_depth"] == 18, p
    else:
        got, p = run_skew(board, turns, depth, 2, skew_half=1, skew_tx=tx)
    assert p["skew_half_launches"] >= 2
    assert np.array_equal(got, want)


def test_skew_half_tiles_need_even_rows(coracle):
    """An odd number of rows cannot split into two equal halves: full tiles."""
    board = coracle.fill_random(16384, 1001, 0x5EED0042)
    want = coracle.run(board, 43)
    got, p = run_skew(board, 43, 20, 2, skew_half=1)
    assert p["skew_launches"] >= 2 and p["skew_half_launches"] == 0
    assert np.array_equal(got, want)


@pytest.mark.parametrize("W,H", [(16384, 3000), (5120, 2048)])
def test_skew_half_tiles_rccl_ring_and_strips(coracle, W, H):
    """Half-wave tiles on a strip's extended rows: a one-rank RCCL ring and
    three in-process strips."""
    board = coracle.fill_random(W, H, 0x5EED0043 + W)
    turns = 130
    want = coracle.run(board, turns)
    with golhip.Board(W, H) as b:
        b.comm_init(golhip.unique_id(), 1, 0)
        b.set_option("force_halo", 1)
        b.set_option("skew", 2)
        b.set_option("skew_half", 1)
        b.set_option("wpl", 2)  # (5120 wide would plan one word per lane)
        b.load_bytes(board)
        b.step(turns)
        assert b.perf()["skew_half_launches"] >= 1
        assert np.array_equal(b.snapshot_bytes(), want)
    bounds = [0, H // 3 * 1 // 2 * 2, 2 * H // 3 // 2 * 2, H]
    strips = [golhip.Board(W, H, row0=bounds[i], rows=bounds[i + 1] - bounds[i]) for i in range(3)]
    try:
        for i, s in enumerate(strips):
            s.set_option("skew", 2)
            s.set_option("skew_half", 1)
            s.set_option("wpl", 2)
            s.load_bytes(board[bounds[i]:bounds[i + 1]])
        golhip.group_step(strips, turns)
        assert sum(s.perf()["skew_half_launches"] for s in strips) >= 1
        got = np.concatenate([s.snapshot_bytes() for s in strips])
        assert np.array_equal(got, want)
    finally:
        for s in strips:
            s.close()


def test_default_plans_by_board_size():
    """The default plan: half-wave tiles at 16384^2 (configs[1]: 4.5 instead
    of 5 waves a row) with 18-turn launches on the pair rule (round 6; 16 on
    the 9-LUT stages before), full tiles and 18-turn launches on the pair
    rule at 65536^2, and the resident kernel for tori whose K1w stacks would
    not fill the CUs (8192^2)."""
    with golhip.Board(16384, 16384) as b:
        b.fill_random(0x5EED0001)
        b.step(36)
        p = b.perf()
        assert p["skew_launches"] == 2 and p["skew_half_launches"] == 2 and p["step_turns"] == 36
        assert p["pair_launches"] == 2 and p["tb_depth"] == 18
    with golhip.Board(65536, 4096) as b:
        b.fill_random(0x5EED0002)
        b.step(18)
        p = b.perf()
        assert p["skew_half_launches"] == 0 and p["skew_launches"] == 1 and p["pair_launches"] == 1
        assert p["tb_depth"] == 18
    with golhip.Board(8192, 8192) as b:
        b.fill_random(0x5EED0003)
        b.step(64)
        p = b.perf()
        assert p["persist_launches"] >= 1 and p["skew_launches"] == 0


@pytest.mark.parametrize("W,H", [(2048, 1024), (4096, 777), (8192, 331), (3968, 2500), (16384, 1600), (7936, 4099)])
@pytest.mark.parametrize("turns", [41, 18, 54, 17])
def test_skew_pairs_matches_oracle(coracle, W, H, turns):
    """The pair rule (option skew_pairs, gol_bits.h pair_sum / pair_rule):
    K1w at 18 turns a launch on full-width tiles, its main loop in two-group
    bodies on the pair state, the fill and drain on the 9-LUT stages with the
    state converted between them (pr_enter / pr_leave), bands in multiples of
    6 rows; remainders on 16 / 12 / ... -turn launches of the other kernels."""
    board = coracle.fill_random(W, H, 0x5EED0071 + W + H)
    want = coracle.run(board, turns)
    got, p = run_skew(board, turns, 20, 2, skew_pairs=1, skew_half=-1)
    if turns >= 18:
        assert p["tb_depth"] == 18 and p["skew_launches"] >= turns // 18, p
    assert np.array_equal(got, want)


@pytest.mark.parametrize("young,tx", [(60, 1), (100, 2), (150, 1)])
def test_skew_pairs_band_shapes(coracle, young, tx):
    """Pair-rule bands of other heights and stacks of 4 bands."""
    board = coracle.fill_random(6080, 3000, 0x5EED0077 + young + tx)
    want = coracle.run(board, 40)
    got, p = run_skew(board, 40, 20, 2, skew_pairs=1, skew_half=-1, skew_young=young, skew_tx=tx)
    assert p["skew_launches"] >= 2
    assert np.array_equal(got, want)
