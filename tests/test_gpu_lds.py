"""GPU parity of resident LDS bands (option "lds_band", gol_kernels.hip K1r) against the C oracle.

K1r keeps each workgroup's band of full-width rows in LDS with `lds_depth`
halo rows on each side, runs super-steps of D turns there (column wrap in
LDS, no tiles) and trades its top and bottom D rows with its two neighbour
workgroups through write-through edge buffers and flags between
super-steps.  Bit-exact against oracle/gol_fastcpu.c (the C restatement
pinned to the reference's fixtures in tests/test_oracle_golden.py) for both
layouts (canonical words, interleaved pairs), depths 1..16, bands of exactly
D rows, uneven bands (rows not a multiple of the band count), one band (its
own neighbour above and below), two bands (one neighbour on both sides),
turn counts that end in a short super-step, non-square boards, the fused
alive count, and the XCD-ordered band assignment on and off.
"""
import numpy as np
import pytest

from oracle.oracle import COracle

pytestmark = pytest.mark.gpu

golhip = pytest.importorskip("golhip")


@pytest.fixture(scope="module")
def coracle():
    return COracle()


def run_lds(board, turns, depth, wpl=2, **opts):
    H, W = board.shape
    with golhip.Board(W, H) as b:
        b.set_option("persistent", 1)
        b.set_option("lds_band", 1)
        b.set_option("lds_depth", depth)
        b.set_option("wpl", wpl)
        for k, v in opts.items():
            b.set_option(k, v)
        b.load_bytes(board)
        b.step(turns)
        p = b.perf()
        out = b.snapshot_bytes()
        cnt, at = b.alive_count()
        assert at == turns
        assert cnt == int((out == 255).sum())
        return out, p


@pytest.mark.parametrize("wpl", [1, 2])
@pytest.mark.parametrize("depth", [1, 2, 3, 5, 8, 12, 16])
@pytest.mark.parametrize("W,H", [(1024, 1024), (2048, 1003), (640, 384), (4096, 256)])
def test_lds_band_matches_oracle(coracle, wpl, depth, W, H):
    board = coracle.fill_random(W, H, 0x5EED0041 + W + H + depth)
    turns = 3 * depth + 2  # ends in a short super-step
    want = coracle.run(board, turns)
    got, p = run_lds(board, turns, depth, wpl)
    assert p["lds_launches"] == 1 and p["persist_launches"] == 1 and p["kernel_variant"] == 4
    assert p["words_per_lane"] == wpl
    assert np.array_equal(got, want)


@pytest.mark.parametrize("H,depth", [(8, 8), (16, 8), (24, 8), (9, 4), (2 * 256 * 8, 8), (256 * 8 + 7, 8)])
def test_lds_band_counts(coracle, H, depth):
    """One band (8 rows at depth 8: its own neighbour on both sides), two
    bands (one neighbour both ways), three, bands of exactly D rows (256 of
    them on a 256-CU device) and uneven bands."""
    W = 512
    board = coracle.fill_random(W, H, 0x5EED0042 + H)
    turns = 5 * depth + 1
    want = coracle.run(board, turns)
    got, p = run_lds(board, turns, depth)
    assert p["lds_launches"] == 1
    assert np.array_equal(got, want)


@pytest.mark.parametrize("turns", [2, 7, 8, 9, 100, 1001])
def test_lds_band_turn_counts(coracle, turns):
    board = coracle.fill_random(1536, 1280, 0x5EED0043 + turns)
    want = coracle.run(board, turns)
    got, p = run_lds(board, turns, 8)
    assert p["lds_launches"] == 1
    assert np.array_equal(got, want)


@pytest.mark.parametrize("xcd", [0, 1])
def test_lds_band_xcd_order(coracle, xcd):
    board = coracle.fill_random(2048, 2048, 0x5EED0044)
    want = coracle.run(board, 50)
    got, p = run_lds(board, 50, 8, lds_xcd=xcd)
    assert p["lds_launches"] == 1
    assert np.array_equal(got, want)


def test_lds_band_fixture_5120(coracle):
    """configs[4]'s board (5120^2, seed 0x5EED0005) through K1r for 200 turns
    vs the oracle, then the auto plan picks K1r for it."""
    with golhip.Board(5120, 5120) as b:
        b.fill_random(0x5EED0005)
        start = b.snapshot_bytes()
        b.step(200)
        p = b.perf()
        assert p["lds_launches"] == 1, p  # the auto plan
        got = b.snapshot_bytes()
    assert np.array_equal(got, coracle.run(start, 200))


def test_lds_band_then_other_kernels(coracle):
    """K1r, then a flip-list turn and per-launch steps on the same handle:
    the buffers and the layout stay consistent across kernels."""
    board = coracle.fill_random(2048, 1024, 0x5EED0045)
    with golhip.Board(2048, 1024) as b:
        b.set_option("persistent", 1)
        b.set_option("lds_band", 1)
        b.load_bytes(board)
        b.step(37)
        b.step(1, want_flips=True)
        b.set_option("persistent", 0)
        b.step(21)
        assert b.perf()["lds_launches"] == 1
        got = b.snapshot_bytes()
    assert np.array_equal(got, coracle.run(board, 59))


@pytest.mark.parametrize("W,H,opts", [(12288, 512, {}),                      # 384 words: the runtime-stride kernel
                                      (2048, 1000, {"lds_stride": 0}),       # 64 words at their own stride
                                      (5120, 640, {"lds_stride": 0}),
                                      (8192, 1024, {"lds_waves": 16}),       # 16 waves a workgroup
                                      (8192, 1024, {"lds_waves": 8}),        # 8192 wide on 8 (auto: 16)
                                      (8192, 1000, {"lds_age": 70}),         # age-weighted runs
                                      (8192, 1000, {"lds_age": 100}),        # equal runs (auto: 60)
                                      (4096, 3001, {"lds_age": 130}),
                                      (8192, 2048, {"lds_age": 40, "lds_waves": 8}),
                                      (5120, 1280, {"lds_age": 60}),         # runs straddling waves
                                      (2048, 1000, {"lds_age": 150}),        # two runs a wave
                                      (5120, 1280, {"lds_waves": 16}),
                                      (8192, 2048, {"lds_wg_cu": 2}),        # two bands a CU
                                      (4096, 3000, {"lds_wg_cu": 2})])
def test_lds_band_variants(coracle, W, H, opts):
    board = coracle.fill_random(W, H, 0x5EED0046 + W + H)
    turns = 29
    want = coracle.run(board, turns)
    got, p = run_lds(board, turns, 8, **opts)
    assert p["lds_launches"] == 1
    assert np.array_equal(got, want)


@pytest.mark.parametrize("W,H", [(128, 3), (128, 5), (256, 4), (256, 13), (384, 12), (128, 1000)])
def test_lds_band_tiny_boards(coracle, W, H):
    """Rows of 2-6 pairs (many runs a wave, neighbours across the row's wrap in
    one run) and boards shorter than the default depth (D = H rows, one band)."""
    board = coracle.fill_random(W, H, 0x5EED0048 + W + H)
    turns = 37
    want = coracle.run(board, turns)
    with golhip.Board(W, H) as b:
        b.set_option("persistent", 1)
        b.load_bytes(board)
        b.step(turns)
        assert b.perf()["lds_launches"] == 1
        got = b.snapshot_bytes()
        assert b.alive_count() == (int((want == 255).sum()), turns)
    assert np.array_equal(got, want)


@pytest.mark.usefixtures("test_hooks")
def test_lds_band_wait_timeout(coracle):
    """Band 0 never publishes its edges (test hook resident_fault): its neighbours'
    flag waits reach the bound, every workgroup drains, and the step is
    restored and re-run on the per-launch kernels, exactly."""
    board = coracle.fill_random(2048, 1024, 0x5EED004A)
    want = coracle.run(board, 51)
    with golhip.Board(2048, 1024) as b:
        b.set_option("persistent", 1)
        b.set_option("resident_fault", 1)
        b.set_option("lds_depth", 8)
        b.set_option("persist_timeout_us", 2000)
        b.load_bytes(board)
        b.step(51)
        p = b.perf()
        got = b.snapshot_bytes()
    assert p["persist_fallbacks"] == 1 and p["lds_launches"] == 0
    assert np.array_equal(got, want)


@pytest.mark.parametrize("W,H,lds", [(12288, 2048, 0), (5120, 1280, 1), (3072, 3072, 1)])
def test_lds_band_auto_choice(coracle, W, H, lds):
    """The auto plan runs K1r only where a row's pairs keep >= 90 % of the
    threads busy (12288 wide: 192 pairs, 384 of 512 threads: K1p, which was
    faster there); the result is exact either way."""
    board = coracle.fill_random(W, H, 0x5EED004B + W)
    want = coracle.run(board, 40)
    with golhip.Board(W, H) as b:
        b.load_bytes(board)
        b.step(40)
        p = b.perf()
        got = b.snapshot_bytes()
    assert p["lds_launches"] == lds and p["persist_launches"] == 1
    assert np.array_equal(got, want)


@pytest.mark.parametrize("pre", [1, 2, 3, 12])
@pytest.mark.parametrize("W,H,depth", [(1024, 1024, 8), (2048, 1003, 12), (8192, 8192, 12), (5120, 5120, 12),
                                       (640, 384, 5), (2048, 2055, 8), (256, 13, 4)])
def test_lds_band_interior_first(coracle, pre, W, H, depth):
    """Interior-first super-steps (option lds_pre): the first `pre` turns on the
    rows that need no halo while the edges travel (the previous flag raised
    after the first of them), then those turns' halo-side rows, then whole
    turns; a short last super-step runs whole turns.  Several steps on one
    handle; pre >= the band height leaves no interior at the later turns."""
    if W * H > 2048 * 2048 and pre not in (2, 3):
        pytest.skip("large boards at two values")
    board = coracle.fill_random(W, H, 0x5EED004C + W + H + pre)
    steps = [3 * depth + 2, 2 * depth, 7]
    want = coracle.run(board, sum(steps))
    with golhip.Board(W, H) as b:
        b.set_option("persistent", 1)
        b.set_option("lds_band", 1)
        b.set_option("lds_pre", pre)
        b.set_option("lds_depth", depth)
        b.load_bytes(board)
        for n in steps:
            b.step(n)
        p = b.perf()
        got = b.snapshot_bytes()
    assert p["lds_launches"] == 3 and p["persist_fallbacks"] == 0
    assert np.array_equal(got, want)


@pytest.mark.usefixtures("test_hooks")
def test_lds_band_interior_first_timeout(coracle):
    board = coracle.fill_random(2048, 1024, 0x5EED004D)
    want = coracle.run(board, 51)
    with golhip.Board(2048, 1024) as b:
        b.set_option("persistent", 1)
        b.set_option("lds_pre", 2)
        b.set_option("resident_fault", 1)
        b.set_option("lds_depth", 8)
        b.set_option("persist_timeout_us", 2000)
        b.load_bytes(board)
        b.step(51)
        p = b.perf()
        got = b.snapshot_bytes()
    assert p["persist_fallbacks"] == 1 and p["lds_launches"] == 0
    assert np.array_equal(got, want)
