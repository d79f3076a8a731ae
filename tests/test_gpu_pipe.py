"""GPU parity of the resident LDS turn pipeline (option "lds_pipe",
gol_pipe.hip K1t) against the C oracle.

K1t runs tori whose rows are one wavefront wide (2048 cells at one word per
lane, 4096 at two, 8192 at four): each workgroup owns a skewed band of rows
(generation t of band b is the rows [r_b + t, r_{b+1} + t)), its eight waves
are eight consecutive turns streaming the band through LDS rings, and the
only hand-off between workgroups is the first two rows of each turn, from the
band below.  Bit-exact against oracle/gol_fastcpu.c / gol_oracle.c (pinned to
the reference's fixtures, tests/test_oracle_golden.py) for the three widths,
square and non-square boards, uneven bands, bands of two rows, one band (its
own band below), few bands (cu_count), turn counts below and above the
eight-turn cycle and the 32-slot edge window, the fused alive count, several
steps on one handle, the XCD band order on and off, and a launch whose waits
time out (restored and re-run on the per-launch kernels).
"""
import numpy as np
import pytest

from oracle.oracle import COracle

pytestmark = pytest.mark.gpu

golhip = pytest.importorskip("golhip")

WPL_OF = {2048: 1, 4096: 2, 8192: 4}


@pytest.fixture(scope="module")
def coracle():
    return COracle()


def run_pipe(board, turns, steps=1, **opts):
    H, W = board.shape
    with golhip.Board(W, H) as b:
        b.set_option("lds_pipe", 1)
        for k, v in opts.items():
            b.set_option(k, v)
        b.load_bytes(board)
        for _ in range(steps):
            b.step(turns)
        p = b.perf()
        out = b.snapshot_bytes()
        cnt, at = b.alive_count()
        assert at == turns * steps
        assert cnt == int((out == 255).sum())
        return out, p


@pytest.mark.parametrize("turns", [1, 2, 9, 100])
@pytest.mark.parametrize("W,H", [(2048, 2048), (4096, 4096), (8192, 8192), (8192, 1000), (4096, 777), (2048, 512),
                                 (4096, 5120)])
def test_pipe_matches_oracle(coracle, W, H, turns):
    board = coracle.fill_random(W, H, 0x5EED0061 + W + H + turns)
    want = coracle.run(board, turns)
    got, p = run_pipe(board, turns)
    assert p["pipe_launches"] == 1 and p["persist_launches"] == 1 and p["kernel_variant"] == 5, p
    assert p["words_per_lane"] == WPL_OF[W]
    assert np.array_equal(got, want)


@pytest.mark.parametrize("W,cus", [(2048, 1), (2048, 2), (2048, 3), (2048, 7), (4096, 3), (8192, 7), (8192, 64)])
def test_pipe_band_counts(coracle, W, cus):
    """One band (its own band below), two, three, uneven bands; the 70 turns
    run past the 32-slot edge window (the econs flow control).  (persistent 1:
    with few CUs the per-launch kernels would otherwise be planned.)"""
    H = 2 * cus + 301
    board = coracle.fill_random(W, H, 0x5EED0062 + W + cus)
    turns = 70
    want = coracle.run(board, turns)
    got, p = run_pipe(board, turns, cu_count=cus, persistent=1)
    assert p["pipe_launches"] == 1
    assert np.array_equal(got, want)


def test_pipe_does_not_fit_tall_bands():
    """A band's rows must fit one workgroup's LDS (8192-wide rows: at most ~60
    a band): with two bands of 150 rows the step runs another kernel."""
    with golhip.Board(8192, 300) as b:
        b.set_option("lds_pipe", 1)
        b.set_option("persistent", 1)
        b.set_option("cu_count", 2)
        b.fill_random(3)
        b.step(5)
        assert b.perf()["pipe_launches"] == 0


@pytest.mark.parametrize("turns", [3, 7, 8, 15, 16, 17, 33, 257])
def test_pipe_turn_counts(coracle, turns):
    """Fewer turns than waves (idle waves), whole and partial eight-turn cycles."""
    board = coracle.fill_random(4096, 1024, 0x5EED0063 + turns)
    want = coracle.run(board, turns)
    got, p = run_pipe(board, turns)
    assert np.array_equal(got, want)


def test_pipe_two_row_bands(coracle):
    """Bands of exactly two rows (256 CUs x 2 rows): every row of a turn is an edge row."""
    board = coracle.fill_random(8192, 512, 0x5EED0064)
    want = coracle.run(board, 41)
    got, p = run_pipe(board, 41)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("xcd", [0, 1])
def test_pipe_steps_and_xcd_order(coracle, xcd):
    """Several steps on one handle (the board shifts by the turns each launch,
    rows land where the torus puts them) with and without the XCD band order."""
    board = coracle.fill_random(8192, 2048, 0x5EED0065 + xcd)
    want = coracle.run(board, 3 * 37)
    got, p = run_pipe(board, 37, steps=3, lds_xcd=xcd)
    assert p["pipe_launches"] == 3
    assert np.array_equal(got, want)


def test_pipe_glider_crosses_bands_and_wrap():
    """A glider travels down-right across many bands and both wraps: after
    4k turns it sits k cells further along each axis (exact positions)."""
    W, H = 4096, 600
    board = np.zeros((H, W), dtype=np.uint8)
    for y, x in [(0, 1), (1, 2), (2, 0), (2, 1), (2, 2)]:  # moves (+1, +1) every 4 turns
        board[(y + 590) % H, (x + 4090) % W] = 255
    got, p = run_pipe(board, 4 * 50)
    want = np.zeros_like(board)
    for y, x in [(0, 1), (1, 2), (2, 0), (2, 1), (2, 2)]:
        want[(y + 590 + 50) % H, (x + 4090 + 50) % W] = 255
    assert np.array_equal(got, want)


def test_pipe_timeout_restores_and_reruns(coracle):
    """A 1-us wait bound makes the launch time out: every wave drains, the
    host restores the board and re-runs the step on the per-launch kernels;
    the result is still exact."""
    board = coracle.fill_random(8192, 4096, 0x5EED0066)
    want = coracle.run(board, 50)
    with golhip.Board(8192, 4096) as b:
        b.set_option("lds_pipe", 1)
        b.set_option("persist_timeout_us", 1)
        b.load_bytes(board)
        b.step(50)
        p = b.perf()
        got = b.snapshot_bytes()
    assert p["persist_fallbacks"] == 1 and p["pipe_launches"] == 0
    assert np.array_equal(got, want)


def test_pipe_off_by_default():
    """K1t runs only when asked for (it is slower than K1r at every width it
    runs): the default plan of its widths stays on K1r."""
    for W, H in [(8192, 8192), (4096, 4096)]:
        with golhip.Board(W, H) as b:
            b.fill_random(1)
            b.step(20)
            p = b.perf()
            assert p["pipe_launches"] == 0 and p["lds_launches"] == 1
