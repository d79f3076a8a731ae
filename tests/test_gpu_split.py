"""GPU parity of split tiling (option "split", gol_kernels.hip K1s) against the C oracle.

K1s computes each launch with two kernels: A streams regions of input rows
from both ends (two waves meeting where their claims meet, possibly streaming
0-2 rows twice) and exports the edge rows of every generation; B computes the
triangles between the bands from those exports.  Bit-exact against
oracle/gol_fastcpu.c (the C restatement pinned to the reference's fixtures in
tests/test_oracle_golden.py) for every instantiated (depth, words per lane),
for boards with one region up to many, odd heights (regions of unequal
length, claims ending in partial groups) and the full-size BASELINE fixtures.
"""
import numpy as np
import pytest

from oracle.oracle import COracle

pytestmark = pytest.mark.gpu

golhip = pytest.importorskip("golhip")

from test_gpu_fullsize import full, run_checkpoints  # noqa: E402,F401


@pytest.fixture(scope="module")
def coracle():
    return COracle()


def run_split(board, turns, depth, wpl, rows_per_wave=0):
    H, W = board.shape
    with golhip.Board(W, H) as b:
        b.set_option("persistent", 0)
        b.set_option("wpl", wpl)
        b.set_option("split", 1)
        b.set_option("skew", 0)
        b.set_tb_depth(depth)
        b.set_rows_per_wave(rows_per_wave)
        b.load_bytes(board)
        b.step(turns)
        p = b.perf()
        out = b.snapshot_bytes()
        cnt, at = b.alive_count()
        assert at == turns
        assert cnt == int((out == 255).sum())
        return out, p


SPLIT = [(8, 2), (12, 2), (16, 2), (20, 2), (8, 4), (9, 4), (16, 1), (32, 1)]


@pytest.mark.parametrize("depth,wpl", SPLIT)
@pytest.mark.parametrize("W,H", [(2048, 1024), (4096, 777), (1024, 200), (8192, 331), (3968, 2500)])
def test_split_matches_oracle(coracle, depth, wpl, W, H):
    if W % (32 * wpl):
        pytest.skip("width not a multiple of the lane chunk")
    board = coracle.fill_random(W, H, 0x5EED0021 + W + H)
    turns = 2 * depth + 3  # two split launches and a remainder on the other kernels
    want = coracle.run(board, turns)
    got, p = run_split(board, turns, depth, wpl)
    assert p["kernel_variant"] in (1, 2)
    assert 1 <= p["split_launches"] <= p["step_launches"]  # the full-depth launches split, the remainder may not
    assert np.array_equal(got, want)


@pytest.mark.parametrize("depth,wpl", SPLIT)
def test_split_single_region(coracle, depth, wpl):
    """A board just tall enough for one region: the torus seam is the region end."""
    P0 = 3 * ((2 * depth + 2) // 3)
    H = 2 * (P0 + 3) + 4
    W = 4096
    board = coracle.fill_random(W, H, 0x5EED0022 + depth)
    want = coracle.run(board, depth)
    got, p = run_split(board, depth, depth, wpl)
    assert p["kernel_variant"] == 2
    assert np.array_equal(got, want)


@pytest.mark.parametrize("depth,wpl", [(16, 2), (20, 2), (8, 4), (9, 4)])
@pytest.mark.parametrize("H", [4096 + 1, 4096 + 2, 4096 + 3, 5000])
def test_split_many_regions_every_remainder(coracle, depth, wpl, H):
    """Region lengths of every residue mod 3 (the meeting claims end in 1-, 2- and 3-row grants)."""
    W = 4096
    board = coracle.fill_random(W, H, 0x5EED0023 + H)
    turns = 5 * depth
    want = coracle.run(board, turns)
    got, _ = run_split(board, turns, depth, wpl)
    assert np.array_equal(got, want)


def test_split_falls_back_below_one_region(coracle):
    """Boards shorter than one region run on the per-launch kernels."""
    board = coracle.fill_random(1024, 40, 0x5EED0024)
    want = coracle.run(board, 60)
    got, p = run_split(board, 60, 20, 2)
    assert p["kernel_variant"] == 1 and p["split_launches"] == 0
    assert np.array_equal(got, want)


# ---------------------------------------------------------------- full-size BASELINE fixtures
def test_split_config1_16384(full):
    run_checkpoints(full, "c1", split=1, persistent=0, skew=0)


def test_split_config2_65536(full):
    run_checkpoints(full, "c2", split=1, skew=0)


def test_split_config3_262144(full):
    run_checkpoints(full, "c3", split=1, skew=0)
