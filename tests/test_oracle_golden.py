"""Pin the CPU oracle against the reference's own fixtures.

The reference's golden data (check/images/*.pgm and check/alive/*.csv) is
committed as fixtures in tests/golden/ (see make_golden.py).  Every oracle the
GPU parity tests trust is checked here first:

* the numpy restatement (oracle.step_np) and the per-cell C restatement
  (oracle/gol_oracle.c) reproduce all 9 golden boards (TestGol/TestPgm matrix,
  gol_test.go:15-47, pgm_test.go:10-42);
* both reproduce all 3 x 10,000 alive counts (count_test.go:17-69,
  sdl_test.go:93-128);
* the worker-pool port (the CPU baseline) gives the same boards;
* PGM bytes rebuilt from the fixtures are byte-identical to the reference
  files (SHA-256 from manifest.json), so io.go's writer format is pinned.
"""
import hashlib

import numpy as np
import pytest

from oracle.oracle import (COracle, alive_cells_np, fill_random_np, flips_np, pack_bits,
                           parse_pgm, pgm_bytes, run_np, step_np, unpack_bits)

CHECKS = [(16, 0), (16, 1), (16, 100), (64, 0), (64, 1), (64, 100), (512, 0), (512, 1), (512, 100)]


@pytest.fixture(scope="module")
def coracle():
    return COracle()


def board(fixtures, key, n):
    return unpack_bits(fixtures[key], n)


@pytest.mark.parametrize("n", [16, 64, 128, 256, 512])
def test_pgm_roundtrip_bytes(fixtures, manifest, n):
    """Input images rebuild byte-identically (io.go:52-59 header format)."""
    b = board(fixtures, f"image_{n}", n)
    data = pgm_bytes(b)
    m = manifest[f"image_{n}"]
    assert data[: len(m["header"])] == m["header"].encode()
    assert hashlib.sha256(data).hexdigest() == m["sha256"]
    assert np.array_equal(parse_pgm(data, n, n), b)


@pytest.mark.parametrize("n,t", CHECKS)
def test_golden_board_bytes(fixtures, manifest, n, t):
    data = pgm_bytes(board(fixtures, f"check_{n}x{t}", n))
    assert hashlib.sha256(data).hexdigest() == manifest[f"check_{n}x{t}"]["sha256"]


@pytest.mark.parametrize("n,t", CHECKS)
def test_numpy_oracle_matches_golden_boards(fixtures, n, t):
    out = run_np(board(fixtures, f"image_{n}", n), t)
    assert np.array_equal(pack_bits(out), fixtures[f"check_{n}x{t}"])


@pytest.mark.parametrize("n,t", CHECKS)
def test_c_oracle_matches_golden_boards(fixtures, coracle, n, t):
    out = coracle.run(board(fixtures, f"image_{n}", n), t)
    assert np.array_equal(pack_bits(out), fixtures[f"check_{n}x{t}"])


@pytest.mark.parametrize("n,t", [(16, 100), (64, 100), (512, 100)])
@pytest.mark.parametrize("threads", [1, 8])
def test_workerpool_port_matches_golden(fixtures, coracle, n, t, threads):
    out, flips = coracle.run_workerpool(board(fixtures, f"image_{n}", n), t, threads)
    assert np.array_equal(pack_bits(out), fixtures[f"check_{n}x{t}"])
    assert flips > 0


@pytest.mark.parametrize("n", [16, 64])
def test_c_oracle_alive_counts_10000(fixtures, coracle, n):
    _, counts = coracle.run_counts(board(fixtures, f"image_{n}", n), 10000)
    assert np.array_equal(counts, fixtures[f"alive_{n}"][1:])


def test_numpy_oracle_alive_counts_512_10000(fixtures):
    """All 10,000 rows of check/alive/512x512.csv (count_test.go:45-55), plus the
    post-10000 rule (even -> 5565, odd -> 5567, count_test.go:45-51)."""
    b = board(fixtures, "image_512", 512)
    exp = fixtures["alive_512"]
    for t in range(1, 10003):
        b = step_np(b)
        got = int((b == 255).sum())
        if t <= 10000:
            assert got == exp[t], t
        else:
            assert got == (5565 if t % 2 == 0 else 5567), t


@pytest.mark.parametrize("n", [16, 64, 512])
def test_initial_alive_matches_csv_turn0(fixtures, n):
    assert int((board(fixtures, f"image_{n}", n) == 255).sum()) == fixtures[f"alive_{n}"][0]


def test_alive_cells_and_flips_agree(fixtures, coracle):
    b0 = board(fixtures, "image_512", 512)
    b1 = step_np(b0)
    assert np.array_equal(coracle.alive_cells(b1), alive_cells_np(b1))
    assert np.array_equal(coracle.flips(b0, b1), flips_np(b0, b1))
    # 512x512 turn 1: flips == |alive(1) - alive(0)| parity sanity
    assert len(flips_np(b0, b1)) >= abs(int((b1 == 255).sum()) - int((b0 == 255).sum()))


def test_fill_random_c_equals_numpy(coracle):
    for (W, H, seed) in [(64, 32, 1), (100, 7, 0x5EED0001), (512, 512, 0x5EED0005)]:
        a = coracle.fill_random(W, H, seed)
        assert np.array_equal(a, fill_random_np(W, H, seed))
        frac = (a == 255).mean()
        assert 0.2 < frac < 0.3


def test_pack_unpack_roundtrip():
    rng = np.random.default_rng(0)
    for (H, W) in [(3, 16), (5, 33), (4, 64), (2, 100)]:
        b = np.where(rng.random((H, W)) < 0.4, 255, 0).astype(np.uint8)
        assert np.array_equal(unpack_bits(pack_bits(b), W), b)


@pytest.mark.parametrize("n,t", [(64, 0), (64, 1), (64, 100), (512, 0), (512, 1), (512, 100)])
def test_fastcpu_comparator_matches_golden_boards(fixtures, coracle, n, t):
    """The bit-packed OpenMP CPU comparator (oracle/gol_fastcpu.c, timed by bench.py) is exact too."""
    out = coracle.run_fast(board(fixtures, f"image_{n}", n), t, threads=3)
    assert np.array_equal(pack_bits(out), fixtures[f"check_{n}x{t}"])


@pytest.mark.parametrize("W,H,turns,threads", [(64, 3, 7, 1), (128, 37, 13, 4), (1024, 99, 20, 8), (192, 200, 33, 5)])
def test_fastcpu_comparator_matches_oracle(coracle, W, H, turns, threads):
    b = coracle.fill_random(W, H, 0x5EED0042 + W)
    assert np.array_equal(coracle.run_fast(b, turns, threads), coracle.run_exact(b, turns))


@pytest.mark.parametrize("W,H,turns", [(4096, 2048, 3), (65536, 96, 2), (128, 8192, 4)])
def test_fastcpu_comparator_matches_oracle_wide_and_tall(coracle, W, H, turns):
    """the large GPU parity cases compare against the bit-packed
    comparator, so pin it to the per-cell oracle on boards as wide and as tall
    as those cases (word and row wrap on a 4096 x 2048 board, the 65536-wide
    rows of configs[2], an 8192-row column)."""
    b = coracle.fill_random(W, H, 0x5EED0046 + W + H)
    assert np.array_equal(coracle.run_fast(b, turns, 8), coracle.run_exact(b, turns))


def test_oracle_run_switches_to_the_comparator_on_large_cases(coracle):
    """run() answers large cases with the comparator: same board as the per-cell oracle."""
    b = coracle.fill_random(2048, 1000, 0x5EED0044)
    assert 2048 * 1000 * 10 >= coracle.FAST_CELL_UPDATES
    assert np.array_equal(coracle.run(b, 10), coracle.run_exact(b, 10))


# ------------------------------------------- full-size fixture generator (make_fullsize.py)
@pytest.mark.parametrize("W,H,seed,row0", [(128, 64, 1, 0), (1024, 300, 0x5EED0005, 0), (640, 17, 7, 33)])
def test_fastcpu_fixture_helpers(coracle, W, H, seed, row0):
    """fastcpu_fill_random / _hash / _popcount (the full-size fixture generator)
    equal the per-cell oracle's board and the host digest of golhip_board_hash."""
    import golhip
    b = coracle.fill_random(W, H + row0, seed)[row0:]
    w = coracle.fill_random64(W, H, seed, 4, row0=row0)
    assert np.array_equal(coracle.unpack64(w, W), b)
    assert coracle.hash64(w, W, 4, word0=row0 * (W // 32)) == golhip.board_hash_np(pack_bits(b), row0=row0)
    assert coracle.popcount64(w, W, 4) == int((b == 255).sum())
    coracle.run_fast_words(w, W, 9, 3)
    want = coracle.run(coracle.fill_random(W, H, seed), 9) if row0 == 0 else None
    if want is not None:
        assert coracle.hash64(w, W, 2) == golhip.board_hash_np(pack_bits(want))


def test_fullsize_fixture_file_is_consistent():
    """tests/golden/fullsize.json covers every GPU config of BASELINE.json and
    its turn-0 entries equal the generator rule (digest of the fresh board)."""
    import json
    import os
    path = os.path.join(os.path.dirname(__file__), "golden", "fullsize.json")
    with open(path) as f:
        js = json.load(f)
    assert {"c1", "c2", "c3", "c4"} <= set(js)
    assert js["c1"]["width"] == 16384 and "10000" in js["c1"]["checkpoints"]
    assert js["c2"]["width"] == 65536 and "1000" in js["c2"]["checkpoints"]
    assert js["c3"]["width"] == 262144 and "100" in js["c3"]["checkpoints"]
    assert js["c4"]["width"] == 5120 and len(js["c4"]["flip_counts"]) == js["c4"]["turns"] == 50
    # configs[3]'s count exceeds 2^31: the 64-bit count path matters
    assert js["c3"]["checkpoints"]["0"]["alive"] > 2 ** 31
    # 16384^2 turn 0 recomputed here (0.3 s)
    co = COracle()
    w = co.fill_random64(16384, 16384, js["c1"]["seed"], 8)
    assert f"{co.hash64(w, 16384, 8):016x}" == js["c1"]["checkpoints"]["0"]["hash"]
    assert co.popcount64(w, 16384, 8) == js["c1"]["checkpoints"]["0"]["alive"]
    co.run_fast_words(w, 16384, 1, 8)
    assert f"{co.hash64(w, 16384, 8):016x}" == js["c1"]["checkpoints"]["1"]["hash"]
