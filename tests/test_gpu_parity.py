"""GPU parity: libgolhip.so (HIP, gfx950) against the oracle and the golden fixtures.

Bar: bit-exact (integer / bit work).  Mirrors the reference's tests:
  TestGol  (gol_test.go:15-47)  final alive set for 16/64/512 x turns {0,1,100}
  TestPgm  (pgm_test.go:10-42)  output PGM equals check/images (here: SHA-256 of the bytes)
  TestAlive(count_test.go:17-69) alive counts vs check/alive/*.csv (every turn 1..10000)
  TestSdl  (sdl_test.go:93-128)  CellFlipped stream applied to a shadow board
and adds what the GPU design needs: every fused depth / strip height, odd
widths, multi-strip (row-strip decomposition) runs and full-size property
checks (BASELINE configs) through the board digest.
"""
import hashlib

import numpy as np
import pytest

from oracle.oracle import (COracle, alive_cells_np, fill_random_np, flips_np, pack_bits, pgm_bytes, run_np,
                           step_np, unpack_bits)

pytestmark = pytest.mark.gpu

golhip = pytest.importorskip("golhip")

CHECKS = [(16, 0), (16, 1), (16, 100), (64, 0), (64, 1), (64, 100), (512, 0), (512, 1), (512, 100)]
DEPTHS = [1, 2, 4, 6, 8, 12, 16, 20, 24, 32]


@pytest.fixture(scope="module")
def coracle():
    return COracle()


def img(fixtures, n):
    return unpack_bits(fixtures[f"image_{n}"], n)


def run_gpu(board, turns, depth=16, rows_per_wave=0, **options):
    H, W = board.shape
    with golhip.Board(W, H) as b:
        for k, v in options.items():
            b.set_option(k, v)
        b.set_tb_depth(depth)
        b.set_rows_per_wave(rows_per_wave)
        b.load_bytes(board)
        b.step(turns)
        out = b.snapshot_bytes()
        cnt, at = b.alive_count()
        assert at == turns
        assert cnt == int((out == 255).sum())
        return out


# ---------------------------------------------------------------- TestGol / TestPgm
@pytest.mark.parametrize("n,t", CHECKS)
def test_gol_final_alive_cells(fixtures, n, t):
    """FinalTurnComplete.Alive == golden alive set (gol_test.go:42, :58-86)."""
    with golhip.Board(n, n) as b:
        b.load_bytes(img(fixtures, n))
        b.step(t)
        got = b.alive_cells()
    expected = alive_cells_np(unpack_bits(fixtures[f"check_{n}x{t}"], n))
    assert np.array_equal(got, expected)


@pytest.mark.parametrize("n,t", CHECKS)
def test_pgm_output_bytes(fixtures, manifest, n, t):
    """out/NxNxT.pgm byte-identical to check/images (io.go:52-81 writer format)."""
    out = run_gpu(img(fixtures, n), t)
    assert hashlib.sha256(pgm_bytes(out)).hexdigest() == manifest[f"check_{n}x{t}"]["sha256"]


@pytest.mark.parametrize("n", [128, 256])
@pytest.mark.parametrize("t", [1, 100, 1000])
def test_unchecked_images_vs_oracle(fixtures, n, t):
    """128x128 and 256x256 have no goldens in the reference: the oracle is the check."""
    board = img(fixtures, n)
    assert np.array_equal(run_gpu(board, t), run_np(board, t))


# ---------------------------------------------------------------- TestAlive
@pytest.mark.parametrize("n", [16, 64, 512])
def test_alive_counts_every_turn(fixtures, n):
    """check/alive/NxN.csv at every turn 1..10000, plus count_test's post-10000 rule."""
    exp = fixtures[f"alive_{n}"]
    with golhip.Board(n, n) as b:
        b.load_bytes(img(fixtures, n))
        assert b.alive_count() == (exp[0], 0)
        for t in range(1, 10001):
            b.step(1)
            cnt, at = b.alive_count()
            assert at == t and cnt == exp[t], (t, cnt, exp[t])
        if n == 512:
            for t in range(10001, 10005):
                b.step(1)
                cnt, _ = b.alive_count()
                assert cnt == (5565 if t % 2 == 0 else 5567)


@pytest.mark.parametrize("depth", DEPTHS)
def test_alive_counts_fused_launches(fixtures, depth):
    """Counts sampled at fused-launch boundaries (the ticker path) match the CSV."""
    exp = fixtures["alive_512"]
    with golhip.Board(512, 512) as b:
        b.set_tb_depth(depth)
        b.load_bytes(img(fixtures, 512))
        t = 0
        for chunk in [1, 3, 32, 64, 100, 1000, 2800]:
            b.step(chunk)
            t += chunk
            assert b.alive_count() == (exp[t], t)


# ---------------------------------------------------------------- TestSdl
def test_sdl_flip_stream_512(fixtures):
    """CellFlipped events applied to a shadow board reproduce every alive count
    (sdl_test.go:58, :107-116); flips also equal the oracle's diff list."""
    board = img(fixtures, 512)
    exp = fixtures["alive_512"]
    shadow = np.zeros((512, 512), dtype=np.uint8)
    with golhip.Board(512, 512) as b:
        b.load_bytes(board)
        init = b.alive_cells()                      # initial CellFlipped (distributor.go:72-80)
        shadow[init[:, 1], init[:, 0]] ^= 0xFF
        prev = board
        for t in range(1, 101):
            b.step(1, want_flips=True)
            fl = b.flips()
            shadow[fl[:, 1], fl[:, 0]] ^= 0xFF
            assert int((shadow == 255).sum()) == exp[t]
            nxt = step_np(prev)
            assert np.array_equal(fl, flips_np(prev, nxt))
            prev = nxt
        assert np.array_equal(shadow, b.snapshot_bytes())


@pytest.mark.parametrize("n", [64, 256])
def test_flips_match_oracle_each_turn(fixtures, n):
    board = img(fixtures, n)
    with golhip.Board(n, n) as b:
        b.load_bytes(board)
        for _ in range(20):
            nxt = step_np(board)
            b.step(1, want_flips=True)
            assert np.array_equal(b.flips(), flips_np(board, nxt))
            board = nxt


def test_flips_after_multi_turn_step(fixtures):
    """want_flips with n > 1: flips of the last turn only."""
    board = img(fixtures, 512)
    with golhip.Board(512, 512) as b:
        b.load_bytes(board)
        b.step(37, want_flips=True)
        a = run_np(board, 36)
        assert np.array_equal(b.flips(), flips_np(a, step_np(a)))


@pytest.mark.parametrize("n,batches", [(512, [1, 7, 32, 60]), (256, [20, 1, 13]), (64, [64, 64]), (48, [9, 4])])
def test_step_flips_batched_stream(fixtures, n, batches):
    """golhip_step_flips: every turn's list of a batch, concatenated, equals the
    oracle's per-turn diffs; the shadow board replays the alive-count CSV
    (sdl_test.go:107-116) where the reference ships one.  48 x 48 takes the
    generic-width kernel."""
    if n == 48:
        rng = np.random.default_rng(48)
        board = np.where(rng.random((n, n)) < 0.35, 255, 0).astype(np.uint8)
    else:
        board = img(fixtures, n)
    exp = fixtures.get(f"alive_{n}")
    shadow = board.copy()
    t = 0
    with golhip.Board(n, n) as b:
        b.load_bytes(board)
        for k in batches:
            xy, counts = b.step_flips(k, cap=k * n * n)
            assert len(counts) == k and int(counts.sum()) == len(xy)
            off = 0
            for c in counts:
                nxt = step_np(board)
                assert np.array_equal(xy[off:off + int(c)], flips_np(board, nxt))
                shadow[xy[off:off + int(c), 1], xy[off:off + int(c), 0]] ^= 0xFF
                board, off, t = nxt, off + int(c), t + 1
                if exp is not None and t < len(exp):
                    assert int((shadow == 255).sum()) == exp[t]
            assert b.alive_count() == (int((board == 255).sum()), t)
        assert np.array_equal(b.snapshot_bytes(), board)
        assert np.array_equal(shadow, board)


def test_step_flips_capacity_and_edges(fixtures):
    """cap too small: ERANGE with the total, the first cap pairs kept, the board
    still advanced; zero turns; a still board gives empty lists."""
    board = img(fixtures, 256)
    with golhip.Board(256, 256) as b:
        b.load_bytes(board)
        xy_all = [flips_np(run_np(board, i), run_np(board, i + 1)) for i in range(5)]
        want = np.concatenate(xy_all)
        buf = np.zeros((100, 2), dtype=np.int32)
        with pytest.raises(golhip.GolHipError) as e:
            b.step_flips(5, cap=100, xy=buf)
        assert e.value.code == golhip.GOLHIP_ERANGE
        assert np.array_equal(buf, want[:100])
        assert np.array_equal(b.snapshot_bytes(), run_np(board, 5))
        xy, counts = b.step_flips(0, cap=0)
        assert len(xy) == 0 and len(counts) == 0
        assert b.alive_count()[1] == 5
    z = np.zeros((64, 64), dtype=np.uint8)
    with golhip.Board(64, 64) as b:
        b.load_bytes(z)
        xy, counts = b.step_flips(10, cap=16)
        assert len(xy) == 0 and list(counts) == [0] * 10


# ---------------------------------------------------------------- kernel geometry sweeps
@pytest.mark.parametrize("depth", DEPTHS)
@pytest.mark.parametrize("rpw", [0, 1, 2, 5, 37, 512])
@pytest.mark.parametrize("fill_skip", [0, 1])
@pytest.mark.parametrize("wpl", [1, 2, 4])
def test_depth_and_strip_height_invariance(fixtures, depth, rpw, fill_skip, wpl):
    board = img(fixtures, 256)
    assert np.array_equal(run_gpu(board, 70, depth, rpw, fill_skip=fill_skip, wpl=wpl), run_np(board, 70))


@pytest.mark.parametrize("W,H", [(32, 1), (32, 3), (64, 2), (96, 7), (2016, 9), (1984, 33), (4000 - 4000 % 32, 40),
                                 (8192, 5), (320, 1000), (6272, 70), (7936, 20), (8064, 12), (128, 64)])
@pytest.mark.parametrize("depth", [1, 8, 12, 20, 32])
@pytest.mark.parametrize("wpl", [1, 2, 4])
def test_random_shapes(W, H, depth, wpl):
    """Widths that are 1..many tiles (62 x wpl stored words/tile), heights below the depth."""
    rng = np.random.default_rng(W * 7 + H)
    board = np.where(rng.random((H, W)) < 0.3, 255, 0).astype(np.uint8)
    assert np.array_equal(run_gpu(board, 45, depth, 16, wpl=wpl), run_np(board, 45))


@pytest.mark.parametrize("W,H", [(16, 16), (1, 1), (3, 5), (17, 9), (48, 20), (100, 37), (33, 64)])
def test_generic_width_kernel(W, H):
    """Widths that are not a multiple of 32 take the generic kernel."""
    rng = np.random.default_rng(W + 100 * H)
    board = np.where(rng.random((H, W)) < 0.35, 255, 0).astype(np.uint8)
    out = run_gpu(board, 23)
    assert np.array_equal(out, run_np(board, 23))


def test_non_binary_bytes_follow_reference_rule():
    """alive <=> byte == 255 (distributor.go:363, :411): other values are dead."""
    rng = np.random.default_rng(5)
    board = rng.choice(np.array([0, 1, 128, 254, 255], dtype=np.uint8), size=(64, 128))
    out = run_gpu(board, 3)
    assert np.array_equal(out, run_np(board, 3))


def test_zero_turns_and_empty_board():
    z = np.zeros((64, 64), dtype=np.uint8)
    assert np.array_equal(run_gpu(z, 0), z)
    assert np.array_equal(run_gpu(z, 10), z)
    with golhip.Board(64, 64) as b:
        b.load_bytes(z)
        assert len(b.alive_cells()) == 0
        b.step(1, want_flips=True)
        assert len(b.flips()) == 0


# ---------------------------------------------------------------- synthetic boards, digest
def test_fill_random_matches_oracle(coracle):
    for (W, H, seed) in [(64, 32, 1), (100, 7, 0x5EED0001), (1024, 300, 0x5EED0005)]:
        with golhip.Board(W, H) as b:
            b.fill_random(seed)
            assert np.array_equal(b.snapshot_bytes(), coracle.fill_random(W, H, seed))


def test_board_hash_matches_host():
    rng = np.random.default_rng(9)
    board = np.where(rng.random((300, 640)) < 0.5, 255, 0).astype(np.uint8)
    with golhip.Board(640, 300) as b:
        b.load_bytes(board)
        assert b.board_hash() == golhip.board_hash_np(pack_bits(board))


def test_random_2048_vs_c_oracle(coracle):
    board = coracle.fill_random(2048, 2048, 0x5EED0001)
    with golhip.Board(2048, 2048) as b:
        b.fill_random(0x5EED0001)
        b.step(40)
        got = b.snapshot_bytes()
    assert np.array_equal(got, coracle.run(board, 40))


# ---------------------------------------------------------------- row strips (multi-GPU decomposition)
@pytest.mark.parametrize("splits", [[64], [32, 32], [10, 20, 34], [1, 1, 62], [16, 16, 16, 16]])
@pytest.mark.parametrize("depth", [1, 4, 32])
def test_group_strips_equal_single_board(fixtures, splits, depth):
    """n strips of one torus, halos exchanged every launch, == the whole board."""
    board = img(fixtures, 64)
    strips, r = [], 0
    for rows in splits:
        s = golhip.Board(64, 64, row0=r, rows=rows)
        s.set_tb_depth(depth)
        s.load_bytes(board[r:r + rows])
        strips.append(s)
        r += rows
    golhip.group_step(strips, 100)
    got = np.concatenate([s.snapshot_bytes() for s in strips])
    assert np.array_equal(got, unpack_bits(fixtures["check_64x100"], 64))
    assert sum(s.alive_count()[0] for s in strips) == fixtures["alive_64"][100]
    digest = sum(s.board_hash() for s in strips) % (1 << 64)
    assert digest == golhip.board_hash_np(pack_bits(got))
    for s in strips:
        s.close()


def test_group_strips_large_random_hash():
    """Config-3 shape in miniature: 8 strips of a 8192^2 torus == one board."""
    W = H = 8192
    seed = 0x5EED0002
    with golhip.Board(W, H) as one:
        one.fill_random(seed)
        one.step(64)
        ref = one.board_hash()
    strips = [golhip.Board(W, H, row0=i * H // 8, rows=H // 8) for i in range(8)]
    for s in strips:
        s.fill_random(seed)
    golhip.group_step(strips, 64)
    assert sum(s.board_hash() for s in strips) % (1 << 64) == ref
    for s in strips:
        s.close()


# ---------------------------------------------------------------- full-size properties
@pytest.mark.parametrize("N,turns", [(16384, 256), (65536, 32), (65536, 100)])
def test_full_size_depth_invariance(N, turns):
    """BASELINE configs 2/3 at full size: fused depths 32 / 16 / 1 agree (digest + count);
    65536^2 x 100 turns is the bench step (launches of 16, 16, 16, 16, 12, 12, 12 turns)."""
    res = []
    for depth in (32, 16, 1):
        with golhip.Board(N, N) as b:
            b.set_tb_depth(depth)
            b.fill_random(0x5EED0001 if N == 16384 else 0x5EED0002)
            b.step(turns)
            res.append((b.board_hash(), b.alive_count()))
    assert res[0] == res[1] == res[2]


def test_full_size_fill_sample_rows(coracle):
    """Sampled rows of the 16384^2 synthetic board equal the host generator."""
    N, seed = 16384, 0x5EED0001
    with golhip.Board(N, N) as b:
        b.fill_random(seed)
        bits = b.snapshot_bits()
    for r in (0, 1, 777, N - 1):
        idx = np.arange(N, dtype=np.uint64) + np.uint64(r * N)
        from oracle.oracle import splitmix64_np
        row = np.where((splitmix64_np(np.uint64(seed) ^ idx) & np.uint64(3)) == 0, 255, 0).astype(np.uint8)
        assert np.array_equal(unpack_bits(bits[r:r + 1], N)[0], row)


# ---------------------------------------------------------------- persistent kernel (K1p)
@pytest.mark.parametrize("N,depth", [(1024, 4), (2048, 8), (2048, 16), (4096, 32), (3968, 16)])
@pytest.mark.parametrize("wpl", [1, 2])
def test_persistent_matches_oracle(coracle, N, depth, wpl):
    """Resident multi-super-step kernel vs the C oracle (and vs the per-launch path)."""
    board = coracle.fill_random(N, N // 2, 0x5EED0007)
    want = coracle.run(board, 3 * depth + 5)
    outs = {}
    for persistent in (1, 0):
        with golhip.Board(N, N // 2) as b:
            b.set_option("wpl", wpl)
            b.set_option("persistent", persistent)
            b.set_tb_depth(depth)
            b.load_bytes(board)
            b.step(3 * depth + 5)
            outs[persistent] = b.snapshot_bytes()
            assert b.alive_count() == (int((want == 255).sum()), 3 * depth + 5)
    assert np.array_equal(outs[1], want) and np.array_equal(outs[0], want)


@pytest.mark.parametrize("N,turns", [(16384, 512), (65536, 64)])
def test_persistent_full_size_matches_per_launch(N, turns):
    res = []
    for persistent in (1, 0):
        with golhip.Board(N, N) as b:
            b.set_option("persistent", persistent)
            b.fill_random(0x5EED0001)
            b.step(turns)
            res.append((b.board_hash(), b.alive_count()))
    assert res[0] == res[1]


@pytest.mark.parametrize("N,depth,wpl,nw", [(2048, 8, 1, 8), (2048, 16, 1, 8), (4096, 8, 2, 8), (4096, 16, 2, 8),
                                            (1024, 8, 1, 8), (4096, 4, 2, 16)])
def test_persistent_waves_per_workgroup(coracle, N, depth, wpl, nw):
    """Persistent kernel with 8 / 16 resident waves per workgroup vs the C oracle."""
    board = coracle.fill_random(N, N // 2, 0x5EED0008)
    turns = 4 * depth + 3
    want = coracle.run(board, turns)
    with golhip.Board(N, N // 2) as b:
        b.set_option("persistent", 1)
        b.set_option("lds_band", 0)  # K1p itself (K1r: tests/test_gpu_lds.py)
        b.set_option("wpl", wpl)
        b.set_option("persist_waves", nw)
        b.set_tb_depth(depth)
        b.load_bytes(board)
        b.step(turns)
        assert b.perf()["persist_launches"] == 1
        assert np.array_equal(b.snapshot_bytes(), want)
        assert b.alive_count() == (int((want == 255).sum()), turns)


# ------------------------------------------------ interleaved pair / quad layouts (wpl = 2, 4)
@pytest.mark.parametrize("W,H", [(1024, 96), (640, 128), (4096, 64), (320, 33)])
@pytest.mark.parametrize("wpl", [2, 4])
def test_interleaved_layout_side_channels(coracle, W, H, wpl):
    """wpl = 2 (4) boards live in the interleaved pair (quad) layout: every
    canonical view (bytes, bits, hash, flips, alive list) must be unaffected,
    including after switching the layout mid-run and after load_bits.  W = 320
    (10 words a row, 33 rows) ends the buffer in half a quad; W % 128 != 0
    runs wpl 4 as wpl 2."""
    board = coracle.fill_random(W, H, 0x5EED000B)
    with golhip.Board(W, H) as b:
        b.set_option("wpl", wpl)
        b.load_bytes(board)
        assert np.array_equal(b.snapshot_bytes(), board)
        assert np.array_equal(b.snapshot_bits(), pack_bits(board))
        assert b.board_hash() == golhip.board_hash_np(pack_bits(board))
        b.step(6, want_flips=True)
        want5 = coracle.run(board, 5)
        want6 = coracle.run(board, 6)
        assert np.array_equal(b.flips(), flips_np(want5, want6))
        assert np.array_equal(b.snapshot_bytes(), want6)
        assert np.array_equal(b.alive_cells(), alive_cells_np(want6))
        assert b.board_hash() == golhip.board_hash_np(pack_bits(want6))
        b.set_option("wpl", 1)      # converted back to canonical at the next step
        b.step(7)
        want13 = coracle.run(board, 13)
        assert np.array_equal(b.snapshot_bits(), pack_bits(want13))
        b.set_option("wpl", wpl)
        b.step(4)
        b.set_option("wpl", 6 - wpl)  # 2 <-> 4 directly
        b.step(5, want_flips=True)
        want21, want22 = coracle.run(board, 21), coracle.run(board, 22)
        assert np.array_equal(b.flips(), flips_np(want21, want22))
        assert np.array_equal(b.snapshot_bytes(), want22)
        b.load_bits(pack_bits(board))
        assert np.array_equal(b.snapshot_bits(), pack_bits(board))
        b.step(22)
        assert np.array_equal(b.snapshot_bytes(), want22)
        assert b.alive_count() == (int((want22 == 255).sum()), 22)


@pytest.mark.parametrize("wpl", [2, 4])
def test_interleaved_fill_random_and_strips(coracle, wpl):
    """fill_random + in-process strips on a wpl = 2 / 4 board vs the C oracle."""
    W, H = 2048, 256
    want = coracle.run(coracle.fill_random(W, H, 0x5EED000C), 40)
    hs = []
    try:
        for r0, rows in ((0, 100), (100, 60), (160, 96)):
            h = golhip.Board(W, H, row0=r0, rows=rows)
            h.set_option("wpl", wpl)
            h.fill_random(0x5EED000C)
            hs.append(h)
        golhip.group_step(hs, 40)
        got = np.concatenate([h.snapshot_bytes() for h in hs])
        assert np.array_equal(got, want)
        assert sum(h.board_hash() for h in hs) & (2**64 - 1) == golhip.board_hash_np(pack_bits(want))
    finally:
        for h in hs:
            h.close()


# ---------------------------------------------------------------- RCCL halo path on one GPU
@pytest.mark.parametrize("W,H,depth", [(512, 512, 16), (512, 512, 4), (1024, 768, 8), (2048, 1024, 32),
                                       (640, 200, 16), (4096, 96, 16), (4096, 40, 16), (1000, 300, 4),
                                       (2048, 2048, 16), (1984, 1500, 8)])
@pytest.mark.parametrize("persistent", [1, 0, -1])
def test_rccl_halo_ring_one_rank(coracle, W, H, depth, persistent):
    """The multi-GPU path (RCCL send/recv of deep halo rows, then the resident
    kernel over the extended rows or per-launch kernels on shrinking ranges)
    run as a one-rank ring over the whole board (option force_halo) vs the C
    oracle."""
    board = coracle.fill_random(W, H, 0x5EED000E)
    turns = 5 * depth + 5
    want = coracle.run(board, turns)
    with golhip.Board(W, H) as b:
        b.comm_init(golhip.unique_id(), 1, 0)
        b.set_option("force_halo", 1)
        b.set_option("persistent", persistent)
        b.set_tb_depth(depth)
        b.load_bytes(board)
        b.step(turns)
        p = b.perf()
        assert p["halo_bytes"] > 0
        if persistent == 0:  # (auto: K1w where its stacks fill the CUs, else the guarded resident kernel)
            assert p["persist_launches"] == 0
        elif W % 32 == 0 and depth >= 4 and H >= 4 * depth:
            assert p["persist_launches"] > 0
        assert np.array_equal(b.snapshot_bytes(), want)
        assert b.alive_count() == (int((want == 255).sum()), turns)
        b.step(1, want_flips=True)
        nxt = coracle.run(want, 1)
        assert np.array_equal(b.flips(), flips_np(want, nxt))


@pytest.mark.parametrize("W,H", [(512, 512), (1024, 300), (100, 64)])
def test_rccl_halo_ring_step_flips(coracle, W, H):
    """golhip_step_flips through the halo path (one RCCL exchange per turn)."""
    board = coracle.fill_random(W, H, 0x5EED0010)
    with golhip.Board(W, H) as b:
        b.comm_init(golhip.unique_id(), 1, 0)
        b.set_option("force_halo", 1)
        b.load_bytes(board)
        xy, counts = b.step_flips(9, cap=9 * W * H)
        off = 0
        for c in counts:
            nxt = coracle.run(board, 1)
            assert np.array_equal(xy[off:off + int(c)], flips_np(board, nxt))
            board, off = nxt, off + int(c)
        assert np.array_equal(b.snapshot_bytes(), board)
        assert b.alive_count() == (int((board == 255).sum()), 9)


@pytest.mark.parametrize("W,H,depth", [(2048, 1024, 16), (4096, 96, 8), (1024, 300, 4)])
def test_rccl_halo_ring_quads(coracle, W, H, depth):
    """The one-rank RCCL ring with four words per lane (interleaved quads,
    launches of at most 8 turns, 16 launches per 128-row exchange)."""
    board = coracle.fill_random(W, H, 0x5EED000F)
    turns = 5 * depth + 5
    want = coracle.run(board, turns)
    with golhip.Board(W, H) as b:
        b.comm_init(golhip.unique_id(), 1, 0)
        b.set_option("force_halo", 1)
        b.set_option("persistent", 0)
        b.set_option("wpl", 4)
        b.set_tb_depth(depth)
        b.load_bytes(board)
        b.step(turns)
        assert b.perf()["halo_bytes"] > 0
        assert np.array_equal(b.snapshot_bytes(), want)
        assert b.alive_count() == (int((want == 255).sum()), turns)


@pytest.mark.parametrize("W,H", [(131072, 2048), (262144, 1024)])
def test_quads_auto_on_wide_boards(W, H):
    """Boards 131072 and 262144 wide pick four words per lane by themselves
    (per-launch path); digest and count equal two words per lane and the
    one-turn launches."""
    res = []
    for wpl, depth in ((0, 16), (2, 16), (0, 1)):
        with golhip.Board(W, H) as b:
            b.set_option("persistent", 0)
            b.set_option("wpl", wpl)
            b.set_tb_depth(depth)
            b.fill_random(0x5EED0003)
            b.step(40)
            res.append((b.board_hash(), b.alive_count(), b.perf()["step_launches"]))
    assert res[0][:2] == res[1][:2] == res[2][:2]
    assert res[0][2] == 5 and res[1][2] == 3  # 5 x 8 turns (quads) vs 16 + 12 + 12 (pairs)


@pytest.mark.parametrize("N,depth,wpl,half", [(2048, 16, 1, 1), (2048, 16, 1, 0), (4096, 8, 2, 1), (2048, 4, 1, 1)])
def test_persistent_half_last_super_step(coracle, N, depth, wpl, half):
    """J D + D/2 turns: one resident launch whose last super-step runs D/2
    turns (persist_half), or a resident launch plus a per-launch kernel."""
    board = coracle.fill_random(N, N, 0x5EED0010)
    turns = 5 * depth + depth // 2
    want = coracle.run(board, turns)
    with golhip.Board(N, N) as b:
        b.set_option("persistent", 1)
        b.set_option("lds_band", 0)  # K1p itself (K1r: tests/test_gpu_lds.py)
        b.set_option("persist_half", half)
        b.set_option("wpl", wpl)
        b.set_tb_depth(depth)
        b.load_bytes(board)
        b.step(turns)
        p = b.perf()
        assert p["persist_launches"] == 1 and p["step_launches"] == (0 if half else 1)
        assert p["persist_turns"] == (turns if half else 5 * depth)
        assert np.array_equal(b.snapshot_bytes(), want)
        assert b.alive_count() == (int((want == 255).sum()), turns)


def test_rccl_halo_ring_full_size():
    """16384^2 through the one-rank RCCL ring (deep halos; resident and per-launch kernels) == the torus kernel."""
    res = []
    for halo in (1, 2, 0):
        with golhip.Board(16384, 16384) as b:
            if halo:
                b.comm_init(golhip.unique_id(), 1, 0)
                b.set_option("force_halo", 1)
                b.set_option("persistent", 1 if halo == 1 else 0)
            b.fill_random(0x5EED0001)
            b.step(200)
            res.append((b.board_hash(), b.alive_count()))
    assert res[0] == res[1] == res[2]


@pytest.mark.parametrize("N,depth,wpl,nw,tx", [(2048, 16, 1, 8, 1), (4096, 16, 2, 8, 1), (2048, 8, 1, 16, 1),
                                              (3968, 16, 1, 8, 1), (4096, 16, 1, 8, 2), (4096, 16, 2, 8, 4),
                                              (3968, 8, 1, 16, 4), (2048, 16, 1, 8, 8)])
def test_persistent_unequal_bands(coracle, N, depth, wpl, nw, tx):
    """Persistent kernel without pairing (paired_bands 0): static taller bands
    for the oldest waves (65 % of the rows at 8 waves, equal at 16) vs the C oracle."""
    board = coracle.fill_random(N, N // 2, 0x5EED000F)
    turns = 4 * depth + 1
    want = coracle.run(board, turns)
    with golhip.Board(N, N // 2) as b:
        b.set_option("wpl", wpl)
        b.set_option("persist_waves", nw)
        b.set_option("paired_bands", 0)
        b.set_option("persist_wg_tx", tx)
        b.set_option("persistent", 1)
        b.set_option("lds_band", 0)  # K1p itself (K1r: tests/test_gpu_lds.py)
        b.set_tb_depth(depth)
        b.load_bytes(board)
        b.step(turns)
        assert b.perf()["persist_launches"] == 1
        assert np.array_equal(b.snapshot_bytes(), want)
        assert b.alive_count() == (int((want == 255).sum()), turns)


@pytest.mark.parametrize("N,rows,depth,wpl,nw,tx", [(2048, 1024, 16, 1, 8, 1), (4096, 2048, 16, 2, 8, 1),
                                                    (2048, 1024, 8, 1, 16, 1), (3968, 1984, 16, 1, 8, 2),
                                                    (4096, 2048, 16, 2, 8, 4), (3968, 1001, 8, 1, 16, 4),
                                                    (2048, 1024, 16, 1, 8, 8), (1984, 999, 4, 2, 16, 2)])
def test_persistent_paired_bands(coracle, N, rows, depth, wpl, nw, tx):
    """SIMD mates streaming a shared two-band region from both ends (dynamic meeting row) vs the C oracle."""
    board = coracle.fill_random(N, rows, 0x5EED0010)
    turns = 5 * depth + 3
    want = coracle.run(board, turns)
    with golhip.Board(N, rows) as b:
        b.set_option("wpl", wpl)
        b.set_option("persist_waves", nw)
        b.set_option("persist_wg_tx", tx)
        b.set_option("paired_bands", 1)
        b.set_option("persistent", 1)
        b.set_option("lds_band", 0)  # K1p itself (K1r: tests/test_gpu_lds.py)
        b.set_tb_depth(depth)
        b.load_bytes(board)
        b.step(turns)
        assert b.perf()["persist_launches"] == 1
        assert np.array_equal(b.snapshot_bytes(), want)
        assert b.alive_count() == (int((want == 255).sum()), turns)


@pytest.mark.parametrize("N,rows,depth,wpl,rpw", [(2048, 1024, 16, 1, 0), (4096, 2048, 16, 2, 0), (1984, 999, 8, 2, 37),
                                                  (3968, 1001, 4, 1, 5), (2048, 77, 2, 1, 3), (1024, 513, 32, 1, 50),
                                                  (4096, 300, 1, 2, 7), (4096, 2048, 20, 2, 0), (2048, 999, 20, 1, 37)])
@pytest.mark.parametrize("paired", [1, 0])
def test_per_launch_paired_bands(coracle, N, rows, depth, wpl, rpw, paired):
    """Per-launch kernel with SIMD mates meeting inside a two-band region (gol_tb_pair_kernel) vs the C oracle."""
    board = coracle.fill_random(N, rows, 0x5EED0011)
    turns = 3 * depth + 1
    want = coracle.run(board, turns)
    with golhip.Board(N, rows) as b:
        b.set_option("persistent", 0)
        b.set_option("skew", 0)
        b.set_option("wpl", wpl)
        b.set_option("paired_bands", paired)
        b.set_tb_depth(depth)
        b.set_rows_per_wave(rpw)
        b.load_bytes(board)
        b.step(turns)
        assert b.perf()["persist_launches"] == 0
        assert np.array_equal(b.snapshot_bytes(), want)
        assert b.alive_count() == (int((want == 255).sum()), turns)


def test_wrong_result_options_need_measurement_consent(monkeypatch):
    """options whose results are wrong by design (halo_skip,
    flip_debug 1-3) are refused unless GOLHIP_MEASUREMENT=1; the exact ones
    (flip_debug 4, the co-residency test hook) stay allowed."""
    monkeypatch.delenv("GOLHIP_MEASUREMENT", raising=False)
    monkeypatch.delenv("GOLHIP_TEST_HOOKS", raising=False)
    with golhip.Board(64, 64) as b:
        for k, v in (("halo_skip", 1), ("flip_debug", 1), ("flip_debug", 3)):
            with pytest.raises(golhip.GolHipError, match="GOLHIP_MEASUREMENT"):
                b.set_option(k, v)
        # test hooks (exact results, forced failure paths): GOLHIP_TEST_HOOKS=1
        for k, v in (("resident_fault", 1), ("flip_debug", 4)):
            with pytest.raises(golhip.GolHipError, match="GOLHIP_TEST_HOOKS"):
                b.set_option(k, v)
        b.set_option("resident_fault", 0)
        monkeypatch.setenv("GOLHIP_TEST_HOOKS", "1")
        b.set_option("flip_debug", 4)
        b.set_option("resident_fault", 1)
        b.set_option("resident_fault", 0)
        b.set_option("halo_skip", 0)
        monkeypatch.setenv("GOLHIP_MEASUREMENT", "1")
        b.set_option("halo_skip", 1)
        b.set_option("halo_skip", 0)


TUNING_KEYS = {"persist_depth": 8, "persist_waves": 8, "dummy_rows": 1, "paired_bands": 0, "persist_half": 0,
               "persist_wg_tx": 1, "trace": 0, "cu_count": 0, "fill_skip": 1, "skew_young": 60, "skew_hcap": 10,
               "skew_prio": 0, "skew_half": 0, "skew_tx": 1, "lds_depth": 8, "lds_waves": 8, "lds_wg_cu": 1,
               "lds_age": 70, "lds_pre": 2, "lds_stride": 1, "lds_xcd": 1, "flip_overlap": 1, "skew_pairs": 0}
PRODUCT_OPTIONS = {"wpl": 0, "persistent": -1, "lds_band": -1, "skew": 1, "timing": 0, "persist_timeout_us": 1000000,
                   "force_halo": 0}


def test_tuning_knobs_need_consent(monkeypatch):
    """the plan's A/B knobs are refused without
    GOLHIP_TUNING=1 (or GOLHIP_MEASUREMENT=1); the product options are not;
    the resident-launch cap is a test hook.  Same lists as
    golhip_build_info() (tests/test_abi_cpu.py::test_product_build_macros)."""
    info = dict(kv.split("=", 1) for kv in golhip.load().golhip_build_info().decode().split())
    assert set(info["CONSENT_TUNING"].split(",")) == set(TUNING_KEYS)
    assert set(info["PRODUCT_OPTIONS"].split(",")) == set(PRODUCT_OPTIONS)
    for var in ("GOLHIP_TUNING", "GOLHIP_MEASUREMENT", "GOLHIP_TEST_HOOKS"):
        monkeypatch.delenv(var, raising=False)
    with golhip.Board(64, 64) as b:
        for k, v in TUNING_KEYS.items():
            with pytest.raises(golhip.GolHipError, match="GOLHIP_TUNING"):
                b.set_option(k, v)
        for k, v in PRODUCT_OPTIONS.items():
            b.set_option(k, v)
        with pytest.raises(golhip.GolHipError, match="GOLHIP_TEST_HOOKS"):
            b.set_option("resident_max_turns", 100)
        monkeypatch.setenv("GOLHIP_TUNING", "1")
        for k, v in TUNING_KEYS.items():
            b.set_option(k, v)
        monkeypatch.setenv("GOLHIP_TUNING", "0")
        monkeypatch.setenv("GOLHIP_MEASUREMENT", "1")
        b.set_option("skew_young", 0)


@pytest.mark.parametrize("n,lds,fault", [(1024, 1, 0), (1024, 1, 1), (1024, 1, 2), (1024, 0, 0), (1024, 0, 1),
                                         (1024, 0, 2)])
def test_resident_launches_past_the_cap(test_hooks, n, lds, fault):
    """a step of more turns than one resident launch takes
    runs several (here the test hook lowers golk::kResidentMaxTurns to 48 and
    40 turns).  With resident_fault 2 only the step's first launch times out
    (a transient starvation) and the later ones are healthy: the error word
    must survive them (each used to clear it, and the step returned OK on a
    drained board), so the step is restored and re-run on the per-launch
    kernels; fault 1 times out every launch.  Bit-exact either way, and the
    fallback is counted."""
    from oracle.oracle import COracle
    board = COracle().fill_random(n, n, 0x5EED0042)
    turns = 200
    want = COracle().run(board, turns)
    with golhip.Board(n, n) as b:
        b.set_option("persistent", 1)
        b.set_option("lds_band", lds)
        b.set_option("persist_timeout_us", 2000)
        b.set_option("resident_max_turns", 48 if lds else 40)
        b.set_option("resident_fault", fault)
        b.load_bytes(board)
        b.step(turns)
        b.sync()
        p = b.perf()
        got = b.snapshot_bytes()
        cnt, at = b.alive_count()
    assert np.array_equal(got, want)
    assert (cnt, at) == (int((want == 255).sum()), turns)
    if fault:
        assert p["persist_fallbacks"] == 1 and p["persist_launches"] == 0, p
    else:
        assert p["persist_fallbacks"] == 0 and p["persist_launches"] >= 4, p
        assert (p["lds_launches"] > 0) == bool(lds), p
