"""The CellFlipped stream (golhip_flip_stream, fused turn + flip-list kernel K5)
and the resident-kernel guard, against the oracle.

Reference: initializeAliveCells (gol/distributor.go:212-220) sends one
CellFlipped per changed cell, row-major, every turn of the loop :93-173;
sdl_test.go:93-128 replays them onto a shadow board.  The engine's stream must
give exactly the oracle's per-turn diff lists, in turn order, never dropping
an entry: a batch that would overflow the caller's buffer stops at the last
turn that fits and leaves the board there.
"""
import numpy as np
import pytest

from oracle.oracle import COracle, flips_np, step_np, unpack_bits

pytestmark = pytest.mark.gpu

golhip = pytest.importorskip("golhip")


@pytest.fixture(scope="module")
def coracle():
    return COracle()


def idx_to_xy(idx, W):
    idx = idx.astype(np.int64)
    return np.stack([idx % W, idx // W], axis=1).astype(np.int32)


def board_for(fixtures, coracle, W, H, seed):
    if W == H and f"image_{W}" in fixtures:
        return unpack_bits(fixtures[f"image_{W}"], W)
    return coracle.fill_random(W, H, seed)


@pytest.mark.parametrize("W,H", [(512, 512), (256, 256), (64, 64), (1024, 300), (4096, 96), (160, 33), (48, 48),
                                 (16, 16), (2048, 1)])
@pytest.mark.parametrize("fmt", [0, 1])
def test_flip_stream_matches_oracle(fixtures, coracle, W, H, fmt):
    """Every turn's list in uneven batches, both formats; widths not a
    multiple of 32 (48, 16) take the generic three-pass path."""
    board = board_for(fixtures, coracle, W, H, 0x5EED0020 + W)
    cur = board
    with golhip.Board(W, H) as b:
        b.load_bytes(board)
        t = 0
        for k in (1, 5, 17, 3):
            ent, counts, done = b.flip_stream(k, cap=k * W * H, fmt=fmt)
            assert done == k and len(counts) == k and int(counts.sum()) == len(ent)
            xy = ent if fmt == 0 else idx_to_xy(ent, W)
            off = 0
            for c in counts:
                nxt = step_np(cur)
                assert np.array_equal(xy[off:off + int(c)], flips_np(cur, nxt)), t
                cur, off, t = nxt, off + int(c), t + 1
        assert b.alive_count() == (int((cur == 255).sum()), t)
        assert np.array_equal(b.snapshot_bytes(), cur)
        b.step(7)  # the per-launch kernels continue from the stream's board
        assert np.array_equal(b.snapshot_bytes(), coracle.run(cur, 7))


@pytest.mark.parametrize("W,H,fmt", [(512, 512, 0), (1024, 300, 1), (48, 48, 0)])
def test_flip_stream_stops_without_loss(fixtures, coracle, W, H, fmt):
    """A small buffer: each call runs the turns that fit, the rest follow in
    the next calls; the concatenation equals the oracle's stream."""
    board = board_for(fixtures, coracle, W, H, 0x5EED0021)
    want, cur = [], board
    for _ in range(40):
        nxt = step_np(cur)
        want.append(flips_np(cur, nxt))
        cur = nxt
    cap = max(len(w) for w in want) * 3  # about three turns per call
    got, turns, calls = [], 0, 0
    with golhip.Board(W, H) as b:
        b.load_bytes(board)
        while turns < 40:
            ent, counts, done = b.flip_stream(40 - turns, cap=cap, fmt=fmt)
            assert 1 <= done <= 40 - turns and len(ent) <= cap
            xy = ent if fmt == 0 else idx_to_xy(ent, W)
            off = 0
            for c in counts:
                got.append(xy[off:off + int(c)])
                off += int(c)
            turns += done
            calls += 1
            assert b.alive_count()[1] == turns
            assert np.array_equal(b.snapshot_bytes(), coracle.run(board, turns))
        assert calls > 5
    assert len(got) == 40
    for t in range(40):
        assert np.array_equal(got[t], want[t]), t


@pytest.mark.parametrize("fmt,overlap,shift", [(0, 1, 0), (1, 1, 0), (0, 1, 1), (1, 1, 3), (0, 0, 0), (1, 0, 1),
                                               (0, 3, 0), (1, 3, 0), (0, 3, 1), (1, 3, 3), (1, 3, 33), (1, 2, 0)])
def test_flip_stream_into_pinned_host_buffer(fixtures, coracle, fmt, overlap, shift):
    """out inside a golhip_host_alloc buffer: the kernels write the entries
    over PCIe themselves -- flip_overlap 3 (2, the default, on larger boards):
    the batch's turns in one resident launch (K5r) whose copy blocks move each
    turn's list while the next turns compute; 1: each launch's copy blocks move the previous turn's
    list, a last copy-only launch the final turn's; 0: the turn's own blocks
    -- same lists, same early stop; `shift` entries into the buffer the
    destination is not 16-byte aligned (4-byte heads and tails; K5r's head
    runs to the next 128-byte line)."""
    W = H = 512
    board = unpack_bits(fixtures["image_512"], 512)
    want, cur = [], board
    for _ in range(30):
        nxt = step_np(cur)
        want.append(flips_np(cur, nxt))
        cur = nxt
    cap = max(len(w) for w in want) * 4
    buf = golhip.host_array((cap + shift, 2) if fmt == 0 else (cap + shift,), np.int32 if fmt == 0 else np.uint32)
    out = buf[shift:]
    got = []
    with golhip.Board(W, H) as b:
        b.set_option("flip_overlap", overlap)
        b.load_bytes(board)
        while len(got) < 30:
            ent, counts, done = b.flip_stream(30 - len(got), cap=cap, fmt=fmt, out=out)
            assert done >= 1
            xy = ent if fmt == 0 else idx_to_xy(ent, W)
            off = 0
            for c in counts:
                got.append(xy[off:off + int(c)].copy())
                off += int(c)
        assert np.array_equal(b.snapshot_bytes(), cur)
        # (2, the default, keeps a board this small on per-turn launches; 3 forces K5r)
        assert (b.perf()["flip_resident_launches"] >= 1) == (overlap == 3)
    for t in range(30):
        assert np.array_equal(got[t], want[t]), t
    del out, buf


def test_flip_stream_first_turn_too_big(fixtures):
    """cap below the first turn's list: ERANGE, *n = what it needs, board untouched."""
    board = unpack_bits(fixtures["image_256"], 256)
    need = len(flips_np(board, step_np(board)))
    with golhip.Board(256, 256) as b:
        b.load_bytes(board)
        with pytest.raises(golhip.GolHipError) as e:
            b.flip_stream(4, cap=need - 1)
        assert e.value.code == golhip.GOLHIP_ERANGE
        assert b.alive_count() == (int((board == 255).sum()), 0)
        assert np.array_equal(b.snapshot_bytes(), board)
        ent, counts, done = b.flip_stream(1, cap=need)
        assert done == 1 and len(ent) == need


@pytest.mark.parametrize("W,H", [(512, 512), (1024, 300)])
def test_flip_stream_one_rank_ring(coracle, W, H):
    """Through the RCCL halo path (one halo row exchanged per turn)."""
    board = coracle.fill_random(W, H, 0x5EED0022)
    cur = board
    with golhip.Board(W, H) as b:
        b.comm_init(golhip.unique_id(), 1, 0)
        b.set_option("force_halo", 1)
        b.load_bytes(board)
        ent, counts, done = b.flip_stream(9, cap=9 * W * H, fmt=1)
        assert done == 9
        xy, off = idx_to_xy(ent, W), 0
        for c in counts:
            nxt = step_np(cur)
            assert np.array_equal(xy[off:off + int(c)], flips_np(cur, nxt))
            cur, off = nxt, off + int(c)
        assert np.array_equal(b.snapshot_bytes(), cur)


def test_flip_stream_dense_blocks(coracle):
    """A board whose blocks flip more cells than the kernel's LDS staging holds
    (the direct-store path): a checkerboard of 2 x 2 blocks dies at once."""
    W, H = 1024, 64
    yy, xx = np.mgrid[0:H, 0:W]
    board = np.where(((yy // 2 + xx // 2) % 2) == 0, 255, 0).astype(np.uint8)
    with golhip.Board(W, H) as b:
        b.load_bytes(board)
        for fmt in (0, 1):
            b.load_bytes(board)
            ent, counts, done = b.flip_stream(3, cap=3 * W * H, fmt=fmt)
            xy = ent if fmt == 0 else idx_to_xy(ent, W)
            cur, off = board, 0
            for c in counts:
                nxt = step_np(cur)
                assert np.array_equal(xy[off:off + int(c)], flips_np(cur, nxt))
                cur, off = nxt, off + int(c)
        assert int(counts[0]) > 16384


@pytest.mark.parametrize("fmt", [0, 1])
@pytest.mark.usefixtures("test_hooks")
def test_flip_stream_coresidency_fallback(fixtures, coracle, fmt):
    """A batch whose blockIdx-ordered prefix sums report a missing
    predecessor (forced by the test hook flip_debug 4) is restored and re-run
    in ticket order with the decoupled look-back: the lists stay exact."""
    board = unpack_bits(fixtures["image_512"], 512)
    cur, want = board, []
    for _ in range(12):
        nxt = step_np(cur)
        want.append(flips_np(cur, nxt))
        cur = nxt
    with golhip.Board(512, 512) as b:
        b.load_bytes(board)
        b.set_option("flip_debug", 4)
        ent, counts, done = b.flip_stream(12, cap=12 * 512 * 512, fmt=fmt)
        assert done == 12 and b.perf()["flip_fallbacks"] == 1
        xy = ent if fmt == 0 else idx_to_xy(ent, 512)
        assert np.array_equal(xy, np.concatenate(want))
        assert np.array_equal(b.snapshot_bytes(), cur)
        ent, counts, done = b.flip_stream(5, cap=5 * 512 * 512, fmt=fmt)  # ticket order from now on
        xy = ent if fmt == 0 else idx_to_xy(ent, 512)
        assert np.array_equal(xy, np.concatenate([flips_np(coracle.run(cur, i), coracle.run(cur, i + 1))
                                                  for i in range(5)]))


@pytest.mark.parametrize("fmt", [0, 1])
@pytest.mark.usefixtures("test_hooks")
def test_flip_stream_resident_fallback(fixtures, fmt):
    """K5r (flip_overlap 3: one resident launch a batch at any size) with the missing-
    predecessor report forced inside it (test hook flip_debug 4): the batch is
    restored and re-run on per-turn launches in ticket order, exact."""
    board = unpack_bits(fixtures["image_512"], 512)
    cur, want = board, []
    for _ in range(12):
        nxt = step_np(cur)
        want.append(flips_np(cur, nxt))
        cur = nxt
    cap = 12 * 512 * 512
    buf = golhip.host_array((cap, 2) if fmt == 0 else (cap,), np.int32 if fmt == 0 else np.uint32)
    with golhip.Board(512, 512) as b:
        b.set_option("flip_overlap", 3)
        b.load_bytes(board)
        b.set_option("flip_debug", 4)
        ent, counts, done = b.flip_stream(12, cap=cap, fmt=fmt, out=buf)
        p = b.perf()
        assert done == 12 and p["flip_fallbacks"] == 1 and p["flip_resident_launches"] == 1, p
        xy = ent if fmt == 0 else idx_to_xy(ent, 512)
        assert np.array_equal(xy, np.concatenate(want))
        assert np.array_equal(b.snapshot_bytes(), cur)
    del buf


@pytest.mark.parametrize("groups", [None, 1, 8])
@pytest.mark.parametrize("W,H", [(5120, 640), (4000, 96), (1024, 3000)])
def test_flip_stream_resident_shapes(coracle, monkeypatch, W, H, groups):
    """K5r on other shapes: a narrow-row board (Ww % 4 != 0: the 4-byte
    path), many blocks a row, and a tall board, 40 turns in batches that stop
    on a small buffer and resume; the lists, board and alive count exact.
    `groups`: the copy blocks in 1 / 8 groups (each copying every 1st / 8th
    turn) besides the default 4 (GOLHIP_FLIP_CP_GROUPS, a tuning override)."""
    if groups is not None:
        monkeypatch.setenv("GOLHIP_TUNING", "1")
        monkeypatch.setenv("GOLHIP_FLIP_CP_GROUPS", str(groups))
    board = coracle.fill_random(W, H, 0x5EED0081 + W)
    cur, want = board, []
    for _ in range(40):
        nxt = coracle.run(cur, 1)
        want.append(flips_np(cur, nxt))
        cur = nxt
    cap = max(len(w) for w in want) * 3
    buf = golhip.host_array((cap,), np.uint32)
    got, calls = [], []
    with golhip.Board(W, H) as b:
        b.set_option("flip_overlap", 3)
        b.load_bytes(board)
        while len(got) < 40:
            ent, counts, done = b.flip_stream(40 - len(got), cap=cap, fmt=golhip.FLIPS_INDEX, out=buf)
            calls.append(done)
            assert done >= 1
            xy = idx_to_xy(ent, W)
            off = 0
            for c in counts:
                got.append(xy[off:off + int(c)].copy())
                off += int(c)
        p = b.perf()
        assert p["flip_fallbacks"] == 0 and p["flip_resident_launches"] >= 2, (calls, p)
        assert np.array_equal(b.snapshot_bytes(), cur)
        assert b.alive_count() == (int((cur == 255).sum()), 40)
    for t in range(40):
        assert np.array_equal(got[t], want[t]), t
    del buf


def test_step_flips_truncates_and_advances(fixtures):
    """golhip_step_flips keeps its contract on the fused kernel: lists cut at
    cap, ERANGE with the total, the board advanced every turn."""
    board = unpack_bits(fixtures["image_256"], 256)
    want, cur = [], board
    for _ in range(5):
        nxt = step_np(cur)
        want.append(flips_np(cur, nxt))
        cur = nxt
    allw = np.concatenate(want)
    with golhip.Board(256, 256) as b:
        b.load_bytes(board)
        buf = np.zeros((100, 2), dtype=np.int32)
        with pytest.raises(golhip.GolHipError) as e:
            b.step_flips(5, cap=100, xy=buf)
        assert e.value.code == golhip.GOLHIP_ERANGE
        assert np.array_equal(buf, allw[:100])
        assert np.array_equal(b.snapshot_bytes(), cur)


# ------------------------------------------------------------ resident-kernel guard
@pytest.mark.parametrize("N,depth,wpl", [(4096, 16, 1), (2048, 8, 2)])
@pytest.mark.parametrize("lds", [0, 1])
@pytest.mark.usefixtures("test_hooks")
def test_persistent_timeout_restores_and_reruns(coracle, N, depth, wpl, lds):
    """A resident launch (K1p, or K1r's LDS bands) whose workgroups give up
    waiting (a 1 us bound stands in for a co-tenant kernel holding CUs) is
    detected, the board restored and the step re-run on the per-launch
    kernels: the result is still exact."""
    board = coracle.fill_random(N, N // 2, 0x5EED0023)
    turns = 6 * depth + 3
    want = coracle.run(board, turns)
    with golhip.Board(N, N // 2) as b:
        b.set_option("persistent", 1)
        b.set_option("lds_band", lds)
        b.set_option("lds_depth", depth)
        b.set_option("wpl", wpl)
        b.set_tb_depth(depth)
        # workgroup / band 0 never reports (test hook): its neighbours' waits
        # reach the bound on every box (a 1 us bound alone did not always)
        b.set_option("resident_fault", 1)
        b.set_option("persist_timeout_us", 2000)
        b.load_bytes(board)
        b.step(turns)
        p = b.perf()
        assert p["persist_fallbacks"] == 1 and p["persist_launches"] == 0 and p["lds_launches"] == 0
        assert np.array_equal(b.snapshot_bytes(), want)
        assert b.alive_count() == (int((want == 255).sum()), turns)
        b.step(10)
        assert np.array_equal(b.snapshot_bytes(), coracle.run(want, 10))


@pytest.mark.parametrize("timeout_us", [1000000, 1])
@pytest.mark.usefixtures("test_hooks")
def test_persistent_timeout_one_rank_ring(coracle, timeout_us):  # 1: workgroup 0 never reports (test hook)
    """A strip run as a one-rank RCCL ring (force_halo) with the resident
    kernel between exchanges: the step is guarded like a torus step, so a
    resident launch that gives up waiting (1 us bound) restores the board and
    re-runs the step on per-launch kernels, exchanges included (safe with no
    other rank; multi-rank rings never run the resident kernel)."""
    # depth 8: one resident launch of 16 super-steps per exchange, i.e. 15
    # neighbour waits per workgroup, each of which the 1 us bound can cut
    N, depth = 4096, 8
    board = coracle.fill_random(N, N // 2, 0x5EED0024)
    turns = 16 * depth + 7
    want = coracle.run(board, turns)
    with golhip.Board(N, N // 2) as b:
        b.comm_init(golhip.unique_id(), 1, 0)
        b.set_option("force_halo", 1)
        b.set_option("persistent", 1)
        b.set_option("wpl", 2)
        b.set_tb_depth(depth)
        b.set_option("persist_timeout_us", timeout_us if timeout_us > 1 else 2000)
        b.set_option("resident_fault", 1 if timeout_us == 1 else 0)
        b.load_bytes(board)
        b.step(turns)
        p = b.perf()
        if timeout_us == 1:
            assert p["persist_fallbacks"] == 1 and p["persist_launches"] == 0
        else:
            assert p["persist_fallbacks"] == 0 and p["persist_launches"] >= 1
        assert p["halo_exchanges"] >= 1
        assert np.array_equal(b.snapshot_bytes(), want)
        assert b.alive_count() == (int((want == 255).sum()), turns)
        b.step(10)
        assert np.array_equal(b.snapshot_bytes(), coracle.run(want, 10))


def test_host_link_probe():
    """golhip_host_link_probe: K5's ceiling, the rate a
    kernel's coalesced 16-byte stores reach page-locked host memory, and the
    DMA copy rate beside it; bad arguments are refused."""
    r = golhip.host_link_probe(0, 16 << 20, 2)
    assert 1.0 < r["kernel_write_GBps"] < 1000.0 and 1.0 < r["dma_d2h_GBps"] < 1000.0, r
    for nbytes, reps in ((100, 1), (4097, 1), (1 << 20, 0)):
        with pytest.raises(golhip.GolHipError):
            golhip.host_link_probe(0, nbytes, reps)
