"""CPU oracle for the Game of Life hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module.  The product (libgolhip.so and its Python binding) never does.

Two independent restatements of the reference algorithm live here:

* ``step_np`` — numpy B3/S23 on a torus (np.roll), restating
  gol/distributor.go:350-417 (calculateNextState + checkNeighbour).
* ``COracle`` — ctypes wrapper over oracle/gol_oracle.c, the literal per-cell
  restatement plus the worker-pool port used for the CPU baseline.

Both are pinned against the reference's own fixtures (check/images and
check/alive, committed as data in tests/golden/) by tests/test_oracle_golden.py.

PGM helpers restate gol/io.go:42-126 (header "P5\\n<W> <H>\\n255\\n" + raw raster).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ALIVE = 255


# --------------------------------------------------------------------------- numpy
def step_np(board: np.ndarray) -> np.ndarray:
    """One turn.  board: (H, W) uint8, alive <=> ==255 (distributor.go:363,411).

    Neighbour count with toroidal wrap (distributor.go:398-409); output 0/255
    (distributor.go:363-375)."""
    a = (board == ALIVE).astype(np.uint8)
    n = np.zeros(a.shape, dtype=np.uint8)
    for dr in (-1, 0, 1):
        for dc in (-1, 0, 1):
            if dr == 0 and dc == 0:
                continue
            n += np.roll(np.roll(a, dr, axis=0), dc, axis=1)
    nxt = (n == 3) | ((a == 1) & (n == 2))
    return np.where(nxt, ALIVE, 0).astype(np.uint8)


def run_np(board: np.ndarray, turns: int) -> np.ndarray:
    b = board
    for _ in range(turns):
        b = step_np(b)
    return b


def alive_cells_np(board: np.ndarray) -> np.ndarray:
    """calculateAliveCells (distributor.go:420-432): row-major (X=col, Y=row)."""
    rows, cols = np.nonzero(board == ALIVE)
    return np.stack([cols, rows], axis=1).astype(np.int32)


def flips_np(old: np.ndarray, new: np.ndarray) -> np.ndarray:
    """initializeAliveCells (distributor.go:212-220): row-major changed cells as
    (col, row) pairs (the reference's Cell{j,i} transposition is a host concern)."""
    rows, cols = np.nonzero(old != new)
    return np.stack([cols, rows], axis=1).astype(np.int32)


def splitmix64_np(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x.astype(np.uint64) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def fill_random_np(W: int, H: int, seed: int) -> np.ndarray:
    """Synthetic board of SURVEY.md §8d: alive <=> splitmix64(seed ^ (y*W+x)) & 3 == 0."""
    idx = np.arange(W * H, dtype=np.uint64).reshape(H, W)
    h = splitmix64_np(np.uint64(seed) ^ idx)
    return np.where((h & np.uint64(3)) == 0, ALIVE, 0).astype(np.uint8)


# --------------------------------------------------------------------------- PGM
def pgm_bytes(board: np.ndarray) -> bytes:
    """writePgmImage (io.go:42-87): "P5\\n" W " " H "\\n" "255\\n" + raster."""
    H, W = board.shape
    return b"P5\n" + f"{W} {H}\n".encode() + b"255\n" + board.astype(np.uint8).tobytes()


def read_pgm(path: str, width: int | None = None, height: int | None = None) -> np.ndarray:
    """readPgmImage (io.go:90-126): whitespace-split header fields P5, W, H, 255;
    the raster is what follows.  Panics (ValueError) on the same conditions."""
    with open(path, "rb") as f:
        data = f.read()
    return parse_pgm(data, width, height)


def parse_pgm(data: bytes, width: int | None = None, height: int | None = None) -> np.ndarray:
    fields = []
    pos = 0
    n = len(data)
    while len(fields) < 4:
        while pos < n and data[pos] in b" \t\n\r\v\f":
            pos += 1
        start = pos
        while pos < n and data[pos] not in b" \t\n\r\v\f":
            pos += 1
        fields.append(data[start:pos])
    pos += 1  # the single whitespace byte after maxval
    if fields[0] != b"P5":
        raise ValueError("Not a pgm file")
    W, H, maxval = int(fields[1]), int(fields[2]), int(fields[3])
    if width is not None and W != width:
        raise ValueError("Incorrect width")
    if height is not None and H != height:
        raise ValueError("Incorrect height")
    if maxval != 255:
        raise ValueError("Incorrect maxval/bit depth")
    raster = np.frombuffer(data, dtype=np.uint8, count=W * H, offset=pos)
    return raster.reshape(H, W).copy()


# --------------------------------------------------------------------------- bits
def pack_bits(board: np.ndarray) -> np.ndarray:
    """(H, W) 0/255 bytes -> (H, ceil(W/32)) uint32 words, cell (r, c) is bit
    c%32 of word c//32 (the device layout, DESIGN.md "Layout")."""
    H, W = board.shape
    Ww = (W + 31) // 32
    b = np.zeros((H, Ww * 32), dtype=np.uint8)
    b[:, :W] = board == ALIVE
    bits = np.packbits(b.reshape(H, Ww, 32), axis=2, bitorder="little")
    return bits.reshape(H, Ww * 4).view(np.uint32).copy()


def unpack_bits(words: np.ndarray, W: int) -> np.ndarray:
    H = words.shape[0]
    u8 = np.ascontiguousarray(words).view(np.uint8).reshape(H, -1)
    bits = np.unpackbits(u8, axis=1, bitorder="little")[:, :W]
    return (bits * ALIVE).astype(np.uint8)


# --------------------------------------------------------------------------- C oracle
class COracle:
    """ctypes binding of oracle/build/liboracle.so (built by oracle/Makefile)."""

    def __init__(self, path: str | None = None):
        path = path or os.path.join(HERE, "build", "liboracle.so")
        if not os.path.exists(path):
            build()
        lib = ctypes.CDLL(path)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        i32p = ctypes.POINTER(ctypes.c_int32)
        i64p = ctypes.POINTER(ctypes.c_int64)
        lib.oracle_step.argtypes = [u8p, u8p, ctypes.c_int, ctypes.c_int]
        lib.oracle_run.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.c_long]
        lib.oracle_run_counts.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.c_long, i64p]
        lib.oracle_alive_cells.argtypes = [u8p, ctypes.c_int, ctypes.c_int, i32p]
        lib.oracle_alive_cells.restype = ctypes.c_int64
        lib.oracle_flips.argtypes = [u8p, u8p, ctypes.c_int, ctypes.c_int, i32p]
        lib.oracle_flips.restype = ctypes.c_int64
        lib.oracle_fill_random.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.c_uint64]
        lib.oracle_run_workerpool.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.c_long, ctypes.c_int]
        lib.oracle_run_workerpool.restype = ctypes.c_int64
        u64p = ctypes.POINTER(ctypes.c_uint64)
        lib.oracle_run_workerpool_events.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.c_long, ctypes.c_int,
                                                     ctypes.c_int, u64p, i64p, i64p, ctypes.c_char_p]
        lib.oracle_run_workerpool_events.restype = ctypes.c_int
        lib.fastcpu_pack.argtypes = [u8p, ctypes.c_int, ctypes.c_int, u64p]
        lib.fastcpu_unpack.argtypes = [u64p, ctypes.c_int, ctypes.c_int, u8p]
        lib.fastcpu_run.argtypes = [u64p, ctypes.c_int, ctypes.c_int, ctypes.c_long, ctypes.c_int]
        lib.fastcpu_fill_random.argtypes = [u64p, ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_uint64,
                                            ctypes.c_int]
        lib.fastcpu_hash.argtypes = [u64p, ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_int]
        lib.fastcpu_hash.restype = ctypes.c_uint64
        lib.fastcpu_popcount.argtypes = [u64p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        lib.fastcpu_popcount.restype = ctypes.c_uint64
        self.lib = lib

    @staticmethod
    def _p(a, t=ctypes.c_uint8):
        return a.ctypes.data_as(ctypes.POINTER(t))

    # Above this many cell-updates run() answers with the bit-packed comparator
    # (gol_fastcpu.c, 16 threads), which tests/test_oracle_golden.py pins to the
    # per-cell oracle and to the reference's check/images boards: the GPU suite's
    # large parity cases then take seconds instead of minutes.
    FAST_CELL_UPDATES = 20_000_000

    def run(self, board: np.ndarray, turns: int) -> np.ndarray:
        H, W = board.shape
        if W % 64 == 0 and W * H * turns >= self.FAST_CELL_UPDATES:
            return self.run_fast(np.ascontiguousarray(board, dtype=np.uint8), turns,
                                 threads=max(1, min(16, os.cpu_count() or 1)))
        return self.run_exact(board, turns)

    def run_exact(self, board: np.ndarray, turns: int) -> np.ndarray:
        """The per-cell restatement (oracle_run), whatever the size."""
        b = np.ascontiguousarray(board, dtype=np.uint8).copy()
        H, W = b.shape
        if self.lib.oracle_run(self._p(b), W, H, turns) != 0:
            raise MemoryError("oracle_run")
        return b

    def run_counts(self, board: np.ndarray, turns: int):
        b = np.ascontiguousarray(board, dtype=np.uint8).copy()
        H, W = b.shape
        counts = np.zeros(turns, dtype=np.int64)
        self.lib.oracle_run_counts(self._p(b), W, H, turns, self._p(counts, ctypes.c_int64))
        return b, counts

    def alive_cells(self, board: np.ndarray) -> np.ndarray:
        b = np.ascontiguousarray(board, dtype=np.uint8)
        H, W = b.shape
        n = self.lib.oracle_alive_cells(self._p(b), W, H, None)
        xy = np.zeros((max(n, 1), 2), dtype=np.int32)
        self.lib.oracle_alive_cells(self._p(b), W, H, self._p(xy, ctypes.c_int32))
        return xy[:n]

    def flips(self, old: np.ndarray, new: np.ndarray) -> np.ndarray:
        a = np.ascontiguousarray(old, dtype=np.uint8)
        b = np.ascontiguousarray(new, dtype=np.uint8)
        H, W = a.shape
        n = self.lib.oracle_flips(self._p(a), self._p(b), W, H, None)
        xy = np.zeros((max(n, 1), 2), dtype=np.int32)
        self.lib.oracle_flips(self._p(a), self._p(b), W, H, self._p(xy, ctypes.c_int32))
        return xy[:n]

    def fill_random(self, W: int, H: int, seed: int) -> np.ndarray:
        b = np.zeros((H, W), dtype=np.uint8)
        self.lib.oracle_fill_random(self._p(b), W, H, seed)
        return b

    def run_workerpool(self, board: np.ndarray, turns: int, threads: int):
        b = np.ascontiguousarray(board, dtype=np.uint8).copy()
        H, W = b.shape
        flips = self.lib.oracle_run_workerpool(self._p(b), W, H, turns, threads)
        if flips < 0:
            raise MemoryError("oracle_run_workerpool")
        return b, flips

    EVENT_NAMES = ["AliveCellsCount", "ImageOutputComplete", "StateChange", "CellFlipped", "TurnComplete",
                   "FinalTurnComplete"]

    def run_workerpool_events(self, board: np.ndarray, turns: int, threads: int, events_cap: int = 0,
                              out_pgm: str | None = None):
        """The port as gol.Run runs it, every event through a channel of
        capacity `events_cap` drained by main.go's loop
        (gol_port_events.cpp).  Returns (board, counts by event name, last
        TurnComplete, len(FinalTurnComplete.Alive))."""
        b = np.ascontiguousarray(board, dtype=np.uint8).copy()
        H, W = b.shape
        counts = np.zeros(6, dtype=np.uint64)
        last, fin = ctypes.c_int64(), ctypes.c_int64()
        rc = self.lib.oracle_run_workerpool_events(self._p(b), W, H, turns, threads, events_cap,
                                                   self._p(counts, ctypes.c_uint64), ctypes.byref(last),
                                                   ctypes.byref(fin), out_pgm.encode() if out_pgm else None)
        if rc != 0:
            raise RuntimeError("oracle_run_workerpool_events failed")
        return b, {self.EVENT_NAMES[k]: int(counts[k]) for k in range(6)}, last.value, fin.value

    # -- bit-packed OpenMP comparator (gol_fastcpu.c), W % 64 == 0
    def pack64(self, board: np.ndarray) -> np.ndarray:
        b = np.ascontiguousarray(board, dtype=np.uint8)
        H, W = b.shape
        w = np.zeros((H, W // 64), dtype=np.uint64)
        if self.lib.fastcpu_pack(self._p(b), W, H, self._p(w, ctypes.c_uint64)) != 0:
            raise ValueError("fastcpu_pack needs W % 64 == 0")
        return w

    def unpack64(self, words: np.ndarray, W: int) -> np.ndarray:
        H = words.shape[0]
        b = np.zeros((H, W), dtype=np.uint8)
        if self.lib.fastcpu_unpack(self._p(np.ascontiguousarray(words), ctypes.c_uint64), W, H, self._p(b)) != 0:
            raise ValueError("fastcpu_unpack needs W % 64 == 0")
        return b

    def run_fast_words(self, words: np.ndarray, W: int, turns: int, threads: int) -> None:
        """In place on H x W/64 packed words."""
        H = words.shape[0]
        if self.lib.fastcpu_run(self._p(words, ctypes.c_uint64), W, H, turns, threads) != 0:
            raise ValueError("fastcpu_run")

    def fill_random64(self, W: int, H: int, seed: int, threads: int, row0: int = 0) -> np.ndarray:
        """Synthetic board (fill_random's rule) packed 64 cells per uint64."""
        w = np.empty((H, W // 64), dtype=np.uint64)
        if self.lib.fastcpu_fill_random(self._p(w, ctypes.c_uint64), W, H, row0, seed, threads) != 0:
            raise ValueError("fastcpu_fill_random needs W % 64 == 0")
        return w

    def hash64(self, words: np.ndarray, W: int, threads: int, word0: int = 0) -> int:
        """golhip_board_hash of packed words (strips: word0 = first global 32-bit word)."""
        return int(self.lib.fastcpu_hash(self._p(np.ascontiguousarray(words), ctypes.c_uint64), W,
                                         words.shape[0], word0, threads))

    def popcount64(self, words: np.ndarray, W: int, threads: int) -> int:
        return int(self.lib.fastcpu_popcount(self._p(np.ascontiguousarray(words), ctypes.c_uint64), W,
                                             words.shape[0], threads))

    def run_fast(self, board: np.ndarray, turns: int, threads: int = 1) -> np.ndarray:
        W = board.shape[1]
        w = self.pack64(board)
        self.run_fast_words(w, W, turns, threads)
        return self.unpack64(w, W)


def build() -> str:
    """Compile oracle/build/liboracle.so with gcc (oracle/Makefile)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return os.path.join(HERE, "build", "liboracle.so")
