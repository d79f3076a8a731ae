"""The bit-sliced B3/S23 circuit of the step kernels (gol_kernels.hip `stage`, LUTs in gol_bits.h),
emulated with the same v_bitop3_b32 truth tables, against the reference rule
(distributor.go:350-379 calculateNextState, :382-417 checkNeighbour) on all
512 3x3 neighbourhoods.  CPU only: this pins the LUT constants the kernel
compiles in, including the one unreachable input the 3-gate rule relies on
(centre alive with a 9-cell sum of 0)."""
import itertools
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = os.path.join(ROOT, "game-of-life-distributed_amd", "csrc", "gol_bits.h")  # the LUTs the kernels share


def bitop3(lut: int, a: int, b: int, c: int) -> int:
    """Bitwise v_bitop3_b32: result bit = lut[a*4 + b*2 + c] per bit position."""
    out = 0
    for i in range(8):
        if lut >> i & 1:
            ma = a if i & 4 else ~a
            mb = b if i & 2 else ~b
            mc = c if i & 1 else ~c
            out |= ma & mb & mc
    return out & 0xFFFFFFFF


def kernel_luts() -> dict:
    src = open(KERNELS).read()
    m = re.search(r"static_assert\(kG1 == (0x[0-9a-fA-F]+) && kG2 == (0x[0-9a-fA-F]+) && kNext == (0x[0-9a-fA-F]+)",
                  src)
    assert m, "rule LUT static_assert not found in gol_bits.h"
    return {"g1": int(m.group(1), 16), "g2": int(m.group(2), 16), "next": int(m.group(3), 16)}


XOR3, MAJ = 0x96, 0xE8


def sliced_next(up: int, mid: int, dn: int, luts: dict) -> int:
    """One word-stage of the kernel on three 32-bit rows (no wrap: bits 1..30 valid)."""
    def row_sum(x):
        west, east = (x << 1) & 0xFFFFFFFF, x >> 1
        return bitop3(XOR3, west, x, east), bitop3(MAJ, west, x, east)

    (a0, a1), (b0, b1), (c0, c1) = row_sum(up), row_sum(mid), row_sum(dn)
    u0, u1 = bitop3(XOR3, a0, b0, c0), bitop3(MAJ, a0, b0, c0)
    v0, v1 = bitop3(XOR3, a1, b1, c1), bitop3(MAJ, a1, b1, c1)
    g1 = bitop3(luts["g1"], u1, v0, v1)
    g2 = bitop3(luts["g2"], u0, v1, mid)
    return bitop3(luts["next"], u0, g1, g2)


def test_rule_circuit_all_neighbourhoods():
    luts = kernel_luts()
    for cells in itertools.product((0, 1), repeat=9):
        up = cells[0] << 4 | cells[1] << 5 | cells[2] << 6
        mid = cells[3] << 4 | cells[4] << 5 | cells[5] << 6
        dn = cells[6] << 4 | cells[7] << 5 | cells[8] << 6
        n = sum(cells) - cells[4]
        want = 1 if (n == 3 or (cells[4] and n == 2)) else 0
        assert (sliced_next(up, mid, dn, luts) >> 5) & 1 == want, cells


def test_rule_circuit_random_words():
    """Whole 32-bit words: interior bits 1..30 against a per-cell count."""
    import numpy as np

    luts = kernel_luts()
    rng = np.random.default_rng(7)
    for _ in range(200):
        up, mid, dn = (int(x) for x in rng.integers(0, 2**32, 3, dtype=np.uint64))
        got = sliced_next(up, mid, dn, luts)
        for b in range(1, 31):
            cnt = sum((r >> (b + d)) & 1 for r in (up, mid, dn) for d in (-1, 0, 1)) - ((mid >> b) & 1)
            alive = (mid >> b) & 1
            assert (got >> b) & 1 == (1 if cnt == 3 or (alive and cnt == 2) else 0)
