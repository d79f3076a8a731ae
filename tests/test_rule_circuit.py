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


def pair_luts() -> dict:
    src = open(KERNELS).read()
    m = re.search(r"static_assert\(kPrA == (0x[0-9a-fA-F]+) && kPrB == (0x[0-9a-fA-F]+) && kPrC == (0x[0-9a-fA-F]+) "
                  r"&& kPrNext == (0x[0-9a-fA-F]+)", src)
    n = re.search(r"static_assert\(kXor2 == (0x[0-9a-fA-F]+) && kAnd2 == (0x[0-9a-fA-F]+) && kBorrow == (0x[0-9a-fA-F]+)",
                  src)
    assert m and n, "pair-rule LUT static_asserts not found in gol_bits.h"
    return {"A": int(m.group(1), 16), "B": int(m.group(2), 16), "C": int(m.group(3), 16), "next": int(m.group(4), 16),
            "xor2": int(n.group(1), 16), "and2": int(n.group(2), 16), "borrow": int(n.group(3), 16)}


def pair_sum(b0, b1, c0, c1, L):
    """gol_bits.h pair_sum: P = B + C as (p0, p1, p2) (the 2-input LUTs repeat an operand)."""
    p0 = bitop3(L["xor2"], b0, c0, c0)
    k = bitop3(L["and2"], b0, c0, c0)
    return p0, bitop3(XOR3, b1, c1, k), bitop3(MAJ, b1, c1, k)


def pair_rule(a0, a1, p0, p1, p2, c, L):
    """gol_bits.h pair_rule: next from the other row's sum A, the pair sum P and the centre."""
    s6 = bitop3(L["A"], a0, p0, c)
    s7 = bitop3(L["B"], a1, p1, p2)
    s8 = bitop3(L["C"], c, s6, s7)
    return bitop3(L["next"], p2, s7, s8)


def test_pair_rule_all_four_row_neighbourhoods():
    """The pair rule of K1w's main loop (gol_kernels.hip stage_pr): the two
    output rows of a pair share the middle rows' vertical sum P; each is the
    4-LUT rule of P, the other row's sum and its centre.  All 4096 four-row
    neighbourhoods (rows a, b, c, d of three cells; outputs: b's and c's
    centres), against the reference rule, with the LUTs the kernels compile."""
    L = pair_luts()
    for bits in range(1 << 12):
        rows = [[(bits >> (3 * r + i)) & 1 for i in range(3)] for r in range(4)]
        words = [row[0] << 4 | row[1] << 5 | row[2] << 6 for row in rows]

        def row_sum(x):
            west, east = (x << 1) & 0xFFFFFFFF, x >> 1
            return bitop3(XOR3, west, x, east), bitop3(MAJ, west, x, east)

        (a0, a1), (b0, b1), (c0, c1), (d0, d1) = (row_sum(w) for w in words)
        p0, p1, p2 = pair_sum(b0, b1, c0, c1, L)
        got_b = (pair_rule(a0, a1, p0, p1, p2, words[1], L) >> 5) & 1
        got_c = (pair_rule(d0, d1, p0, p1, p2, words[2], L) >> 5) & 1
        for out, centre, window in ((got_b, rows[1][1], rows[0:3]), (got_c, rows[2][1], rows[1:4])):
            n = sum(sum(r) for r in window) - centre
            assert out == (1 if n == 3 or (centre and n == 2) else 0), (bits, rows)


def test_pair_unsum_inverts_pair_sum():
    """pair_unsum (pr_leave: the pair state back to per-row sums) recovers B
    from P and C for every pair of row sums (B, C in 0..3)."""
    L = pair_luts()
    for b in range(4):
        for c in range(4):
            b0, b1, c0, c1 = -(b & 1), -(b >> 1), -(c & 1), -(c >> 1)  # all-ones / all-zeros words
            p0, p1, p2 = pair_sum(b0, b1, c0, c1, L)
            assert ((p0 & 1) + 2 * (p1 & 1) + 4 * (p2 & 1)) == b + c
            r0 = bitop3(L["xor2"], p0, c0 & 0xFFFFFFFF, c0 & 0xFFFFFFFF)
            br = bitop3(L["borrow"], p0, c0 & 0xFFFFFFFF, c0 & 0xFFFFFFFF)
            r1 = bitop3(XOR3, p1, c1 & 0xFFFFFFFF, br)
            assert (r0 & 1) + 2 * (r1 & 1) == b, (b, c)
