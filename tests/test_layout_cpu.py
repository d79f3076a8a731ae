"""Code-layout guard (CPU): the bench kernels' main loops keep their 8-byte
instructions on the fast address parity (4 mod 8; the other
parity costs ~20 % on gfx950, profiles/r2la).  Reads the built libgolhip.so
(no GPU); skipped when it is not built."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "game-of-life-distributed_amd", "golhip", "libgolhip.so")
sys.path.insert(0, os.path.join(ROOT, "scripts"))

pytestmark = pytest.mark.skipif(not os.path.exists(LIB) or not shutil.which("/opt/rocm/lib/llvm/bin/llvm-objdump"),
                                reason="libgolhip.so not built or no LLVM tools")


@pytest.fixture(scope="module")
def disasm():
    import loop_parity
    return loop_parity.disassemble(LIB)


@pytest.mark.parametrize("kernel", [
    "gol_persist_kernelILi16ELi2ELi8E",      # configs[1]: 16384^2 resident
    "gol_tb_pair_kernelILi20ELi2ELb0E",      # the paired-band kernel (skew off)
])
def test_main_loop_on_fast_parity(disasm, kernel):
    import loop_parity
    good, n = loop_parity.main_loop_parity(disasm, kernel)
    assert n > 500, (kernel, n)
    assert good >= 0.9, f"{kernel}: {good:.2f} of {n} 8-byte instructions at 4 (mod 8)"


@pytest.mark.parametrize("kernel,nph", [
    ("gol_skew_kernelILi20ELi2ELb0E", 6),   # configs[2] and its strips (default K1w)
    ("gol_skew_kernelILi16ELi2ELb0E", 5),
    ("gol_skew_kernelILi9ELi4ELb0E", 2),    # configs[3]
    ("gol_skew_kernelILi20ELi2ELb1E", 6),   # configs[1] (half-wave tiles)
    ("gol_skew_kernelILi16ELi2ELb1E", 5),
    # the pair rule (round 6, the default at 65536^2): its drain runs on the
    # pair state too, the last phase (6 pushes) as straight-line code, so 4 loops
    ("gol_skew_kernelILi18ELi2ELb0ELb1E", 4),
    ("gol_skew_kernelILi18ELi2ELb1ELb1E", 4),
    ("gol_skew_kernelILi8ELi4ELb0ELb1E", 2),   # quads on the pair rule (skew_pairs bit 2)
])
def test_skew_main_and_drain_loops_on_fast_parity(disasm, kernel, nph):
    """K1w: the main loop and the nph drain-phase loops after it (the
    kernel's last loops; SkewPlan::NPH of the depth)."""
    import loop_parity
    lps = loop_parity.inner_loops(disasm, kernel, min_b8=100)
    assert len(lps) >= nph + 2, (kernel, len(lps))
    last = lps[-(nph + 1):]
    main = max(last, key=lambda l: l[2])  # the main loop: all D stages
    for start, good, n in last:
        # the main loop must sit on the fast parity; the short drain loops (2-17
        # stages, two groups a launch) may have a few instructions off it
        bound = 0.9 if (start, good, n) == main else 0.85
        assert good >= bound, f"{kernel} loop at {start:#x}: {good:.2f} of {n} 8-byte instructions at 4 (mod 8)"
