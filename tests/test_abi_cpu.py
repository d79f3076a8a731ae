"""CPU-side checks of the C-ABI boundary (no GPU needed).

* libgolhip.so loads and exports every function include/golhip.h declares;
* the library refuses to run without a HIP device (no silent CPU fallback);
* the halo plan (shared by the RCCL ring and the in-process strip group) is
  self-consistent: what rank r sends up lands in rank r-1's bottom halo, etc.
"""
import ctypes

import pytest

golhip = pytest.importorskip("golhip")


def test_library_exports_every_header_symbol():
    lib = golhip.load()
    syms = golhip.header_symbols()
    assert len(syms) >= 25
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_version_and_error_string():
    lib = golhip.load()
    assert b"gfx950" in lib.golhip_version()
    rc = lib.golhip_create(0, 0, 0, 0, ctypes.byref(ctypes.c_void_p()))
    assert rc == -1
    assert b"bad board" in lib.golhip_last_error()


def test_no_device_fails_loudly():
    """On a host without a GPU the product path raises instead of falling back."""
    try:
        n = golhip.device_count()
    except golhip.GolHipError as e:
        assert e.code == -2
        with pytest.raises(golhip.GolHipError):
            golhip.Board(64, 64)
        return
    if n == 0:
        with pytest.raises(golhip.GolHipError):
            golhip.Board(64, 64)


@pytest.mark.parametrize("nranks", [1, 2, 3, 8])
@pytest.mark.parametrize("depth", [1, 4, 32, 64])
def test_halo_plan_pairs_up(nranks, depth):
    rows = 80
    plans = [golhip.halo_plan(2048, rows, nranks, r, depth) for r in range(nranks)]
    halo = golhip.HALO_ROWS
    for r, p in enumerate(plans):
        assert p["prev_rank"] == (r - 1) % nranks and p["next_rank"] == (r + 1) % nranks
        assert p["rows"] == depth and p["bytes"] == depth * 2048 // 8
        # my first `depth` rows go up, my last go down
        assert p["send_up_row"] == halo and p["send_down_row"] == halo + rows - depth
        # received rows sit directly above / below my rows
        assert p["recv_top_row"] + depth == halo and p["recv_bottom_row"] == halo + rows


def test_halo_plan_rejects_depth_above_strip():
    with pytest.raises(golhip.GolHipError):
        golhip.halo_plan(64, 3, 2, 0, 4)
    with pytest.raises(golhip.GolHipError):
        golhip.halo_plan(64, 128, 2, 0, golhip.HALO_ROWS + 1)


@pytest.mark.parametrize("rows,tb,left,want", [(16384, 16, 1000, (16, 8)), (16384, 16, 40, (16, 1)),
                                               (16384, 32, 1000, (32, 4)), (40, 16, 1000, (16, 2)),
                                               (10, 16, 1000, (8, 1)), (16384, 16, 7, (6, 1)),
                                               (16384, 1, 100, (1, 100)), (16384, 1, 1000, (1, 128)),
                                               (100, 16, 1000, (16, 6))])
def test_halo_schedule(rows, tb, left, want):
    """k launches of d turns per exchange of k * d <= GOLHIP_HALO_ROWS rows, k * d <= strip rows."""
    d, k = golhip.halo_schedule(rows, tb, left)
    assert (d, k) == want
    assert d * k <= min(golhip.HALO_ROWS, max(rows, d)) and d * k <= left


@pytest.mark.parametrize("rows,tb,left,want", [
    (65536, 16, 100, [(16, 4), (12, 3)]),          # not 6 x 16 + 4: no short tail launch
    (16384, 16, 40, [(16, 1), (12, 2)]),
    (16384, 32, 100, [(32, 1), (24, 2), (20, 1)]),
    (65536, 20, 1000, [(20, 6)] * 8 + [(20, 2)]),
    (16384, 16, 20, [(12, 1), (8, 1)]),
    (16384, 16, 7, [(6, 1), (1, 1)]),
    (65536, 8, 100, [(8, 11), (6, 2)]),              # quads: no 4-turn tail
    (65536, 9, 100, [(9, 4), (8, 8)]),               # quads' own depth 9: 12 launches, the smallest 8
    (16384, 16, 36, [(12, 3)]),
])
def test_halo_schedule_sequence(rows, tb, left, want):
    """The whole schedule (golhip.hip depth_plan): fewest launches, then the
    largest smallest launch, in descending depth order."""
    seq, l = [], left
    while l > 0:
        d, k = golhip.halo_schedule(rows, tb, l)
        seq.append((d, k))
        l -= d * k
    assert seq == want


@pytest.mark.parametrize("tb", [1, 4, 12, 16, 32])
def test_halo_schedule_covers_turns(tb):
    for left in list(range(1, 200)) + [999, 1000, 10000]:
        seq, l = [], left
        while l > 0:
            d, k = golhip.halo_schedule(1 << 20, tb, l)
            assert 1 <= d <= tb and 1 <= k and d * k <= min(golhip.HALO_ROWS, l)
            seq += [d] * k
            l -= d * k
        assert sum(seq) == left and seq == sorted(seq, reverse=True)
        # never more launches than the greedy power-of-two schedule
        g, r = 0, left
        while r > 0:
            d = 1 << (min(r, tb).bit_length() - 1)
            r -= d
            g += 1
        assert len(seq) <= g


def test_product_build_macros():
    """The shipped libgolhip.so is built with the default tuning macros: no
    A/B or layout-experiment build (GOL_LOOP_PAD etc.) is mistaken for the
    product.  Macros that gave wrong results (GOL_SPLIT_NOHOOK) are gone:
    defining one is a compile error."""
    info = golhip.load().golhip_build_info().decode()
    want = {"GOL_LOOP_PAD": "0", "GOL_PARITY_FIX": "1", "GOL_PERSIST_STORE": "6", "GOL_PAIR_STORE": "-1",
            "GOL_PAIR_G2": "0", "GOL_FILL_PHASES": "4", "GOL_SKEW_STORE_CPOL": "16", "GOL_PERSIST_WG_COUNT": "1",
            "GOL_COMPACT_WPT": "4", "GOL_SKEW_WAIT_TRACE": "0", "GOL_K5R_NOCOPY": "0",
            # options that give wrong results by design need
            # GOLHIP_MEASUREMENT=1, test hooks GOLHIP_TEST_HOOKS=1 (refused otherwise:
            # tests/test_gpu_parity.py::test_wrong_result_options_need_measurement_consent)
            "CONSENT_MEASUREMENT": "halo_skip,flip_debug:1-3",
            "CONSENT_TEST_HOOKS": "resident_fault,resident_max_turns,flip_debug:4,golhip_test_ring_init",
            # the A/B knobs no default plan varies need
            # GOLHIP_TUNING=1; a product caller has the options below alone
            "CONSENT_TUNING": "persist_depth,persist_waves,dummy_rows,paired_bands,persist_half,persist_wg_tx,trace,"
                              "cu_count,fill_skip,skew_young,skew_hcap,skew_prio,skew_half,skew_tx,lds_depth,lds_waves,"
                              "lds_wg_cu,lds_age,lds_pre,lds_stride,lds_xcd,flip_overlap,skew_pairs",
            "PRODUCT_OPTIONS": "wpl,persistent,lds_band,skew,timing,persist_timeout_us,force_halo"}
    got = dict(kv.split("=", 1) for kv in info.split())
    assert got == want, info


def test_wrong_result_macro_is_a_compile_error(tmp_path):
    import os
    import subprocess
    src = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(golhip.__file__)), "..", "csrc",
                                        "gol_kernels.hip"))
    p = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-std=c++17", "-fsyntax-only",
                        "-DGOL_SPLIT_NOHOOK=1", src], capture_output=True, text=True, timeout=300)
    assert p.returncode != 0 and "GOL_SPLIT_NOHOOK" in p.stderr


def test_resident_turn_bound(tmp_path):
    """K1r's / K1p's super-step arithmetic is 32-bit.  A step of
    more than golk::kResidentMaxTurns turns runs as several resident launches
    of at most that many (golhip.hip step_locked), and at that bound
    J = ceil(turns / D), j * D and turns - j * D fit an int for every depth
    the kernels take (1..64): checked here with g++ on csrc/gol_limits.h."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = tmp_path / "bound.cpp"
    src.write_text(r'''
#include <climits>
#include <cstdio>
#include <initializer_list>
#include "gol_limits.h"
int main() {
    using namespace golk;
    for (long long left : {2ll, 1000ll, (long long)INT_MAX, (long long)INT_MAX + 1, 10000000000ll, LLONG_MAX / 2}) {
        const long long run = resident_turns(left);
        if (run < 1 || run > left || run > kResidentMaxTurns) return 1;
        if (left <= kResidentMaxTurns && run != left) return 2;
        for (int D = 1; D <= kResidentMaxDepth; ++D) {
            const long long J = (run + D - 1) / D;  // the kernel's int J, int j * D
            if (J > INT_MAX || (J - 1) * D > INT_MAX || (long long)run + D - 1 > INT_MAX) return 3;
        }
    }
    // 10^10 turns (main.go:37-41's default) in launches of the bound: 10 launches, none wraps
    long long left = 10000000000ll, n = 0;
    while (left > 0) { left -= resident_turns(left); ++n; }
    if (n != 10) return 4;
    std::puts("ok");
    return 0;
}
''')
    exe = tmp_path / "bound"
    subprocess.run(["g++", "-std=c++17", "-O1", "-I", os.path.join(root, "game-of-life-distributed_amd", "csrc"),
                    str(src), "-o", str(exe)], check=True, timeout=120)
    assert subprocess.run([str(exe)], capture_output=True, text=True, timeout=60).stdout.strip() == "ok"
