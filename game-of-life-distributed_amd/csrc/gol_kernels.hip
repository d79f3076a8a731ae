// gol_kernels.hip — gfx950 kernels of libgolhip.so.
//
// K1 gol_tb_kernel   : the B3/S23 torus turn (distributor.go:350-417, worker
//                      pool :304-347) for `DEPTH` fused turns per launch.
// K1g generic kernel : same turn for widths that are not a multiple of 32.
// K2 popcount        : len(calculateAliveCells(world)) (:420-432, ticker :292).
// K3 compaction      : initializeAliveCells flip list (:212-220) and the
//                      FinalTurnComplete alive list (:180), row-major.
// K4 pack / unpack   : 0/255 bytes <-> bits at the io boundary (:66-80, :186-191).
// K6 fill_random     : synthetic boards (BASELINE configs 2-5).
//
// Layout (DESIGN.md "Layout in HBM"): rows of Ww = ceil(W/32) uint32 words;
// cell (y, x) = bit x%32 of word x/32.  Everything here is integer work bound
// by HBM or VALU; none of it is matrix-shaped, so there is no MFMA.
#include "gol_kernels.h"
#include "gol_bits.h"

#include <algorithm>
#include <climits>
#include <type_traits>
#include <utility>

namespace golk {
#ifndef GOL_LOOP_PAD
#define GOL_LOOP_PAD 0  // code-layout experiments: 4-byte s_nop pads ahead of the main loops (profiles/r2la)
#endif
#ifndef GOL_FILL_PHASES
#define GOL_FILL_PHASES 4  // K1 fill phases: quarters (8: eighths, round-1 A/B, profiles/r1*)
#endif

template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F &&f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>()), ...);
}
// f(integral_constant<int, i>) for i = 0 .. N-1, unrolled at compile time
template <int N, typename F>
__device__ __forceinline__ void static_for(F &&f) {
    static_for_impl(f, std::make_integer_sequence<int, N>());
}

// ---------------------------------------------------------------------------
// Interleaved pair layout (boards run with two words per lane, W % 64 == 0).
// A row's canonical words (2c, 2c+1) hold cells 64c .. 64c+63 in order; the
// interleaved pair holds the even cells 64c+2k in bit k of word 2c and the
// odd cells 64c+2k+1 in bit k of word 2c+1.  Rows stay rows, so halo rows,
// strips and popcounts are layout-agnostic; only cell positions change.
// ---------------------------------------------------------------------------
__host__ __device__ __forceinline__ uint32_t unshuffle32(uint32_t x) {  // even bits -> low half, odd -> high
    uint32_t t;
    t = (x ^ (x >> 1)) & 0x22222222u; x ^= t ^ (t << 1);
    t = (x ^ (x >> 2)) & 0x0C0C0C0Cu; x ^= t ^ (t << 2);
    t = (x ^ (x >> 4)) & 0x00F000F0u; x ^= t ^ (t << 4);
    t = (x ^ (x >> 8)) & 0x0000FF00u; x ^= t ^ (t << 8);
    return x;
}
__host__ __device__ __forceinline__ uint32_t shuffle32(uint32_t x) {  // inverse of unshuffle32
    uint32_t t;
    t = (x ^ (x >> 8)) & 0x0000FF00u; x ^= t ^ (t << 8);
    t = (x ^ (x >> 4)) & 0x00F000F0u; x ^= t ^ (t << 4);
    t = (x ^ (x >> 2)) & 0x0C0C0C0Cu; x ^= t ^ (t << 2);
    t = (x ^ (x >> 1)) & 0x22222222u; x ^= t ^ (t << 1);
    return x;
}
__host__ __device__ __forceinline__ void il_encode(uint32_t a, uint32_t b, uint32_t &e, uint32_t &o) {
    const uint32_t ua = unshuffle32(a), ub = unshuffle32(b);
    e = (ua & 0xFFFFu) | (ub << 16);
    o = (ua >> 16) | (ub & 0xFFFF0000u);
}
__host__ __device__ __forceinline__ void il_decode(uint32_t e, uint32_t o, uint32_t &a, uint32_t &b) {
    a = shuffle32((e & 0xFFFFu) | (o << 16));
    b = shuffle32((e >> 16) | (o & 0xFFFF0000u));
}
// Interleaved quad layout (four words per lane, W % 128 == 0): word 4q + j of
// a row holds the cells 128q + 4k + j in bit k.  It is the pair layout applied
// twice: the pair encoding of (a, b) and (c, d) gives the even and odd cells
// of each 64-cell half; pairing the two even-cell words (e1, e2) again splits
// them into cells 4k (j = 0) and 4k + 2 (j = 2), the odd-cell words into
// 4k + 1 (j = 1) and 4k + 3 (j = 3).
__host__ __device__ __forceinline__ void il4_encode(const uint32_t (&c)[4], uint32_t (&w)[4]) {
    uint32_t e1, o1, e2, o2;
    il_encode(c[0], c[1], e1, o1);
    il_encode(c[2], c[3], e2, o2);
    il_encode(e1, e2, w[0], w[2]);
    il_encode(o1, o2, w[1], w[3]);
}
__host__ __device__ __forceinline__ void il4_decode(const uint32_t (&w)[4], uint32_t (&c)[4]) {
    uint32_t e1, o1, e2, o2;
    il_decode(w[0], w[2], e1, e2);
    il_decode(w[1], w[3], o1, o2);
    il_decode(e1, o1, c[0], c[1]);
    il_decode(e2, o2, c[2], c[3]);
}
// Canonical word i of a board stored in layout `il` (0 canonical, 2 pairs, 4 quads).
__device__ __forceinline__ uint32_t canon_word(const uint32_t *w, int64_t i, int il) {
    if (il == 0) return w[i];
    if (il == 2) {
        uint32_t a, b;
        il_decode(w[i & ~(int64_t)1], w[i | 1], a, b);
        return (i & 1) ? b : a;
    }
    const uint4 q = *reinterpret_cast<const uint4 *>(w + (i & ~(int64_t)3));
    uint32_t c[4];
    il4_decode({q.x, q.y, q.z, q.w}, c);
    return c[i & 3];
}

// In place, one quad of words per thread: layout `from` -> canonical -> `to`.
// Layout 4 implies W % 128 == 0 (whole quads); layout 2 only W % 64 == 0, so
// the last "quad" of the buffer may be a single pair.
__global__ __launch_bounds__(256) void convert_layout_kernel(uint32_t *__restrict__ w, int64_t nwords, int from, int to) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (4 * i >= nwords) return;
    if (4 * i + 4 > nwords) {  // a trailing pair: layouts 0 and 2 only
        uint32_t *p = w + 4 * i, a = p[0], b = p[1];
        if (from == 2) il_decode(p[0], p[1], a, b);
        if (to == 2) il_encode(a, b, p[0], p[1]);
        else p[0] = a, p[1] = b;
        return;
    }
    const uint4 v = reinterpret_cast<uint4 *>(w)[i];
    uint32_t x[4] = {v.x, v.y, v.z, v.w}, c[4];
    if (from == 4) {
        il4_decode(x, c);
    } else if (from == 2) {
        il_decode(x[0], x[1], c[0], c[1]);
        il_decode(x[2], x[3], c[2], c[3]);
    } else {
        for (int k = 0; k < 4; ++k) c[k] = x[k];
    }
    if (to == 4) {
        il4_encode(c, x);
    } else if (to == 2) {
        il_encode(c[0], c[1], x[0], x[1]);
        il_encode(c[2], c[3], x[2], x[3]);
    } else {
        for (int k = 0; k < 4; ++k) x[k] = c[k];
    }
    reinterpret_cast<uint4 *>(w)[i] = make_uint4(x[0], x[1], x[2], x[3]);
}

hipError_t launch_convert_layout(uint32_t *words, int64_t nwords, int from, int to, hipStream_t s) {
    if (from == to) return hipSuccess;
    const int64_t nq = (nwords + 3) / 4;
    if (nq == 0) return hipSuccess;
    hipLaunchKernelGGL(convert_layout_kernel, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, s, words, nwords, from, to);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// K1: temporal-blocked bit-sliced step.
//
// One wavefront = one tile of 64 lanes x WPL consecutive words of a row band
// (lane j holds words t0 + WPL*(j-1) ...); it streams the band's rows top to
// bottom through a D-stage register pipeline.  Stage t turns generation t-1
// row i into generation t row i-1, so after 2D rows of fill every input row
// yields one row D generations ahead.  Horizontal neighbours: the lane's own
// words plus one edge word from each adjacent lane (DPP); lanes 0 and 63 are
// the halo: their error front moves one cell per turn, so with D <= 32 lanes
// 1..62 are exact and stored.  Vertically a wave reads D extra rows above and
// below its band.
// Per stage, row and word: 2/WPL DPP + 2 alignbit + 2 bitop3 (3-cell row sum,
// shared by the three output rows that use it) + 7 bitop3 (column sum + rule).
// DPP and alignbit issue at half rate on gfx950, bitop3 at full rate, so
// WPL = 2 cuts a word-turn from ~17 to ~15 full-rate slots.
// HBM traffic per launch ~ 2 bits per cell (read + write) for D turns.
// ---------------------------------------------------------------------------
template <int WPL>
struct Lanes {
    uint32_t w[WPL];
};

// Horizontal 3-cell sums of one row (s0 + 2 s1 per cell, centre included).
// WPL == 1: the lane's word plus one edge bit from each adjacent lane
// (alignbit).  WPL == 2 uses the interleaved pair layout (see il_encode): w0
// holds the even cells 2k and w1 the odd cells 2k+1 of the lane's 64-cell
// chunk, so the west neighbour of an odd cell and the east neighbour of an
// even cell are the other word as is; only one word per side needs a one-bit
// funnel shift with the edge lane's bit.  WPL == 4: interleaved quads, word j
// holds cells 4k + j, so every neighbour word but two is another word of the
// lane as is.
template <int WPL>
__device__ __forceinline__ void row_sums(const Lanes<WPL> &x, uint32_t (&s0)[WPL], uint32_t (&s1)[WPL]) {
    uint32_t west[WPL], east[WPL];
    if constexpr (WPL == 1) {
        const uint32_t l = from_left_lane(x.w[0]);
        const uint32_t r = from_right_lane(x.w[0]);
        west[0] = __builtin_amdgcn_alignbit(x.w[0], l, 31);  // bit b = cell b-1
        east[0] = __builtin_amdgcn_alignbit(r, x.w[0], 1);   // bit b = cell b+1
    } else if constexpr (WPL == 4) {
        const uint32_t l3 = from_left_lane(x.w[3]);   // left chunk's cells 4k + 3 (bit 31 = its cell 127)
        const uint32_t r0 = from_right_lane(x.w[0]);  // right chunk's cells 4k (bit 0 = its cell 0)
        west[0] = __builtin_amdgcn_alignbit(x.w[3], l3, 31);  // cell 4k - 1
        west[1] = x.w[0];
        west[2] = x.w[1];
        west[3] = x.w[2];
        east[0] = x.w[1];
        east[1] = x.w[2];
        east[2] = x.w[3];
        east[3] = __builtin_amdgcn_alignbit(r0, x.w[0], 1);   // cell 4k + 4
    } else {
        const uint32_t l1 = from_left_lane(x.w[1]);   // left chunk's odd cells (bit 31 = its cell 63)
        const uint32_t r0 = from_right_lane(x.w[0]);  // right chunk's even cells (bit 0 = its cell 0)
        west[0] = __builtin_amdgcn_alignbit(x.w[1], l1, 31);  // cell 2k-1
        east[0] = x.w[1];                                     // cell 2k+1
        west[1] = x.w[0];                                     // cell 2k
        east[1] = __builtin_amdgcn_alignbit(r0, x.w[0], 1);   // cell 2k+2
    }
#pragma unroll
    for (int k = 0; k < WPL; ++k) {
        s0[k] = bop<kXor3>(west[k], x.w[k], east[k]);
        s1[k] = bop<kMaj>(west[k], x.w[k], east[k]);
    }
}

// One stage (turn t) for the row entering with role R (R = input index % 3).
template <int D, int R, int WPL>
__device__ __forceinline__ void stage(int t, Lanes<WPL> &x, uint32_t (&h0)[3][D][WPL], uint32_t (&h1)[3][D][WPL],
                                      uint32_t (&cc)[3][D][WPL]) {
    constexpr int N = R;            // slot of the row entering now
    constexpr int C = (R + 2) % 3;  // previous row (the one we emit)
    constexpr int P = (R + 1) % 3;  // the row before it
    // Horizontal 3-cell sums, as row_sums (kept inline here: the same code
    // through the helper allocates registers differently in the step kernels).
    uint32_t west[WPL], east[WPL];
    if constexpr (WPL == 1) {
        const uint32_t l = from_left_lane(x.w[0]);
        const uint32_t r = from_right_lane(x.w[0]);
        west[0] = __builtin_amdgcn_alignbit(x.w[0], l, 31);  // bit b = cell b-1
        east[0] = __builtin_amdgcn_alignbit(r, x.w[0], 1);   // bit b = cell b+1
    } else if constexpr (WPL == 4) {
        const uint32_t l3 = from_left_lane(x.w[3]);   // left chunk's cells 4k + 3 (bit 31 = its cell 127)
        const uint32_t r0 = from_right_lane(x.w[0]);  // right chunk's cells 4k (bit 0 = its cell 0)
        west[0] = __builtin_amdgcn_alignbit(x.w[3], l3, 31);  // cell 4k - 1
        west[1] = x.w[0];
        west[2] = x.w[1];
        west[3] = x.w[2];
        east[0] = x.w[1];
        east[1] = x.w[2];
        east[2] = x.w[3];
        east[3] = __builtin_amdgcn_alignbit(r0, x.w[0], 1);   // cell 4k + 4
    } else {
        const uint32_t l1 = from_left_lane(x.w[1]);   // left chunk's odd cells (bit 31 = its cell 63)
        const uint32_t r0 = from_right_lane(x.w[0]);  // right chunk's even cells (bit 0 = its cell 0)
        west[0] = __builtin_amdgcn_alignbit(x.w[1], l1, 31);  // cell 2k-1
        east[0] = x.w[1];                                     // cell 2k+1
        west[1] = x.w[0];                                     // cell 2k
        east[1] = __builtin_amdgcn_alignbit(r0, x.w[0], 1);   // cell 2k+2
    }
    uint32_t nx[WPL];
#pragma unroll
    for (int k = 0; k < WPL; ++k) {
        h0[N][t][k] = bop<kXor3>(west[k], x.w[k], east[k]);
        h1[N][t][k] = bop<kMaj>(west[k], x.w[k], east[k]);
        const uint32_t u0 = bop<kXor3>(h0[P][t][k], h0[C][t][k], h0[N][t][k]);
        const uint32_t u1 = bop<kMaj>(h0[P][t][k], h0[C][t][k], h0[N][t][k]);
        const uint32_t v0 = bop<kXor3>(h1[P][t][k], h1[C][t][k], h1[N][t][k]);
        const uint32_t v1 = bop<kMaj>(h1[P][t][k], h1[C][t][k], h1[N][t][k]);
        const uint32_t g1 = bop<kG1>(u1, v0, v1);
        const uint32_t g2 = bop<kG2>(u0, v1, cc[C][t][k]);
        nx[k] = bop<kNext>(u0, g1, g2);
    }
#pragma unroll
    for (int k = 0; k < WPL; ++k) {
        cc[N][t][k] = x.w[k];
        x.w[k] = nx[k];
    }
}

// Code layout.  On gfx950 the step kernels' 8-byte VALU instructions issue
// ~20 % faster at addresses = 4 (mod 8) than at 0 (mod 8): the same kernel
// shifted by one 4-byte instruction runs 65536^2 at 97 instead of 120 TCUPS,
// 262144^2 110 vs 133, 16384^2 52.5 vs 61.9 (profiles/r2la, same box).  The
// compiler does not track this, and every odd run of 4-byte instructions
// (SALU, s_waitcnt, s_nop hazard pads, VOP1/VOP2) flips the parity of all
// code after it.  parity_fix re-anchors it: `.p2align 3` then one s_nop puts
// the next instruction at 4 (mod 8) whatever came before (one or two
// s_nops executed), once per 3-row group (pinned by sched barriers; 2 =
// every pipeline step as well, which the hazard pads then mis-anchor).  The
// tree before it happened to sit on the fast parity in every main loop; the
// fix keeps it there whatever changes upstream of a loop (scripts/
// loop_parity.py reports the parity of every hot loop of a build).
#ifndef GOL_PARITY_FIX
#define GOL_PARITY_FIX 1  // profiles/r2lc: 16384^2 +1.2 %, the others within 0.6 % of the lucky layout
#endif
template <int LEVEL>
__device__ __forceinline__ void parity_fix() {
    if constexpr (GOL_PARITY_FIX >= LEVEL) {  // pinned: nothing is scheduled across it
        __builtin_amdgcn_sched_barrier(0);
        asm volatile(".p2align 3\n\ts_nop 0");
        __builtin_amdgcn_sched_barrier(0);
    }
}

// A group of 3 consecutive input rows through the first A of the D stages.
// Stage t of row i+1 needs stage t of row i (its row sum), so the rows run
// skewed by one stage: (row0, t), (row1, t-1), (row2, t-2) are independent and
// interleave, which hides the VALU->DPP hazard of each stage's serial chain.
// A < D is used while the pipeline fills: stage t only sees real rows from
// input index 2t on, so later stages would only compute garbage.
template <int D, int A, int WPL>
__device__ __forceinline__ void push_group(Lanes<WPL> &x0, Lanes<WPL> &x1, Lanes<WPL> &x2,
                                           uint32_t (&h0)[3][D][WPL], uint32_t (&h1)[3][D][WPL],
                                           uint32_t (&cc)[3][D][WPL]) {
    parity_fix<1>();
#pragma unroll
    for (int s = 0; s < A + 2; ++s) {
        parity_fix<2>();
        if (s < A) stage<D, 0, WPL>(s, x0, h0, h1, cc);
        if (s >= 1 && s - 1 < A) stage<D, 1, WPL>(s - 1, x1, h0, h1, cc);
        if (s >= 2 && s - 2 < A) stage<D, 2, WPL>(s - 2, x2, h0, h1, cc);
    }
}

template <int WPL>
__device__ __forceinline__ Lanes<WPL> vmov(const Lanes<WPL> &v) {
    Lanes<WPL> r;
#pragma unroll
    for (int k = 0; k < WPL; ++k) asm volatile("v_mov_b32 %0, %1" : "=v"(r.w[k]) : "v"(v.w[k]));
    return r;
}

// One wavefront streams output rows [r0, r0 + rows_here) of the tile whose
// first stored word is t0, D turns ahead; returns the popcount of its stored
// output words.  Shared by the per-launch and the persistent kernel.
// dir = -1 streams the band bottom to top (the rule is symmetric in y).
// With `claim` (an LDS counter shared with the wave streaming the same band
// from the other end) the wave takes its output rows three at a time from the
// counter and stops when the two fronts meet, so the band splits wherever the
// SIMD arbiter's service left the two waves.
// Output stores (STORE): kStoreDeferred = masked, one group late (K1);
// kStoreMasked = masked, right after the group; kStoreDummy = unconditional,
// masked rows to a dummy row (wave_id % dummy_rows of dst).
// kStoreAfterLoads = one group late like kStoreDeferred, but unconditional
// (masked rows / lanes to the dummy row) and issued AFTER the next group's
// prefetch loads: vmcnt counts in issue order, so the wait for those loads
// at the bottom of the body no longer waits for the stores' acks too.
// kStoreMaskedAfterLoads = the same, but masked stores (no dummy row).
// kStoreBufAfterLoads = after the loads, as buffer stores whose masked lanes
// carry an out-of-range offset (the hardware drops them): no branch, no dummy
// row, and a static vmcnt.  Needs each wave's band < 2 GiB (host-checked).
// kStoreBufImmediate = buffer stores right after the group (no deferral).
[[maybe_unused]] constexpr int kStoreDeferred = 0, kStoreMasked = 1, kStoreDummy = 2, kStoreAfterLoads = 3,
                               kStoreMaskedAfterLoads = 4, kStoreBufAfterLoads = 5, kStoreBufImmediate = 6;
#ifndef GOL_PERSIST_STORE
#define GOL_PERSIST_STORE 6  // immediate buffer stores: 16384^2 58.5 -> 59.0 TCUPS vs dummy-row stores (profiles/r2n)
#endif
#ifndef GOL_PAIR_STORE
#define GOL_PAIR_STORE -1  // -1: by words per lane (A/B builds override)
#endif
// K1's stores, measured per words per lane (profiles/r2m, same box): buffer
// stores after the loads 65536^2 114.6 -> 116.5 TCUPS (WPL 2); quads keep the
// deferred masked stores (262144^2: 129.0 vs 116.0 with buffer stores).
template <int WPL>
constexpr int pair_store() {
    return GOL_PAIR_STORE >= 0 ? GOL_PAIR_STORE : (WPL == 4 ? kStoreDeferred : kStoreBufAfterLoads);
}
#ifdef GOL_SPLIT_NOHOOK
#error "GOL_SPLIT_NOHOOK (round-2 timing experiment, wrong results) was removed"
#endif
#ifndef GOL_PAIR_G2
#define GOL_PAIR_G2 0
#endif
template <int WPL>
constexpr bool pair_g2() {
    return GOL_PAIR_G2 && pair_store<WPL>() == kStoreBufAfterLoads;
}

// G2 (kStoreBufAfterLoads only): the main loop takes two 3-row groups per
// body, so each body's prefetch loads have two groups of compute to land.
template <int D, bool SKIP, int WPL, int STORE = kStoreDeferred, bool LATE_CLAIM = true, bool G2 = false>
__device__ __forceinline__ uint32_t stream_band(const StepArgs &a, int r0, int rows_here, int t0, int wave_id,
                                                int dir = 1, int *claim = nullptr) {
    const int lane = threadIdx.x & 63;
    const int Ww = a.Ww;
    int col = (t0 + WPL * (lane - 1)) % Ww;  // WPL = 2 (4) needs Ww % 2 (4) == 0: a pair (quad) never wraps
    if (col < 0) col += Ww;
    const bool keep = lane >= 1 && lane <= kTileValid && (t0 + WPL * (lane - 1)) < Ww;

    // input row cursor (wave-uniform)
    int r = (dir > 0 ? r0 - D : r0 + rows_here - 1 + D) + a.in.off;
    const int wrap = a.in.wrap > 0 ? a.in.wrap : INT_MAX;
    if (a.in.wrap > 0) {
        r %= a.in.wrap;
        if (r < 0) r += a.in.wrap;
    }
    const uint32_t *__restrict__ src = a.src + col;
    auto load_next = [&]() -> Lanes<WPL> {
        const int pr = a.in.base + min(r, a.in.rmax);
        Lanes<WPL> v;
        if constexpr (WPL == 1) {
            v.w[0] = src[(size_t)pr * Ww];
        } else if constexpr (WPL == 4) {
            const uint4 q = *reinterpret_cast<const uint4 *>(src + (size_t)pr * Ww);
            v.w[0] = q.x;
            v.w[1] = q.y;
            v.w[2] = q.z;
            v.w[3] = q.w;
        } else {
            const uint2 q = *reinterpret_cast<const uint2 *>(src + (size_t)pr * Ww);
            v.w[0] = q.x;
            v.w[1] = q.y;
        }
        if (dir > 0)
            r = (r + 1 == wrap) ? 0 : r + 1;
        else
            r = (r == 0) ? wrap - 1 : r - 1;  // no wrap: only prefetched rows past the band go below 0
        return v;
    };

    // Output stores, by STORE: kStoreDeferred stores under the lane mask
    // (halo lanes, pipeline-fill rows and rows past the band or the meeting
    // row store nothing) and one group late: a group's stores are issued at
    // the top of the next body, just before its prefetch loads, so the
    // in-order vmcnt wait for those loads at the bottom of that body also
    // covers the stores, a whole group after they were issued (stores issued
    // right after the group are followed straight away by that wait, which
    // then stalls on their acks: 97 -> 115 TCUPS for K1 at 65536^2 on the
    // boxes where it did).  kStoreMasked stores right away under the mask;
    // kStoreDummy stores unconditionally, masked rows/lanes to a dummy row
    // (one of the first `dummy_rows` physical rows of dst, spread over waves).
    uint32_t *const dst_row0 = a.dst + (size_t)(a.dst_base + (dir > 0 ? r0 : r0 + rows_here - 1)) * Ww + col;
    const ptrdiff_t dst_step = dir > 0 ? (ptrdiff_t)Ww : -(ptrdiff_t)Ww;
    int lim = claim ? 0 : rows_here;  // output rows [0, lim) of this wave's order are its own
    uint32_t *const dummy = a.dst + (size_t)(wave_id % a.dummy_rows) * Ww + col;
    uint32_t cnt = 0;
    // kStoreBufAfterLoads: one buffer resource over the wave's output rows
    // [r0, r0 + rows_here) of dst (wave-uniform), a byte offset per lane
    const __amdgpu_buffer_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc(
        a.dst + (size_t)(a.dst_base + r0) * Ww, (short)0,
        (STORE == kStoreBufAfterLoads || STORE == kStoreBufImmediate) ? rows_here * Ww * 4 : 0,
        0x00020000);
    // output rows counted into the popcount, in this wave's out_idx order
    const int clo = dir > 0 ? a.count_lo - r0 : r0 + rows_here - a.count_hi;
    const int chi = dir > 0 ? a.count_hi - r0 : r0 + rows_here - a.count_lo;
    auto emit = [&](const Lanes<WPL> &y, int out_idx) {
        const bool ok = keep && (unsigned)out_idx < (unsigned)lim;
        uint32_t pc = 0;
        auto put = [&](uint32_t *p) {
            if constexpr (WPL == 1)
                *p = y.w[0];
            else if constexpr (WPL == 4)
                *reinterpret_cast<uint4 *>(p) = make_uint4(y.w[0], y.w[1], y.w[2], y.w[3]);
            else
                *reinterpret_cast<uint2 *>(p) = make_uint2(y.w[0], y.w[1]);
        };
        if constexpr (STORE == kStoreBufAfterLoads || STORE == kStoreBufImmediate) {
            const int rel = dir > 0 ? out_idx : rows_here - 1 - out_idx;
            const int off = ok ? (rel * Ww + col) * 4 : INT_MAX;  // out of range: dropped
            if constexpr (WPL == 1)
                __builtin_amdgcn_raw_buffer_store_b32(y.w[0], brs, off, 0, 0);
            else if constexpr (WPL == 2)
                __builtin_amdgcn_raw_buffer_store_b64((__attribute__((ext_vector_type(2))) unsigned)
                                                      {y.w[0], y.w[1]}, brs, off, 0, 0);
            else
                __builtin_amdgcn_raw_buffer_store_b128((__attribute__((ext_vector_type(4))) unsigned)
                                                       {y.w[0], y.w[1], y.w[2], y.w[3]}, brs, off, 0, 0);
        } else if constexpr (STORE == kStoreDummy || STORE == kStoreAfterLoads)
            put(ok ? dst_row0 + (ptrdiff_t)out_idx * dst_step : dummy);
        else if (ok)
            put(dst_row0 + (ptrdiff_t)out_idx * dst_step);
#pragma unroll
        for (int k = 0; k < WPL; ++k) pc += __builtin_popcount(y.w[k]);
        cnt += (ok && out_idx >= clo && out_idx < chi) ? pc : 0u;
    };

    uint32_t h0[3][D][WPL], h1[3][D][WPL], cc[3][D][WPL];
#pragma unroll
    for (int s = 0; s < 3; ++s)
#pragma unroll
        for (int t = 0; t < D; ++t)
#pragma unroll
            for (int k = 0; k < WPL; ++k) h0[s][t][k] = h1[s][t][k] = cc[s][t][k] = 0u;

    // Prefetch: the next group's rows are issued at the top of the body and
    // moved into place at the bottom (an inline-asm v_mov: a plain copy lets
    // the register allocator merge the registers and hoist the copy, and its
    // vmcnt wait, to the loop top), so the wait lands a full group of compute
    // after issue.  The first group also goes through vmov, so no load is
    // pending on the loop's entry edge either.
    Lanes<WPL> x0 = vmov(load_next()), x1 = vmov(load_next()), x2 = vmov(load_next());
    int oi = -2 * D;  // output row of the group's first input row (input index oi + 2D)
    // Pipeline fill in three steps: while the group's last input index
    // i = oi + 2D + 2 satisfies i/2 + 1 <= A, stages >= A cannot see real rows
    // yet, so a body with only the first A = D/4, D/2, 3D/4 stages runs.
    // Runtime loops keep the code small (a fully unrolled triangular fill
    // thrashes the instruction cache beside the main loop).
    auto fill = [&](auto a_tag) {
        constexpr int A = decltype(a_tag)::value;
        if constexpr (SKIP && A >= 1 && A < D) {
            for (; (oi + 2 * D + 2) / 2 + 1 <= A; oi += 3) {
                const Lanes<WPL> n0 = load_next(), n1 = load_next(), n2 = load_next();
                __builtin_amdgcn_sched_barrier(0);
                Lanes<WPL> y0 = x0, y1 = x1, y2 = x2;
                push_group<D, A, WPL>(y0, y1, y2, h0, h1, cc);
                __builtin_amdgcn_sched_barrier(0);
                x0 = vmov(n0);
                x1 = vmov(n1);
                x2 = vmov(n2);
            }
        }
    };
#if GOL_FILL_PHASES == 8
    if constexpr (D >= 8) {  // eighths: closer to the exact triangle, more code
        fill(std::integral_constant<int, D / 8>());
        fill(std::integral_constant<int, 2 * D / 8>());
        fill(std::integral_constant<int, 3 * D / 8>());
        fill(std::integral_constant<int, 4 * D / 8>());
        fill(std::integral_constant<int, 5 * D / 8>());
        fill(std::integral_constant<int, 6 * D / 8>());
        fill(std::integral_constant<int, 7 * D / 8>());
    } else
#endif
    {
        fill(std::integral_constant<int, D / 4>());
        fill(std::integral_constant<int, D / 2>());
        fill(std::integral_constant<int, 3 * D / 4>());
    }
    bool more = true, pend = false;
    Lanes<WPL> q0, q1, q2;  // the previous group's output rows (stored one body late)
    int qoi = 0;
    if constexpr (STORE == kStoreAfterLoads || STORE == kStoreBufAfterLoads) {  // the first body stores nothing real
#pragma unroll
        for (int k = 0; k < WPL; ++k) q0.w[k] = q1.w[k] = q2.w[k] = 0u;
        qoi = -8;
    }
    if constexpr (G2) {
        static_assert(STORE == kStoreBufAfterLoads, "G2 needs static store counts");
        Lanes<WPL> x3 = vmov(load_next()), x4 = vmov(load_next()), x5 = vmov(load_next());
        Lanes<WPL> q3 = q0, q4 = q0, q5 = q0;
        for (; claim ? more : oi < rows_here; oi += 6) {
            const Lanes<WPL> n0 = load_next(), n1 = load_next(), n2 = load_next();
            const Lanes<WPL> n3 = load_next(), n4 = load_next(), n5 = load_next();
            emit(q0, qoi);
            emit(q1, qoi + 1);
            emit(q2, qoi + 2);
            emit(q3, qoi + 3);
            emit(q4, qoi + 4);
            emit(q5, qoi + 5);
            const int need = claim ? min(6, max(0, oi + 6)) : 0;
            int old = 0, o = 0;
            if (need > 0 && lane == 0)
                o = __hip_atomic_fetch_add(claim, -need, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __builtin_amdgcn_sched_barrier(0);
            Lanes<WPL> y0 = x0, y1 = x1, y2 = x2, y3 = x3, y4 = x4, y5 = x5;
            push_group<D, D, WPL>(y0, y1, y2, h0, h1, cc);
            push_group<D, D, WPL>(y3, y4, y5, h0, h1, cc);
            if (need > 0) {
                asm volatile("" : "+v"(o));  // the LDS wait after both groups
                old = __builtin_amdgcn_readfirstlane(o);
                lim = max(oi, 0) + min(need, max(0, old));
                more = old > need;
            }
            q0 = y0;
            q1 = y1;
            q2 = y2;
            q3 = y3;
            q4 = y4;
            q5 = y5;
            qoi = oi;
            pend = true;
            __builtin_amdgcn_sched_barrier(0);
            x0 = vmov(n0);
            x1 = vmov(n1);
            x2 = vmov(n2);
            x3 = vmov(n3);
            x4 = vmov(n4);
            x5 = vmov(n5);
        }
        if (pend) {
            emit(q0, qoi);
            emit(q1, qoi + 1);
            emit(q2, qoi + 2);
            emit(q3, qoi + 3);
            emit(q4, qoi + 4);
            emit(q5, qoi + 5);
        }
        return cnt;
    }
    for (int i = 0; i < GOL_LOOP_PAD; ++i) asm volatile("s_nop 0");
    for (; claim ? more : oi < rows_here; oi += 3) {
        if (STORE == kStoreDeferred && pend) {
            emit(q0, qoi);
            emit(q1, qoi + 1);
            emit(q2, qoi + 2);
        }
        const Lanes<WPL> n0 = load_next(), n1 = load_next(), n2 = load_next();
        if constexpr (STORE == kStoreAfterLoads || STORE == kStoreBufAfterLoads) {
            emit(q0, qoi);
            emit(q1, qoi + 1);
            emit(q2, qoi + 2);
        } else if (STORE == kStoreMaskedAfterLoads && pend) {
            emit(q0, qoi);
            emit(q1, qoi + 1);
            emit(q2, qoi + 2);
        }
        // claim this group's rows >= 0; the LDS round trip hides under the group
        const int need = claim ? min(3, max(0, oi + 3)) : 0;
        // LATE_CLAIM: wait for the LDS round trip after the group rather than
        // before it.  Measured per kernel (profiles/r1g): K1 65536^2 115 (late)
        // vs 96 TCUPS (early); K1p 16384^2 54 (late) vs 59 (early).
        int old = 0, o = 0;
        if constexpr (LATE_CLAIM) {
            if (need > 0 && lane == 0)
                o = __hip_atomic_fetch_add(claim, -need, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else if (need > 0) {
            if (lane == 0) o = __hip_atomic_fetch_add(claim, -need, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            old = __builtin_amdgcn_readfirstlane(o);
        }
        __builtin_amdgcn_sched_barrier(0);
        Lanes<WPL> y0 = x0, y1 = x1, y2 = x2;
        push_group<D, D, WPL>(y0, y1, y2, h0, h1, cc);
        if (need > 0) {
            if constexpr (LATE_CLAIM) {
                asm volatile("" : "+v"(o));  // keep the LDS wait here, after the group
                old = __builtin_amdgcn_readfirstlane(o);
            }
            lim = max(oi, 0) + min(need, max(0, old));
            more = old > need;
        }
        if constexpr (STORE == kStoreDeferred || STORE == kStoreAfterLoads || STORE == kStoreMaskedAfterLoads ||
                      STORE == kStoreBufAfterLoads) {
            q0 = y0;
            q1 = y1;
            q2 = y2;
            qoi = oi;
            pend = true;
        } else {
            emit(y0, oi);
            emit(y1, oi + 1);
            emit(y2, oi + 2);
        }
        __builtin_amdgcn_sched_barrier(0);
        x0 = vmov(n0);
        x1 = vmov(n1);
        x2 = vmov(n2);
    }
    if ((STORE == kStoreDeferred || STORE == kStoreAfterLoads || STORE == kStoreMaskedAfterLoads ||
         STORE == kStoreBufAfterLoads) && pend) {
        emit(q0, qoi);
        emit(q1, qoi + 1);
        emit(q2, qoi + 2);
    }
    return cnt;
}

__host__ __device__ constexpr int tile_words(int wpl) { return kTileValid * wpl; }

template <int D, bool SKIP, int WPL>
__global__ __launch_bounds__(256) void gol_tb_kernel(StepArgs a) {
    const int wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    const int tiles_x = (a.Ww + tile_words(WPL) - 1) / tile_words(WPL);
    const int S = a.rows_per_wave;
    const int strip = wave / tiles_x;
    const int tile = wave - strip * tiles_x;
    const int r0 = strip * S;
    if (r0 >= a.rows_out) return;  // wave-uniform
    const uint32_t cnt = stream_band<D, SKIP, WPL>(a, r0, min(S, a.rows_out - r0), tile * tile_words(WPL), wave);
    if (a.alive) {
        const uint32_t tot = wave_sum_u32(cnt);
        if ((threadIdx.x & 63) == 0) atomicAdd(a.alive, (unsigned long long)tot);
    }
}

// K1 with paired bands: a workgroup of 8 waves covers 4 consecutive (region,
// tile) pairs in row-major order, a region being 2 S rows of one tile; the
// two waves of each SIMD (w and w + 4, the older and the younger) stream
// pair w & 3 from the top and from the bottom and claim output rows from a
// shared LDS counter until they meet, so the SIMD arbiter's oldest-first
// service no longer leaves the younger wave running alone at the end of the
// launch.
template <int D, int WPL, bool CNT>
__global__ __launch_bounds__(512) void gol_tb_pair_kernel(StepArgs a) {
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int tiles_x = (a.Ww + tile_words(WPL) - 1) / tile_words(WPL);
    const int S = a.rows_per_wave;
    const int q = blockIdx.x * 4 + (w & 3);
    const int region = q / tiles_x;
    const int tile = q - region * tiles_x;
    const int r0 = region * 2 * S;
    const int len = r0 < a.rows_out ? min(2 * S, a.rows_out - r0) : 0;
    __shared__ int s_claim[4];
    __shared__ unsigned long long s_cnt;  // (waves arrived << 40) | cells, for the fused count
    if (w < 4 && lane == 0) s_claim[w] = len;
    if (CNT && threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
    if (len == 0) return;  // wave-uniform, after the only barrier
    const uint32_t cnt = stream_band<D, true, WPL, pair_store<WPL>(), true, pair_g2<WPL>()>(a, r0, len, tile * tile_words(WPL), blockIdx.x * 8 + w,
                                                   w < 4 ? 1 : -1, &s_claim[w & 3]);
    if constexpr (!CNT) {
        if (a.alive) {
            const uint32_t tot = wave_sum_u32(cnt);
            if (lane == 0 && tot) atomicAdd(a.alive, (unsigned long long)tot);
        }
    } else if (a.alive) {
        // The counting instance (last launch of a step): one device atomic per
        // workgroup, by the last wave to arrive.  Device atomics on one address
        // serialise (~20 ns each); per wave they cost a 1-turn launch at 5120^2
        // (3 840 waves finishing together) 78 us on 10 us.  A separate
        // instance because the extra code slowed the count-free launches.
        const uint32_t tot = wave_sum_u32(cnt);
        int active = 0;
        for (int i = 0; i < 4; ++i) {
            const int qi = blockIdx.x * 4 + i;
            active += (qi / tiles_x) * 2 * S < a.rows_out ? 2 : 0;
        }
        if (lane == 0) {
            const unsigned long long mine = (1ull << 40) | tot;
            const unsigned long long now = atomicAdd(&s_cnt, mine) + mine;
            const unsigned long long sum = now & ((1ull << 40) - 1);
            if ((int)(now >> 40) == active && sum) atomicAdd(a.alive, sum);
        }
    }
}

// Popcount of a workgroup's waves into *alive with one device atomic (the
// last of `active` waves to arrive adds the sum).
__device__ __forceinline__ void wg_count(unsigned long long *alive, unsigned long long *s_cnt, uint32_t cnt, int active) {
    const uint32_t tot = wave_sum_u32(cnt);
    if ((threadIdx.x & 63) == 0) {
        const unsigned long long mine = (1ull << 40) | tot;
        const unsigned long long now = atomicAdd(s_cnt, mine) + mine;
        const unsigned long long sum = now & ((1ull << 40) - 1);
        if ((int)(now >> 40) == active && sum) atomicAdd(alive, sum);
    }
}

// Row helpers of the skewed band stacks (K1w below): one tile row as lanes.
template <int WPL>
__device__ __forceinline__ void put_lanes(uint32_t *row, const uint32_t (&v)[WPL]) {
    const int lane = threadIdx.x & 63;
    if constexpr (WPL == 1)
        row[lane] = v[0];
    else if constexpr (WPL == 2)
        reinterpret_cast<uint2 *>(row)[lane] = make_uint2(v[0], v[1]);
    else
        reinterpret_cast<uint4 *>(row)[lane] = make_uint4(v[0], v[1], v[2], v[3]);
}
template <int WPL>
__device__ __forceinline__ Lanes<WPL> get_lanes(const uint32_t *row) {
    const int lane = threadIdx.x & 63;
    Lanes<WPL> v;
    if constexpr (WPL == 1) {
        v.w[0] = row[lane];
    } else if constexpr (WPL == 2) {
        const uint2 q = reinterpret_cast<const uint2 *>(row)[lane];
        v.w[0] = q.x;
        v.w[1] = q.y;
    } else {
        const uint4 q = reinterpret_cast<const uint4 *>(row)[lane];
        v.w[0] = q.x;
        v.w[1] = q.y;
        v.w[2] = q.z;
        v.w[3] = q.w;
    }
    return v;
}
template <int WPL>
__device__ __forceinline__ Lanes<WPL> load_row(const uint32_t *p) {
    Lanes<WPL> v;
    if constexpr (WPL == 1) {
        v.w[0] = *p;
    } else if constexpr (WPL == 2) {
        const uint2 q = *reinterpret_cast<const uint2 *>(p);
        v.w[0] = q.x;
        v.w[1] = q.y;
    } else {
        const uint4 q = *reinterpret_cast<const uint4 *>(p);
        v.w[0] = q.x;
        v.w[1] = q.y;
        v.w[2] = q.z;
        v.w[3] = q.w;
    }
    return v;
}
// push_group for the fill of a skewed band: before stage t of a row with input
// index ii in {2t, 2t + 1} (its first two valid rows), hook(t, ii, x) exports it.
template <int D, int A, int WPL, typename Hook>
__device__ __forceinline__ void push_group_exp(Lanes<WPL> &x0, Lanes<WPL> &x1, Lanes<WPL> &x2,
                                               uint32_t (&h0)[3][D][WPL], uint32_t (&h1)[3][D][WPL],
                                               uint32_t (&cc)[3][D][WPL], int ii0, Hook &&hook) {
    parity_fix<1>();
#pragma unroll
    for (int s = 0; s < A + 2; ++s) {
        // every step: the hook's export stores (4-byte SALU address work) flip
        // the parity; 65536^2 +0.5 %, quads -0.5 % (profiles/r2pf), so pairs only
        if constexpr (WPL <= 2) parity_fix<1>();
        if (s < A) {
            hook(s, ii0, x0);
            stage<D, 0, WPL>(s, x0, h0, h1, cc);
        }
        if (s >= 1 && s - 1 < A) {
            hook(s - 1, ii0 + 1, x1);
            stage<D, 1, WPL>(s - 1, x1, h0, h1, cc);
        }
        if (s >= 2 && s - 2 < A) {
            hook(s - 2, ii0 + 2, x2);
            stage<D, 2, WPL>(s - 2, x2, h0, h1, cc);
        }
    }
}
// ---------------------------------------------------------------------------
// K1w: skewed band stacks (round 3; torus and row strips, per launch).
//
// K1 computes the D-turn trapezoid at both ends of every band (~1.25 D^2
// extra stage-rows a band); K1s computes every stage-row once but leaves the
// triangles between bands to a second, latency-bound kernel.  K1w skews
// the bands instead: band [a, e) of input rows owns generation g of the rows
// [a + g, e + g).  Generation g + 1 of its rows needs generation g of
// [a + g, e + g + 1]: its own rows and, at the bottom, the first two rows of
// the band below it -- rows that band computes first, in its pipeline fill.
// So no band needs anything from above, the band below hands over its top
// rows early, and nobody computes a triangle.
//
// Pipeline (as stream_band): at push j (generation-0 row j entering), stage s
// receives generation s of row j - s and emits generation s + 1 of row
// j - s - 1; the band needs stage s at the pushes j in [a + 2 s + 2,
// e + 2 s + 2), gen D goes out at j in [a + 2 D, e + 2 D).  Pushes run in
// groups of 3 rows from a:
//  * fill (j - a < 2 D): stages [0, A) only (phases A = D/4, D/2, 3D/4, D),
//    exporting to LDS generation P of the rows a + P + m (the input of stage
//    P at push a + 2 P + m) for the drain phases P = D/4, D/2, 3D/4 of the
//    band above;
//  * main: all stages on board rows, until the drain;
//  * drain (d = j - e in [2 P, 2 P')): only stages [P, D) are needed; their
//    input is generation P of row e + d - P, the band below's export (its
//    rows a' + P + m, a' = e).  A group runs in the phase of its first row,
//    so each phase exports 2 rows beyond its pushes.  The drain computes
//    1.25 D^2 stage-rows instead of the exact D^2 (the triangle).
// A stack of bands is one workgroup of one tile column (LDS hand-offs only,
// no cross-workgroup wait); its bottom band has no band below in the
// workgroup and computes its drain in full from board rows (2 D^2), so it
// is shorter by `hcap` rows.  Torus: the input rows [-D, H - D) produce
// generation D of [0, H) without wrapping the output; row strips: the
// halo rows feed the top band's first D rows and the bottom band's drain.
// ---------------------------------------------------------------------------
#ifndef GOL_SKEW_WAIT_TRACE
#define GOL_SKEW_WAIT_TRACE 0  // diagnostic builds: per-wave load-wait ticks of K1w (option "trace")
#endif
#ifndef GOL_SKEW_STORE_CPOL
#define GOL_SKEW_STORE_CPOL 16  // K1w output stores sc1 (16384^2 +3.6 %, 8192-row strips +1.9 % in a round-3 A/B whose scratch data was not kept; 0 plain, 2 nt)
#endif
// Pipeline phases of a band: fill phase i runs stages [0, STEP (i + 1))
// (then [0, D)), drain phase j stages [P(j), D) with P(j) = STEP (j + 1).
// Bands other than a stack's bottom one are multiples of 3 rows, so drain
// groups start at d = 0 (mod 3) and, STEP being a multiple of 3, never
// straddle a drain phase: phase j imports exactly the 2 (P(j+1) - P(j))
// rows of generation P(j) its pushes d in [2 P(j), 2 P(j+1)) take in.
// Coarser phases compute more stage-rows nobody needs (both at the fill and
// at the drain, about D^2 / 4 each for phases of D / 4 stages); finer ones
// more code (each phase is a loop of its own).
template <int D>
struct SkewPlan {
    static constexpr int STEP = D > 20 ? 6 : 3;
    static constexpr int NPH = (D - 1) / STEP;  // drain phases (also the fill phases before the full one)
    static constexpr int P(int j) { return (j + 1) * STEP; }
    static constexpr int NROWS(int j) { return 2 * ((j + 1 < NPH ? P(j + 1) : D) - P(j)); }
    static constexpr int BASE(int j) {
        int b = 0;
        for (int i = 0; i < j; ++i) b += NROWS(i);
        return b;
    }
    static constexpr int NEXP = BASE(NPH);  // row NEXP of a wave's LDS slot = dummy (fill rows not exported)
    static_assert(NPH >= 1 && STEP % 3 == 0, "skew depth >= 4");
};


// ---------------------------------------------------------------------------
// The pair rule in K1w's main loop (round 6; gol_bits.h pair_sum / pair_rule).
// Generation-t rows pair up as (2m, 2m + 1) by the parity of their index in
// the band's input frame (push j brings row j - t to stage t, so a row's
// parity is that of j + t).  Per stage the state alternates:
//  * before an odd row 2m + 1 arrives: a = S(2m - 1), b = S(2m), c = row 2m;
//    the odd row completes the pair: p = b + S(2m + 1), out row 2m =
//    pair_rule(a, p, c); then a = S(2m + 1), c = row 2m + 1 (b is dead);
//  * before an even row 2m + 2 arrives: p, a = S(2m + 1), c = row 2m + 1;
//    out row 2m + 1 = pair_rule(S(2m + 2), p, c); then b = S(2m + 2),
//    c = row 2m + 2 (p is dead).
// So a stage's live state is 5 words (a, b, c) or 6 (p, a, c) per word of a
// lane, where the 9-LUT stage keeps 5: half the stages are in each phase, so
// the pipeline costs 10 % more VGPRs and runs at most 18 turns a launch at two
// words per lane (242 VGPRs at 20 with the 9-LUT stage).  Groups still hold 3
// rows, so the phase of (group row q, stage t) flips from group to group: the
// main loop takes two groups a body (KQ = parity of the group's first push).
// The fill keeps the 9-LUT stages (on the pair state it spills, DESIGN.md
// §5.13); pr_enter converts the state before the main loop, and the drain
// continues on the pair state (push_group_pr_hi) where D = 0 mod 3, else
// pr_leave converts it back (b from p and a: pair_unsum).
// ---------------------------------------------------------------------------
template <int D, int WPL>
struct PairSt {
    uint32_t a0[D][WPL], a1[D][WPL];
    uint32_t b0[D][WPL], b1[D][WPL];
    uint32_t p0[D][WPL], p1[D][WPL], p2[D][WPL];
    uint32_t c[D][WPL];
};

// One stage (turn t) of a row of phase PH (1: odd row, completes its pair).
template <int D, int PH, int WPL>
__device__ __forceinline__ void stage_pr(int t, Lanes<WPL> &x, PairSt<D, WPL> &st) {
    uint32_t west[WPL], east[WPL];
    if constexpr (WPL == 1) {
        const uint32_t l = from_left_lane(x.w[0]);
        const uint32_t r = from_right_lane(x.w[0]);
        west[0] = __builtin_amdgcn_alignbit(x.w[0], l, 31);
        east[0] = __builtin_amdgcn_alignbit(r, x.w[0], 1);
    } else if constexpr (WPL == 4) {
        const uint32_t l3 = from_left_lane(x.w[3]);
        const uint32_t r0 = from_right_lane(x.w[0]);
        west[0] = __builtin_amdgcn_alignbit(x.w[3], l3, 31);
        west[1] = x.w[0];
        west[2] = x.w[1];
        west[3] = x.w[2];
        east[0] = x.w[1];
        east[1] = x.w[2];
        east[2] = x.w[3];
        east[3] = __builtin_amdgcn_alignbit(r0, x.w[0], 1);
    } else {
        const uint32_t l1 = from_left_lane(x.w[1]);
        const uint32_t r0 = from_right_lane(x.w[0]);
        west[0] = __builtin_amdgcn_alignbit(x.w[1], l1, 31);
        east[0] = x.w[1];
        west[1] = x.w[0];
        east[1] = __builtin_amdgcn_alignbit(r0, x.w[0], 1);
    }
    uint32_t nx[WPL];
#pragma unroll
    for (int k = 0; k < WPL; ++k) {
        const uint32_t n0 = bop<kXor3>(west[k], x.w[k], east[k]);
        const uint32_t n1 = bop<kMaj>(west[k], x.w[k], east[k]);
        if constexpr (PH == 1) {
            uint32_t p0, p1, p2;
            pair_sum(st.b0[t][k], st.b1[t][k], n0, n1, p0, p1, p2);
            nx[k] = pair_rule(st.a0[t][k], st.a1[t][k], p0, p1, p2, st.c[t][k]);
            st.p0[t][k] = p0;
            st.p1[t][k] = p1;
            st.p2[t][k] = p2;
            st.a0[t][k] = n0;
            st.a1[t][k] = n1;
        } else {
            nx[k] = pair_rule(n0, n1, st.p0[t][k], st.p1[t][k], st.p2[t][k], st.c[t][k]);
            st.b0[t][k] = n0;
            st.b1[t][k] = n1;
        }
    }
#pragma unroll
    for (int k = 0; k < WPL; ++k) {
        st.c[t][k] = x.w[k];
        x.w[k] = nx[k];
    }
}

// push_group on the pair state: rows of pushes KQ + 0, 1, 2 (mod 2).
template <int D, int KQ, int WPL>
__device__ __forceinline__ void push_group_pr(Lanes<WPL> &x0, Lanes<WPL> &x1, Lanes<WPL> &x2,
                                              PairSt<D, WPL> &st) {
    parity_fix<1>();
    static_for<D + 2>([&](auto s_tag) {
        constexpr int s = decltype(s_tag)::value;
        parity_fix<2>();
        if constexpr (s < D) stage_pr<D, (KQ + 0 + s) & 1, WPL>(s, x0, st);
        if constexpr (s >= 1 && s - 1 < D) stage_pr<D, (KQ + 1 + s - 1) & 1, WPL>(s - 1, x1, st);
        if constexpr (s >= 2) stage_pr<D, (KQ + 2 + s - 2) & 1, WPL>(s - 2, x2, st);
    });
}

// push_group_pr for the last stages only (the drain): the group's rows enter
// stage LO (push_group_hi on the pair state; the stages below LO are dead).
template <int D, int KQ, int LO, int WPL>
__device__ __forceinline__ void push_group_pr_hi(Lanes<WPL> &x0, Lanes<WPL> &x1, Lanes<WPL> &x2,
                                                 PairSt<D, WPL> &st) {
    parity_fix<1>();
    static_for<D + 2>([&](auto s_tag) {
        constexpr int s = decltype(s_tag)::value;
        if constexpr (s >= LO) {
            parity_fix<2>();
            if constexpr (s < D) stage_pr<D, (KQ + 0 + s) & 1, WPL>(s, x0, st);
            if constexpr (s - 1 >= LO && s - 1 < D) stage_pr<D, (KQ + 1 + s - 1) & 1, WPL>(s - 1, x1, st);
            if constexpr (s - 2 >= LO) stage_pr<D, (KQ + 2 + s - 2) & 1, WPL>(s - 2, x2, st);
        }
    });
}

// 9-LUT stage state (slots 1, 2 = pushes k - 2, k - 1 of a push k = 0 mod 3)
// -> pair state before push k (parity KQ); pr_leave the inverse.
template <int D, int KQ, int WPL>
__device__ __forceinline__ void pr_enter(const uint32_t (&h0)[3][D][WPL], const uint32_t (&h1)[3][D][WPL],
                                         const uint32_t (&cc)[3][D][WPL], PairSt<D, WPL> &st) {
#pragma unroll
    for (int t = 0; t < D; ++t)
#pragma unroll
        for (int k = 0; k < WPL; ++k) {
            st.c[t][k] = cc[2][t][k];
            if (((KQ + t) & 1) == 1) {  // the next row completes a pair
                st.a0[t][k] = h0[1][t][k];
                st.a1[t][k] = h1[1][t][k];
                st.b0[t][k] = h0[2][t][k];
                st.b1[t][k] = h1[2][t][k];
            } else {
                pair_sum(h0[1][t][k], h1[1][t][k], h0[2][t][k], h1[2][t][k], st.p0[t][k], st.p1[t][k], st.p2[t][k]);
                st.a0[t][k] = h0[2][t][k];
                st.a1[t][k] = h1[2][t][k];
            }
        }
}
template <int D, int KQ, int WPL>
__device__ __forceinline__ void pr_leave(const PairSt<D, WPL> &st, uint32_t (&h0)[3][D][WPL],
                                         uint32_t (&h1)[3][D][WPL], uint32_t (&cc)[3][D][WPL]) {
#pragma unroll
    for (int t = 0; t < D; ++t)
#pragma unroll
        for (int k = 0; k < WPL; ++k) {
            cc[2][t][k] = st.c[t][k];
            if (((KQ + t) & 1) == 1) {
                h0[1][t][k] = st.a0[t][k];
                h1[1][t][k] = st.a1[t][k];
                h0[2][t][k] = st.b0[t][k];
                h1[2][t][k] = st.b1[t][k];
            } else {
                h0[2][t][k] = st.a0[t][k];
                h1[2][t][k] = st.a1[t][k];
                pair_unsum(st.p0[t][k], st.p1[t][k], st.a0[t][k], st.a1[t][k], h0[1][t][k], h1[1][t][k]);
            }
        }
}

// push_group for the last stages only: the group's rows enter stage LO.
template <int D, int LO, int WPL>
__device__ __forceinline__ void push_group_hi(Lanes<WPL> &x0, Lanes<WPL> &x1, Lanes<WPL> &x2,
                                              uint32_t (&h0)[3][D][WPL], uint32_t (&h1)[3][D][WPL],
                                              uint32_t (&cc)[3][D][WPL]) {
    parity_fix<1>();
#pragma unroll
    for (int s = LO; s < D + 2; ++s) {
        parity_fix<2>();
        if (s < D) stage<D, 0, WPL>(s, x0, h0, h1, cc);
        if (s - 1 >= LO && s - 1 < D) stage<D, 1, WPL>(s - 1, x1, h0, h1, cc);
        if (s - 2 >= LO) stage<D, 2, WPL>(s - 2, x2, h0, h1, cc);
    }
}

// One band [ab, eb) of input rows (StepArgs frame) of tile `tile`.  self: no
// band below in the workgroup (compute the drain from board rows).  Exports
// go to exp_mine (LDS slot of this wave), imports come from exp_next.
// HALF (half-wave tiles): lanes 0-31 and 32-63 are two tiles of 30 stored
// lanes each (lanes 0, 31, 32, 63 are their halos), of the same tile column
// but rows `dr` apart (the same band of two stacks): narrow boards waste less
// of a wave on padding (16384^2: nine 60-word tiles for 512 words instead of
// five 124-word ones).  Everything lane-wise (loads, stores, LDS hand-offs)
// just takes the upper half's rows `dr` further down.
template <int D, int WPL, bool HALF = false, bool PR = false>
__device__ __forceinline__ uint32_t stream_skew(const StepArgs &a, int ab, int eb, int tile, bool self,
                                                uint32_t *exp_mine, const uint32_t *exp_next, int *flag_mine,
                                                int *flag_next, unsigned *error, unsigned long long *phase_tr,
                                                int dr = 0) {
    using SP = SkewPlan<D>;
    constexpr int ROW = 64 * WPL;  // words of one LDS row
    constexpr int TV = HALF ? kHalfTileValid : kTileValid;
    const int lane = threadIdx.x & 63;
    const int hl = HALF ? (lane & 31) : lane;        // lane within its tile
    const int rofs = (HALF && lane >= 32) ? dr : 0;  // the upper half's rows
    const int Ww = a.Ww;
    const int S = eb - ab;
    const int t0 = tile * TV * WPL;
    int col = (t0 + WPL * (hl - 1)) % Ww;
    if (col < 0) col += Ww;
    const bool keep = hl >= 1 && hl <= TV && (t0 + WPL * (hl - 1)) < Ww;
    // input rows ab, ab + 1, ... through the row map (torus wrap or halo clamp)
    int r = ab + rofs + a.in.off;
    const int wrap = a.in.wrap > 0 ? a.in.wrap : INT_MAX;
    if (a.in.wrap > 0) {
        r %= a.in.wrap;
        if (r < 0) r += a.in.wrap;
    }
    const uint32_t *__restrict__ src = a.src + col;
    auto load_next = [&]() -> Lanes<WPL> {
        const Lanes<WPL> v = load_row<WPL>(src + (size_t)(a.in.base + min(r, a.in.rmax)) * Ww);
        r = (r + 1 == wrap) ? 0 : r + 1;
        return v;
    };
    // generation D of row ab + D + oi leaves at push ab + 2 D + oi
    // (buffer stores for every width: a masked store's branch and EXEC writes
    // put hazard s_nops between parity_fix and the group's first DPP)
    const __amdgpu_buffer_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc(
        a.dst + (size_t)(a.dst_base + ab + D) * Ww, (short)0, (S + (HALF ? dr : 0)) * Ww * 4, 0x00020000);
    const int clo = a.count_lo - (ab + D + rofs), chi = a.count_hi - (ab + D + rofs);
    const int colw = col + rofs * Ww;  // the lane's word offset from the band's first output row
    uint32_t cnt = 0;
    auto emit = [&](const Lanes<WPL> &y, int oi) {
        const bool ok = keep && (unsigned)oi < (unsigned)S;
        const int off = ok ? (oi * Ww + colw) * 4 : INT_MAX;  // out of range: dropped
        if constexpr (WPL == 1)
            __builtin_amdgcn_raw_buffer_store_b32(y.w[0], brs, off, 0, GOL_SKEW_STORE_CPOL);
        else if constexpr (WPL == 2)
            __builtin_amdgcn_raw_buffer_store_b64((__attribute__((ext_vector_type(2))) unsigned){y.w[0], y.w[1]}, brs,
                                                  off, 0, GOL_SKEW_STORE_CPOL);
        else
            __builtin_amdgcn_raw_buffer_store_b128(
                (__attribute__((ext_vector_type(4))) unsigned){y.w[0], y.w[1], y.w[2], y.w[3]}, brs, off, 0,
                GOL_SKEW_STORE_CPOL);
        uint32_t pc = 0;
#pragma unroll
        for (int k = 0; k < WPL; ++k) pc += __builtin_popcount(y.w[k]);
        cnt += (ok && oi >= clo && oi < chi) ? pc : 0u;
    };
    // fill exports: the input of stage P (generation P of row ab + P + m) at
    // fill push 2 P + m, for the band above's drain phase P
    auto hook = [&](int s, int k, const Lanes<WPL> &x) {
        if (s % SP::STEP != 0 || s == 0 || s / SP::STEP > SP::NPH) return;  // s = P(j), folded per stage
        const int j = s / SP::STEP - 1;
        const int m = k - 2 * SP::P(j);
        const int row = (unsigned)m < (unsigned)SP::NROWS(j) ? SP::BASE(j) + m : SP::NEXP;
        put_lanes<WPL>(exp_mine + row * ROW, x.w);
    };

    uint32_t h0[3][D][WPL], h1[3][D][WPL], cc[3][D][WPL];
#pragma unroll
    for (int s = 0; s < 3; ++s)
#pragma unroll
        for (int t = 0; t < D; ++t)
#pragma unroll
            for (int k = 0; k < WPL; ++k) h0[s][t][k] = h1[s][t][k] = cc[s][t][k] = 0u;

    Lanes<WPL> x0 = vmov(load_next()), x1 = vmov(load_next()), x2 = vmov(load_next());
    int k = 0;  // push index of x0, from ab
    // GOL_SKEW_WAIT_TRACE (diagnostic build, option "trace"): s_memrealtime
    // ticks each wave spends waiting for its next group's rows
    [[maybe_unused]] unsigned long long wt0 = 0, wmain = 0, nmain = 0, wfill = 0, nfill = 0;
    auto fill = [&](auto a_tag) {
        constexpr int A = decltype(a_tag)::value;
        for (; A == D ? k <= 2 * D - 1 : (k + 2) / 2 <= A - 1; k += 3) {
            const Lanes<WPL> n0 = load_next(), n1 = load_next(), n2 = load_next();
            __builtin_amdgcn_sched_barrier(0);
            Lanes<WPL> y0 = x0, y1 = x1, y2 = x2;
            push_group_exp<D, A, WPL>(y0, y1, y2, h0, h1, cc, k, hook);
            if constexpr (A == D) {
                emit(y0, k - 2 * D);
                emit(y1, k + 1 - 2 * D);
                emit(y2, k + 2 - 2 * D);
            }
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (GOL_SKEW_WAIT_TRACE) wt0 = __builtin_amdgcn_s_memrealtime();
            x0 = vmov(n0);
            x1 = vmov(n1);
            x2 = vmov(n2);
            if constexpr (GOL_SKEW_WAIT_TRACE) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                wfill += __builtin_amdgcn_s_memrealtime() - wt0;
                ++nfill;
            }
        }
    };
    static_for<SP::NPH>([&](auto j) { fill(std::integral_constant<int, SP::P(decltype(j)::value)>()); });
    fill(std::integral_constant<int, D>());
    if (phase_tr && lane == 0) phase_tr[0] = (unsigned long long)__builtin_amdgcn_s_memrealtime();  // fill done
    // exports done: this wave's LDS writes complete before the flag (LDS
    // operations of a wave complete in order; no wait on its global loads)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_store(flag_mine, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);

    Lanes<WPL> q0, q1, q2;
#pragma unroll
    for (int i = 0; i < WPL; ++i) q0.w[i] = q1.w[i] = q2.w[i] = 0u;
    int qoi = -8;  // the first body stores nothing real
    [[maybe_unused]] PairSt<D, WPL> st;  // PR: the main loop's and the drain's stage state
    // main: every stage on board rows (the bottom band of a stack to the end)
    const int kmain = S + (self ? 2 * D : 2 * SP::P(0));
    for (int i = 0; i < GOL_LOOP_PAD; ++i) asm volatile("s_nop 0");
    if constexpr (PR) {
        // the pair rule, two groups a body: the fill leaves k at KSTART (= 0
        // mod 6), other bands are multiples of 6 rows (gol_skew_kernel), so
        // the loop ends exactly at kmain where a drain follows; a stack's
        // bottom band may run up to 5 rows past its end (masked stores)
        constexpr int KSTART = 3 * ((2 * D + 2) / 3);
        static_assert(KSTART % 6 == 0, "the pair main loop starts at an even push");
        {
            pr_enter<D, 0, WPL>(h0, h1, cc, st);
            for (; k < kmain; k += 6) {
                {
                    const Lanes<WPL> n0 = load_next(), n1 = load_next(), n2 = load_next();
                    emit(q0, qoi);
                    emit(q1, qoi + 1);
                    emit(q2, qoi + 2);
                    __builtin_amdgcn_sched_barrier(0);
                    Lanes<WPL> y0 = x0, y1 = x1, y2 = x2;
                    push_group_pr<D, 0, WPL>(y0, y1, y2, st);
                    q0 = y0;
                    q1 = y1;
                    q2 = y2;
                    qoi = k - 2 * D;
                    __builtin_amdgcn_sched_barrier(0);
                    x0 = vmov(n0);
                    x1 = vmov(n1);
                    x2 = vmov(n2);
                }
                {
                    const Lanes<WPL> n0 = load_next(), n1 = load_next(), n2 = load_next();
                    emit(q0, qoi);
                    emit(q1, qoi + 1);
                    emit(q2, qoi + 2);
                    __builtin_amdgcn_sched_barrier(0);
                    Lanes<WPL> y0 = x0, y1 = x1, y2 = x2;
                    push_group_pr<D, 1, WPL>(y0, y1, y2, st);
                    q0 = y0;
                    q1 = y1;
                    q2 = y2;
                    qoi = k + 3 - 2 * D;
                    __builtin_amdgcn_sched_barrier(0);
                    x0 = vmov(n0);
                    x1 = vmov(n1);
                    x2 = vmov(n2);
                }
            }
            // the drain continues on the pair state (h0 / h1 / cc dead here)
            // where its phases are whole two-group bodies, else on the 9-LUT one
            if constexpr (D % 3 != 0) pr_leave<D, 0, WPL>(st, h0, h1, cc);
        }
    }
    for (; !PR && k < kmain; k += 3) {
        const Lanes<WPL> n0 = load_next(), n1 = load_next(), n2 = load_next();
        emit(q0, qoi);
        emit(q1, qoi + 1);
        emit(q2, qoi + 2);
        __builtin_amdgcn_sched_barrier(0);
        Lanes<WPL> y0 = x0, y1 = x1, y2 = x2;
        push_group<D, D, WPL>(y0, y1, y2, h0, h1, cc);
        q0 = y0;
        q1 = y1;
        q2 = y2;
        qoi = k - 2 * D;
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (GOL_SKEW_WAIT_TRACE) wt0 = __builtin_amdgcn_s_memrealtime();
        x0 = vmov(n0);
        x1 = vmov(n1);
        x2 = vmov(n2);
        if constexpr (GOL_SKEW_WAIT_TRACE) {
            asm volatile("s_waitcnt vmcnt(3)" ::: "memory");  // the rows have landed
            wmain += __builtin_amdgcn_s_memrealtime() - wt0;
            ++nmain;
        }
    }
    if constexpr (GOL_SKEW_WAIT_TRACE) {
        if (phase_tr && lane == 0) {
            phase_tr[32] = wmain;  // (block, 32 + wave): main-loop wait ticks, groups
            phase_tr[33] = nmain;
            phase_tr[64] = wfill;  // (block, 48 + wave): fill wait ticks, groups
            phase_tr[65] = nfill;
        }
    }
    if (phase_tr && lane == 0) phase_tr[1] = (unsigned long long)__builtin_amdgcn_s_memrealtime();  // main done
    if (!self) {
        // the band below has exported its top rows (almost always long ago)
        if (__hip_atomic_load(flag_next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0) {
            const long long t_start = (long long)__builtin_amdgcn_s_memrealtime();
            while (__hip_atomic_load(flag_next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0) {
                if ((long long)__builtin_amdgcn_s_memrealtime() - t_start > 200000000ll) {  // 2 s: never
                    if (error && lane == 0) __hip_atomic_store(error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the flag read before the imports
        // the imports of the group at push kg: generation P of rows e + d - P
        // (d = kg - S + row), P the phase of the group's first row
        auto imports = [&](int kg, Lanes<WPL> &y0, Lanes<WPL> &y1, Lanes<WPL> &y2) {
            const int d = kg - S;
            int base = SP::BASE(0) - 2 * SP::P(0);
            static_for<SP::NPH>([&](auto j) {
                constexpr int J = decltype(j)::value;
                if (J > 0 && d >= 2 * SP::P(J)) base = SP::BASE(J) - 2 * SP::P(J);
            });
            const int top = SP::NEXP - 1;  // the last phase clamps (rows past the drain)
            y0 = get_lanes<WPL>(exp_next + min(base + d, top) * ROW);
            y1 = get_lanes<WPL>(exp_next + min(base + d + 1, top) * ROW);
            y2 = get_lanes<WPL>(exp_next + min(base + d + 2, top) * ROW);
        };
        {
            Lanes<WPL> n0, n1, n2;
            imports(k, n0, n1, n2);
            x0 = vmov(n0);  // waited here, not at the loop head (keeps parity_fix next to the group)
            x1 = vmov(n1);
            x2 = vmov(n2);
        }
        // the pair rule: two groups a body (KQ 0, 1), as in the main loop; the
        // drain phases span multiples of 6 pushes when D = 0 mod 3 (2 P(j) with
        // STEP = 3 or 6, 2 D), so the parity of k stays that of KSTART
        auto drain_pr = [&](auto kq_tag, auto lo_tag) {
            constexpr int KQ = decltype(kq_tag)::value, LO = decltype(lo_tag)::value;
            Lanes<WPL> n0, n1, n2;
            imports(k + 3, n0, n1, n2);
            __builtin_amdgcn_sched_barrier(0);
            Lanes<WPL> y0 = x0, y1 = x1, y2 = x2;
            push_group_pr_hi<D, KQ, LO, WPL>(y0, y1, y2, st);
            parity_fix<1>();  // (the stores and LDS loads: most of a short phase's body)
            emit(q0, qoi);
            emit(q1, qoi + 1);
            emit(q2, qoi + 2);
            q0 = y0;
            q1 = y1;
            q2 = y2;
            qoi = k - 2 * D;
            __builtin_amdgcn_sched_barrier(0);
            x0 = vmov(n0);
            x1 = vmov(n1);
            x2 = vmov(n2);
            k += 3;
        };
        auto drain = [&](auto lo_tag, int kend) {
            constexpr int LO = decltype(lo_tag)::value;
            if constexpr (PR && D % 3 == 0) {
                if constexpr (LO == SP::P(SP::NPH - 1) && D - LO <= 6) {
                    // the last phase, 2 (D - LO) pushes: straight-line bodies (as a
                    // loop of one or two trips its hazard pads moved most of it
                    // off the fast code parity)
                    static_for<(D - LO) / 3>([&](auto) {
                        drain_pr(std::integral_constant<int, 0>(), lo_tag);
                        drain_pr(std::integral_constant<int, 1>(), lo_tag);
                    });
                    return;
                }
                while (k < kend) {
                    drain_pr(std::integral_constant<int, 0>(), lo_tag);
                    drain_pr(std::integral_constant<int, 1>(), lo_tag);
                }
                return;
            }
            for (; k < kend; k += 3) {
                Lanes<WPL> n0, n1, n2;
                imports(k + 3, n0, n1, n2);
                __builtin_amdgcn_sched_barrier(0);
                Lanes<WPL> y0 = x0, y1 = x1, y2 = x2;
                // the previous group's stores after this group: their offset
                // and count arithmetic right before the group put a hazard
                // s_nop between parity_fix and the first DPP (slow parity)
                push_group_hi<D, LO, WPL>(y0, y1, y2, h0, h1, cc);
                __builtin_amdgcn_sched_barrier(0);
                emit(q0, qoi);
                emit(q1, qoi + 1);
                emit(q2, qoi + 2);
                q0 = y0;
                q1 = y1;
                q2 = y2;
                qoi = k - 2 * D;
                __builtin_amdgcn_sched_barrier(0);
                x0 = vmov(n0);
                x1 = vmov(n1);
                x2 = vmov(n2);
            }
        };
        static_for<SP::NPH>([&](auto j) {
            constexpr int J = decltype(j)::value;
            drain(std::integral_constant<int, SP::P(J)>(), S + 2 * (J + 1 < SP::NPH ? SP::P(J + 1) : D));
        });
    }
    emit(q0, qoi);
    emit(q1, qoi + 1);
    emit(q2, qoi + 2);
    return cnt;
}

// K1w: one workgroup = one stack = tx tiles x (8 / tx) bands; wave w takes
// tile w % tx and stack position w / tx (top to bottom).
template <int D, int WPL, bool HALF = false, bool PR = false>
__global__ __launch_bounds__(512) void gol_skew_kernel(SkewArgs p) {
    using SP = SkewPlan<D>;
    constexpr int ROW = 64 * WPL;
    __shared__ uint32_t s_exp[8][(SP::NEXP + 1) * ROW];
    __shared__ int s_flag[8];
    __shared__ unsigned long long s_cnt;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int sy = 8 / p.tx;
    const int tcols = (p.tiles_x + p.tx - 1) / p.tx;
    const int stack = blockIdx.x / tcols, tc = blockIdx.x - stack * tcols;
    const int tile = tc * p.tx + w % p.tx, pos = w / p.tx;
    if (lane == 0) s_flag[w] = 0;
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
    if (tile >= p.tiles_x) return;  // wave-uniform, after the only barrier (its stack's waves all leave)
    if (p.prio_young && w >= 4) __builtin_amdgcn_s_setprio(1);
    // HALF: the stacks split the first half of the rows; each wave's upper
    // lanes take the same band L / 2 rows further down (L even, host-checked)
    const int L = HALF ? p.base.rows_out / 2 : p.base.rows_out;
    const int A0 = (int)((int64_t)stack * L / p.nst) - D, E0 = (int)((int64_t)(stack + 1) * L / p.nst) - D;
    const int64_t Ls = (int64_t)(E0 - A0) + p.hcap;
    int cum = 0, tot = 0;
    for (int q = 0; q < sy; ++q) {
        tot += p.wgt[q];
        cum += q < pos ? p.wgt[q] : 0;
    }
    const bool bottom = pos == sy - 1;
    // band boundaries at multiples of 3 rows from the stack start (drain
    // groups aligned with the drain phases, SkewPlan; 6 for the pair rule's
    // two-group main-loop body); the bottom band takes the rest
    constexpr int G = PR ? 6 : 3;
    const int ab = A0 + (int)(Ls * cum / tot) / G * G;
    const int eb = bottom ? E0 : A0 + (int)(Ls * (cum + p.wgt[pos]) / tot) / G * G;
    const long long t_start = p.trace ? (long long)__builtin_amdgcn_s_memrealtime() : 0;
    const uint32_t cnt = stream_skew<D, WPL, HALF, PR>(p.base, ab, eb, tile, bottom, s_exp[w], bottom ? nullptr : s_exp[w + p.tx],
                                             &s_flag[w], bottom ? nullptr : &s_flag[w + p.tx], p.error,
                                             (p.trace && blockIdx.x < 1024) ? p.trace + 8 + 2 * (blockIdx.x * 64 + 16 + w)
                                                                            : nullptr,
                                             L);
    if (p.trace && lane == 0 && blockIdx.x < 1024) {
        p.trace[8 + 2 * (blockIdx.x * 64 + w)] = (unsigned long long)t_start;
        p.trace[8 + 2 * (blockIdx.x * 64 + w) + 1] = (unsigned long long)__builtin_amdgcn_s_memrealtime();
    }
    if (p.base.alive) wg_count(p.base.alive, &s_cnt, cnt, sy * min(p.tx, p.tiles_x - tc * p.tx));
}

// ---------------------------------------------------------------------------
// K1p: persistent multi-super-step kernel (torus mode, one device).
//
// One workgroup of NW wavefronts per CU stays resident for J super-steps of
// D turns.  Workgroup (wy, wx) owns a wg_tx x wg_sy block of (tile, strip)
// units; super-step j reads generation jD from buf[(first + j) & 1] and
// writes generation (j+1)D to the other buffer.  Its inputs are the outputs
// of its 3 x 3 workgroup neighbourhood at super-step j-1, and the buffer it
// overwrites was last read by that same neighbourhood during j-1, so the one
// wait "all 9 neighbours finished j-1" covers both hazards.  Hand-off per
// MI355X guide Guideline 16: stores -> vmcnt(0) -> barrier -> lane 0
// release fence -> vmcnt(0) -> relaxed agent store of the progress counter;
// consumer: relaxed agent polls -> lane 0 acquire fence -> vmcnt(0) ->
// barrier -> loads.  Every spin is bounded: on timeout the kernel sets
// *error and all workgroups drain out.
// ---------------------------------------------------------------------------
__host__ __device__ constexpr int persist_waves(int depth, int wpl) { return depth * wpl <= 16 ? 16 : 8; }

#ifndef GOL_PERSIST_WG_COUNT
#define GOL_PERSIST_WG_COUNT 1  // per-workgroup count atomic in K1p (0 = per wave, A/B builds)
#endif
template <int D, int WPL, int NW>
__global__ __launch_bounds__(NW * 64) void gol_persist_kernel(PersistArgs p) {
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int b = blockIdx.x;
    const int wx = b % p.cols, wy = b / p.cols;
    const int tile = wx * p.wg_tx + w % p.wg_tx;
    int r0, band, dir = 1;
    const int ry = w / p.wg_tx;  // band row within the workgroup stack
    // paired bands: wave w (band row ry < wg_sy/2) and wave w + NW/2 (the
    // younger wave on the same SIMD) share the two-band region of pair
    // ry % (wg_sy/2), streaming it from the top and from the bottom
    const bool paired = p.paired != 0;
    if (paired) {
        const int hr = p.wg_sy / 2;
        r0 = wy * p.wg_sy * p.S + 2 * (ry % hr) * p.S;
        band = 2 * p.S;
        dir = ry < hr ? 1 : -1;
    } else if (p.S_old > 0) {
        // unequal bands: the SIMD arbiter serves the oldest wave first, so the
        // band rows of waves 0 .. NW/2-1 (the first on each SIMD) are taller
        // than those of their younger SIMD mates (see try_persist)
        const int hr = p.wg_sy / 2;
        const int base = wy * p.wg_sy * p.S;
        r0 = base + (ry < hr ? ry * p.S_old : hr * p.S_old + (ry - hr) * p.S_young);
        band = ry < hr ? p.S_old : p.S_young;
        if (ry == p.wg_sy - 1) band = base + p.wg_sy * p.S - r0;  // the last band row takes the rounding
    } else {
        r0 = (wy * p.wg_sy + ry) * p.S;
        band = p.S;
    }
    const int rows_here = (tile < p.tiles_x && r0 < p.base.rows_out) ? min(band, p.base.rows_out - r0) : 0;

    // neighbour workgroup polled by lane k < 9
    int nb = b;
    if (lane < 9) {
        const int ny = (wy + lane / 3 - 1 + p.wg_y) % p.wg_y;
        const int nx = (wx + lane % 3 - 1 + p.cols) % p.cols;
        nb = ny * p.cols + nx;
    }
    __shared__ int s_abort;
    __shared__ int s_claim[2][NW / 2];  // per pair, double-buffered over super-steps
#if GOL_PERSIST_WG_COUNT
    __shared__ unsigned long long s_cnt;  // (waves arrived << 40) | cells, for the fused count
    if (threadIdx.x == 0) s_cnt = 0;
#endif
    if (threadIdx.x == 0) s_abort = 0;
    if (paired && w < NW / 2 && lane == 0) s_claim[0][w] = rows_here;
    __syncthreads();

    uint32_t cnt = 0;
    long long tr_wait = 0, tr_band = 0, tr_max = 0;
    const long long tr_t0 = (long long)__builtin_amdgcn_s_memrealtime();
    for (int j = 0; j < p.J; ++j) {
        const long long tr_w0 = (long long)__builtin_amdgcn_s_memrealtime();
        if (j > 0) {
            if (w == NW - 1) {  // the last wave polls: wave 0 polling cost 16 % at 65536^2 wpl 2 (r1e)
                const long long t_start = (long long)__builtin_amdgcn_s_memrealtime();
                for (;;) {
                    const unsigned v = __hip_atomic_load(&p.progress[nb], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (__all(v >= (unsigned)j)) break;
                    const unsigned err = __hip_atomic_load(p.error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (err || (long long)__builtin_amdgcn_s_memrealtime() - t_start > p.timeout_ticks) {
                        if (lane == 0) {
                            atomicOr(p.error, 1u);
                            s_abort = 1;
                        }
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
                if (lane == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            __syncthreads();
            if (s_abort) return;  // uniform over the workgroup
        }
        const long long tr_b0 = (long long)__builtin_amdgcn_s_memrealtime();
        tr_wait += tr_b0 - tr_w0;
        StepArgs a = p.base;
        const bool odd = ((p.first + j) & 1) != 0;
        a.src = odd ? p.buf1 : p.buf0;
        a.dst = odd ? p.buf0 : p.buf1;
        int *claim = nullptr;
        if (paired) {
            claim = &s_claim[j & 1][w % (NW / 2)];
            // every claim of super-step j-1 is done (barrier above): re-arm its counter for j+1
            if (w < NW / 2 && lane == 0) s_claim[(j + 1) & 1][w] = rows_here;
        }
        // half_last: a step of J D - D/2 turns ends with a D/2-turn super-step
        // here instead of a separate per-launch kernel (16384^2: 110 us for 8
        // turns as a K1 launch vs ~37 us at the resident rate)
        if (rows_here <= 0)
            cnt = 0u;
        else if (D >= 2 && p.half_last && j == p.J - 1)
            cnt = stream_band<(D >= 2 ? D / 2 : 1), true, WPL, GOL_PERSIST_STORE, false>(
                a, r0, rows_here, tile * tile_words(WPL), b * NW + w, dir, claim);
        else
            cnt = stream_band<D, true, WPL, GOL_PERSIST_STORE, false>(a, r0, rows_here, tile * tile_words(WPL),
                                                                       b * NW + w, dir, claim);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        {
            const long long tr_e = (long long)__builtin_amdgcn_s_memrealtime();
            const long long d = tr_e - tr_b0;
            tr_band += d;
            tr_max = d > tr_max ? d : tr_max;
            if (p.trace && j == p.J / 2 && lane == 0) {  // per-wave (start, end) of one super-step
                p.trace[8 + 2 * (b * 64 + w)] = (unsigned long long)tr_b0;
                p.trace[8 + 2 * (b * 64 + w) + 1] = (unsigned long long)tr_e;
            }
        }
        __syncthreads();
        if (threadIdx.x == (NW - 1) * 64 && !(p.fault && b == 0)) {  // (tests: workgroup 0 never reports)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(&p.progress[b], (unsigned)(j + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if (p.trace && lane == 0) {  // diagnostics: per-wave band time, workgroup wait time
        atomicAdd(&p.trace[0], (unsigned long long)tr_band);
        atomicMax(&p.trace[1], (unsigned long long)tr_max);
        if (w == 0) {
            atomicAdd(&p.trace[2], (unsigned long long)tr_wait);
            atomicAdd(&p.trace[3], (unsigned long long)((long long)__builtin_amdgcn_s_memrealtime() - tr_t0));
            atomicAdd(&p.trace[4], 1ull);
        }
    }
    if (p.base.alive) {
        const uint32_t tot = wave_sum_u32(cnt);
#if GOL_PERSIST_WG_COUNT
        // one device atomic per workgroup (see gol_tb_pair_kernel<D, WPL, true>)
        if (lane == 0) {
            const unsigned long long mine = (1ull << 40) | tot;
            const unsigned long long now = atomicAdd(&s_cnt, mine) + mine;
            const unsigned long long sum = now & ((1ull << 40) - 1);
            if ((int)(now >> 40) == NW && sum) atomicAdd(p.base.alive, sum);
        }
#else
        if (lane == 0 && tot) atomicAdd(p.base.alive, (unsigned long long)tot);
#endif
    }
}

// ---------------------------------------------------------------------------
// K1r: resident LDS bands (small tori, one workgroup of 8 waves per CU).
//
// Boards up to ~8192^2 hold too few cells per wave for the register
// pipelines: K1w's bands there are 20-40 rows against a 20-stage pipeline,
// K1p recomputes 2 D halo rows per 16-row band.  K1r keeps each band in LDS
// instead.  Workgroup b owns the full-width rows [r0, r0 + h) and holds them
// with D halo rows above and below (R = h + 2D rows, two buffers); a
// super-step runs D turns in LDS, turn t computing rows [t, R - t) (the
// halo rows go stale one row a turn), with the column wrap of the torus
// taken in LDS, so there are no halo lanes and no tiles.  Between
// super-steps the band's top and bottom D rows go to global memory and the
// neighbours' come back: Guideline 16's write-through hand-off (sc1 buffer
// stores, every wave's vmcnt(0), a barrier, one sc1 flag store; the
// consumer's wave 0 polls both neighbours' flags with sc1 loads, a barrier,
// then sc1 buffer loads), no cache-wide fence.  The edge buffers alternate
// by super-step parity: the wait for a neighbour's super-step j flag also
// proves it read our j - 1 edges, which the slot we overwrite held.
// Per row and word: the lane's word (pair) and one neighbour word each side
// from LDS, the row sums (2 LUTs, and a funnel shift per pair side), the
// column sums and the rule (7 LUTs), one LDS store; each buffer has 3 spare
// rows for the row loop's prefetch.  Every wait is bounded (error word, all drain).
// Pairs (WPL 2) sit in LDS as two planes (round 5): a row of LS = Ww + 8
// words holds the even-cell words E[c] at [0, P) and the odd-cell words O[c]
// at [PO + 1, PO + 1 + P), PO = LS / 2, with one ghost word each for the
// column wrap: E[P] (= E[0]) at P and O[-1] (= O[P - 1]) at PO.  A lane's
// four words E[c], E[c + 1], O[c - 1], O[c] are then two ds_read2_b32 of
// consecutive words across the lanes (the interleaved layout's odd-word
// reads were 2-way bank conflicts: 33 % of LDS cycles, profiles/r4k1rfinal),
// and its store one ds_write2_b32 plus the ghost store (the lanes of
// columns 0 and P - 1 write the ghosts, the others rewrite their E[c]).
// ---------------------------------------------------------------------------
// A row's words as loaded: the lane's own word (pair) and one neighbour word on each side.
constexpr int kHaloRegs = 4;  // K1r: 16-B halo granules per thread loaded ahead (more: loaded at the store)

template <int WPL>
struct LdsRaw {
    uint32_t c[WPL], l, r;
};

// The lane's word (pair) of an LDS row and the one neighbour word on each
// side its row sums need: three ds_reads.  (Taking the neighbour words from
// the adjacent lanes by DPP instead, with only the wave-edge lanes reading
// theirs, saved the 2-way bank conflicts of every-second-word reads but ran
// 8192^2 at 24-26 instead of 31-32 TCUPS: load -> DPP -> alignbit is a longer
// dependent chain at two waves per SIMD; profiles/r4o.)
// WPL 1: o, ol, orr are the lane's word and its neighbours'; WPL 2 (planes):
// o = c, and po the plane offset (compile-time where the stride is).
template <int WPL>
__device__ __forceinline__ LdsRaw<WPL> lds_load(const uint32_t *row, int o, int ol, int orr, int po) {
    LdsRaw<WPL> x;
    if constexpr (WPL == 1) {
        x.c[0] = row[o];
        x.l = row[ol];   // the left word
        x.r = row[orr];  // the right word
    } else {
        const lds_word *r = (const lds_word *)(row + o);
        x.c[0] = lds_get(r);           // E[c]
        x.r = lds_get(r + 1);          // E[c + 1]: the right pair's even cells (bit 0 = its cell 0)
        x.l = lds_get(r + po);         // O[c - 1]: the left pair's odd cells (bit 31 = its cell 63)
        x.c[1] = lds_get(r + po + 1);  // O[c]
    }
    return x;
}

template <int WPL>
__device__ __forceinline__ void lds_sums(const LdsRaw<WPL> &x, LdsRow<WPL> &s) {
    uint32_t west[WPL], east[WPL];
    if constexpr (WPL == 1) {
        west[0] = __builtin_amdgcn_alignbit(x.c[0], x.l, 31);  // cell b-1 (bit 31 of the left word for b = 0)
        east[0] = __builtin_amdgcn_alignbit(x.r, x.c[0], 1);   // cell b+1
    } else {
        west[0] = __builtin_amdgcn_alignbit(x.c[1], x.l, 31);  // cell 2k-1
        east[0] = x.c[1];                                      // cell 2k+1
        west[1] = x.c[0];                                      // cell 2k
        east[1] = __builtin_amdgcn_alignbit(x.r, x.c[0], 1);   // cell 2k+2
    }
#pragma unroll
    for (int k = 0; k < WPL; ++k) {
        s.c[k] = x.c[k];
        s.s0[k] = bop<kXor3>(west[k], x.c[k], east[k]);
        s.s1[k] = bop<kMaj>(west[k], x.c[k], east[k]);
    }
}


// S > 0: LDS rows S words apart (>= Ww, a compile-time stride: the row
// loop's loads and stores of consecutive rows take immediate offsets); 0: Ww.
template <int WPL, int NT, int S>
__global__ __launch_bounds__(NT) void gol_lds_band_kernel(LdsBandArgs p) {
    extern __shared__ uint4 lds_band_smem[];
    uint32_t *const L0 = reinterpret_cast<uint32_t *>(lds_band_smem);
    const int Ww = p.Ww, D = p.D, nb = p.nb;
    const int LS = S > 0 ? S : p.stride;  // LDS row stride (words)
    const int PO = LS / 2;                // WPL 2: the odd plane's offset (ghost O[-1] at PO)
    // pairs at an instantiated stride: the pairs per row at compile time (the
    // stride is exactly Ww + 8), so a wave's runs are uniform when they fill it
    constexpr int PC = (S > 0 && WPL == 2) ? (S - 8) / 2 : 0;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // blocks are dealt round-robin over the 8 XCDs: give each XCD a run of
    // consecutive bands so most neighbours share an L2 (speed only)
    const int b = (p.xcd && nb % 8 == 0) ? (int)(blockIdx.x % 8) * (nb / 8) + (int)(blockIdx.x / 8) : (int)blockIdx.x;
    const int r0 = (int)((int64_t)b * p.rows / nb);
    const int h = (int)((int64_t)(b + 1) * p.rows / nb) - r0;
    const int R = h + 2 * D;
    const int Rmax = p.hmax + 2 * D + 3;  // + 3 spare rows for the row loop's prefetch
    uint32_t *A = L0, *B = L0 + (size_t)Rmax * LS;
    const int up = (b + nb - 1) % nb, down = (b + 1) % nb;
    __shared__ int s_abort;
    if (threadIdx.x == 0) s_abort = 0;

    const int P = PC > 0 ? PC : Ww / WPL;  // words (wpl 1) or pairs per row
    // generation 0: board rows r0 - D .. r0 + h + D - 1 (mod rows), 16-B words
    // (pairs: 8-B pairs into the two planes and their ghosts)
    const int q4 = Ww / 4;
    if constexpr (WPL == 1) {
        for (int i = threadIdx.x; i < R * q4; i += NT) {
            const int r = i / q4, c = i - r * q4;
            int br = r0 - D + r;
            br = ((br % p.rows) + p.rows) % p.rows;
            reinterpret_cast<uint4 *>(A + (size_t)r * LS)[c] = reinterpret_cast<const uint4 *>(p.src + (size_t)br * Ww)[c];
        }
    } else {
        for (int i = threadIdx.x; i < R * P; i += NT) {
            const int r = i / P, c = i - r * P;
            int br = r0 - D + r;
            br = ((br % p.rows) + p.rows) % p.rows;
            const uint2 v = reinterpret_cast<const uint2 *>(p.src + (size_t)br * Ww)[c];
            uint32_t *row = A + (size_t)r * LS;
            row[c] = v.x;
            row[PO + 1 + c] = v.y;
            if (c == 0) row[P] = v.x;
            if (c == P - 1) row[PO] = v.y;
        }
    }
    __syncthreads();

    const __amdgpu_buffer_rsrc_t ers = __builtin_amdgcn_make_buffer_rsrc(
        p.edge, (short)0, (int)(lds_band_edge_words(nb, D, LS) * 4), 0x00020000);
    const int K = max(1, NT / P);        // row runs per column
    const int units = P * K;
    const int J = (int)(((int64_t)p.turns + D - 1) / D);  // turns <= kResidentMaxTurns (gol_limits.h)
    const int rq4 = WPL == 1 ? q4 : LS / 4;  // 16-B granules of an edge row (pairs: the whole LDS row)
    const int eq4 = D * rq4;                 // 16-B granules of one edge side
    // diagnostics (option "trace"): s_memrealtime ticks summed over the
    // workgroups in compute, publish, neighbour wait and halo load
    long long tr[4] = {0, 0, 0, 0}, tr_t = p.trace ? (long long)__builtin_amdgcn_s_memrealtime() : 0;
    auto lap = [&](int k) {
        if (p.trace) {
            const long long now = (long long)__builtin_amdgcn_s_memrealtime();
            tr[k] += now - tr_t;
            tr_t = now;
        }
    };
    long long bar_ticks = 0, bar_turns = 0;  // option trace
    // age-weighted runs (PC % 64 == 0): cumulative weights of runs [0, k) and
    // [0, k + 1) for this wave's run k, and of all K runs
    int run_m0 = 0, run_m1 = 65536;  // this thread's run: row-share bounds in [0, 1], 16-bit fixed point
    if (p.age != 100) {
        const int kme = (int)threadIdx.x / P;
        int wgt = 1 << 12, w0 = 0, w1 = 0, wsum = 0;
        for (int k = 0, rank = 0; k < K; ++k) {
            const int r = (k * P / 64) / 4;  // the age rank of the wave of run k's first column (4 SIMDs)
            for (; rank < r; ++rank) wgt = wgt * p.age / 100;
            if (k == kme) w0 = wsum;
            wsum += max(wgt, 1);
            if (k == kme) w1 = wsum;
        }
        run_m0 = (int)(((int64_t)w0 << 16) / wsum);
        run_m1 = kme >= K - 1 ? 65536 : (int)(((int64_t)w1 << 16) / wsum);
        if constexpr (PC > 0 && PC % 64 == 0) {  // (a wave's lanes share their run)
            run_m0 = __builtin_amdgcn_readfirstlane(run_m0);
            run_m1 = __builtin_amdgcn_readfirstlane(run_m1);
        }
    }
    bool pending = false;  // lds_pre: our last edges are out, their flag not yet raised
    for (int j = 0; j < J; ++j) {
        const int Dj = min(D, p.turns - j * D);
        const bool more = j + 1 < J;
        // One run of rows [lo, hi) of pair (word) column c: the new generation
        // of those rows from Ab into Bb.
        auto run_rows = [&](const uint32_t *Ab, uint32_t *Bb, int lo, int hi, int c) {
            const int cl = c == 0 ? P - 1 : c - 1, cr = c == P - 1 ? 0 : c + 1;
            const int o = c, ol = cl, orr = cr;  // (pairs: ol, orr unused, the ghosts wrap)
            // pairs: the ghost store's word (E[P] for column 0, O[-1] for P - 1, else E[c] again)
            const int goff = c == 0 ? P : c == P - 1 ? PO : c;
            const bool godd = c == P - 1;
            // Loop-carried: the sums of rows r - 1, r, r + 1 (sa, sb, sc; computed,
            // so carrying them needs no wait).  An iteration of three rows issues
            // the loads of rows r + 2 .. r + 4 first, then computes row r, the
            // sums of r + 2, row r + 1, the sums of r + 3, row r + 2, the sums of
            // r + 4: each load is consumed one to three rows after it was issued
            // and none crosses the back edge (a loaded word carried over it made
            // the compiler wait for every load at the loop head).  Rows past
            // R - 1 land in the buffer's 3 spare rows (never used).
            auto rule_store = [&](const LdsRow<WPL> &a, const LdsRow<WPL> &b, const LdsRow<WPL> &n, uint32_t *st,
                                  uint32_t *gst) {
                uint32_t out[WPL];
#pragma unroll
                for (int m = 0; m < WPL; ++m)
                    out[m] = rule_word(a.s0[m], a.s1[m], b.s0[m], b.s1[m], n.s0[m], n.s1[m], b.c[m]);
                if constexpr (WPL == 1) {
                    *st = out[0];
                } else {
                    lds_put((lds_word *)st, out[0]);
                    lds_put((lds_word *)(st + PO + 1), out[1]);
                    lds_put((lds_word *)gst, godd ? out[1] : out[0]);
                }
            };
            LdsRow<WPL> sa, sb, sc;
            {
                const LdsRaw<WPL> x0 = lds_load<WPL>(Ab + (lo - 1) * LS, o, ol, orr, PO);
                const LdsRaw<WPL> x1 = lds_load<WPL>(Ab + lo * LS, o, ol, orr, PO);
                const LdsRaw<WPL> x2 = lds_load<WPL>(Ab + (lo + 1) * LS, o, ol, orr, PO);
                lds_sums<WPL>(x0, sa);
                lds_sums<WPL>(x1, sb);
                lds_sums<WPL>(x2, sc);
            }
            const uint32_t *ld = Ab + (lo + 2) * LS;
            uint32_t *st = Bb + lo * LS + o;
            uint32_t *gst = Bb + lo * LS + goff;
            int r = lo;
            for (; r + 3 <= hi; r += 3) {
                const LdsRaw<WPL> x0 = lds_load<WPL>(ld, o, ol, orr, PO);
                const LdsRaw<WPL> x1 = lds_load<WPL>(ld + LS, o, ol, orr, PO);
                const LdsRaw<WPL> x2 = lds_load<WPL>(ld + 2 * LS, o, ol, orr, PO);
                // the loads first, row r's rule behind them (it needs none of them)
                __builtin_amdgcn_sched_barrier(0);
                rule_store(sa, sb, sc, st, gst);
                __builtin_amdgcn_sched_barrier(0);  // (and only then the first wait)
                lds_sums<WPL>(x0, sa);
                rule_store(sb, sc, sa, st + LS, gst + LS);
                lds_sums<WPL>(x1, sb);
                rule_store(sc, sa, sb, st + 2 * LS, gst + 2 * LS);
                lds_sums<WPL>(x2, sc);
                ld += 3 * LS;
                st += 3 * LS;
                gst += 3 * LS;
            }
            if (r < hi) {
                rule_store(sa, sb, sc, st, gst);
                if (r + 1 < hi) {
                    LdsRow<WPL> sd;
                    lds_sums<WPL>(lds_load<WPL>(ld, o, ol, orr, PO), sd);
                    rule_store(sb, sc, sd, st + LS, gst + LS);
                }
            }
        };
        // One turn over the rows [lo0, hi0) and [lo1, hi1) (either may be empty):
        // K runs per column over the two ranges laid end to end, then a barrier.
        auto do_turn = [&](const uint32_t *Ab, uint32_t *Bb, int lo0, int hi0, int lo1, int hi1) {
            const int n0 = max(0, hi0 - lo0), n = n0 + max(0, hi1 - lo1);
            const int len = (n + K - 1) / K;
            for (int u = threadIdx.x; u < units; u += NT) {
                int k = u / P;
                // a wave's lanes share k when whole waves fit a row: scalar run bounds
                if constexpr (PC > 0 && PC % 64 == 0) k = __builtin_amdgcn_readfirstlane(k);
                const int c = u - k * P;
                int v0 = k * len, v1 = min(v0 + len, n);
                // age-weighted runs: the SIMD arbiter serves a SIMD's older waves
                // first, so run k (the wave of its first column: rank = wave / 4)
                // gets (age / 100)^rank of the oldest rank's row share
                if (p.age != 100) {  // 16-bit fixed point (a scalar division costs ~40 instructions)
                    v0 = (n * run_m0 + 32768) >> 16;
                    v1 = (n * run_m1 + 32768) >> 16;
                }
                if (v0 >= v1) continue;
                if (v0 < n0) run_rows(Ab, Bb, lo0 + v0, lo0 + min(v1, n0), c);
                if (v1 > n0) run_rows(Ab, Bb, lo1 + max(v0, n0) - n0, lo1 + v1 - n0, c);
            }
            if (p.trace) {  // (option trace: each wave's ticks in the turn barrier)
                const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
                __syncthreads();
                bar_ticks += (long long)__builtin_amdgcn_s_memrealtime() - t0;
                ++bar_turns;
            } else {
                __syncthreads();
            }
        };
        // Edge rows of generation (j + 1) D from F: [D, 2D) (side 0) and [h, h + D)
        // (side 1) to slot (j + 1) & 1, write-through; signal() waits for them
        // (every wave's vmcnt(0), a barrier) and raises the flag.
        auto publish = [&](const uint32_t *F) {
            if (p.fault && b == 0) return;  // test hook: band 0 never publishes (its neighbours time out)
            const int slot = (j + 1) & 1;
            const int e0 = (((slot * nb + b) * 2) * eq4) * 16;
            for (int i = threadIdx.x; i < 2 * eq4; i += NT) {
                const bool top = i < eq4;
                const int g = top ? i : i - eq4;
                const uint4 v = *reinterpret_cast<const uint4 *>(F + (size_t)(top ? D : h) * LS + 4 * (g % rq4) + (size_t)(g / rq4) * LS);
                __builtin_amdgcn_raw_buffer_store_b128((v4u32){v.x, v.y, v.z, v.w}, ers,
                                                       e0 + (top ? 0 : eq4 * 16) + g * 16, 0, kCpolSc1);
            }
        };
        auto signal = [&](unsigned v) {  // progress = v: the edges of generation v D are out
            if (p.fault && b == 0) return;   // (b is uniform over the workgroup)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (threadIdx.x == 0)
                __hip_atomic_store(&p.progress[b], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        };
        // Neighbours' super-step j edges (generation j D) into the halo rows of A;
        // false if the wait timed out (every workgroup drains).
        // Neighbours' super-step j edges (generation j D) into the halo rows of
        // A, in three parts: wait_flags (wave 0 polls both flags; false if the
        // wait timed out, every workgroup drains), halo_issue (every thread's
        // first kHaloRegs 16-B granules in flight at once, into registers) and
        // halo_store (those to LDS, any further granules loaded and stored, a
        // barrier): the granules of a thread travel together, not one round
        // trip after another.
        auto wait_flags = [&]() -> bool {
            if (w == 0) {
                const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
                const int nbr = lane == 0 ? up : down;
                for (;;) {
                    const unsigned v = lane < 2 ? __hip_atomic_load(&p.progress[nbr], __ATOMIC_RELAXED,
                                                                    __HIP_MEMORY_SCOPE_AGENT)
                                                : (unsigned)j;
                    if (__all(v >= (unsigned)j)) break;
                    const unsigned err = __hip_atomic_load(p.error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (err || (long long)__builtin_amdgcn_s_memrealtime() - t0 > p.timeout_ticks) {
                        if (lane == 0) {
                            atomicOr(p.error, 1u);
                            s_abort = 1;
                        }
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            __syncthreads();
            if (s_abort) return false;  // uniform over the workgroup
            lap(2);
            return true;
        };
        const int eu = (((j & 1) * nb + up) * 2 + 1) * eq4 * 16;    // up's bottom D rows -> rows [0, D)
        const int ed = (((j & 1) * nb + down) * 2 + 0) * eq4 * 16;  // down's top D rows -> rows [D + h, R)
        auto halo_load = [&](int i) -> v4u32 {
            const bool top = i < eq4;
            return __builtin_amdgcn_raw_buffer_load_b128(ers, (top ? eu : ed) + (top ? i : i - eq4) * 16, 0, kCpolSc1);
        };
        auto halo_put = [&](int i, const v4u32 &v) {
            const bool top = i < eq4;
            const int g = top ? i : i - eq4;
            uint32_t *dstw = A + (size_t)(top ? 0 : D + h) * LS + 4 * (g % rq4) + (size_t)(g / rq4) * LS;
            *reinterpret_cast<uint4 *>(dstw) = make_uint4(v.x, v.y, v.z, v.w);
        };
        v4u32 hreg[kHaloRegs];
        auto halo_issue = [&]() {
#pragma unroll
            for (int k = 0; k < kHaloRegs; ++k) {
                const int i = (int)threadIdx.x + k * NT;
                if (i < 2 * eq4) hreg[k] = halo_load(i);
            }
        };
        auto halo_store = [&]() {
#pragma unroll
            for (int k = 0; k < kHaloRegs; ++k) {
                const int i = (int)threadIdx.x + k * NT;
                if (i < 2 * eq4) halo_put(i, hreg[k]);
            }
            for (int i = (int)threadIdx.x + kHaloRegs * NT; i < 2 * eq4; i += NT) halo_put(i, halo_load(i));
            __syncthreads();
            lap(3);
        };
        // interior first (option lds_pre = k): the first k turns of a full
        // super-step run on the rows that need no halo, [D + t, D + h - t), while
        // the neighbours' edges travel (and the previous edges' signal goes out
        // after the first of them); then the halo-adjacent rows of those turns,
        // [t, D + t) and [D + h - t, R - t), then whole turns.  Turn t's halo-side
        // rows read turn t - 1's interior rows D + t - 1, D + t (bottom: D + h - t
        // - 1, D + h - t), which the interior turns t + 1, t + 3, .. (same buffer)
        // never reach.  Turn t's buffer is A for even t, B for odd.
        const int pre = (j > 0 && Dj == D) ? min(p.pre, D) : 0;
        if (pre > 0) {
            for (int t = 1; t <= pre; ++t) {
                do_turn((t & 1) ? A : B, (t & 1) ? B : A, D + t, D + h - t, 0, 0);
                if (t == 1 && pending) {
                    signal((unsigned)j);
                    pending = false;
                }
            }
            lap(0);
            // (the flags waited for before the last interior turn and the loads
            // in flight during it ran 8192^2 39.0 vs 40.9 TCUPS: the earlier
            // wait costs more than the hidden loads save; profiles/r5t)
            if (!wait_flags()) return;
            halo_issue();
            halo_store();
            for (int t = 1; t <= pre; ++t)
                do_turn((t & 1) ? A : B, (t & 1) ? B : A, t, D + t, D + h - t, R - t);
            for (int t = pre + 1; t <= D; ++t) do_turn((t & 1) ? A : B, (t & 1) ? B : A, t, R - t, 0, 0);
            uint32_t *F = (D & 1) ? B : A;
            if (F != A) {
                B = A;
                A = F;
            }
            lap(0);
            if (more) {
                publish(A);
                pending = true;  // signalled after the next super-step's first interior turn
            }
            lap(1);
            continue;
        }
        if (pending) {
            signal((unsigned)j);
            pending = false;
        }
        if (j > 0) {
            if (!wait_flags()) return;
            halo_issue();
            halo_store();
        }
        // whole turns (a shorter last super-step needs only Dj halo rows of the D)
        const int skip = D - Dj;
        for (int t = 1; t <= Dj; ++t) {
            do_turn(A, B, skip + t, R - skip - t, 0, 0);
            uint32_t *T = A;
            A = B;
            B = T;
        }
        lap(0);
        if (more) {
            publish(A);
            // the next super-step signals after its first interior turn when it
            // runs interior first (full, lds_pre), else now
            if (p.pre > 0 && min(D, p.turns - (j + 1) * D) == D)
                pending = true;
            else
                signal((unsigned)(j + 1));
        }
        lap(1);
    }
    if (p.trace && threadIdx.x == 0) {
        for (int k = 0; k < 4; ++k) atomicAdd(&p.trace[k], (unsigned long long)tr[k]);
        atomicAdd(&p.trace[4], 1ull);
    }
    if (p.trace && lane == 0 && blockIdx.x < 1024) {  // (workgroup, wave): barrier ticks, turns
        p.trace[8 + 2 * (blockIdx.x * 64 + w)] = (unsigned long long)bar_ticks;
        p.trace[8 + 2 * (blockIdx.x * 64 + w) + 1] = (unsigned long long)bar_turns;
    }
    // the band's last generation: rows [D, D + h) of A -> board rows [r0, r0 + h)
    uint32_t cnt = 0;
    if constexpr (WPL == 1) {
        for (int i = threadIdx.x; i < h * q4; i += NT) {
            const int r = i / q4, c = i - r * q4;
            const uint4 v = reinterpret_cast<const uint4 *>(A + (size_t)(D + r) * LS)[c];
            reinterpret_cast<uint4 *>(p.dst + (size_t)(r0 + r) * Ww)[c] = v;
            cnt += __builtin_popcount(v.x) + __builtin_popcount(v.y) + __builtin_popcount(v.z) + __builtin_popcount(v.w);
        }
    } else {
        for (int i = threadIdx.x; i < h * P; i += NT) {
            const int r = i / P, c = i - r * P;
            const uint32_t *row = A + (size_t)(D + r) * LS;
            const uint2 v = make_uint2(row[c], row[PO + 1 + c]);
            reinterpret_cast<uint2 *>(p.dst + (size_t)(r0 + r) * Ww)[c] = v;
            cnt += __builtin_popcount(v.x) + __builtin_popcount(v.y);
        }
    }
    if (p.alive) {
        const uint32_t tot = wave_sum_u32(cnt);
        if (lane == 0 && tot) atomicAdd(p.alive, (unsigned long long)tot);
    }
}

template <typename F>
static hipError_t dispatch_lds_band(int wpl, int nt, int stride, F &&f) {
#define GOL_LCASE(WP, NT, S) \
    if (wpl == WP && nt == NT && stride == S) return f(gol_lds_band_kernel<WP, NT, S>, NT);
    // pairs: the plane stride Ww + 8 of 1024^2, 2048^2, 4096^2, 5120^2, 8192^2
    GOL_LCASE(2, 512, 0) GOL_LCASE(2, 512, 40) GOL_LCASE(2, 512, 72) GOL_LCASE(2, 512, 136) GOL_LCASE(2, 512, 168)
    GOL_LCASE(2, 512, 264) GOL_LCASE(2, 1024, 0) GOL_LCASE(2, 1024, 264)
    GOL_LCASE(1, 512, 0) GOL_LCASE(1, 1024, 0)
#undef GOL_LCASE
    return hipErrorInvalidValue;
}
// The template stride of the kernel that runs LDS rows `stride` words apart:
// that stride where instantiated, else 0 (the runtime-stride kernel, stride == Ww).
static int lds_tmpl_stride(int wpl, int nt, int stride) {
    return dispatch_lds_band(wpl, nt, stride, [](auto, int) { return hipSuccess; }) == hipSuccess ? stride : 0;
}
int lds_band_stride(int Ww, int wpl, int nt) {
    (void)nt;
    return wpl == 2 ? Ww + 8 : Ww;  // pairs: the two-plane row (its kernel instantiated or not)
}

int lds_band_blocks_per_cu(int wpl, int nt, int stride, int64_t lds_bytes) {
    int n = 0;
    hipError_t e = dispatch_lds_band(wpl, nt, lds_tmpl_stride(wpl, nt, stride), [&](auto kern, int t) {
        hipError_t r = hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes);
        return r == hipSuccess ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kern, t, (size_t)lds_bytes) : r;
    });
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}

hipError_t launch_lds_band(const LdsBandArgs &p, int wpl, hipStream_t s) {
    const size_t bytes = (size_t)lds_band_lds_bytes(p.hmax, p.D, p.stride);
    const int S = p.rt_stride ? 0 : lds_tmpl_stride(wpl, p.nt, p.stride);
    if (p.stride != lds_band_stride(p.Ww, wpl, p.nt)) return hipErrorInvalidValue;
    return dispatch_lds_band(wpl, p.nt, S, [&](auto kern, int t) {
        hipLaunchKernelGGL(kern, dim3(p.nb), dim3(t), bytes, s, p);
        return hipGetLastError();
    });
}

// ---- host-side dispatch over (depth, fill skip, words per lane) ----------
// Depths 1, 2, 4, 6, 8, 12, 16, 20 (and 24, 32 for WPL = 1: depth 24 at
// WPL = 2 would exceed 256 VGPRs; WPL = 4 stops at 9, an extra depth of its
// own); the host's depth_plan picks among them.
template <typename F>
static hipError_t dispatch(int depth, bool skip, int wpl, F &&f) {
#define GOL_CASE(D, SK, WP) \
    if (depth == D && skip == SK && wpl == WP) return f(gol_tb_kernel<D, SK, WP>);
    GOL_CASE(1, true, 1) GOL_CASE(2, true, 1) GOL_CASE(4, true, 1) GOL_CASE(8, true, 1) GOL_CASE(16, true, 1)
    GOL_CASE(32, true, 1) GOL_CASE(1, false, 1) GOL_CASE(2, false, 1) GOL_CASE(4, false, 1) GOL_CASE(8, false, 1)
    GOL_CASE(16, false, 1) GOL_CASE(32, false, 1)
    GOL_CASE(12, true, 1) GOL_CASE(24, true, 1) GOL_CASE(12, false, 1) GOL_CASE(24, false, 1)
    GOL_CASE(12, true, 2) GOL_CASE(12, false, 2)
    GOL_CASE(1, true, 4) GOL_CASE(2, true, 4) GOL_CASE(4, true, 4) GOL_CASE(8, true, 4) GOL_CASE(9, true, 4)
    GOL_CASE(1, false, 4) GOL_CASE(2, false, 4) GOL_CASE(4, false, 4) GOL_CASE(8, false, 4) GOL_CASE(9, false, 4)
    GOL_CASE(6, true, 1) GOL_CASE(6, false, 1) GOL_CASE(6, true, 2) GOL_CASE(6, false, 2)
    GOL_CASE(6, true, 4) GOL_CASE(6, false, 4)
    GOL_CASE(1, true, 2) GOL_CASE(2, true, 2) GOL_CASE(4, true, 2) GOL_CASE(8, true, 2) GOL_CASE(16, true, 2)
    GOL_CASE(1, false, 2) GOL_CASE(2, false, 2) GOL_CASE(4, false, 2) GOL_CASE(8, false, 2) GOL_CASE(16, false, 2)
    GOL_CASE(20, true, 1) GOL_CASE(20, false, 1) GOL_CASE(20, true, 2) GOL_CASE(20, false, 2)
    GOL_CASE(18, true, 2) GOL_CASE(18, false, 2)  // the pair rule's depth where a strip's K1w does not plan
#undef GOL_CASE
    return hipErrorInvalidValue;
}

// Per-launch kernels: WPL 2 fits 20 stages in 242 VGPRs (two waves per SIMD,
// no scratch), WPL 4 nine in 248-250 (depth 9 exists for quads only: the host
// plans it only under a cap of exactly 9, see depth_cap); the resident kernel
// keeps 16 / 8 (its instantiations).
int max_depth_for(int wpl) { return wpl == 4 ? 9 : wpl == 2 ? 20 : 32; }
int persist_max_depth(int wpl) { return wpl == 4 ? 8 : wpl == 2 ? 16 : 32; }

int tb_tiles(int Ww, int wpl) { return (Ww + tile_words(wpl) - 1) / tile_words(wpl); }

int tb_waves(const StepArgs &a, int wpl) {
    const int strips = (a.rows_out + a.rows_per_wave - 1) / a.rows_per_wave;
    return tb_tiles(a.Ww, wpl) * strips;
}

template <typename F>
static hipError_t dispatch_pair(int depth, int wpl, F &&f, bool cnt = false) {
#define GOL_QCASE(D, WP) \
    if (depth == D && wpl == WP) return cnt ? f(gol_tb_pair_kernel<D, WP, true>) : f(gol_tb_pair_kernel<D, WP, false>);
    GOL_QCASE(1, 1) GOL_QCASE(2, 1) GOL_QCASE(4, 1) GOL_QCASE(8, 1) GOL_QCASE(16, 1) GOL_QCASE(32, 1)
    GOL_QCASE(1, 2) GOL_QCASE(2, 2) GOL_QCASE(4, 2) GOL_QCASE(8, 2) GOL_QCASE(16, 2)
    GOL_QCASE(12, 1) GOL_QCASE(24, 1) GOL_QCASE(12, 2) GOL_QCASE(1, 4) GOL_QCASE(2, 4) GOL_QCASE(4, 4) GOL_QCASE(8, 4)
    GOL_QCASE(6, 1) GOL_QCASE(6, 2) GOL_QCASE(6, 4) GOL_QCASE(9, 4) GOL_QCASE(20, 1) GOL_QCASE(20, 2)
    GOL_QCASE(18, 2)
#undef GOL_QCASE
    return hipErrorInvalidValue;
}

int tb_pair_blocks(const StepArgs &a, int wpl) {
    const int regions = (a.rows_out + 2 * a.rows_per_wave - 1) / (2 * a.rows_per_wave);
    return (tb_tiles(a.Ww, wpl) * regions + 3) / 4;
}

hipError_t launch_step_tb(const StepArgs &a, int depth, hipStream_t s, bool fill_skip, int wpl, bool paired) {
    if (paired && fill_skip) {
        const dim3 grid(tb_pair_blocks(a, wpl)), block(512);
        return dispatch_pair(
            depth, wpl,
            [&](auto kern) {
                hipLaunchKernelGGL(kern, grid, block, 0, s, a);
                return hipGetLastError();
            },
            a.alive != nullptr);
    }
    const int waves = tb_waves(a, wpl);
    const dim3 grid((waves + 3) / 4), block(256);
    return dispatch(depth, fill_skip, wpl, [&](auto kern) {
        hipLaunchKernelGGL(kern, grid, block, 0, s, a);
        return hipGetLastError();
    });
}

template <typename F>
static hipError_t dispatch_skew(int depth, int wpl, bool half, bool pr, F &&f) {
#define GOL_WCASE(D, WP) \
    if (!pr && !half && depth == D && wpl == WP) return f(gol_skew_kernel<D, WP>);
#define GOL_HCASE(D, WP) \
    if (!pr && half && depth == D && wpl == WP) return f(gol_skew_kernel<D, WP, true>);
#define GOL_RCASE(D, WP, HF) \
    if (pr && half == HF && depth == D && wpl == WP) return f(gol_skew_kernel<D, WP, HF, true>);
    GOL_WCASE(8, 2) GOL_WCASE(12, 2) GOL_WCASE(16, 2) GOL_WCASE(20, 2) GOL_WCASE(6, 4) GOL_WCASE(8, 4)
    GOL_WCASE(9, 4) GOL_WCASE(16, 1) GOL_WCASE(32, 1)
    GOL_HCASE(16, 2) GOL_HCASE(20, 2)
    GOL_RCASE(18, 2, false) GOL_RCASE(18, 2, true) GOL_RCASE(8, 4, false)
#undef GOL_WCASE
#undef GOL_HCASE
#undef GOL_RCASE
    return hipErrorInvalidValue;
}

bool skew_supported(int depth, int wpl, bool half, bool pr) {
    return dispatch_skew(depth, wpl, half, pr, [](auto) { return hipSuccess; }) == hipSuccess;
}

int skew_blocks_per_cu(int depth, int wpl, bool half, bool pr) {
    int b = 0;
    hipError_t e = dispatch_skew(depth, wpl, half, pr, [&](auto kern) {
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, kern, 512, 0);
    });
    return e == hipSuccess ? b : 0;
}

hipError_t launch_skew(const SkewArgs &p, int depth, int wpl, hipStream_t s) {
    const int tcols = (p.tiles_x + p.tx - 1) / p.tx;
    return dispatch_skew(depth, wpl, p.half != 0, p.pairs != 0, [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(tcols * p.nst), dim3(512), 0, s, p);
        return hipGetLastError();
    });
}

int tb_blocks_per_cu(int depth, int wpl) {
    int b = 0;
    hipError_t e = dispatch(depth, true, wpl, [&](auto kern) {
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, kern, 256, 0);
    });
    return (e == hipSuccess && b > 0) ? b : 1;
}

int tb_wave_slots_per_cu(int depth, int wpl, bool paired) {
    if (!paired) return 4 * tb_blocks_per_cu(depth, wpl);
    int b = 0;
    hipError_t e = dispatch_pair(depth, wpl, [&](auto kern) {
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, kern, 512, 0);
    });
    return 8 * ((e == hipSuccess && b > 0) ? b : 1);
}

int auto_rows_per_wave(int Ww, int rows, int depth, int wave_slots, bool fill_skip, int wpl, bool paired) {
    // Each wave streams S + 2*depth rows (~S + 1.25*depth row-equivalents of
    // work when the fill skips dead stages); waves run in ceil(waves / slots)
    // rounds.  Minimise rounds * work (fill overhead vs tail).
    const int tiles_x = tb_tiles(Ww, wpl);
    int best_s = rows;
    double best = 1e300;
    for (int strips = 1; strips <= rows; ++strips) {
        const int S = (rows + strips - 1) / strips;
        const long long waves = paired ? 2LL * tiles_x * ((rows + 2 * S - 1) / (2 * S))
                                       : (long long)tiles_x * ((rows + S - 1) / S);
        const long long rounds = (waves + wave_slots - 1) / wave_slots;
        const double cost = (double)rounds * (S + (fill_skip ? 2 * depth - 0.75 * depth : 2 * depth));
        if (cost < best * 0.999) {
            best = cost;
            best_s = S;
        }
        if (S <= 2) break;
    }
    return best_s;
}

// nw = waves per workgroup (one workgroup per CU): 4, 8 or 16; 0 = default.
template <typename F>
static hipError_t dispatch_persist(int depth, int wpl, int nw, F &&f) {
    if (nw == 0) nw = persist_waves(depth, wpl);
#define GOL_PCASE(D, WP, NW) \
    if (depth == D && wpl == WP && nw == NW) return f(gol_persist_kernel<D, WP, NW>, NW);
    GOL_PCASE(4, 1, 16) GOL_PCASE(8, 1, 16) GOL_PCASE(16, 1, 16) GOL_PCASE(32, 1, 8) GOL_PCASE(4, 2, 16)
    GOL_PCASE(8, 2, 16) GOL_PCASE(16, 2, 8) GOL_PCASE(8, 1, 8) GOL_PCASE(16, 1, 8) GOL_PCASE(8, 2, 8)
#undef GOL_PCASE
    return hipErrorInvalidValue;
}

int persist_waves_for(int depth, int wpl) { return persist_waves(depth, wpl); }

int persist_blocks_per_cu(int depth, int wpl, int nw) {
    int b = 0;
    hipError_t e = dispatch_persist(depth, wpl, nw, [&](auto kern, int n) {
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, kern, 64 * n, 0);
    });
    return e == hipSuccess ? b : 0;
}

bool plan_persist(int Ww, int rows, int depth, int cus, int wpl, int units, PersistArgs *p, int force_tx) {
    const int NW = units;
    const int tiles_x = tb_tiles(Ww, wpl);
    bool found = false;
    long best_s = 0;
    for (int wg_tx = 1; wg_tx <= NW; wg_tx *= 2) {
        if (force_tx > 0 && wg_tx != force_tx) continue;
        const int wg_sy = NW / wg_tx;
        const int cols = (tiles_x + wg_tx - 1) / wg_tx;
        // as many workgroup rows as CUs allow, but bands of >= depth rows
        int wg_y = std::min(cus / cols, rows / (wg_sy * depth));
        if (wg_y < 1) continue;
        const int strips = wg_y * wg_sy;
        const int S = (rows + strips - 1) / strips;
        if (S < depth) continue;                         // halo rows from the adjacent strip only
        wg_y = (rows + wg_sy * S - 1) / (wg_sy * S);     // rounding S up can leave trailing rows empty
        // every workgroup row must hold >= depth real rows (its neighbours' halos)
        const int last_rows = rows - (wg_y - 1) * wg_sy * S;
        if (last_rows < depth) continue;
        if (!found || S < best_s) {
            found = true;
            best_s = S;
            p->wg_tx = wg_tx;
            p->wg_sy = wg_sy;
            p->cols = cols;
            p->wg_y = wg_y;
            p->S = S;
            p->tiles_x = tiles_x;
        }
    }
    return found;
}

hipError_t launch_persist(const PersistArgs &p, int depth, int wpl, hipStream_t s) {
    return dispatch_persist(depth, wpl, p.nw, [&](auto kern, int nw) {
        hipLaunchKernelGGL(kern, dim3(p.cols * p.wg_y), dim3(64 * nw), 0, s, p);
        return hipGetLastError();
    });
}

// ---------------------------------------------------------------------------
// K1g: one turn, any width (bit-by-bit neighbour fetch with column wrap).
// Only used for widths that are not a multiple of 32 (the 16x16 fixture).
// ---------------------------------------------------------------------------
__device__ __forceinline__ int map_in_row(const RowMap &m, int i) {
    int r = i + m.off;
    if (m.wrap > 0) {
        r %= m.wrap;
        if (r < 0) r += m.wrap;
    }
    return m.base + min(r, m.rmax);
}

__global__ __launch_bounds__(256) void gol_generic_kernel(StepArgs a) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int Ww = a.Ww, W = a.W;
    uint32_t cnt = 0;
    if (idx < (int64_t)a.rows_out * Ww) {
        const int row = (int)(idx / Ww);
        const int wc = (int)(idx - (int64_t)row * Ww);
        const uint32_t *up = a.src + (size_t)map_in_row(a.in, row - 1) * Ww;
        const uint32_t *mid = a.src + (size_t)map_in_row(a.in, row) * Ww;
        const uint32_t *dn = a.src + (size_t)map_in_row(a.in, row + 1) * Ww;
        auto bit = [&](const uint32_t *p, int x) -> int {
            x = x < 0 ? x + W : (x >= W ? x - W : x);
            return (p[x >> 5] >> (x & 31)) & 1;
        };
        uint32_t out = 0;
        for (int b = 0; b < 32; ++b) {
            const int x = wc * 32 + b;
            if (x >= W) break;
            const int n = bit(up, x - 1) + bit(up, x) + bit(up, x + 1) + bit(mid, x - 1) + bit(mid, x + 1) +
                          bit(dn, x - 1) + bit(dn, x) + bit(dn, x + 1);
            const int c = bit(mid, x);
            if (n == 3 || (c && n == 2)) out |= 1u << b;
        }
        a.dst[(size_t)(a.dst_base + row) * Ww + wc] = out;
        cnt = __builtin_popcount(out);
    }
    if (a.alive) {
        const uint32_t tot = wave_sum_u32(cnt);
        if ((threadIdx.x & 63) == 0 && tot) atomicAdd(a.alive, (unsigned long long)tot);
    }
}

hipError_t launch_step_generic(const StepArgs &a, hipStream_t s) {
    const int64_t n = (int64_t)a.rows_out * a.Ww;
    hipLaunchKernelGGL(gol_generic_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// K5: one turn + its CellFlipped list, fused (the event stream of
// distributor.go:93-173 with initializeAliveCells :212-220, BASELINE
// configs[4]).  Per block of 256 threads, 1024 consecutive canonical words
// (word k * 256 + tid of the block: every load and board store is a
// coalesced 256-word access):
//   1. the turn: three input rows per word, the column neighbours from the
//      adjacent lanes (DPP; a row's first / last word and the wave's edge
//      lanes load theirs), the bit-sliced row sums and the 3-LUT rule of K1;
//   2. flips = old ^ new, counted per word into a packed 4 x 16-bit vector
//      (one field per k) so ONE block scan orders the block's words;
//   3. decoupled look-back (blocks take virtual ids from a ticket, so every
//      predecessor is already running): the block publishes its aggregate,
//      wave 0 reads up to 64 predecessors per step (one lane each) until the
//      nearest one holding an inclusive prefix, then publishes its own;
//      status words are 64-bit agent-scope atomics carrying (flag, epoch,
//      value) together, so there is no separate payload to hand off;
//   4. entries (row-major: word order, then bit order) go to LDS at their
//      block-relative positions and leave in one coalesced copy (blocks
//      with more entries than LDS holds store them directly).
// HBM traffic per turn: the board read once (neighbour words hit L1/L2),
// written once, plus the entries.
// ---------------------------------------------------------------------------
constexpr int kFtThreads = 256, kFtK = 4, kFtWords = kFtThreads * kFtK;
// 32 KiB of entry staging: four blocks per CU, so a 5120^2 turn (800 blocks)
// is resident at once; a block with more entries stores them directly.
constexpr int kFtLdsBytes = 32768;
constexpr unsigned long long kFtAgg = 1ull << 62, kFtPrefix = 2ull << 62;
constexpr unsigned long long kFtValMask = (1ull << 40) - 1;

__device__ __forceinline__ unsigned long long ft_word(unsigned long long flag, unsigned epoch, unsigned long long v) {
    return flag | ((unsigned long long)(epoch & 0x3FFFFFu) << 40) | (v & kFtValMask);
}

// 3-LUT B3/S23 rule of K1 on three rows' words with their west / east
// neighbour words already aligned (bit b = cell b -+ 1).
__device__ __forceinline__ uint32_t ft_rule(const uint32_t (&w)[3], const uint32_t (&x)[3], const uint32_t (&e)[3]) {
    uint32_t h0[3], h1[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        h0[j] = bop<kXor3>(w[j], x[j], e[j]);
        h1[j] = bop<kMaj>(w[j], x[j], e[j]);
    }
    const uint32_t u0 = bop<kXor3>(h0[0], h0[1], h0[2]), u1 = bop<kMaj>(h0[0], h0[1], h0[2]);
    const uint32_t v0 = bop<kXor3>(h1[0], h1[1], h1[2]), v1 = bop<kMaj>(h1[0], h1[1], h1[2]);
    const uint32_t g1 = bop<kG1>(u1, v0, v1), g2 = bop<kG2>(u0, v1, x[1]);
    return bop<kNext>(u0, g1, g2);
}

// The copy blocks of a K5 launch: the previous turn's entries, device list
// -> host list, in 16-byte stores to the destination's 16-byte boundaries
// (4-byte heads and tails), spread over the copy blocks.  They never wait on
// anything, so the turn's own blocks keep their co-residency, and their host
// stores are in their own waves: the turn's loads never wait behind them
// (vmcnt is per wave).  Whether the previous turn is delivered follows from
// its run bounds alone (a stop flag set by this launch's own blocks must not
// cancel the copy of a turn that did fit).
__device__ void flip_copy_prev(const FlipTurnArgs &a, unsigned cb, unsigned ncb) {
    const unsigned long long s = a.cp_run[0], e0 = a.cp_run[1];
    if (a.stop_on_overflow && e0 > a.cap) return;  // that turn did not fit: the host rolls back to it
    const unsigned long long e = e0 < a.cap ? e0 : a.cap;
    if (e <= s) return;
    const unsigned wpe = a.format == kFlipFormatXY ? 2u : 1u;  // 32-bit words per entry
    const uint32_t *src = reinterpret_cast<const uint32_t *>(a.out) + s * wpe;
    uint32_t *d = reinterpret_cast<uint32_t *>(a.cp_dst) + s * wpe;
    const unsigned long long nw = (e - s) * wpe;
    const unsigned long long head = min(nw, (unsigned long long)((4u - (unsigned)(((uintptr_t)d >> 2) & 3u)) & 3u));
    const unsigned long long nq = (nw - head) / 4;
    const unsigned long long gt = (unsigned long long)cb * kFtThreads + threadIdx.x, gn = (unsigned long long)ncb * kFtThreads;
    if (gt < head) d[gt] = src[gt];
    for (unsigned long long q = gt; q < nq; q += gn) {
        const unsigned long long w = head + 4 * q;
        *reinterpret_cast<uint4 *>(d + w) = make_uint4(src[w], src[w + 1], src[w + 2], src[w + 3]);
    }
    const unsigned long long t0 = head + 4 * nq;
    if (t0 + gt < nw) d[t0 + gt] = src[t0 + gt];
}

// Shared memory of one K5 block.
struct FtShared {
    unsigned long long wsum[4], part[4];
    unsigned long long excl;
    int stop;  // K5r: this turn is not delivered (an earlier turn overflowed, or a wait timed out)
    uint32_t alive[4];
    alignas(16) unsigned char buf[kFtLdsBytes];
};

// One block's share of a K5 turn: words vid * 1024 .. + 1023 of the board;
// false when the turn is not delivered (K5r: the block stops).
// CONTIG (Ww % 4 == 0): thread tid of the block owns the 4 consecutive words
// base + 4 tid .. + 3 of one row (16-byte loads and stores); otherwise word
// base + k * 256 + tid for k = 0..3 (4-byte accesses, any Ww).
// SC1 (K5r): every board and entry access is a write-through (sc1) buffer
// access, the hand-off form that needs no fence (MI355X_MICROARCH.md, valid
// forms); the block reports its turn done once its stores have drained.
template <bool CONTIG, bool SC1>
__device__ __forceinline__ bool flip_turn_block(const FlipTurnArgs &a, const unsigned vid, FtShared &sh) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    // (unused, and dropped, without SC1)
    const __amdgpu_buffer_rsrc_t srs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t *>(a.src), (short)0, (int)a.board_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t drs = __builtin_amdgcn_make_buffer_rsrc(a.dst, (short)0, (int)a.board_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(a.out, (short)0, (int)a.out_bytes, 0x00020000);
    auto src_ld4 = [&](size_t w) -> uint4 {
        if constexpr (SC1) {
            const v4u32 v = __builtin_amdgcn_raw_buffer_load_b128(srs, (int)(w * 4), 0, kCpolSc1);
            return make_uint4(v.x, v.y, v.z, v.w);
        } else {
            return *reinterpret_cast<const uint4 *>(a.src + w);
        }
    };
    auto src_ld1 = [&](size_t w) -> uint32_t {
        if constexpr (SC1) return __builtin_amdgcn_raw_buffer_load_b32(srs, (int)(w * 4), 0, kCpolSc1);
        else return a.src[w];
    };
    auto dst_st4 = [&](size_t w, const uint4 &v) {
        if constexpr (SC1) __builtin_amdgcn_raw_buffer_store_b128((v4u32){v.x, v.y, v.z, v.w}, drs, (int)(w * 4), 0, kCpolSc1);
        else *reinterpret_cast<uint4 *>(a.dst + w) = v;
    };
    auto dst_st1 = [&](size_t w, uint32_t v) {
        if constexpr (SC1) __builtin_amdgcn_raw_buffer_store_b32(v, drs, (int)(w * 4), 0, kCpolSc1);
        else a.dst[w] = v;
    };
    auto out_st4 = [&](unsigned long long w, const uint4 &v) {
        if constexpr (SC1) __builtin_amdgcn_raw_buffer_store_b128((v4u32){v.x, v.y, v.z, v.w}, ors, (int)(w * 4), 0, kCpolSc1);
        else *reinterpret_cast<uint4 *>(static_cast<uint32_t *>(a.out) + w) = v;
    };
    auto out_st1 = [&](unsigned long long w, uint32_t v) {
        if constexpr (SC1) __builtin_amdgcn_raw_buffer_store_b32(v, ors, (int)(w * 4), 0, kCpolSc1);
        else static_cast<uint32_t *>(a.out)[w] = v;
    };
    // the turn's run bounds: read by the next turn's blocks and the copy blocks
    // (K5r: stored with kFtRunReady set, which the next turn's blocks wait for)
    auto run_get = [&](int i) {
        return __hip_atomic_load(&a.run[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & ~kFtRunReady;
    };
    auto run_set = [&](unsigned long long v) {
        __hip_atomic_store(&a.run[1], SC1 ? v | kFtRunReady : v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    // K5r: this block is done with the turn once every wave's stores have
    // drained (sc1: written through): its own turn count (the next turn's
    // neighbours wait on it), then one count on its shard (the copy blocks)
    auto signal_done = [&]() {
        if constexpr (SC1) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) {
                __hip_atomic_store(&a.blk_done[vid], a.turn + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_fetch_add(&a.done[(vid % kFtShards) * kFtShardStride], 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    };
    // K5r: run[0] (this turn's first entry) is the previous turn's last
    // block's prefix: needed only for the entries, so waited for here, not at
    // the turn's start; the last block stores it with kFtRunReady right after
    // its look-back (before its own board and entries).  Thread 0 only.
    auto wait_run = [&]() {
        if constexpr (SC1) {
            if (a.turn > 0) {
                const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
                while (!(__hip_atomic_load(&a.run[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & kFtRunReady)) {
                    if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > 200000000ll) {  // 2 s: never
                        atomicOr(&a.ctl[1], 1u);
                        sh.stop = 1;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
        }
    };
    if constexpr (SC1) {
        if (tid == 0) sh.stop = 0;  // (read after the scan's barriers)
    }
    const unsigned Ww = (unsigned)a.Ww;
    const unsigned nwords = (unsigned)a.rows * Ww;  // host: < 2^32
    const unsigned base = vid * (unsigned)kFtWords;

    uint32_t flip[kFtK];
    unsigned long long packed = 0;  // CONTIG: the thread's count in field 0; else one 16-bit field per k
    uint32_t alive_c = 0;
    // K5r holds the new board words until the turn is known to be delivered
    // (no earlier turn of the batch overflowed: that turn's rollback board is
    // the buffer this turn writes)
    uint32_t held[kFtK];
    size_t held_at[kFtK];
    bool held_ok[kFtK];
    if constexpr (CONTIG) {
        const unsigned i0 = base + 4u * (unsigned)tid;
        const bool valid = i0 < nwords;
        const unsigned ii = valid ? i0 : nwords - 4;  // every lane stays active for the DPP moves
        const unsigned y = ii / Ww, c = ii - y * Ww;
        const size_t rows[3] = {(size_t)map_in_row(a.in, (int)y - 1) * Ww, (size_t)map_in_row(a.in, (int)y) * Ww,
                                (size_t)map_in_row(a.in, (int)y + 1) * Ww};
        const unsigned cl = c == 0 ? Ww - 1 : c - 1, cr = c + 4 == Ww ? 0 : c + 4;
        const bool ledge = lane == 0 || c == 0, redge = lane == 63 || c + 4 == Ww;
        // all loads first (the edge words unconditionally: L1 hits beside the 16-B loads)
        uint4 q[3];
        uint32_t le[3], re[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            q[j] = src_ld4(rows[j] + c);
            le[j] = src_ld1(rows[j] + cl);
            re[j] = src_ld1(rows[j] + cr);
        }
        uint32_t x[4][3], wv[4][3], ev[4][3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const uint32_t v[4] = {q[j].x, q[j].y, q[j].z, q[j].w};
            uint32_t l = from_left_lane(v[3]), r = from_right_lane(v[0]);
            l = ledge ? le[j] : l;
            r = redge ? re[j] : r;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                x[k][j] = v[k];
                wv[k][j] = __builtin_amdgcn_alignbit(v[k], k == 0 ? l : v[k - 1], 31);  // bit b = cell b-1
                ev[k][j] = __builtin_amdgcn_alignbit(k == 3 ? r : v[k + 1], v[k], 1);  // bit b = cell b+1
            }
        }
        uint32_t nx[4], cnt = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            nx[k] = ft_rule(wv[k], x[k], ev[k]);
            flip[k] = valid ? (nx[k] ^ x[k][1]) : 0u;
            cnt += (uint32_t)__builtin_popcount(flip[k]);
            alive_c += valid ? (uint32_t)__builtin_popcount(nx[k]) : 0u;
        }
        if constexpr (SC1) {
#pragma unroll
            for (int k = 0; k < 4; ++k) held[k] = nx[k];
            held_at[0] = (size_t)(a.dst_base + (int)y) * Ww + c;
            held_ok[0] = valid;
        } else {
            if (valid) dst_st4((size_t)(a.dst_base + (int)y) * Ww + c, make_uint4(nx[0], nx[1], nx[2], nx[3]));
        }
        packed = cnt;
    } else {
#pragma unroll
        for (int k = 0; k < kFtK; ++k) {
            const unsigned i = base + (unsigned)(k * kFtThreads + tid);
            const bool valid = i < nwords;
            const unsigned ii = valid ? i : nwords - 1;
            const unsigned y = ii / Ww, c = ii - y * Ww;
            const size_t rows[3] = {(size_t)map_in_row(a.in, (int)y - 1) * Ww, (size_t)map_in_row(a.in, (int)y) * Ww,
                                    (size_t)map_in_row(a.in, (int)y + 1) * Ww};
            const bool ledge = lane == 0 || c == 0, redge = lane == 63 || c == Ww - 1;
            const unsigned cl = c == 0 ? Ww - 1 : c - 1, cr = c == Ww - 1 ? 0 : c + 1;
            uint32_t x[3], le[3], re[3], w[3], e[3];
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                x[j] = src_ld1(rows[j] + c);
                le[j] = src_ld1(rows[j] + cl);
                re[j] = src_ld1(rows[j] + cr);
            }
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                uint32_t l = from_left_lane(x[j]), r = from_right_lane(x[j]);
                l = ledge ? le[j] : l;
                r = redge ? re[j] : r;
                w[j] = __builtin_amdgcn_alignbit(x[j], l, 31);
                e[j] = __builtin_amdgcn_alignbit(r, x[j], 1);
            }
            const uint32_t nx = ft_rule(w, x, e);
            if constexpr (SC1) {
                held[k] = nx;
                held_at[k] = (size_t)(a.dst_base + (int)y) * Ww + c;
                held_ok[k] = valid;
            } else {
                if (valid) dst_st1((size_t)(a.dst_base + (int)y) * Ww + c, nx);
            }
            flip[k] = valid ? (nx ^ x[1]) : 0u;
            alive_c += valid ? (uint32_t)__builtin_popcount(nx) : 0u;
            packed |= (unsigned long long)__builtin_popcount(flip[k]) << (16 * k);
        }
    }

    // block scan of the packed counts (each field <= 256 x 128 < 2^16)
    unsigned long long inc = packed;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long t = __shfl_up(inc, o, 64);
        if (lane >= o) inc += t;
    }
    if (lane == 63) sh.wsum[wid] = inc;
    if (a.alive) {
        const uint32_t t = wave_sum_u32(alive_c);
        if (lane == 0) sh.alive[wid] = t;
    }
    __syncthreads();
    unsigned long long pre = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        if (w < wid) pre += sh.wsum[w];
        tot += sh.wsum[w];
    }
    const unsigned long long excl_packed = pre + inc - packed;
    uint32_t pos[kFtK], T = 0;
    if constexpr (CONTIG) {
        T = (uint32_t)(tot & 0xFFFFu);
        pos[0] = (uint32_t)(excl_packed & 0xFFFFu);
#pragma unroll
        for (int k = 1; k < kFtK; ++k) pos[k] = pos[k - 1] + (uint32_t)__builtin_popcount(flip[k - 1]);
    } else {
#pragma unroll
        for (int k = 0; k < kFtK; ++k) {
            pos[k] = T + (uint32_t)((excl_packed >> (16 * k)) & 0xFFFFu);
            T += (uint32_t)((tot >> (16 * k)) & 0xFFFFu);
        }
    }

    if (a.dbg & 1) {  // measurement only: no look-back (entries overlap)
        if (tid == 0) {
            wait_run();
            const unsigned long long r0 = run_get(0);
            sh.excl = r0;
            if (vid == (unsigned)a.ncompute - 1) run_set(r0);
        }
    } else if (a.coresident) {
        // publish the aggregate, then every thread sums its share of ALL
        // predecessors' aggregates (<= 4 words each at 5120^2): one round of
        // loads instead of a chain of look-back windows
        if (tid == 0)
            __hip_atomic_store(&a.status[vid], ft_word(kFtAgg, a.epoch, T), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long ep = (unsigned long long)(a.epoch & 0x3FFFFFu);
        unsigned long long part = 0;
        for (unsigned j = (unsigned)tid; j < vid; j += kFtThreads) {
            unsigned long long st;
            int spins = 0;
            for (;;) {
                st = __hip_atomic_load(&a.status[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((st >> 62) != 0 && ((st >> 40) & 0x3FFFFFull) == ep) break;
                if (++spins > (1 << 22)) {  // a predecessor never ran: not co-resident after all
                    atomicOr(&a.ctl[1], 1u);
                    st = 0;
                    break;
                }
                if constexpr (SC1) {
                    // K5r: a turn overflowed while this one waits: this is the turn
                    // after it (the blocks that saw the overflow first never start
                    // it, so it never completes): not delivered
                    if ((spins & 63) == 0 && __hip_atomic_load(&a.ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                        sh.stop = 1;
                        st = 0;
                        break;
                    }
                }
                __builtin_amdgcn_s_sleep(1);
            }
            part += st & kFtValMask;
        }
        if ((a.dbg & 4) && tid == 0 && vid == 0) atomicOr(&a.ctl[1], 1u);  // test hook: the fallback
        part = wave_sum_u64(part);
        if (lane == 0) sh.part[wid] = part;
        __syncthreads();
        if (tid == 0) {
            wait_run();
            const unsigned long long excl = run_get(0) + sh.part[0] + sh.part[1] + sh.part[2] + sh.part[3];
            sh.excl = excl;
            if (vid == (unsigned)a.ncompute - 1) {
                const unsigned long long end = excl + T;
                run_set(end);
                if (a.stop_on_overflow && end > a.cap) atomicOr(&a.ctl[0], 1u);
            }
            if (a.alive) {
                const uint32_t al = sh.alive[0] + sh.alive[1] + sh.alive[2] + sh.alive[3];
                if (al) atomicAdd(a.alive, (unsigned long long)al);
            }
        }
    } else if (wid == 0) {
        unsigned long long excl = 0;
        if (vid == 0) {
            excl = run_get(0);
            if (lane == 0)
                __hip_atomic_store(&a.status[0], ft_word(kFtPrefix, a.epoch, excl + T), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        } else {
            if (lane == 0)
                __hip_atomic_store(&a.status[vid], ft_word(kFtAgg, a.epoch, T), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            long long j = (long long)vid - 1 - lane;  // this lane's predecessor
            const unsigned long long ep = (unsigned long long)(a.epoch & 0x3FFFFFu);
            for (;;) {
                unsigned long long st = kFtPrefix;  // lanes past block 0: an empty prefix (never reached)
                if (j >= 0) {
                    int spins = 0;
                    for (;;) {
                        st = __hip_atomic_load(&a.status[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if ((st >> 62) != 0 && ((st >> 40) & 0x3FFFFFull) == ep) break;
                        if (++spins > (1 << 22)) {  // bounded: record, then treat as an empty prefix
                            atomicOr(&a.ctl[1], 1u);
                            st = kFtPrefix | (ep << 40);
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                    }
                }
                const unsigned long long pm = __ballot((st >> 62) == 2);
                if (pm) {
                    const int first = __builtin_ctzll(pm);  // nearest predecessor with an inclusive prefix
                    excl += wave_sum_u64(lane <= first ? (st & kFtValMask) : 0ull);
                    break;
                }
                excl += wave_sum_u64(st & kFtValMask);
                j -= 64;
            }
            if (lane == 0)
                __hip_atomic_store(&a.status[vid], ft_word(kFtPrefix, a.epoch, excl + T), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) {
            sh.excl = excl;
            if (vid == (unsigned)a.ncompute - 1) {  // the last block's inclusive prefix closes the turn
                const unsigned long long end = excl + T;
                run_set(end);
                if (a.stop_on_overflow && end > a.cap) atomicOr(&a.ctl[0], 1u);
            }
            if (a.alive) {
                const uint32_t al = sh.alive[0] + sh.alive[1] + sh.alive[2] + sh.alive[3];
                if (al) atomicAdd(a.alive, (unsigned long long)al);
            }
        }
    }
    __syncthreads();
    if constexpr (SC1) {
        // the turn is delivered unless an earlier turn overflowed (its entries
        // start past cap: the host rolls back to that turn, whose board is the
        // buffer this turn writes) or a wait timed out
        if (tid == 0 && a.stop_on_overflow && run_get(0) > a.cap) sh.stop = 1;
        __syncthreads();
        if (sh.stop) return false;
        if constexpr (CONTIG) {
            if (held_ok[0]) dst_st4(held_at[0], make_uint4(held[0], held[1], held[2], held[3]));
        } else {
#pragma unroll
            for (int k = 0; k < kFtK; ++k)
                if (held_ok[k]) dst_st1(held_at[k], held[k]);
        }
    }
    if (a.dbg & 2) {  // measurement only: no entries
        signal_done();
        return true;
    }
    const unsigned long long bex = sh.excl;
    const int esz = a.format == kFlipFormatXY ? 8 : 4;
    const bool staged = T <= (uint32_t)(kFtLdsBytes / esz);
    auto put = [&](uint32_t p, unsigned x, unsigned y) {
        const unsigned long long gy = (unsigned long long)a.row0 + y;
        if (staged) {
            if (a.format == kFlipFormatXY)
                reinterpret_cast<int2 *>(sh.buf)[p] = make_int2((int)x, (int)gy);
            else
                reinterpret_cast<uint32_t *>(sh.buf)[p] = (uint32_t)(gy * (unsigned)a.W + x);
        } else if (bex + p < a.cap) {
            if (a.format == kFlipFormatXY) {
                out_st1(2 * (bex + p), x);
                out_st1(2 * (bex + p) + 1, (uint32_t)gy);
            } else {
                out_st1(bex + p, (uint32_t)(gy * (unsigned)a.W + x));
            }
        }
    };
#pragma unroll
    for (int k = 0; k < kFtK; ++k) {
        uint32_t m = flip[k];
        if (!m) continue;
        uint32_t p = pos[k];
        const unsigned i = CONTIG ? base + 4u * (unsigned)tid + (unsigned)k : base + (unsigned)(k * kFtThreads + tid);
        const unsigned y = i / Ww, c = i - y * Ww;
        while (m) {
            const int b = __builtin_ctz(m);
            m &= m - 1;
            put(p++, c * 32u + (unsigned)b, y);
        }
    }
    if (!staged) {
        signal_done();
        return true;
    }
    __syncthreads();
    const unsigned long long lim = bex >= a.cap ? 0ull : (a.cap - bex < T ? a.cap - bex : (unsigned long long)T);
    // copy out in 16-byte stores (4 indices or 2 pairs a lane: wider writes
    // when `out` is host memory across PCIe), with 4-byte-word heads and tails
    // up to the 16-byte boundaries of the destination
    const unsigned wpe = (unsigned)esz / 4;                  // 32-bit words per entry
    uint32_t *d = reinterpret_cast<uint32_t *>(a.out) + bex * wpe;
    const uint32_t *sb = reinterpret_cast<const uint32_t *>(sh.buf);
    const unsigned long long nw = lim * wpe;                 // words to copy
    const unsigned long long head = min(nw, (unsigned long long)((4u - (unsigned)(((uintptr_t)d >> 2) & 3u)) & 3u));
    const unsigned long long nq = (nw - head) / 4;           // whole 16-byte groups
    const unsigned long long dw = bex * wpe;                  // d's word offset in `out`
    if ((unsigned long long)tid < head) out_st1(dw + tid, sb[tid]);
    for (unsigned long long q = tid; q < nq; q += kFtThreads) {
        const unsigned long long w = head + 4 * q;
        out_st4(dw + w, make_uint4(sb[w], sb[w + 1], sb[w + 2], sb[w + 3]));
    }
    const unsigned long long t0 = head + 4 * nq;
    if (t0 + (unsigned long long)tid < nw) out_st1(dw + t0 + tid, sb[t0 + tid]);
    signal_done();
    return true;
}

template <bool CONTIG>
__global__ __launch_bounds__(256) void gol_flip_turn_kernel(FlipTurnArgs a) {
    // copy blocks first in the grid: dispatched at once, their host stores
    // stream while the turn's blocks compute (behind them, they waited for
    // the whole turn's dispatch: 42 us a 5120^2 turn either way)
    const unsigned ncp = a.cp_run ? (unsigned)a.cp_blocks : 0u;
    if (blockIdx.x < ncp) {
        flip_copy_prev(a, blockIdx.x, ncp);
        return;
    }
    if (a.ctl[0]) return;  // an earlier turn of the batch overflowed: the host rolls back to it
    __shared__ unsigned s_vid;
    __shared__ FtShared sh;
    // Block order: blockIdx when every block is resident at once (no
    // contended counter: 800 returning atomics on one word cost ~9 us);
    // otherwise a ticket, so every predecessor is already running.
    unsigned vid = blockIdx.x - ncp;
    if (!a.coresident) {
        if (threadIdx.x == 0) s_vid = atomicAdd(a.ticket, 1u);
        __syncthreads();
        vid = s_vid;
    }
    flip_turn_block<CONTIG, false>(a, vid, sh);
}

// K5r: the turns of a batch in one resident launch (flip_overlap 2; see
// FlipStreamArgs).  The host launches it only when every block is resident
// at once; a wait past timeout_ticks sets ctl[1] and the host restores the
// batch and re-runs it on K5 launches in ticket order.
//  * compute blocks (vid = blockIdx - ncopy): turn t once every compute block
//    has finished turn t - 1 (the done counts), the board ping-ponging
//    between buf0 / buf1; an overflowing turn (ctl[0]) ends the launch after
//    it;
//  * copy blocks: turn t's entries, device list -> host list, once turn t is
//    done (none when stop_on_overflow and the turn overflowed).
constexpr int kFtCopyBatch = 8;  // K5r copy blocks: 16-byte loads in flight a thread
#ifndef GOL_K5R_NOCOPY
#define GOL_K5R_NOCOPY 0  // diagnostic builds: K5r's copy blocks copy nothing (the turn loop's own time; WRONG host lists)
#endif

template <bool CONTIG>
__global__ __launch_bounds__(256) void gol_flip_stream_kernel(FlipStreamArgs s) {
    __shared__ FtShared sh;
    __shared__ int s_go;
    const unsigned ncompute = (unsigned)s.turn.ncompute;
    // every compute block done with turn t (thread 0 polls the shards, the
    // block learns the verdict through s_go): 1 go on; 0 stop (a turn
    // overflowed and this one never runs, or the wait timed out: ctl[1])
    auto wait_turn = [&](int t, bool stop_on_ctl0) {
        if (threadIdx.x == 0) {
            const unsigned *d = s.done + (size_t)kFtShards * kFtShardStride * t;
            const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
            int go = 1;
            for (;;) {
                unsigned n = 0;
#pragma unroll
                for (int i = 0; i < kFtShards; ++i)
                    n += __hip_atomic_load(&d[i * kFtShardStride], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (n >= ncompute) break;
                if (stop_on_ctl0 && __hip_atomic_load(&s.turn.ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                    // turn u overflowed: the turns before it are done, u is not
                    // delivered (the host rolls back to it), later turns never run
                    unsigned m = 0;
#pragma unroll
                    for (int i = 0; i < kFtShards; ++i)
                        m += __hip_atomic_load(&d[i * kFtShardStride], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    go = m >= ncompute;
                    break;
                }
                if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > s.timeout_ticks) {
                    atomicOr(&s.turn.ctl[1], 1u);
                    go = 0;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            s_go = go;
        }
        __syncthreads();
        const int go = s_go;
        __syncthreads();  // s_go is rewritten by the next wait
        return go;
    };
    if (blockIdx.x < (unsigned)s.ncopy) {
        const __amdgpu_buffer_rsrc_t ors =
            __builtin_amdgcn_make_buffer_rsrc(s.turn.out, (short)0, (int)s.turn.out_bytes, 0x00020000);
        // group g = blockIdx mod G copies turns g, g + G, ...: a block's next
        // loads wait for its host stores' acknowledgements (vmcnt is in
        // order), a gap in the link that the other groups' stores fill
        const unsigned G = (unsigned)s.cp_groups, g = blockIdx.x % G;
        const unsigned gb = ((unsigned)s.ncopy - g + G - 1) / G;  // blocks in group g
        const unsigned long long gt = (unsigned long long)(blockIdx.x / G) * blockDim.x + threadIdx.x;
        const unsigned long long gn = (unsigned long long)gb * blockDim.x;
        const unsigned wpe = s.turn.format == kFlipFormatXY ? 2u : 1u;
        for (int t = (int)g; t < s.nturns; t += (int)G) {
            if (!wait_turn(t, true)) return;
            const unsigned long long b0 =
                __hip_atomic_load(&s.run[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & ~kFtRunReady;
            const unsigned long long e0 =
                __hip_atomic_load(&s.run[t + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & ~kFtRunReady;
            if (s.turn.stop_on_overflow && e0 > s.turn.cap) continue;
            const unsigned long long e = e0 < s.turn.cap ? e0 : s.turn.cap;
            if (e <= b0 || GOL_K5R_NOCOPY) continue;
            uint32_t *d = static_cast<uint32_t *>(s.cp_dst) + b0 * wpe;
            const unsigned long long sw = b0 * wpe;  // word offset of the turn's list in `out`
            const unsigned long long nw = (e - b0) * wpe;
            // both lists start 16-byte aligned: after a head up to the
            // destination's next 128-byte line, 16-byte loads and stores
            const unsigned long long head = min(nw, (unsigned long long)(((128u - ((uintptr_t)d & 127u)) & 127u) / 4u));
            const unsigned long long nq = (nw - head) / 4;
            if (gt < head) d[gt] = __builtin_amdgcn_raw_buffer_load_b32(ors, (int)((sw + gt) * 4), 0, kCpolSc1);
            // kFtCopyBatch loads in flight a thread, then their stores: vmcnt
            // counts loads and stores in order, so a load issued behind a host
            // store waits for that store's acknowledgement, which takes as
            // long as the link's queue (one round trip a batch, not a load)
            for (unsigned long long q0 = gt; q0 < nq; q0 += gn * kFtCopyBatch) {
                v4u32 v[kFtCopyBatch];
#pragma unroll
                for (int i = 0; i < kFtCopyBatch; ++i)
                    if (q0 + i * gn < nq)
                        v[i] = __builtin_amdgcn_raw_buffer_load_b128(ors, (int)((sw + head + 4 * (q0 + i * gn)) * 4), 0,
                                                                    kCpolSc1);
#pragma unroll
                for (int i = 0; i < kFtCopyBatch; ++i)
                    if (q0 + i * gn < nq)
                        *reinterpret_cast<uint4 *>(d + head + 4 * (q0 + i * gn)) = make_uint4(v[i].x, v[i].y, v[i].z, v[i].w);
            }
            const unsigned long long t1 = head + 4 * nq;
            if (t1 + gt < nw) d[t1 + gt] = __builtin_amdgcn_raw_buffer_load_b32(ors, (int)((sw + t1 + gt) * 4), 0, kCpolSc1);
        }
        return;
    }
    const unsigned vid = blockIdx.x - (unsigned)s.ncopy;
    FlipTurnArgs a = s.turn;
    a.blk_done = s.blk_done;
    // the blocks whose turn-t board words this block's turn t + 1 reads (rows
    // y0 - 1 .. y1 + 1 of a torus), which are also the blocks that read the
    // words it overwrites: at most three ranges of block ids
    const unsigned Ww = (unsigned)a.Ww, H = (unsigned)a.rows, nwords = H * Ww;
    const unsigned w0 = vid * (unsigned)kFtWords, w1 = min(w0 + (unsigned)kFtWords, nwords) - 1;
    const unsigned y0 = w0 / Ww, y1 = w1 / Ww;
    auto blk = [&](unsigned w) { return w / (unsigned)kFtWords; };
    unsigned rlo[3], rhi[3];
    int nr = 0;
    rlo[nr] = blk((y0 > 0 ? y0 - 1 : 0) * Ww);
    rhi[nr++] = blk(((y1 + 1 < H ? y1 + 1 : H - 1) + 1) * Ww - 1);
    if (y0 == 0) {  // row H - 1 (torus)
        rlo[nr] = blk((H - 1) * Ww);
        rhi[nr++] = blk(nwords - 1);
    }
    if (y1 == H - 1) {  // row 0
        rlo[nr] = 0;
        rhi[nr++] = blk(Ww - 1);
    }
    const unsigned nc0 = rhi[0] - rlo[0] + 1, nc1 = nr > 1 ? rhi[1] - rlo[1] + 1 : 0u,
                   nblk = nc0 + nc1 + (nr > 2 ? rhi[2] - rlo[2] + 1 : 0u);
    for (int t = 0; t < s.nturns; ++t) {
        if (t > 0) {
            // turn t - 1 finished in every block this turn reads from or writes
            // over: wave 0 polls them together, one block a lane
            if (threadIdx.x < 64) {
                const unsigned lane = threadIdx.x;
                const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
                int go = 1;
                for (unsigned k0 = 0; k0 < nblk && go; k0 += 64) {
                    const unsigned k = k0 + lane;
                    const unsigned b = k < nc0 ? rlo[0] + k : k < nc0 + nc1 ? rlo[1] + (k - nc0) : rlo[2] + (k - nc0 - nc1);
                    int bad = 0;
                    if (k < nblk)
                        while (__hip_atomic_load(&s.blk_done[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)t) {
                            if (__hip_atomic_load(&a.ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                                bad = 1;  // a turn overflowed: this one never runs
                                break;
                            }
                            if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > s.timeout_ticks) {
                                atomicOr(&a.ctl[1], 1u);
                                bad = 1;
                                break;
                            }
                            __builtin_amdgcn_s_sleep(1);
                        }
                    if (__ballot(bad)) go = 0;
                }
                // (an overflow in turn t - 1 ends the launch here for every block)
                if (go && __hip_atomic_load(&a.ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) go = 0;
                if (lane == 0) s_go = go;
            }
            __syncthreads();
            const int go = s_go;
            __syncthreads();
            if (!go) return;
        }
        const bool odd = ((s.first + t) & 1) != 0;
        a.src = odd ? s.buf1 : s.buf0;
        a.dst = odd ? s.buf0 : s.buf1;
        a.run = s.run + t;
        // the look-back words rotate over three sets: a block publishes turn
        // t + 3 only after the previous turn's last block finished turn t + 1,
        // whose look-back needed every block's turn-(t + 1) aggregate, which a
        // block publishes after its own turn-t look-back reads (two sets do
        // not suffice: the publish comes before the block's wait on run[0])
        a.status = s.turn.status + (size_t)(t % 3) * ncompute;
        a.done = s.done + (size_t)kFtShards * kFtShardStride * t;
        a.turn = (unsigned)t;
        a.epoch = (s.epoch0 + (unsigned)t) & 0x3FFFFFu;
        a.alive = t == s.nturns - 1 ? s.alive : nullptr;
        const bool more = flip_turn_block<CONTIG, true>(a, vid, sh);
        __syncthreads();  // sh is reused by the next turn
        if (!more) return;  // (uniform: a turn not delivered ends the launch for this block)
    }
}

int64_t flip_turn_blocks(int64_t nwords) { return (nwords + kFtWords - 1) / kFtWords; }

int flip_turn_blocks_per_cu(bool contig) {
    int b = 0;
    const hipError_t e = contig ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, gol_flip_turn_kernel<true>, kFtThreads, 0)
                                : hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, gol_flip_turn_kernel<false>, kFtThreads, 0);
    return e == hipSuccess ? b : 0;
}

hipError_t launch_flip_stream(const FlipStreamArgs &a, hipStream_t s) {
    const int64_t grid = (int64_t)a.turn.ncompute + a.ncopy;
    if (grid == 0 || a.nturns <= 0) return hipSuccess;
    if (a.turn.Ww % 4 == 0)
        hipLaunchKernelGGL(gol_flip_stream_kernel<true>, dim3((unsigned)grid), dim3(kFtThreads), 0, s, a);
    else
        hipLaunchKernelGGL(gol_flip_stream_kernel<false>, dim3((unsigned)grid), dim3(kFtThreads), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_flip_turn(const FlipTurnArgs &a, hipStream_t s) {
    const int64_t grid = (int64_t)a.ncompute + (a.cp_run ? a.cp_blocks : 0);
    if (grid == 0) return hipSuccess;
    if (a.Ww % 4 == 0)
        hipLaunchKernelGGL(gol_flip_turn_kernel<true>, dim3((unsigned)grid), dim3(kFtThreads), 0, s, a);
    else
        hipLaunchKernelGGL(gol_flip_turn_kernel<false>, dim3((unsigned)grid), dim3(kFtThreads), 0, s, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// K4: pack (0/255 bytes -> bits, alive <=> == 255) and unpack (bits -> 0/255).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void pack_kernel(const uint8_t *__restrict__ bytes, uint32_t *__restrict__ words,
                                                    int W, int Ww, int rows) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (int64_t)rows * Ww) return;
    const int row = (int)(idx / Ww);
    const int wc = (int)(idx - (int64_t)row * Ww);
    const uint8_t *p = bytes + (size_t)row * W + (size_t)wc * 32;
    const int n = min(32, W - wc * 32);
    uint32_t w = 0;
    if (n == 32 && (W & 15) == 0) {
        const uint4 *q = reinterpret_cast<const uint4 *>(p);
        const uint4 v0 = q[0], v1 = q[1];
        const uint32_t d[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
        for (int k = 0; k < 8; ++k)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (((d[k] >> (8 * j)) & 0xFFu) == 0xFFu) w |= 1u << (4 * k + j);
    } else {
        for (int b = 0; b < n; ++b)
            if (p[b] == 0xFF) w |= 1u << b;
    }
    words[idx] = w;
}

__global__ __launch_bounds__(256) void unpack_kernel(const uint32_t *__restrict__ words, uint8_t *__restrict__ bytes,
                                                      int W, int Ww, int rows, int il) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (int64_t)rows * Ww) return;
    const int row = (int)(idx / Ww);
    const int wc = (int)(idx - (int64_t)row * Ww);
    uint8_t *p = bytes + (size_t)row * W + (size_t)wc * 32;
    const int n = min(32, W - wc * 32);
    const uint32_t w = canon_word(words, idx, il);
    if (n == 32 && (W & 15) == 0) {
        uint32_t d[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            uint32_t v = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) v |= ((w >> (4 * k + j)) & 1u) ? (0xFFu << (8 * j)) : 0u;
            d[k] = v;
        }
        uint4 *q = reinterpret_cast<uint4 *>(p);
        q[0] = make_uint4(d[0], d[1], d[2], d[3]);
        q[1] = make_uint4(d[4], d[5], d[6], d[7]);
    } else {
        for (int b = 0; b < n; ++b) p[b] = ((w >> b) & 1u) ? 0xFF : 0x00;
    }
}

hipError_t launch_pack(const uint8_t *bytes, uint32_t *words, int W, int Ww, int rows, hipStream_t s) {
    const int64_t n = (int64_t)rows * Ww;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(pack_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, bytes, words, W, Ww, rows);
    return hipGetLastError();
}

hipError_t launch_unpack(const uint32_t *words, uint8_t *bytes, int W, int Ww, int rows, int il, hipStream_t s) {
    const int64_t n = (int64_t)rows * Ww;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(unpack_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, words, bytes, W, Ww,
                       rows, il);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// K6: synthetic board, cell (y, x) alive <=> (splitmix64(seed ^ (y*W + x)) & 3) == 0.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void fill_random_kernel(uint32_t *__restrict__ words, int W, int Ww, int rows,
                                                           int64_t row0, uint64_t seed) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (int64_t)rows * Ww) return;
    const int64_t row = idx / Ww;
    const int wc = (int)(idx - row * Ww);
    const uint64_t base = (uint64_t)(row0 + row) * (uint64_t)W + (uint64_t)wc * 32u;
    const int n = min(32, W - wc * 32);
    uint32_t w = 0;
    for (int b = 0; b < n; ++b)
        if ((splitmix64(seed ^ (base + (uint64_t)b)) & 3u) == 0) w |= 1u << b;
    words[idx] = w;
}

hipError_t launch_fill_random(uint32_t *words, int W, int Ww, int rows, int64_t row0, uint64_t seed,
                              hipStream_t s) {
    const int64_t n = (int64_t)rows * Ww;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(fill_random_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, words, W, Ww, rows,
                       row0, seed);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// K2: popcount reduction (one atomic per wave) and the board digest.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void popcount_kernel(const uint32_t *__restrict__ w, int64_t n,
                                                        unsigned long long *out) {
    uint32_t c = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        c += __builtin_popcount(w[i]);
    const uint32_t tot = wave_sum_u32(c);
    if ((threadIdx.x & 63) == 0 && tot) atomicAdd(out, (unsigned long long)tot);
}

hipError_t launch_popcount(const uint32_t *words, int64_t nwords, unsigned long long *out, hipStream_t s) {
    if (nwords == 0) return hipSuccess;
    const int64_t blocks = std::min<int64_t>((nwords + 255) / 256, 4096);
    hipLaunchKernelGGL(popcount_kernel, dim3((unsigned)blocks), dim3(256), 0, s, words, nwords, out);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void hash_kernel(const uint32_t *__restrict__ w, int64_t n, int64_t word0,
                                                    unsigned long long *out, int il) {
    unsigned long long h = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        h += splitmix64(((uint64_t)(word0 + i) << 32) | (uint64_t)canon_word(w, i, il));
    h = wave_sum_u64(h);
    if ((threadIdx.x & 63) == 0) atomicAdd(out, h);
}

hipError_t launch_hash(const uint32_t *words, int64_t nwords, int64_t word0, unsigned long long *out, int il,
                       hipStream_t s) {
    if (nwords == 0) return hipSuccess;
    const int64_t blocks = std::min<int64_t>((nwords + 255) / 256, 4096);
    hipLaunchKernelGGL(hash_kernel, dim3((unsigned)blocks), dim3(256), 0, s, words, nwords, word0, out, il);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// K3: ordered stream compaction of set bits (flip list / alive list).
// Thread t of block b owns words [b*kBlkWords + t*kWpt, +kWpt): a block
// count pass, a single-block exclusive scan of block counts, and a scatter
// pass that re-scans inside the block keep the output strictly row-major.
// ---------------------------------------------------------------------------
#ifndef GOL_COMPACT_WPT
#define GOL_COMPACT_WPT 4  // words per thread (A/B builds override)
#endif
constexpr int kWpt = GOL_COMPACT_WPT;
constexpr int kBlkWords = 256 * kWpt;

int64_t compact_blocks(int64_t nwords) { return (nwords + kBlkWords - 1) / kBlkWords; }

__device__ __forceinline__ uint32_t cword(const uint32_t *a, const uint32_t *b, int64_t i) {
    return b ? (a[i] ^ b[i]) : a[i];
}
// Canonical (row-major cell order) word i of a ^ b.  Per block and per
// thread chunk (kWpt even) the set-bit count is the same in either layout.
__device__ __forceinline__ uint32_t cword_canon(const uint32_t *a, const uint32_t *b, int64_t i, int il) {
    return b ? (canon_word(a, i, il) ^ canon_word(b, i, il)) : canon_word(a, i, il);
}
static_assert(kWpt % 4 == 0, "pairs and quads must not straddle compaction chunks");

__device__ uint32_t block_excl_scan(uint32_t v, uint32_t *total) {
    __shared__ uint32_t wsum[4];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(inc, o, 64);
        if (lane >= o) inc += t;
    }
    if (lane == 63) wsum[wid] = inc;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        if (w < wid) pre += wsum[w];
        tot += wsum[w];
    }
    if (total) *total = tot;
    return pre + inc - v;
}

__global__ __launch_bounds__(256) void compact_count_kernel(const uint32_t *__restrict__ a,
                                                             const uint32_t *__restrict__ b, int64_t n,
                                                             unsigned long long *blk) {
    const int64_t base = (int64_t)blockIdx.x * kBlkWords + (int64_t)threadIdx.x * kWpt;
    uint32_t c = 0;
    for (int k = 0; k < kWpt; ++k)
        if (base + k < n) c += __builtin_popcount(cword(a, b, base + k));
    __shared__ uint32_t ws[4];
    const uint32_t tot = wave_sum_u32(c);
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = tot;
    __syncthreads();
    if (threadIdx.x == 0) blk[blockIdx.x] = (unsigned long long)ws[0] + ws[1] + ws[2] + ws[3];
}

__global__ __launch_bounds__(1024) void compact_scan_kernel(unsigned long long *blk, int64_t nblk,
                                                             const unsigned long long *base,
                                                             unsigned long long *total) {
    const unsigned long long b0 = base ? *base : 0ull;  // batched lists: running offset
    __shared__ unsigned long long part[1024];
    const int64_t per = (nblk + 1023) / 1024;
    const int64_t beg = (int64_t)threadIdx.x * per;
    const int64_t end = min<int64_t>(beg + per, nblk);
    unsigned long long s = 0;
    for (int64_t i = beg; i < end; ++i) s += blk[i];
    part[threadIdx.x] = s;
    __syncthreads();
    // Hillis-Steele inclusive scan over 1024 partials
    for (int o = 1; o < 1024; o <<= 1) {
        const unsigned long long t = threadIdx.x >= (unsigned)o ? part[threadIdx.x - o] : 0ull;
        __syncthreads();
        part[threadIdx.x] += t;
        __syncthreads();
    }
    unsigned long long run = part[threadIdx.x] - s + b0;  // exclusive
    for (int64_t i = beg; i < end; ++i) {
        const unsigned long long v = blk[i];
        blk[i] = run;
        run += v;
    }
    if (threadIdx.x == 1023) *total = part[1023] + b0;
}

__global__ __launch_bounds__(256) void compact_scatter_kernel(const uint32_t *__restrict__ a,
                                                               const uint32_t *__restrict__ b, int64_t n, int Ww,
                                                               int64_t row0, const unsigned long long *blk_off,
                                                               int32_t *__restrict__ xy, unsigned long long cap,
                                                               int il) {
    const int64_t base = (int64_t)blockIdx.x * kBlkWords + (int64_t)threadIdx.x * kWpt;
    uint32_t c = 0;
    for (int k = 0; k < kWpt; ++k)
        if (base + k < n) c += __builtin_popcount(cword(a, b, base + k));
    const uint32_t pre = block_excl_scan(c, nullptr);
    unsigned long long o = blk_off[blockIdx.x] + pre;
    for (int k = 0; k < kWpt; ++k) {
        const int64_t i = base + k;
        if (i >= n) break;
        uint32_t m = cword_canon(a, b, i, il);
        if (!m) continue;
        const int64_t row = i / Ww;
        const int wc = (int)(i - row * Ww);
        while (m) {
            const int bit = __builtin_ctz(m);
            m &= m - 1;
            if (o < cap) {  // batched lists stop at the caller's capacity
                xy[2 * o] = wc * 32 + bit;
                xy[2 * o + 1] = (int32_t)(row0 + row);
            }
            ++o;
        }
    }
}

hipError_t launch_compact_count(const uint32_t *a, const uint32_t *b, int64_t nwords, unsigned long long *blk,
                                hipStream_t s) {
    const int64_t nb = compact_blocks(nwords);
    if (nb == 0) return hipSuccess;
    hipLaunchKernelGGL(compact_count_kernel, dim3((unsigned)nb), dim3(256), 0, s, a, b, nwords, blk);
    return hipGetLastError();
}

hipError_t launch_compact_scan(unsigned long long *blk, int64_t nblk, unsigned long long *total, hipStream_t s,
                              const unsigned long long *base) {
    hipLaunchKernelGGL(compact_scan_kernel, dim3(1), dim3(1024), 0, s, blk, nblk, base, total);
    return hipGetLastError();
}

hipError_t launch_compact_scatter(const uint32_t *a, const uint32_t *b, int64_t nwords, int Ww, int64_t row0,
                                  const unsigned long long *blk_off, int32_t *xy, int il, hipStream_t s,
                                  unsigned long long cap) {
    const int64_t nb = compact_blocks(nwords);
    if (nb == 0) return hipSuccess;
    hipLaunchKernelGGL(compact_scatter_kernel, dim3((unsigned)nb), dim3(256), 0, s, a, b, nwords, Ww, row0, blk_off,
                       xy, cap, il);
    return hipGetLastError();
}

// The build's tuning macros (A/B builds override them; the product build
// uses the defaults, tests/test_abi_cpu.py::test_product_build_macros).
#define GOL_STR2(x) #x
#define GOL_STR(x) GOL_STR2(x)
const char *build_info() {
    return "GOL_LOOP_PAD=" GOL_STR(GOL_LOOP_PAD) " GOL_PARITY_FIX=" GOL_STR(GOL_PARITY_FIX)
           " GOL_PERSIST_STORE=" GOL_STR(GOL_PERSIST_STORE) " GOL_PAIR_STORE=" GOL_STR(GOL_PAIR_STORE)
           " GOL_PAIR_G2=" GOL_STR(GOL_PAIR_G2) " GOL_FILL_PHASES=" GOL_STR(GOL_FILL_PHASES)
           " GOL_SKEW_STORE_CPOL=" GOL_STR(GOL_SKEW_STORE_CPOL) " GOL_PERSIST_WG_COUNT=" GOL_STR(GOL_PERSIST_WG_COUNT)
           " GOL_COMPACT_WPT=" GOL_STR(GOL_COMPACT_WPT) " GOL_SKEW_WAIT_TRACE=" GOL_STR(GOL_SKEW_WAIT_TRACE) " GOL_K5R_NOCOPY=" GOL_STR(GOL_K5R_NOCOPY);
}

}  // namespace golk
