// gol_bits.h — device helpers of the step kernels (gol_kernels.hip): the
// bit-sliced B3/S23 circuit (v_bitop3 LUTs), LDS word access, DPP lane
// shifts, wave reductions, the counter hash of the synthetic boards and the
// write-through buffer-access policy bit.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace golk {

// ---------------------------------------------------------------------------
// bit-sliced helpers
// ---------------------------------------------------------------------------
template <typename F>
constexpr unsigned tt3(F f) {
    unsigned r = 0;
    for (int i = 0; i < 8; ++i)
        if (f((i >> 2) & 1, (i >> 1) & 1, i & 1)) r |= 1u << i;
    return r;
}
// v_bitop3_b32 truth tables, operand order (a, b, c) -> index a*4 + b*2 + c.
constexpr unsigned kXor3 = tt3([](int a, int b, int c) { return (a ^ b ^ c) != 0; });       // 0x96
constexpr unsigned kMaj = tt3([](int a, int b, int c) { return a + b + c >= 2; });          // 0xE8
// Column sum of three 2-bit row sums (h0 + 2 h1 each, centre included):
//   u = sum of the h0 bits = u0 + 2 u1,  v = sum of the h1 bits = v0 + 2 v1,
//   sum9 = u0 + 2 T with T = u1 + v0 + 2 v1.
// next = (sum9 == 3) | (centre & sum9 == 4) in three LUTs, found by exhaustive
// search over 3-gate circuits; it leans on one unreachable input (centre
// alive with sum9 == 0) and is checked against all 512 neighbourhoods in
// tests/test_rule_circuit.py:
//   g1   = [T == 0 or T == 2]
//   g2   = !v1 & (!centre | u0) | !u0 & !centre
//   next = u0 ? (!g1 & g2) : (g1 & !g2)
constexpr unsigned kG1 = tt3([](int u1, int v0, int v1) { int T = u1 + v0 + 2 * v1; return T == 0 || T == 2; });
constexpr unsigned kG2 = tt3([](int u0, int v1, int c) { return (!v1 && (!c || u0)) || (!u0 && !c); });
constexpr unsigned kNext = tt3([](int u0, int g1, int g2) { return u0 ? (!g1 && g2) : (g1 && !g2); });
static_assert(kG1 == 0x43 && kG2 == 0x35 && kNext == 0x24, "rule LUTs");
static_assert(kXor3 == 0x96 && kMaj == 0xE8, "bitop3 table order");

// Pair rule (round 6, K1w's main loop with `PR`): the two output rows 2m and
// 2m + 1 share the middle pair of their input rows, so they share that
// pair's vertical sum P = S(2m) + S(2m + 1) of the row sums S = s0 + 2 s1:
// P in 0..6 as three bits from four LUTs (a half adder on the s0 bits, a
// full adder on the s1 bits and its carry), two LUTs a row.  Each output row
// is then a 4-LUT circuit of the other input row's sum A (a0 + 2 a1, the row
// above for 2m, below for 2m + 1), P and its centre c: sum9 = A + P and
// next = (sum9 == 3) | (c & sum9 == 4).  Found by exhaustive search over
// 4-gate circuits (none with 3 exists); it leans on the unreachable input
// c & P == 0 and is checked on all 4096 four-row neighbourhoods in
// tests/test_rule_circuit.py:
//   s6   = [exactly one of a0, p0, c]
//   s7   = [(a1, p1, p2) in {000, 001, 110}]
//   s8   = [(c, s6, s7) in {010, 100, 111}]
//   next = s8 & (s7 | !p2)
// 2 (row sum) + 2 (pair) + 4 = 8 LUTs a word-turn instead of 9.
constexpr unsigned kXor2 = tt3([](int a, int b, int) { return (a ^ b) != 0; });   // 0x3C
constexpr unsigned kAnd2 = tt3([](int a, int b, int) { return a && b; });         // 0xC0
constexpr unsigned kBorrow = tt3([](int a, int b, int) { return !a && b; });      // 0x0C: a - b borrows
constexpr unsigned kPrA = tt3([](int a0, int p0, int c) { return a0 + p0 + c == 1; });
constexpr unsigned kPrB = tt3([](int a1, int p1, int p2) {
    return (!a1 && !p1) || (a1 && p1 && !p2);
});
constexpr unsigned kPrC = tt3([](int c, int s6, int s7) { return (!c && s6 && !s7) || (c && !s6 && !s7) || (c && s6 && s7); });
constexpr unsigned kPrNext = tt3([](int p2, int s7, int s8) { return s8 && (s7 || !p2); });
static_assert(kPrA == 0x16 && kPrB == 0x43 && kPrC == 0x94 && kPrNext == 0x8a, "pair rule LUTs");
static_assert(kXor2 == 0x3C && kAnd2 == 0xC0 && kBorrow == 0x0C, "pair adder LUTs");

template <unsigned IMM>
__device__ __forceinline__ uint32_t bop(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, IMM);
}

// P = B + C of two row sums (b0 + 2 b1, c0 + 2 c1): p0 + 2 p1 + 4 p2.  The
// two-input LUTs repeat an operand (8-byte bitop3 keeps the step kernels'
// instruction stream on its code parity; a VOP2 v_xor would not).
__device__ __forceinline__ void pair_sum(uint32_t b0, uint32_t b1, uint32_t c0, uint32_t c1, uint32_t &p0,
                                         uint32_t &p1, uint32_t &p2) {
    p0 = bop<kXor2>(b0, c0, c0);
    const uint32_t k = bop<kAnd2>(b0, c0, c0);
    p1 = bop<kXor3>(b1, c1, k);
    p2 = bop<kMaj>(b1, c1, k);
}
// B = P - C (the inverse, for a pipeline leaving the pair layout; B <= 3)
__device__ __forceinline__ void pair_unsum(uint32_t p0, uint32_t p1, uint32_t c0, uint32_t c1, uint32_t &b0,
                                           uint32_t &b1) {
    b0 = bop<kXor2>(p0, c0, c0);
    const uint32_t br = bop<kBorrow>(p0, c0, c0);
    b1 = bop<kXor3>(p1, c1, br);
}
__device__ __forceinline__ uint32_t pair_rule(uint32_t a0, uint32_t a1, uint32_t p0, uint32_t p1, uint32_t p2,
                                              uint32_t c) {
    const uint32_t s6 = bop<kPrA>(a0, p0, c);
    const uint32_t s7 = bop<kPrB>(a1, p1, p2);
    const uint32_t s8 = bop<kPrC>(c, s6, s7);
    return bop<kPrNext>(p2, s7, s8);
}
// Whole-wavefront lane shifts (DPP wave_shr:1 / wave_shl:1): lane i receives
// lane i-1 / i+1; bound_ctrl zero-fills the edge lane (no `old` operand, so
// no extra v_mov).  Edge lanes are the tile halo.
__device__ __forceinline__ uint32_t from_left_lane(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x138, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t from_right_lane(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x130, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// The B3/S23 rule from the row sums of the rows above (a), at (b) and below
// (c) and the centre word: column sums + the 3-LUT rule (kG1, kG2, kNext).
__device__ __forceinline__ uint32_t rule_word(uint32_t a0, uint32_t a1, uint32_t b0, uint32_t b1, uint32_t c0,
                                              uint32_t c1, uint32_t centre) {
    const uint32_t u0 = bop<kXor3>(a0, b0, c0);
    const uint32_t u1 = bop<kMaj>(a0, b0, c0);
    const uint32_t v0 = bop<kXor3>(a1, b1, c1);
    const uint32_t v1 = bop<kMaj>(a1, b1, c1);
    const uint32_t g1 = bop<kG1>(u1, v0, v1);
    const uint32_t g2 = bop<kG2>(u0, v1, centre);
    return bop<kNext>(u0, g1, g2);
}

// Row sums and centre words of one row (K1r).
template <int WPL>
struct LdsRow {
    uint32_t s0[WPL], s1[WPL], c[WPL];
};
typedef unsigned v4u32 __attribute__((ext_vector_type(4)));
constexpr int kCpolSc1 = 16;  // buffer load/store aux bit: sc1 (write-through store, L1-bypassing load)

// LDS words read / written as relaxed workgroup-scope atomics through an
// address-space-3 pointer: plain ds_read_b32 / ds_write_b32 at immediate
// offsets that the compiler neither caches in registers, nor turns into flat
// accesses, nor merges into ds_read2 / ds_write2 (whose 8-bit offsets cost a
// VALU address add per row once rows are more than 1 KB apart)
typedef __attribute__((address_space(3))) uint32_t lds_word;
__device__ __forceinline__ uint32_t lds_get(const lds_word *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_put(lds_word *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

}  // namespace golk
