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

template <unsigned IMM>
__device__ __forceinline__ uint32_t bop(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, IMM);
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
