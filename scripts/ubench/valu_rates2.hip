// gfx950 VALU throughput of candidate ops for the bit-sliced Life stage.
// Each kernel: ITER x CH independent asm ops; 8 waves/SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITER 16384
#define CH 8
#define PRE uint32_t v[CH]; uint64_t w[CH]; \
  for (int i = 0; i < CH; ++i) { v[i] = seed * (threadIdx.x + 7 * i + 1); w[i] = v[i] * 3ull; } \
  for (int it = 0; it < ITER; ++it) { _Pragma("unroll") for (int i = 0; i < CH; ++i) {
#define POST }} uint32_t r = 0; for (int i = 0; i < CH; ++i) r ^= v[i] ^ (uint32_t)w[i]; out[blockIdx.x * blockDim.x + threadIdx.x] = r;
#define A1 : "=v"(v[i]) : "v"(v[(i + 1) % CH])
#define A2 : "=v"(v[i]) : "v"(v[(i + 1) % CH]), "v"(v[(i + 2) % CH]) : "vcc"
#define A3 : "=v"(v[i]) : "v"(v[(i + 1) % CH]), "v"(v[(i + 2) % CH]), "v"(v[(i + 3) % CH])
#define K(n, body) __global__ __launch_bounds__(256) void k##n(uint32_t* out, uint32_t seed) { PRE body; POST }
K(0, asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" A3))
K(1, asm volatile("v_or3_b32 %0, %1, %2, %3" A3))
K(2, asm volatile("v_alignbit_b32 %0, %1, %2, 31" A2))
K(3, asm volatile("v_lshl_or_b32 %0, %1, 1, %2" A2))
K(4, asm volatile("v_lshlrev_b32 %0, 1, %1" A1))
K(5, asm volatile("v_or_b32 %0, %1, %2" A2))
K(6, asm volatile("v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" A1))
K(7, asm volatile("v_or_b32_dpp %0, %1, %2 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" A2))
K(8, asm volatile("v_cndmask_b32 %0, %1, %2, vcc" A2))
K(9, asm volatile("v_addc_co_u32 %0, vcc, %1, %2, vcc" A2))
K(10, asm volatile("v_lshrrev_b64 %0, 1, %1" : "=v"(w[i]) : "v"(w[(i + 1) % CH])))
K(11, asm volatile("v_and_or_b32 %0, %1, %2, %3" A3))
K(12, asm volatile("v_bfi_b32 %0, %1, %2, %3" A3))
K(13, asm volatile("v_perm_b32 %0, %1, %2, %3" A3))
K(14, asm volatile("v_alignbyte_b32 %0, %1, %2, 1" A2))
K(15, asm volatile("v_lshl_add_u32 %0, %1, 1, %2" A2))
K(16, asm volatile("v_cmp_gt_i32_e32 vcc, 0, %0" :: "v"(v[(i + 1) % CH]) : "vcc"))
K(17, asm volatile("v_bitop3_b32 %0, %1, %2, 0 bitop3:0x96" A2))
K(18, asm volatile("v_alignbit_b32 %0, %1, %2, %3" A3))
K(19, asm volatile("v_lshrrev_b32 %0, 1, %1" A1))
K(20, asm volatile("v_bitop3_b32 %0, %1, %1, %2 bitop3:0x96" A2))
typedef void (*kf)(uint32_t*, uint32_t);
int main() {
  int blocks = 256 * 8;
  uint32_t* d; hipMalloc(&d, blocks * 256 * 4);
  kf ks[] = {k0,k1,k2,k3,k4,k5,k6,k7,k8,k9,k10,k11,k12,k13,k14,k15,k16,k17,k18,k19,k20};
  const char* names[] = {"v_bitop3_b32 (3 vgpr)", "v_or3_b32", "v_alignbit_b32 imm", "v_lshl_or_b32", "v_lshlrev_b32",
    "v_or_b32", "v_mov_b32_dpp wave_shr", "v_or_b32_dpp wave_shr", "v_cndmask_b32", "v_addc_co_u32",
    "v_lshrrev_b64", "v_and_or_b32", "v_bfi_b32", "v_perm_b32", "v_alignbyte_b32", "v_lshl_add_u32",
    "v_cmp_gt_i32 vcc", "v_bitop3 2vgpr+0", "v_alignbit_b32 vgpr sh", "v_lshrrev_b32", "v_bitop3 a,a,b"};
  float best[21];
  for (int n = 0; n < 21; ++n) best[n] = 1e30f;
  for (int pass = 0; pass < 3; ++pass)
    for (int n = 0; n < 21; ++n) {
      hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
      hipLaunchKernelGGL(ks[n], dim3(blocks), dim3(256), 0, 0, d, 3u);
      hipEventRecord(a);
      for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(ks[n], dim3(blocks), dim3(256), 0, 0, d, 3u);
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b); ms /= 3;
      if (ms < best[n]) best[n] = ms;
    }
  for (int n = 0; n < 21; ++n) {
    double instr = (double)blocks * 4 * ITER * CH;
    printf("%-26s %8.3f ms  %.3f wave-instr/cycle/SIMD @2.4GHz\n", names[n], best[n], instr / (best[n] * 1e-3) / 1024 / 2.4e9);
  }
  return 0;
}
