// Throughput of the VALU ops the step kernel is made of (gfx950).
// Each kernel runs ITER x 8 independent chains of one op; time -> ops/s.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITER 4096
#define CH 8
template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t* out, uint32_t seed) {
  uint32_t v[CH];
#pragma unroll
  for (int i = 0; i < CH; ++i) v[i] = seed * (threadIdx.x + 7 * i + 1);
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      if constexpr (OP == 0) v[i] = v[i] ^ (v[(i + 1) % CH]);
      if constexpr (OP == 1) v[i] = __builtin_amdgcn_bitop3_b32(v[i], v[(i + 1) % CH], v[(i + 2) % CH], 0x96);
      if constexpr (OP == 2) v[i] = __builtin_amdgcn_alignbit(v[i], v[(i + 1) % CH], 31);
      if constexpr (OP == 3) v[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)v[i], 0x138, 0xF, 0xF, true) ^ v[(i+3)%CH];
      if constexpr (OP == 4) v[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)v[i], 0x111, 0xF, 0xF, true) ^ v[(i+3)%CH]; // row_shr:1
    }
  }
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < CH; ++i) r ^= v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
template <int OP> float run(uint32_t* d, int blocks) {
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, 3u);
  hipEventRecord(a);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, 3u);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b); return ms / 5;
}
int main() {
  int blocks = 256 * 8;  // 8 blocks per CU = 8 waves/SIMD
  uint32_t* d; hipMalloc(&d, blocks * 256 * 4);
  const char* names[] = {"v_xor_b32", "v_bitop3_b32", "v_alignbit_b32", "dpp wave_shr + xor (2 instr)", "dpp row_shr + xor (2 instr)"};
  float ms[5] = {run<0>(d, blocks), run<1>(d, blocks), run<2>(d, blocks), run<3>(d, blocks), run<4>(d, blocks)};
  for (int i = 0; i < 5; ++i) {
    double instr = (double)blocks * 4 * ITER * CH * (i >= 3 ? 2 : 1);  // wave-instructions
    double per_simd_cycle = instr / (ms[i] * 1e-3) / 1024 / 2.4e9;
    printf("%-30s %8.3f ms  %.3f wave-instr/cycle/SIMD @2.4GHz (peak 0.5)\n", names[i], ms[i], per_simd_cycle);
  }
  return 0;
}
