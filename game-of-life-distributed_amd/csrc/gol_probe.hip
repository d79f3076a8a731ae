// gol_probe.hip — the host-link ceiling of the event stream (VERDICT r5
// item 3).  K5 (gol_flip_turn_kernel) writes each turn's CellFlipped list
// straight into page-locked host memory (golhip_host_alloc) with 16-byte
// stores; this kernel streams the same kind of stores, coalesced, over a
// buffer of the same kind, so bench.py can price K5's host bytes against what
// the link actually takes on the box.  Its own translation unit: adding it
// leaves the step kernels' code object (and its layout) alone.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gol_kernels.h"

namespace golk {

__global__ __launch_bounds__(256) void host_write_probe_kernel(uint4 *__restrict__ dst, uint64_t n16, uint32_t tag) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
        const uint32_t v = (uint32_t)i ^ tag;
        dst[i] = make_uint4(v, v + 1, v + 2, v + 3);
    }
}

hipError_t launch_host_write_probe(void *dst, uint64_t bytes, int blocks, uint32_t tag, hipStream_t s) {
    hipLaunchKernelGGL(host_write_probe_kernel, dim3((unsigned)blocks), dim3(256), 0, s,
                       reinterpret_cast<uint4 *>(dst), bytes / 16, tag);
    return hipGetLastError();
}

}  // namespace golk
