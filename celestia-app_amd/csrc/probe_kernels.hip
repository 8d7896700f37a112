// Same-run ceilings for the bench line (include/celestia_eds.h, cel_probe_*): what this box,
// at this moment, gives the two bounds the hot path is priced against.
//   k_probe_sha   the NMT kernels' SHA-256 compression (cel::sha256_compress) chained in
//                 registers on every lane, no memory traffic: the NMT phase's measured peak
//                 (tools/microbench/sha_rate.hip is the sweep this probe fixes one point of,
//                 16 workgroups of 256 per CU, 64 compressions per lane). Each wave also reads
//                 the shader-clock counter (s_memtime) and the constant-rate counter
//                 (s_memrealtime) at its start and end, so the sustained clock under a
//                 VALU-bound load comes from the same launch.
//   k_probe_copy  a streaming copy (dwordx4, non-temporal like the RS kernels' accesses):
//                 achievable HBM bytes/s, read + write.
#include <hip/hip_runtime.h>

#include "cel_internal.hpp"
#include "sha256_device.hpp"

namespace cel {

__global__ __launch_bounds__(256, 4) void k_probe_sha(uint32_t* out, unsigned long long* clk, uint32_t seed, int n) {
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  uint32_t st[8], w[16];
  sha256_init(st);
  const uint32_t t = blockIdx.x * 256u + threadIdx.x;
#pragma unroll
  for (int i = 0; i < 16; i++) w[i] = seed * (t + 1) + i * 0x9E3779B9u;
#pragma unroll 1
  for (int c = 0; c < n; c++) {
    sha256_compress(st, w);
#pragma unroll
    for (int i = 0; i < 8; i++) w[i] ^= st[i];
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s ^= st[i];
  out[t] = s;
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63u) == 0) {
    const uint32_t wv = t >> 6;
    clk[2 * wv] = t1 - t0;
    clk[2 * wv + 1] = r1 - r0;
  }
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_probe_copy(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                    uint64_t n16) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
    const u32x4 v = __builtin_nontemporal_load(src + i);
    __builtin_nontemporal_store(v, dst + i);
  }
}

hipError_t launch_probe_sha(uint32_t* out, unsigned long long* clk, uint32_t blocks, int n, hipStream_t s) {
  hipLaunchKernelGGL(k_probe_sha, dim3(blocks), dim3(256), 0, s, out, clk, 1u, n);
  return hipGetLastError();
}

hipError_t launch_probe_copy(const void* src, void* dst, uint64_t bytes, uint32_t blocks, hipStream_t s) {
  hipLaunchKernelGGL(k_probe_copy, dim3(blocks), dim3(256), 0, s, static_cast<const u32x4*>(src),
                     static_cast<u32x4*>(dst), bytes / 16);
  return hipGetLastError();
}

}  // namespace cel
