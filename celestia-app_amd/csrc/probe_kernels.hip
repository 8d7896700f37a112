// Same-run ceilings for the bench line (include/celestia_eds.h, cel_probe_*): what this box,
// at this moment, gives the two bounds the hot path is priced against.
//   k_probe_sha   the NMT kernels' SHA-256 compression (cel::sha256_compress) chained in
//                 registers on every lane, no memory traffic: the NMT phase's measured peak
//                 (tools/microbench/sha_rate.hip is the sweep this probe fixes one point of,
//                 16 workgroups of 256 per CU, 64 compressions per lane). Each wave also reads
//                 the shader-clock counter (s_memtime) and the constant-rate counter
//                 (s_memrealtime) at its start and end, so the sustained clock under a
//                 VALU-bound load comes from the same launch.
//   k_probe_copy  a streaming copy (16 KiB chunks per workgroup, four dwordx4 loads in
//                 flight per lane, non-temporal or default policy): achievable HBM bytes/s,
//                 read + write.
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

// Each workgroup copies contiguous 16 KiB chunks (four dwordx4 loads in flight per lane
// before their stores), chunk index grid-strided: the fastest shape of the sweep in
// tools/microbench/hbm_copy.hip (profiles/r5_hbm_copy_sweep.txt: 5.6-5.8 TB/s non-temporal
// at 4-16 workgroups per CU, against 4.6-5.5 for grid-strided lanes). NT = non-temporal.
template <bool NT>
__global__ __launch_bounds__(256) void k_probe_copy(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                    uint64_t n16) {
  constexpr uint64_t kPer = 256 * 4;
  for (uint64_t c = blockIdx.x; c * kPer < n16; c += gridDim.x) {
    const uint64_t b = c * kPer + threadIdx.x;
    if (b + 3 * 256 < n16) {
      u32x4 v[4];
#pragma unroll
      for (int j = 0; j < 4; j++) v[j] = NT ? __builtin_nontemporal_load(src + b + j * 256) : src[b + j * 256];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        if (NT)
          __builtin_nontemporal_store(v[j], dst + b + j * 256);
        else
          dst[b + j * 256] = v[j];
      }
    } else {
      for (uint64_t i = b; i < n16 && i < c * kPer + kPer; i += 256) dst[i] = src[i];
    }
  }
}

hipError_t launch_probe_sha(uint32_t* out, unsigned long long* clk, uint32_t blocks, int n, hipStream_t s) {
  hipLaunchKernelGGL(k_probe_sha, dim3(blocks), dim3(256), 0, s, out, clk, 1u, n);
  return hipGetLastError();
}

hipError_t launch_probe_copy(const void* src, void* dst, uint64_t bytes, uint32_t blocks, bool nt, hipStream_t s) {
  if (nt)
    hipLaunchKernelGGL(k_probe_copy<true>, dim3(blocks), dim3(256), 0, s, static_cast<const u32x4*>(src),
                       static_cast<u32x4*>(dst), bytes / 16);
  else
    hipLaunchKernelGGL(k_probe_copy<false>, dim3(blocks), dim3(256), 0, s, static_cast<const u32x4*>(src),
                       static_cast<u32x4*>(dst), bytes / 16);
  return hipGetLastError();
}

}  // namespace cel
