// Same-run ceilings for the bench line (include/celestia_eds.h, cel_probe_*): what this box,
// at this moment, gives the two bounds the hot path is priced against.
//   k_probe_sha   the NMT kernels' SHA-256 compression (cel::sha256_compress) chained in
//                 registers on every lane, no memory traffic: the NMT phase's measured peak
//                 (tools/microbench/sha_rate.hip is the sweep this probe fixes one point of,
//                 16 workgroups of 256 per CU, 64 compressions per lane). Each wave also reads
//                 the shader-clock counter (s_memtime) and the constant-rate counter
//                 (s_memrealtime) at its start and end, so the sustained clock under a
//                 VALU-bound load comes from the same launch.
//   k_probe_copy  a streaming copy (one 16-byte element per lane, non-temporal or default
//                 policy): achievable HBM bytes/s, read + write; and the read-only and
//                 write-only streams of the same elements.
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

// The streaming copy, one 16-byte element per lane and one lane per element (n / 256
// workgroups, no loop: MI355X_MICROARCH.md's float4 copy), non-temporal or default policy:
// 6.49-6.53 TB/s read + write on MI355X at 1-8 GiB, against 5.4-5.8 for the 16 KiB
// chunk-per-workgroup shape of rounds 1-5 (profiles/r6_hbm_copy.txt). MODE 0 copies, 1 only
// reads (the xor of every element, kept live by a test that never passes), 2 and 3 only
// write (16 / 4 bytes per lane): HBM writes stream at ~5.5 TB/s at best against ~7 for
// reads, which prices a write-heavy kernel (the RS extension writes 3 bytes per byte read).
template <bool NT, int MODE>
__global__ __launch_bounds__(256) void k_probe_copy(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                    uint64_t n16) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (MODE == 2) {  // write only: grid-strided (a read-free stream needs few lanes in flight)
    const u32x4 v = {(uint32_t)i, 1u, 2u, 3u};
    for (uint64_t j = i; j < n16; j += (uint64_t)gridDim.x * 256) __builtin_nontemporal_store(v, dst + j);
    return;
  }
  if (MODE == 3) {  // write only, 4 bytes per lane (the RS kernels' store width): 5.5-5.6 TB/s
    // against 4.0-4.6 for 16 bytes per lane (profiles/r6_hbm_write.txt)
    uint32_t* d4 = reinterpret_cast<uint32_t*>(dst);
    for (uint64_t j = i; j < 4 * n16; j += (uint64_t)gridDim.x * 256) d4[j] = (uint32_t)j;
    return;
  }
  if (MODE == 1) {
    u32x4 acc = {0, 0, 0, 0};
    for (uint64_t j = i; j < n16; j += (uint64_t)gridDim.x * 256) acc ^= __builtin_nontemporal_load(src + j);
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9E3779B9u && i == 0) dst[0] = acc;
    return;
  }
  if (i < n16) {
    if (NT)
      __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
    else
      dst[i] = src[i];
  }
}

hipError_t launch_probe_sha(uint32_t* out, unsigned long long* clk, uint32_t blocks, int n, hipStream_t s) {
  hipLaunchKernelGGL(k_probe_sha, dim3(blocks), dim3(256), 0, s, out, clk, 1u, n);
  return hipGetLastError();
}

hipError_t launch_probe_copy(const void* src, void* dst, uint64_t bytes, uint32_t blocks, int mode, bool nt,
                             hipStream_t s) {
  const uint64_t n16 = bytes / 16;
  const auto* sp = static_cast<const u32x4*>(src);
  auto* dp = static_cast<u32x4*>(dst);
  if (mode == 0) {
    const uint64_t g = (n16 + 255) / 256;  // one lane per element
    if (g > 0x7FFFFFFFull) return hipErrorInvalidValue;
    if (nt)
      hipLaunchKernelGGL((k_probe_copy<true, 0>), dim3((unsigned)g), dim3(256), 0, s, sp, dp, n16);
    else
      hipLaunchKernelGGL((k_probe_copy<false, 0>), dim3((unsigned)g), dim3(256), 0, s, sp, dp, n16);
  } else if (mode == 1) {
    hipLaunchKernelGGL((k_probe_copy<true, 1>), dim3(blocks), dim3(256), 0, s, sp, dp, n16);
  } else if (mode == 2) {
    hipLaunchKernelGGL((k_probe_copy<true, 2>), dim3(blocks), dim3(256), 0, s, sp, dp, n16);
  } else {
    hipLaunchKernelGGL((k_probe_copy<false, 3>), dim3(blocks), dim3(256), 0, s, sp, dp, n16);
  }
  return hipGetLastError();
}

}  // namespace cel
