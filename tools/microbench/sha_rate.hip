// SHA-256 compression throughput on gfx950 with no memory traffic: every lane runs a chain
// of N compressions of its own message (the same sha256_compress the NMT kernels use; each
// output feeds the next message, so nothing folds away), at several waves per SIMD.
// Gives the achieved SHA-256 peak the NMT phase is measured against.
// Build: hipcc --offload-arch=gfx950 -O3 -I../../celestia-app_amd/csrc -o sha_rate sha_rate.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "sha256_device.hpp"

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

template <int WAVES>
__global__ __launch_bounds__(256, WAVES) void k_sha(uint32_t* out, uint32_t seed, int n) {
  uint32_t st[8], w[16];
  cel::sha256_init(st);
  const uint32_t t = blockIdx.x * 256u + threadIdx.x;
#pragma unroll
  for (int i = 0; i < 16; i++) w[i] = seed * (t + 1) + i * 0x9E3779B9u;
#pragma unroll 1
  for (int c = 0; c < n; c++) {
    cel::sha256_compress(st, w);
#pragma unroll
    for (int i = 0; i < 8; i++) w[i] ^= st[i];
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s ^= st[i];
  out[t] = s;
}

// the same compression with the three 16-round schedule bodies unrolled (no loop)
__device__ __forceinline__ void compress_unrolled(uint32_t (&st)[8], uint32_t (&w)[16]) {
  cel::ShaRegs r{st[0], st[1], st[2], st[3], st[4], st[5], st[6], st[7]};
#pragma unroll
  for (int i = 0; i < 16; i++) cel::sha_round(r, w[i] + cel::kSha256K[i]);
#pragma unroll
  for (int base = 16; base < 64; base += 16) {
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const uint32_t w15 = w[(j + 1) & 15], w2 = w[(j + 14) & 15];
      const uint32_t s0 = cel::xor3(cel::rotr32(w15, 7), cel::rotr32(w15, 18), w15 >> 3);
      const uint32_t s1 = cel::xor3(cel::rotr32(w2, 17), cel::rotr32(w2, 19), w2 >> 10);
      w[j] = w[j] + s0 + w[(j + 9) & 15] + s1;
      cel::sha_round(r, w[j] + cel::kSha256K[base + j]);
    }
  }
  st[0] += r.a; st[1] += r.b; st[2] += r.c; st[3] += r.d;
  st[4] += r.e; st[5] += r.f; st[6] += r.g; st[7] += r.h;
}

template <int WAVES>
__global__ __launch_bounds__(256, WAVES) void k_sha_u(uint32_t* out, uint32_t seed, int n) {
  uint32_t st[8], w[16];
  cel::sha256_init(st);
  const uint32_t t = blockIdx.x * 256u + threadIdx.x;
#pragma unroll
  for (int i = 0; i < 16; i++) w[i] = seed * (t + 1) + i * 0x9E3779B9u;
#pragma unroll 1
  for (int c = 0; c < n; c++) {
    compress_unrolled(st, w);
#pragma unroll
    for (int i = 0; i < 8; i++) w[i] ^= st[i];
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s ^= st[i];
  out[t] = s;
}

template <int WAVES>
static void run_u(uint32_t* out, int blocks_per_cu) {
  const int n = 64;
  dim3 grid(256 * blocks_per_cu), block(256);
  hipLaunchKernelGGL(k_sha_u<WAVES>, grid, block, 0, 0, out, 1u, n);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a));
  for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k_sha_u<WAVES>, grid, block, 0, 0, out, 1u, n);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= 5;
  const double comp = (double)grid.x * 256 * n;
  printf("unrolled, bound %d, %2d WG/CU:  %8.3f ms  %6.2f G compressions/s\n", WAVES, blocks_per_cu, ms,
         comp / (ms * 1e-3) / 1e9);
}

template <int WAVES>
static void run(uint32_t* out, int blocks_per_cu) {
  const int n = 64;
  dim3 grid(256 * blocks_per_cu), block(256);
  hipLaunchKernelGGL(k_sha<WAVES>, grid, block, 0, 0, out, 1u, n);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a));
  for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k_sha<WAVES>, grid, block, 0, 0, out, 1u, n);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= 5;
  const double comp = (double)grid.x * 256 * n;
  printf("waves/SIMD bound %d, %2d WG/CU: %8.3f ms  %6.2f G compressions/s\n", WAVES, blocks_per_cu, ms,
         comp / (ms * 1e-3) / 1e9);
}

int main() {
  uint32_t* out;
  CK(hipMalloc(&out, 256 * 64 * 256 * 4));
  for (int b : {4, 8, 16, 32}) run<1>(out, b);
  for (int b : {8, 16, 32}) run<4>(out, b);
  for (int b : {16, 32, 64}) run<8>(out, b);
  for (int b : {16, 32}) run_u<4>(out, b);
  for (int b : {16, 32}) run_u<1>(out, b);
  CK(hipFree(out));
  return 0;
}
