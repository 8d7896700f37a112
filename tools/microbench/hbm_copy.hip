// Streaming-copy sweep on gfx950: which copy shape reaches the achievable HBM rate the
// library's cel_probe_hbm_copy should report (MI355X_MICROARCH.md: 6.29 TB/s float4 copy).
// Shapes: grid-stride vs contiguous chunk per workgroup; loads in flight per lane; cache
// policy; workgroups per CU. Bytes = read + written.
// Build: hipcc --offload-arch=gfx950 -O3 -o hbm_copy hbm_copy.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void k_stride(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t n) {
  const uint64_t st = (uint64_t)gridDim.x * 256;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i + (U - 1) * st < n; i += U * st) {
    u32x4 v[U];
#pragma unroll
    for (int j = 0; j < U; j++) v[j] = NT ? __builtin_nontemporal_load(s + i + j * st) : s[i + j * st];
#pragma unroll
    for (int j = 0; j < U; j++) {
      if (NT) __builtin_nontemporal_store(v[j], d + i + j * st);
      else d[i + j * st] = v[j];
    }
  }
}

// each workgroup copies contiguous chunks of 256 * U * 16 bytes, chunk index grid-strided
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_chunk(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t n) {
  const uint64_t per = 256 * U;
  for (uint64_t c = blockIdx.x; c * per < n; c += gridDim.x) {
    const uint64_t b = c * per + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int j = 0; j < U; j++) v[j] = NT ? __builtin_nontemporal_load(s + b + j * 256) : s[b + j * 256];
#pragma unroll
    for (int j = 0; j < U; j++) {
      if (NT) __builtin_nontemporal_store(v[j], d + b + j * 256);
      else d[b + j * 256] = v[j];
    }
  }
}

template <class K>
static void run(const char* name, K kern, int wgcu, const u32x4* s, u32x4* d, uint64_t n) {
  dim3 grid(256 * wgcu), block(256);
  hipLaunchKernelGGL(kern, grid, block, 0, 0, s, d, n);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float best = 1e30f;
  for (int r = 0; r < 5; r++) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(kern, grid, block, 0, 0, s, d, n);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  printf("%-22s WG/CU %2d: %8.3f ms  %7.0f GB/s\n", name, wgcu, best, 2.0 * n * 16 / (best * 1e-3) / 1e9);
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
}

int main(int argc, char** argv) {
  const uint64_t half = (argc > 1 ? strtoull(argv[1], nullptr, 0) : (2ull << 30));
  const uint64_t n = half / 16;
  u32x4 *s, *d;
  CK(hipMalloc(&s, half));
  CK(hipMalloc(&d, half));
  CK(hipMemset(s, 0x5A, half));
  CK(hipDeviceSynchronize());
  for (int w : {4, 8, 16}) {
    run("stride U1 default", k_stride<1, false>, w, s, d, n);
    run("stride U4 default", k_stride<4, false>, w, s, d, n);
    run("stride U4 nt", k_stride<4, true>, w, s, d, n);
    run("chunk U4 default", k_chunk<4, false>, w, s, d, n);
    run("chunk U4 nt", k_chunk<4, true>, w, s, d, n);
    run("chunk U8 default", k_chunk<8, false>, w, s, d, n);
    run("chunk U8 nt", k_chunk<8, true>, w, s, d, n);
  }
  CK(hipFree(s));
  CK(hipFree(d));
  return 0;
}
