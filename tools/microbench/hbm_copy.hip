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

// round 6: the canonical float4 copy (one element per thread, one thread per element, no
// loop: n / 256 workgroups), and read-only / write-only streams of the same shape
template <bool NT>
__global__ __launch_bounds__(256) void k_flat(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) {
    if (NT) __builtin_nontemporal_store(__builtin_nontemporal_load(s + i), d + i);
    else d[i] = s[i];
  }
}
__global__ __launch_bounds__(256) void k_read(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t n) {
  const uint64_t st = (uint64_t)gridDim.x * 256;
  u32x4 acc = {0, 0, 0, 0};
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += st) acc ^= __builtin_nontemporal_load(s + i);
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) d[0] = acc;  // keeps the loads live
}
__global__ __launch_bounds__(256) void k_write(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t n) {
  const uint64_t st = (uint64_t)gridDim.x * 256;
  const u32x4 v = {(uint32_t)threadIdx.x, 1u, 2u, 3u};
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += st) __builtin_nontemporal_store(v, d + i);
}

// write-only forms: 16 B or 4 B per lane, non-temporal or default policy, grid-strided
template <int W, bool NT>
__global__ __launch_bounds__(256) void k_write_form(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t n) {
  const uint64_t st = (uint64_t)gridDim.x * 256;
  if (W == 16) {
    const u32x4 v = {(uint32_t)threadIdx.x, 1u, 2u, 3u};
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += st) {
      if (NT) __builtin_nontemporal_store(v, d + i);
      else d[i] = v;
    }
  } else {
    uint32_t* d4 = reinterpret_cast<uint32_t*>(d);
    const uint32_t v = threadIdx.x;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < 4 * n; i += st) {
      if (NT) __builtin_nontemporal_store(v, d4 + i);
      else d4[i] = v;
    }
  }
}

template <class K>
static float time_grid(K kern, dim3 grid, const u32x4* s, u32x4* d, uint64_t n) {
  hipLaunchKernelGGL(kern, grid, dim3(256), 0, 0, s, d, n);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float best = 1e30f;
  for (int r = 0; r < 5; r++) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(kern, grid, dim3(256), 0, 0, s, d, n);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return best;
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
  {
    const dim3 flat((unsigned)((n + 255) / 256));
    float ms = time_grid(k_flat<false>, flat, s, d, n);
    printf("%-22s          : %8.3f ms  %7.0f GB/s\n", "flat float4 default", ms, 2.0 * n * 16 / (ms * 1e-3) / 1e9);
    ms = time_grid(k_flat<true>, flat, s, d, n);
    printf("%-22s          : %8.3f ms  %7.0f GB/s\n", "flat float4 nt", ms, 2.0 * n * 16 / (ms * 1e-3) / 1e9);
    for (int w : {4, 8, 16}) {
      ms = time_grid(k_read, dim3(256 * w), s, d, n);
      printf("%-22s WG/CU %2d: %8.3f ms  %7.0f GB/s (read only)\n", "read nt", w, ms, 1.0 * n * 16 / (ms * 1e-3) / 1e9);
      ms = time_grid(k_write, dim3(256 * w), s, d, n);
      printf("%-22s WG/CU %2d: %8.3f ms  %7.0f GB/s (write only)\n", "write nt", w, ms, 1.0 * n * 16 / (ms * 1e-3) / 1e9);
    }
  }
  for (int w : {4, 8, 16}) {
    float ms = time_grid(k_write_form<16, false>, dim3(256 * w), s, d, n);
    printf("%-22s WG/CU %2d: %8.3f ms  %7.0f GB/s (write only)\n", "write x4 default", w, ms, 1.0 * n * 16 / (ms * 1e-3) / 1e9);
    ms = time_grid(k_write_form<4, true>, dim3(256 * w), s, d, n);
    printf("%-22s WG/CU %2d: %8.3f ms  %7.0f GB/s (write only)\n", "write dword nt", w, ms, 1.0 * n * 16 / (ms * 1e-3) / 1e9);
    ms = time_grid(k_write_form<4, false>, dim3(256 * w), s, d, n);
    printf("%-22s WG/CU %2d: %8.3f ms  %7.0f GB/s (write only)\n", "write dword default", w, ms, 1.0 * n * 16 / (ms * 1e-3) / 1e9);
  }
  if (argc > 2) return 0;  // the flat / read / write lines only
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
