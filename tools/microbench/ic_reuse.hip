// Infinity-Cache reuse probe for the two-pass RS extension.
//
// Question: when the column pass re-reads [Q0|Q1] right after the row pass wrote Q1,
// does the read come from the 256 MiB Infinity Cache (faster than HBM)?
//   cold   : read S bytes after streaming 1 GiB through another buffer
//   rd-rd  : read S bytes right after reading the same S bytes
//   wr-rd  : read S bytes right after writing the same S bytes
// plus streaming read / write / copy rates and the column-shaped access (256-B
// segments at a 128 KiB stride, 2 adjacent segments per wave pair) against contiguous.
// Build: hipcc --offload-arch=gfx950 -O3 -o ic_reuse ic_reuse.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

// one dword per lane, 256 B per wave instruction, grid-stride over n dwords
__global__ void k_read(const uint32_t* __restrict__ p, size_t n, uint32_t* sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    acc ^= p[i];
  if (acc == 0x12345679u) sink[0] = acc;
}
__global__ void k_write(uint32_t* __restrict__ p, size_t n, uint32_t v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = v ^ (uint32_t)i;
}
__global__ void k_copy(const uint32_t* __restrict__ a, uint32_t* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    b[i] = a[i];
}
// Column-shaped read like the RS column pass: wave w reads K segments of 256 B,
// segment i at base(w) + i*stride. Waves of a 4-wave group cover 4 adjacent 256-B
// segments (2 cells x 2 slices). Each wave holds K loads in flight like the kernel.
template <int K>
__global__ __launch_bounds__(256) void k_colread(const uint32_t* __restrict__ p, uint32_t ncols, uint32_t stride_dw,
                                                 uint32_t sq_dw, uint32_t nsq, uint32_t* sink) {
  const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint32_t per_sq = ncols;  // 256-B column segments per square
  if (wave >= per_sq * nsq) return;
  const uint32_t z = wave / per_sq, c = wave % per_sq;
  const uint32_t* b = p + (size_t)z * sq_dw + (size_t)c * 64 + lane;
  uint32_t w[K];
#pragma unroll
  for (int i = 0; i < K; i++) w[i] = b[(size_t)i * stride_dw];
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < K; i++) acc ^= w[i];
  if (acc == 0x12345679u) sink[0] = acc;
}

// Column-shaped write, same geometry as k_colread.
template <int K>
__global__ __launch_bounds__(256) void k_colwrite(uint32_t* __restrict__ p, uint32_t ncols, uint32_t stride_dw,
                                                  uint32_t sq_dw, uint32_t nsq) {
  const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (wave >= ncols * nsq) return;
  const uint32_t z = wave / ncols, c = wave % ncols;
  uint32_t* b = p + (size_t)z * sq_dw + (size_t)c * 64 + lane;
#pragma unroll
  for (int i = 0; i < K; i++) b[(size_t)i * stride_dw] = wave ^ (uint32_t)i;
}
// Row-shaped read: wave reads K consecutive 256-B segments (32 KiB contiguous at K=128).
template <int K>
__global__ __launch_bounds__(256) void k_rowread(const uint32_t* __restrict__ p, uint32_t nwaves, uint32_t* sink) {
  const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (wave >= nwaves) return;
  const uint32_t* b = p + (size_t)wave * K * 64 + lane;
  uint32_t w[K];
#pragma unroll
  for (int i = 0; i < K; i++) w[i] = b[(size_t)i * 64];
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < K; i++) acc ^= w[i];
  if (acc == 0x12345679u) sink[0] = acc;
}

int main() {
  const size_t GB = 1ull << 30, MB = 1ull << 20;
  uint32_t *big, *x, *sink;
  CK(hipMalloc(&big, 2 * GB));
  CK(hipMalloc(&x, 512 * MB));
  CK(hipMalloc(&sink, 64));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int grid = 256 * 16, blk = 256;
  auto tm = [&](auto&& f) {
    CK(hipEventRecord(e0));
    f();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e-3;
  };
  auto flush = [&] { hipLaunchKernelGGL(k_write, dim3(grid), dim3(blk), 0, 0, big, GB / 4, 7u); };
  // streaming rates on 1 GiB
  flush();
  CK(hipDeviceSynchronize());
  for (int r = 0; r < 2; r++) {
    double t = tm([&] { hipLaunchKernelGGL(k_read, dim3(grid), dim3(blk), 0, 0, big, GB / 4, sink); });
    printf("stream read  1 GiB: %.3f ms = %.2f TB/s\n", t * 1e3, GB / t / 1e12);
    t = tm([&] { hipLaunchKernelGGL(k_write, dim3(grid), dim3(blk), 0, 0, big, GB / 4, 3u); });
    printf("stream write 1 GiB: %.3f ms = %.2f TB/s\n", t * 1e3, GB / t / 1e12);
    t = tm([&] { hipLaunchKernelGGL(k_copy, dim3(grid), dim3(blk), 0, 0, big, big + GB / 4, GB / 8); });
    printf("stream copy 512 MiB -> 512 MiB: %.3f ms = %.2f TB/s (r+w)\n", t * 1e3, GB / t / 1e12);
  }
  const size_t sizes[] = {16 * MB, 32 * MB, 64 * MB, 128 * MB, 192 * MB, 256 * MB, 512 * MB};
  for (size_t S : sizes) {
    double cold = 0, rdrd = 0, wrrd = 0, wr = 0;
    const int reps = 3;
    for (int r = 0; r < reps; r++) {
      flush();
      cold += tm([&] { hipLaunchKernelGGL(k_read, dim3(grid), dim3(blk), 0, 0, x, S / 4, sink); });
      rdrd += tm([&] { hipLaunchKernelGGL(k_read, dim3(grid), dim3(blk), 0, 0, x, S / 4, sink); });
      flush();
      wr += tm([&] { hipLaunchKernelGGL(k_write, dim3(grid), dim3(blk), 0, 0, x, S / 4, 5u); });
      wrrd += tm([&] { hipLaunchKernelGGL(k_read, dim3(grid), dim3(blk), 0, 0, x, S / 4, sink); });
    }
    auto bw = [&](double t) { return S / (t / reps) / 1e12; };
    printf("S=%4zu MiB: read cold %.2f TB/s | read after read %.2f | write (cold) %.2f | read after write %.2f TB/s\n",
           S / MB, bw(cold), bw(rdrd), bw(wr), bw(wrrd));
  }
  // column-shaped reads, k=128 geometry: EDS row = 256 cells x 512 B = 128 KiB; a
  // column of the top half = 128 cells; 512 segments of 256 B per row (2 per cell).
  {
    const uint32_t ncols = 512, K = 128, stride_dw = 128 * 1024 / 4, sq_dw = 32 * MB / 4;
    const uint32_t nsq = 8;  // 8 squares of 32 MiB: 256 MiB span, 128 MiB read (top halves)
    const size_t bytes = (size_t)nsq * ncols * K * 256;
    const dim3 g((ncols * nsq + 3) / 4);
    double tc = 0, tw = 0, tr = 0, tcont = 0;
    for (int r = 0; r < 3; r++) {
      flush();
      tc += tm([&] { hipLaunchKernelGGL(k_colread<128>, g, dim3(256), 0, 0, x, ncols, stride_dw, sq_dw, nsq, sink); });
      tr += tm([&] { hipLaunchKernelGGL(k_colread<128>, g, dim3(256), 0, 0, x, ncols, stride_dw, sq_dw, nsq, sink); });
      flush();
      tw += tm([&] { hipLaunchKernelGGL(k_write, dim3(grid), dim3(blk), 0, 0, x, 256 * MB / 4, 9u); });
      tw -= 0;
      double t = tm([&] { hipLaunchKernelGGL(k_colread<128>, g, dim3(256), 0, 0, x, ncols, stride_dw, sq_dw, nsq, sink); });
      tcont += t;
    }
    printf("column-shaped read of 128 MiB (k=128 top halves of 8 squares): cold %.2f TB/s | after read %.2f | after write %.2f TB/s\n",
           bytes / (tc / 3) / 1e12, bytes / (tr / 3) / 1e12, bytes / (tcont / 3) / 1e12);
  }
  {
    const uint32_t ncols = 512, stride_dw = 128 * 1024 / 4, sq_dw = 32 * MB / 4, nsq = 8;
    const size_t bytes = (size_t)nsq * ncols * 128 * 256;
    const dim3 g((ncols * nsq + 3) / 4);
    double tw = 0, tr = 0;
    for (int r = 0; r < 3; r++) {
      flush();
      tw += tm([&] { hipLaunchKernelGGL(k_colwrite<128>, g, dim3(256), 0, 0, x, ncols, stride_dw, sq_dw, nsq); });
      flush();
      tr += tm([&] { hipLaunchKernelGGL(k_rowread<128>, dim3((uint32_t)(bytes / 32768 / 4)), dim3(256), 0, 0, x,
                                        (uint32_t)(bytes / 32768), sink); });
    }
    printf("column-shaped write of 128 MiB (cold): %.2f TB/s | row-shaped read of 128 MiB (cold, 32 KiB per wave): %.2f TB/s\n",
           bytes / (tw / 3) / 1e12, bytes / (tr / 3) / 1e12);
    // big row-shaped read: 1 GiB
    double tb = 0;
    for (int r = 0; r < 3; r++) {
      flush();
      tb += tm([&] { hipLaunchKernelGGL(k_rowread<128>, dim3(GB / 32768 / 4), dim3(256), 0, 0, big + GB / 4, GB / 32768, sink); });
    }
    printf("row-shaped read of 1 GiB (cold): %.2f TB/s\n", GB / (tb / 3) / 1e12);
  }
  return 0;
}
