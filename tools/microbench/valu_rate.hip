// Microbenchmark: VALU issue rate per op type on gfx950, and the cost of running
// several distinct large straight-line code variants per workgroup (I-cache).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define N_ACC 8
template <int OP>
__global__ __launch_bounds__(256) void k_rate(uint32_t* out, uint32_t seed, int iters) {
  uint32_t a[N_ACC];
  float f[N_ACC];
  uint64_t b[N_ACC];
  for (int i = 0; i < N_ACC; i++) { a[i] = seed * (threadIdx.x + 1) + i; f[i] = (float)a[i]; b[i] = ((uint64_t)a[i] << 32) | a[i]; }
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int r = 0; r < 16; r++)
#pragma unroll
      for (int i = 0; i < N_ACC; i++) {
        if (OP == 0) a[i] = a[i] ^ (a[(i + 1) % N_ACC] + r);        // v_xor (+ v_add)
        if (OP == 1) a[i] = __builtin_amdgcn_bitop3_b32(a[i], a[(i + 1) % N_ACC], a[(i + 3) % N_ACC], 0x96);
        if (OP == 2) a[i] = __builtin_amdgcn_alignbit(a[i], a[(i + 1) % N_ACC], 7);
        if (OP == 3) a[i] = a[i] + a[(i + 1) % N_ACC] + a[(i + 2) % N_ACC];  // v_add3
        if (OP == 4) f[i] = __builtin_fmaf(f[i], 1.0001f, f[(i + 1) % N_ACC]);
        if (OP == 5) a[i] = __builtin_amdgcn_perm(a[i], a[(i + 1) % N_ACC], 0x05040100u + r);
        if (OP == 6) asm volatile("v_lshrrev_b64 %0, 7, %1" : "=v"(b[i]) : "v"(b[(i + 1) % N_ACC]));
        if (OP == 7) a[i] = (a[(i + 1) % N_ACC] << 7) | a[i];  // v_lshl_or_b32
        if (OP == 8) a[i] = __builtin_amdgcn_alignbyte(a[i], a[(i + 1) % N_ACC], 3);
        if (OP == 9) a[i] = a[i] + a[(i + 1) % N_ACC];  // v_add_u32 alone
      }
  }
  uint32_t s = 0;
  for (int i = 0; i < N_ACC; i++) s ^= a[i] ^ __float_as_uint(f[i]) ^ (uint32_t)b[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// NV distinct straight-line variants (~VLEN ops each); wave w of a workgroup runs
// variant (w % NV) if SPREAD else variant 0.
template <int V>
__device__ __forceinline__ void variant(uint32_t (&a)[N_ACC]) {
#pragma unroll
  for (int r = 0; r < 256; r++)
#pragma unroll
    for (int i = 0; i < N_ACC; i++)
      a[i] = __builtin_amdgcn_bitop3_b32(a[i], a[(i + 1 + V) % N_ACC], a[(i + 3 + r) % N_ACC] + (V * 977 + r), 0x96);
}

template <bool SPREAD>
__global__ __launch_bounds__(512) void k_icache(uint32_t* out, uint32_t seed, int iters) {
  uint32_t a[N_ACC];
  for (int i = 0; i < N_ACC; i++) a[i] = seed * (threadIdx.x + 1) + i;
  const int w = SPREAD ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : 0;
  for (int it = 0; it < iters; it++) {
    switch (w) {
      case 0: variant<0>(a); break;
      case 1: variant<1>(a); break;
      case 2: variant<2>(a); break;
      case 3: variant<3>(a); break;
      case 4: variant<4>(a); break;
      case 5: variant<5>(a); break;
      case 6: variant<6>(a); break;
      default: variant<7>(a); break;
    }
  }
  uint32_t s = 0;
  for (int i = 0; i < N_ACC; i++) s ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K>
static float time_kernel(K kern, dim3 grid, dim3 block, uint32_t* out, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, grid, block, 0, 0, out, 1u, iters);
  hipEventRecord(e0);
  for (int rep = 0; rep < 5; rep++) hipLaunchKernelGGL(kern, grid, block, 0, 0, out, 1u, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  uint32_t* out;
  hipMalloc(&out, 256 * 8 * 512 * 4 * 8);
  const int iters = 200;
  const char* names[] = {"xor+add (2 ops)", "bitop3", "alignbit", "add3", "fma_f32", "perm", "lshrrev_b64", "lshl_or", "alignbyte", "add_u32"};
  for (int op = 0; op < 10; op++) {
    for (int wpc : {4, 8, 16}) {  // waves per CU
      dim3 grid(256 * wpc / 4), block(256);
      float ms = 0;
      switch (op) {
        case 0: ms = time_kernel(k_rate<0>, grid, block, out, iters); break;
        case 1: ms = time_kernel(k_rate<1>, grid, block, out, iters); break;
        case 2: ms = time_kernel(k_rate<2>, grid, block, out, iters); break;
        case 3: ms = time_kernel(k_rate<3>, grid, block, out, iters); break;
        case 4: ms = time_kernel(k_rate<4>, grid, block, out, iters); break;
        case 5: ms = time_kernel(k_rate<5>, grid, block, out, iters); break;
        case 6: ms = time_kernel(k_rate<6>, grid, block, out, iters); break;
        case 7: ms = time_kernel(k_rate<7>, grid, block, out, iters); break;
        case 8: ms = time_kernel(k_rate<8>, grid, block, out, iters); break;
        case 9: ms = time_kernel(k_rate<9>, grid, block, out, iters); break;
      }
      const double ops = (double)grid.x * 256 * iters * 16 * N_ACC * (op == 0 ? 2 : 1);
      printf("%-16s waves/CU=%2d  %8.3f ms  %7.2f T lane-ops/s\n", names[op], wpc, ms, ops / (ms * 1e-3) / 1e12);
    }
  }
  for (int spread = 0; spread < 2; spread++) {
    dim3 grid(256 * 2), block(512);
    float ms = spread ? time_kernel(k_icache<true>, grid, block, out, 20) : time_kernel(k_icache<false>, grid, block, out, 20);
    const double ops = (double)grid.x * 512 * 20 * 256 * N_ACC * 2;
    printf("icache spread=%d: %8.3f ms  %7.2f T lane-ops/s\n", spread, ms, ops / (ms * 1e-3) / 1e12);
  }
  return 0;
}
