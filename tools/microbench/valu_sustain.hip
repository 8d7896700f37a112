// Sustained VALU rate vs kernel duration: the same independent-chain v_alignbit / v_add3
// loop as valu_rate.hip run for ~0.1 ms to ~100 ms. A falling lane-op rate on the long
// runs means the clock drops under sustained integer load (power management), which
// prices every VALU-bound kernel of this repo below the 2.4 GHz ceiling.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define N_ACC 8
template <int OP>
__global__ __launch_bounds__(256) void k_rate(uint32_t* out, uint32_t seed, int iters) {
  uint32_t a[N_ACC];
  for (int i = 0; i < N_ACC; i++) a[i] = seed * (threadIdx.x + 1) + i;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int r = 0; r < 16; r++)
#pragma unroll
      for (int i = 0; i < N_ACC; i++) {
        if (OP == 0) a[i] = __builtin_amdgcn_alignbit(a[i], a[(i + 1) % N_ACC], 7);
        if (OP == 1) a[i] = a[i] + a[(i + 1) % N_ACC] + a[(i + 2) % N_ACC];
        if (OP == 2) a[i] = __builtin_amdgcn_bitop3_b32(a[i], a[(i + 1) % N_ACC], a[(i + 3) % N_ACC], 0x96);
      }
  }
  uint32_t s = 0;
  for (int i = 0; i < N_ACC; i++) s ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  uint32_t* out;
  const dim3 grid(256 * 4), block(256);  // 4 waves per SIMD
  hipMalloc(&out, (size_t)grid.x * block.x * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[3] = {"alignbit", "add3", "bitop3"};
  for (int op = 0; op < 3; op++) {
    for (int iters : {50, 500, 5000, 50000}) {
      auto launch = [&] {
        if (op == 0) hipLaunchKernelGGL(k_rate<0>, grid, block, 0, 0, out, 1u, iters);
        if (op == 1) hipLaunchKernelGGL(k_rate<1>, grid, block, 0, 0, out, 1u, iters);
        if (op == 2) hipLaunchKernelGGL(k_rate<2>, grid, block, 0, 0, out, 1u, iters);
      };
      launch();
      hipDeviceSynchronize();
      hipEventRecord(e0);
      launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double ops = (double)grid.x * block.x * iters * 16 * N_ACC;
      printf("%-9s iters=%6d  %9.3f ms  %6.2f T lane-ops/s\n", names[op], iters, ms, ops / (ms * 1e-3) / 1e12);
    }
  }
  return 0;
}
