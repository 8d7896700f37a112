// Memory-pattern probe for the GF(2^16) register kernel (rs_gf16x.hip), K = 512, one
// 512-byte-share square (EDS 1024 x 1024 cells, row pitch 512 KiB).
//
// Question: why does the column pass (shards = rows, 512 KiB apart) run 1.5x slower per
// byte than the row pass (shards = cells, 512 B apart) with the same instruction shapes?
// Each wave moves 512 shards x 64 B in and out like k_rs_gf16x (no transform; VALU filler
// of F dependent xors per loaded dword stands in for it) under:
//   map 0: lane = j + 8L, L = shard bits 5-7 (the kernel's arrangement A)
//   map 1: L = shard bits 0-2 (8 consecutive shards per instruction)
//   map 2: dwordx4 loads/stores, 4 lanes per 64-B block, 16 consecutive shards per instr
//   map 3: two dwordx4 per shard group (lo 32 B, hi 32 B), 2 lanes per half, 32 shards
//          per instruction (consecutive)
//   map 4: map 2 with the shards of arrangement A (S0 = shard bit 0, S1..S3 = bits 5-7)
//   map 7: dwordx2, 8 lanes per 64-B block, 8 consecutive shards per instruction
//   map 8: map 7 with lane group L = shard bits 5-7 (arrangement A)
// Build: hipcc --offload-arch=gfx950 -O3 -o gf16_mem gf16_mem.hip
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

typedef uint32_t uint32_t4 __attribute__((ext_vector_type(4)));
typedef uint32_t uint32_t2 __attribute__((ext_vector_type(2)));

struct Geo {
  const uint8_t* in;
  uint8_t* out;
  uint32_t in_shard, in_axis, out_shard, out_axis, axes;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}

// byte offset of wide access i (0..31) of lane `lane`
template <int MAP>
__device__ __forceinline__ uint32_t woff(int i, uint32_t lane, uint32_t shard) {
  if constexpr (MAP == 2) {
    return ((uint32_t)i * 16u + (lane >> 2)) * shard + (lane & 3u) * 16u;
  } else if constexpr (MAP == 3) {
    const uint32_t s = (uint32_t)(i >> 1) * 32u + (lane >> 1);
    return s * shard + (uint32_t)(i & 1) * 32u + (lane & 1u) * 16u;
  } else {
    const uint32_t S = lane >> 2;
    const uint32_t s = (S & 1u) | ((uint32_t)(i & 15) << 1) | ((S >> 1) << 5) | ((uint32_t)(i >> 4) << 8);
    return s * shard + (lane & 3u) * 16u;
  }
}

template <int MAP, int F>
__global__ __launch_bounds__(256, 3) void k_mem(Geo g) {
  constexpr int K = 512, NR = K / 8;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t tile = blockIdx.x * 4u + (threadIdx.x >> 6);
  if (tile >= g.axes * 8u) return;
  const uint32_t cb = tile % 8u, x = tile / 8u;
  const auto rin = rsrc(g.in + (uint64_t)x * g.in_axis + cb * 64u);
  const auto rout = rsrc(g.out + (uint64_t)x * g.out_axis + cb * 64u);
  uint32_t w[2 * NR];
  if constexpr (MAP >= 7) {
    const uint32_t L = lane >> 3;
#pragma unroll
    for (int i = 0; i < NR; i++) {
      const uint32_t s = MAP == 8 ? ((uint32_t)(i & 31) | (L << 5) | ((uint32_t)(i >> 5) << 8)) : ((uint32_t)i * 8u + L);
      const auto v = __builtin_amdgcn_raw_buffer_load_b64(rin, s * g.in_shard + (lane & 7u) * 8u, 0, 2);
      w[2 * i] = v[0];
      w[2 * i + 1] = v[1];
    }
  } else if constexpr (MAP >= 2) {
    uint32_t4 v[NR / 2];
#pragma unroll
    for (int i = 0; i < NR / 2; i++) v[i] = __builtin_amdgcn_raw_buffer_load_b128(rin, woff<MAP>(i, lane, g.in_shard), 0, 2);
#pragma unroll
    for (int i = 0; i < NR / 2; i++) {
      w[4 * i] = v[i].x;
      w[4 * i + 1] = v[i].y;
      w[4 * i + 2] = v[i].z;
      w[4 * i + 3] = v[i].w;
    }
  } else {
    const uint32_t j = lane & 7u, L = lane >> 3;
#pragma unroll
    for (int i = 0; i < NR; i++) {
      const uint32_t s = MAP == 0 ? ((uint32_t)(i & 31) | (L << 5) | ((uint32_t)(i >> 5) << 8)) : ((uint32_t)i * 8u + L);
      w[2 * i] = __builtin_amdgcn_raw_buffer_load_b32(rin, s * g.in_shard + j * 4u, 0, 2);
      w[2 * i + 1] = __builtin_amdgcn_raw_buffer_load_b32(rin, s * g.in_shard + j * 4u + 32u, 0, 2);
    }
  }
  // filler: F rounds of a dependent xor-rotate chain over every register
#pragma unroll 1
  for (int f = 0; f < F; f++) {
#pragma unroll
    for (int i = 0; i < 2 * NR; i++) w[i] = __builtin_amdgcn_alignbit(w[i], w[(i + 1) & (2 * NR - 1)], 7) ^ w[i];
  }
  if constexpr (MAP >= 7) {
    const uint32_t L = lane >> 3;
#pragma unroll
    for (int i = 0; i < NR; i++) {
      const uint32_t s = MAP == 8 ? ((uint32_t)(i & 31) | (L << 5) | ((uint32_t)(i >> 5) << 8)) : ((uint32_t)i * 8u + L);
      uint32_t2 v = {w[2 * i], w[2 * i + 1]};
      __builtin_amdgcn_raw_buffer_store_b64(v, rout, s * g.out_shard + (lane & 7u) * 8u, 0, 2);
    }
  } else if constexpr (MAP >= 2) {
#pragma unroll
    for (int i = 0; i < NR / 2; i++) {
      uint32_t4 v = {w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]};
      __builtin_amdgcn_raw_buffer_store_b128(v, rout, woff<MAP>(i, lane, g.out_shard), 0, 2);
    }
  } else {
    const uint32_t j = lane & 7u, L = lane >> 3;
#pragma unroll
    for (int i = 0; i < NR; i++) {
      const uint32_t s = MAP == 0 ? ((uint32_t)(i & 31) | (L << 5) | ((uint32_t)(i >> 5) << 8)) : ((uint32_t)i * 8u + L);
      __builtin_amdgcn_raw_buffer_store_b32(w[2 * i], rout, s * g.out_shard + j * 4u, 0, 2);
      __builtin_amdgcn_raw_buffer_store_b32(w[2 * i + 1], rout, s * g.out_shard + j * 4u + 32u, 0, 2);
    }
  }
}

template <int MAP, int F>
static float run(const Geo& g, int reps) {
  const uint32_t tiles = g.axes * 8u;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL((k_mem<MAP, F>), dim3((tiles + 3) / 4), dim3(256), 0, 0, g);
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; r++) hipLaunchKernelGGL((k_mem<MAP, F>), dim3((tiles + 3) / 4), dim3(256), 0, 0, g);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1e3f / reps;
}

int main(int argc, char** argv) {
  const size_t W = 1024, share = 512;
  // argv[1] = "pad": the row pitch sweep (is the column pass's loss the 512 KiB stride?)
  if (argc > 1) {
    const size_t pads[] = {0, 256, 512, 2048, 4096, 8192 + 256};
    for (size_t pad : pads) {
      const size_t pitch = W * share + pad;
      uint8_t* d;
      CK(hipMalloc(&d, W * pitch));
      CK(hipMemset(d, 1, W * pitch));
      const Geo rows{d, d + 512 * share, share, (uint32_t)pitch, share, (uint32_t)pitch, 512};
      const Geo cols{d, d + 512 * pitch, (uint32_t)pitch, share, (uint32_t)pitch, share, 1024};
      const float r = run<8, 0>(rows, 5), c = run<8, 0>(cols, 5);
      const float r2 = run<8, 54>(rows, 5), c2 = run<8, 54>(cols, 5);
      printf("pitch pad %6zu B: map 8 rows %7.1f us cols %7.1f us (%5.2f TB/s); with filler rows %7.1f cols %7.1f us\n",
             pad, r, c, 2.0 * 1024 * 512 * 512 / c / 1e6, r2, c2);
      CK(hipFree(d));
    }
    return 0;
  }
  const size_t pitch = W * share, eds = W * pitch;  // 512 MiB
  uint8_t* d;
  CK(hipMalloc(&d, eds));
  CK(hipMemset(d, 1, eds));
  // rows: Q0 rows (512) -> Q1; cols: all 1024 columns, rows 0..511 -> rows 512..1023
  const Geo rows{d, d + 512 * share, share, (uint32_t)pitch, share, (uint32_t)pitch, 512};
  const Geo cols{d, d + 512 * pitch, (uint32_t)pitch, share, (uint32_t)pitch, share, 1024};
  const int reps = 5;
  printf("bytes moved: rows %.0f MB, cols %.0f MB\n", 2.0 * 512 * 512 * 512 / 1e6, 2.0 * 1024 * 512 * 512 / 1e6);
#define ONE(MAP, F)                                                                                        \
  {                                                                                                        \
    const float r = run<MAP, F>(rows, reps), c = run<MAP, F>(cols, reps);                                  \
    printf("map %d filler %3d: rows %8.1f us (%5.2f TB/s)  cols %8.1f us (%5.2f TB/s)  cols/rows per B %.2f\n", \
           MAP, F, r, 2.0 * 512 * 512 * 512 / r / 1e6, c, 2.0 * 1024 * 512 * 512 / c / 1e6, c / r / 2);     \
  }
  ONE(0, 0)
  ONE(2, 0)
  ONE(4, 0)
  ONE(7, 0)
  ONE(8, 0)
  ONE(0, 54)
  ONE(2, 54)
  ONE(4, 54)
  ONE(7, 54)
  ONE(8, 54)
  CK(hipFree(d));
  return 0;
}
