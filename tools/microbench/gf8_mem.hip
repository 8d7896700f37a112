// Memory-pattern probe for the GF(2^8) wave-per-axis kernel (rs_axis.hip k_rs_axis_gf8),
// k = 128, 512-byte shares, B squares (EDS 256 x 256 cells, row pitch 128 KiB).
//
// Question: is the kernel's access shape (one 256-byte shard slice per wave instruction,
// dword per lane) below what wider accesses stream? Each wave moves the 128 data shards of
// its (square, axis, 256-byte slice) in and 128 parity shards out, like the row pass
// (shards 512 B apart: Q0 row -> Q1 row) and the column pass (shards 128 KiB apart:
// [Q0|Q1] column -> [Q2|Q3] column); no transform (F dependent xor rounds as filler):
//   map 0: dword per lane, 64 lanes = one shard's 256-byte slice (the kernel's shape)
//   map 1: dwordx2 per lane, 32 lanes per slice, 2 shards per instruction
//   map 2: dwordx4 per lane, 16 lanes per slice, 4 shards per instruction
// Build: hipcc --offload-arch=gfx950 -O3 -o gf8_mem gf8_mem.hip
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

typedef uint32_t u4 __attribute__((ext_vector_type(4)));
typedef uint32_t u2 __attribute__((ext_vector_type(2)));

struct Geo {
  const uint8_t* in;
  uint8_t* out;
  uint32_t in_shard, out_shard;
  uint64_t in_axis, out_axis, sq;
  uint32_t axes, nsq;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}

template <int MAP, int F, int POL = 2>
__global__ __launch_bounds__(256, 3) void k_mem(Geo g) {
  constexpr int K = 128;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t tile = blockIdx.x * 4u + (threadIdx.x >> 6);
  if (tile >= g.axes * 2u * g.nsq) return;
  const uint32_t sl = tile % 2u, r = tile / 2u, x = r % g.axes, z = r / g.axes;
  const auto rin = rsrc(g.in + z * g.sq + x * g.in_axis + sl * 256u);
  const auto rout = rsrc(g.out + z * g.sq + x * g.out_axis + sl * 256u);
  uint32_t w[K];
  if constexpr (MAP == 0) {
#pragma unroll
    for (int i = 0; i < K; i++) w[i] = __builtin_amdgcn_raw_buffer_load_b32(rin, lane * 4u, i * g.in_shard, POL);
  } else if constexpr (MAP == 1) {
    const uint32_t s = lane >> 5, o = (lane & 31u) * 8u;
#pragma unroll
    for (int i = 0; i < K / 2; i++) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b64(rin, s * g.in_shard + o, 2 * i * g.in_shard, 2);
      w[2 * i] = v[0];
      w[2 * i + 1] = v[1];
    }
  } else {
    const uint32_t s = lane >> 4, o = (lane & 15u) * 16u;
#pragma unroll
    for (int i = 0; i < K / 4; i++) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(rin, s * g.in_shard + o, 4 * i * g.in_shard, 2);
      w[4 * i] = v[0];
      w[4 * i + 1] = v[1];
      w[4 * i + 2] = v[2];
      w[4 * i + 3] = v[3];
    }
  }
#pragma unroll 1
  for (int f = 0; f < F; f++) {
#pragma unroll
    for (int i = 0; i < K; i++) w[i] = __builtin_amdgcn_alignbit(w[i], w[(i + 1) & (K - 1)], 7) ^ w[i];
  }
  if constexpr (MAP == 0) {
#pragma unroll
    for (int i = 0; i < K; i++) __builtin_amdgcn_raw_buffer_store_b32(w[i], rout, lane * 4u, i * g.out_shard, POL);
  } else if constexpr (MAP == 1) {
    const uint32_t s = lane >> 5, o = (lane & 31u) * 8u;
#pragma unroll
    for (int i = 0; i < K / 2; i++) {
      u2 v = {w[2 * i], w[2 * i + 1]};
      __builtin_amdgcn_raw_buffer_store_b64(v, rout, s * g.out_shard + o, 2 * i * g.out_shard, 2);
    }
  } else {
    const uint32_t s = lane >> 4, o = (lane & 15u) * 16u;
#pragma unroll
    for (int i = 0; i < K / 4; i++) {
      u4 v = {w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]};
      __builtin_amdgcn_raw_buffer_store_b128(v, rout, s * g.out_shard + o, 4 * i * g.out_shard, 2);
    }
  }
}

// rows then columns of C squares at a time (the Infinity-Cache schedule: a chunk's [Q0|Q1]
// is re-read by its column pass while it may still sit in the 256 MB MALL)
template <int POL>
static float run_chunked(Geo rows, Geo cols, uint32_t C, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto once = [&]() {
    for (uint32_t z = 0; z < rows.nsq; z += C) {
      Geo r = rows, c = cols;
      r.in += z * rows.sq; r.out += z * rows.sq; r.nsq = C;
      c.in += z * cols.sq; c.out += z * cols.sq; c.nsq = C;
      hipLaunchKernelGGL((k_mem<0, 0, POL>), dim3((r.axes * 2u * C + 3) / 4), dim3(256), 0, 0, r);
      hipLaunchKernelGGL((k_mem<0, 0, POL>), dim3((c.axes * 2u * C + 3) / 4), dim3(256), 0, 0, c);
    }
  };
  once();
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; i++) once();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

template <int MAP, int F>
static float run(Geo g, int reps) {
  const uint32_t tiles = g.axes * 2u * g.nsq;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL((k_mem<MAP, F>), dim3((tiles + 3) / 4), dim3(256), 0, 0, g);
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; i++) hipLaunchKernelGGL((k_mem<MAP, F>), dim3((tiles + 3) / 4), dim3(256), 0, 0, g);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main() {
  const uint32_t k = 128, W = 2 * k, B = 64;
  const uint64_t sq = (uint64_t)W * W * 512;
  uint8_t* eds;
  CK(hipMalloc(&eds, sq * B));
  CK(hipMemset(eds, 1, sq * B));
  // row pass: axis = row r < k: in = cells (r, 0..k-1), out = (r, k..2k-1)
  Geo rows{eds, eds + (uint64_t)k * 512, 512, 512, (uint64_t)W * 512, (uint64_t)W * 512, sq, k, B};
  // column pass: axis = column c < 2k: in = cells (0..k-1, c), out = (k..2k-1, c)
  Geo cols{eds, eds + (uint64_t)k * W * 512, W * 512, W * 512, 512, 512, sq, W, B};
  const double rb = 2.0 * k * k * 512 * B, cb = 2.0 * 2 * k * k * 512 * B;  // bytes moved per launch
  auto rep = [&](const char* name, float ms, double bytes) {
    printf("%-28s %8.1f us  %6.2f TB/s\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e12);
  };
  rep("rows map0 (b32, kernel)", run<0, 0>(rows, 10), rb);
  rep("rows map1 (b64)", run<1, 0>(rows, 10), rb);
  rep("rows map2 (b128)", run<2, 0>(rows, 10), rb);
  rep("cols map0 (b32, kernel)", run<0, 0>(cols, 10), cb);
  rep("cols map1 (b64)", run<1, 0>(cols, 10), cb);
  rep("cols map2 (b128)", run<2, 0>(cols, 10), cb);
  rep("rows map0 F=8", run<0, 8>(rows, 10), rb);
  rep("rows map2 F=8", run<2, 8>(rows, 10), rb);
  rep("cols map0 F=8", run<0, 8>(cols, 10), cb);
  rep("cols map2 F=8", run<2, 8>(cols, 10), cb);
  for (uint32_t C : {64u, 16u, 8u, 4u, 2u}) {
    char n1[64], n2[64];
    snprintf(n1, sizeof n1, "pair chunk %u nt", C);
    snprintf(n2, sizeof n2, "pair chunk %u default", C);
    rep(n1, run_chunked<2>(rows, cols, C, 5), rb + cb);
    rep(n2, run_chunked<0>(rows, cols, C, 5), rb + cb);
  }
  CK(hipFree(eds));
  return 0;
}
