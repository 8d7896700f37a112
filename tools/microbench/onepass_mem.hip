// Memory-side probe of a ONE-PASS GF(2^8) extension data flow (VERDICT r3 ask 1), against
// the shipped two-pass flow's memory shape, with no transform in either (what the data flow
// alone costs; the transform is the same arithmetic in both).
//
// Two-pass (shipped, rs_axis.hip): rows pass reads Q0 and writes Q1, columns pass reads
// [Q0|Q1] again and writes [Q2|Q3]: 1.5x the algorithmic 2048 k^2 bytes per square.
//
// One-pass: a workgroup owns an S-byte slice of EVERY cell of one square. It loads the Q0
// slice (k^2 x S bytes) into LDS once, and writes the Q1, Q2, Q3 slices from there (the
// row transform, the column transform and the Q2-row transform would run on that image):
// 1.0x traffic. The slice must fit the 160 KiB LDS: k^2 S <= 160 KiB, so S = 8 at k = 128
// (128 KiB, one workgroup per CU) and S = 32 at k = 64. Every access moves S bytes per cell
// (cells are 512 B apart), so the L2 sees one request per S bytes instead of per 64-128 B;
// the 512/S workgroups of a square read the same lines. Placements:
//   xcd: the slices of a square are dealt to one XCD (blockIdx b -> XCD b % 8 under the
//        observed round-robin dispatch, MI355X_MICROARCH.md), so the 16 (S = 8) workgroups
//        sharing a 128-byte line run on one L2 at about the same time
//   rr : plain blockIdx order (a square's slices spread over the 8 XCDs)
// Build: hipcc --offload-arch=gfx950 -O3 -o onepass_mem onepass_mem.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

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

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}

// ---------------------------------------------------------------- two-pass (shipped shape)
// one wave per (square, axis, 256-byte slice): 128 data shards in (dword per lane), 128
// parity shards out; rows: shards 512 B apart, columns: a row pitch (128 KiB) apart
struct Geo {
  uint8_t* eds;
  uint32_t in_shard;
  uint64_t in_axis, out_off, sq;
  uint32_t axes, nsq;
};

template <int K>
__global__ __launch_bounds__(256, 3) void k_two(Geo g) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t tile = blockIdx.x * 4u + (threadIdx.x >> 6);
  if (tile >= g.axes * 2u * g.nsq) return;
  const uint32_t sl = tile % 2u, r = tile / 2u, x = r % g.axes, z = r / g.axes;
  const auto rin = rsrc(g.eds + z * g.sq + x * g.in_axis + sl * 256u);
  const auto rout = rsrc(g.eds + z * g.sq + x * g.in_axis + g.out_off + sl * 256u);
  uint32_t w[K];
#pragma unroll
  for (int i = 0; i < K; i++) w[i] = __builtin_amdgcn_raw_buffer_load_b32(rin, lane * 4u, i * g.in_shard, 2);
#pragma unroll
  for (int i = 0; i < K; i++) __builtin_amdgcn_raw_buffer_store_b32(w[i] ^ (uint32_t)i, rout, lane * 4u, i * g.in_shard, 2);
}

// ---------------------------------------------------------------- one-pass
template <int S>
__device__ __forceinline__ void ld(const __amdgpu_buffer_rsrc_t& r, uint32_t off, uint32_t (&v)[S / 4], int pol) {
  if constexpr (S == 4) {
    v[0] = pol ? __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 2) : __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
  } else if constexpr (S == 8) {
    const u2 x = pol ? __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 2) : __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
    v[0] = x[0]; v[1] = x[1];
  } else {
#pragma unroll
    for (int q = 0; q < S / 16; q++) {
      const u4 x = pol ? __builtin_amdgcn_raw_buffer_load_b128(r, off + 16 * q, 0, 2)
                       : __builtin_amdgcn_raw_buffer_load_b128(r, off + 16 * q, 0, 0);
      v[4 * q] = x[0]; v[4 * q + 1] = x[1]; v[4 * q + 2] = x[2]; v[4 * q + 3] = x[3];
    }
  }
}
template <int S>
__device__ __forceinline__ void st(const __amdgpu_buffer_rsrc_t& r, uint32_t off, const uint32_t (&v)[S / 4], int pol) {
  if constexpr (S == 4) {
    if (pol) __builtin_amdgcn_raw_buffer_store_b32(v[0], r, off, 0, 2);
    else __builtin_amdgcn_raw_buffer_store_b32(v[0], r, off, 0, 0);
  } else if constexpr (S == 8) {
    const u2 x = {v[0], v[1]};
    if (pol) __builtin_amdgcn_raw_buffer_store_b64(x, r, off, 0, 2);
    else __builtin_amdgcn_raw_buffer_store_b64(x, r, off, 0, 0);
  } else {
#pragma unroll
    for (int q = 0; q < S / 16; q++) {
      const u4 x = {v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
      if (pol) __builtin_amdgcn_raw_buffer_store_b128(x, r, off + 16 * q, 0, 2);
      else __builtin_amdgcn_raw_buffer_store_b128(x, r, off + 16 * q, 0, 0);
    }
  }
}

// grid: nsq * (512 / S) workgroups of 256 threads, one (square, slice) each
template <int K, int S>
__global__ __launch_bounds__(256, 1) void k_one(uint8_t* eds, uint64_t sq, uint32_t nsq, int xcd, int pol) {
  constexpr uint32_t W = 2 * K, NS = 512 / S, DW = S / 4;
  __shared__ uint32_t img[K * K * DW];  // the Q0 slice, cell-major
  uint32_t b = blockIdx.x;
  if (xcd) b = (b % 8u) * (gridDim.x / 8u) + b / 8u;  // consecutive slices on one XCD
  const uint32_t z = b / NS, s = b % NS;
  if (z >= nsq) return;
  const auto r = rsrc(eds + z * sq + s * S);
  const uint32_t row = W * 512u;
  for (uint32_t cell = threadIdx.x; cell < K * K; cell += 256u) {
    const uint32_t rr = cell / K, cc = cell % K;
    uint32_t v[DW];
    ld<S>(r, rr * row + cc * 512u, v, pol);
#pragma unroll
    for (int q = 0; q < (int)DW; q++) img[cell * DW + q] = v[q];
  }
  __syncthreads();
  for (uint32_t cell = threadIdx.x; cell < K * K; cell += 256u) {
    const uint32_t rr = cell / K, cc = cell % K;
    uint32_t a[DW], t[DW], c3[DW];
#pragma unroll
    for (int q = 0; q < (int)DW; q++) {
      a[q] = img[cell * DW + q] ^ 1u;               // Q1 (r, k + c): the row transform's output
      t[q] = img[cell * DW + q] ^ 2u;               // Q2 (k + r, c): the column transform's
      c3[q] = img[cell * DW + q] ^ 3u;              // Q3 (k + r, k + c)
    }
    st<S>(r, rr * row + (K + cc) * 512u, a, pol);
    st<S>(r, (K + rr) * row + cc * 512u, t, pol);
    st<S>(r, (K + rr) * row + (K + cc) * 512u, c3, pol);
  }
}

static hipEvent_t ev0, ev1;

template <typename F>
static float timeit(F f, int reps) {
  f();
  CK(hipEventRecord(ev0));
  for (int i = 0; i < reps; i++) f();
  CK(hipEventRecord(ev1));
  CK(hipEventSynchronize(ev1));
  float ms;
  CK(hipEventElapsedTime(&ms, ev0, ev1));
  return ms / reps;
}

// usage: onepass_mem [only]   (only: run the lines whose name contains this substring,
// e.g. "two-pass" or "S=8 xcd default", for one PMC pass per data flow)
int main(int argc, char** argv) {
  const char* only = argc > 1 ? argv[1] : nullptr;
  CK(hipEventCreate(&ev0));
  CK(hipEventCreate(&ev1));
  const uint32_t B = 64;
  for (uint32_t k : {128u, 64u}) {
    const uint32_t W = 2 * k;
    const uint64_t sq = (uint64_t)W * W * 512;
    const uint32_t nsq = k == 128 ? B : 4 * B;
    uint8_t* eds;
    CK(hipMalloc(&eds, sq * nsq));
    CK(hipMemset(eds, 1, sq * nsq));
    const double alg = 2048.0 * k * k * nsq;
    auto want = [&](const char* name) { return !only || strstr(name, only) != nullptr; };
    auto rep = [&](const char* name, float ms) {
      printf("k=%3u %-40s %9.1f us  %6.2f us/square  %5.2f TB/s algorithmic (frac %.3f of 8 TB/s)\n", k, name,
             ms * 1e3, ms * 1e3 / nsq, alg / (ms * 1e-3) / 1e12, alg / (ms * 1e-3) / 8e12);
    };
    auto go = [&](const char* name, auto f, int reps) {
      if (want(name)) rep(name, timeit(f, reps));
    };
    Geo rows{eds, 512, (uint64_t)W * 512, (uint64_t)k * 512, sq, k, nsq};
    Geo cols{eds, W * 512, 512, (uint64_t)k * W * 512, sq, W, nsq};
    go("two-pass rows + cols (dword, nt)", [&] {
          if (k == 128) {
            hipLaunchKernelGGL(k_two<128>, dim3((rows.axes * 2 * nsq + 3) / 4), dim3(256), 0, 0, rows);
            hipLaunchKernelGGL(k_two<128>, dim3((cols.axes * 2 * nsq + 3) / 4), dim3(256), 0, 0, cols);
          } else {
            hipLaunchKernelGGL(k_two<64>, dim3((rows.axes * 2 * nsq + 3) / 4), dim3(256), 0, 0, rows);
            hipLaunchKernelGGL(k_two<64>, dim3((cols.axes * 2 * nsq + 3) / 4), dim3(256), 0, 0, cols);
          }
        }, 10);
    if (k == 128) {
      for (int pol = 0; pol < 2; pol++)
        for (int xcd = 1; xcd >= 0; xcd--) {
          char n[64];
          snprintf(n, sizeof n, "one-pass S=8 %s %s", xcd ? "xcd" : "rr", pol ? "nt" : "default");
          go(n, [&] { hipLaunchKernelGGL((k_one<128, 8>), dim3(nsq * 64), dim3(256), 0, 0, eds, sq, nsq, xcd, pol); }, 5);
        }
      go("one-pass S=4 xcd default", [&] { hipLaunchKernelGGL((k_one<128, 4>), dim3(nsq * 128), dim3(256), 0, 0, eds, sq, nsq, 1, 0); }, 5);
    } else {
      for (int xcd = 1; xcd >= 0; xcd--) {
        char n[64];
        snprintf(n, sizeof n, "one-pass S=32 %s default", xcd ? "xcd" : "rr");
        go(n, [&] { hipLaunchKernelGGL((k_one<64, 32>), dim3(nsq * 16), dim3(256), 0, 0, eds, sq, nsq, xcd, 0); }, 5);
      }
      go("one-pass S=16 xcd default", [&] { hipLaunchKernelGGL((k_one<64, 16>), dim3(nsq * 32), dim3(256), 0, 0, eds, sq, nsq, 1, 0); }, 5);
    }
    CK(hipFree(eds));
  }
  return 0;
}
