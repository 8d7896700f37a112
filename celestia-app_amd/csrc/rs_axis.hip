// Leopard GF(2^8) encode, one wave per axis slice (32 <= k <= 128).
//
// The transform of SURVEY.md Appendix A.2 in radix-2 form (see the header of
// rs_kernels.hip), laid out so that nothing is shared between waves:
//   - a wave owns one tile = (square, axis, 256-byte slice); lane l holds dword l of
//     the slice of every one of the K data shards of the axis in VGPRs (K <= 128);
//   - every radix-2 layer is lane-local, so there is no LDS image and no barrier: the
//     waves of a CU drift apart and one wave's loads and stores run under the
//     butterflies of the others;
//   - the skew index of every butterfly is a compile-time constant, so the v_perm
//     product tables are immediates (no table loads), "multiply by zero" butterflies
//     (skew == 255) lose their multiply and "multiply by one" becomes an xor.
// Multiply: the byte splits into 3+3+2 bits, each looked up with one v_perm_b32 in
// an 8/8/4-entry product table (as rs_kernels.hip gf8_mul4).
#include <hip/hip_runtime.h>

#include "cel_internal.hpp"
#include "bitslice8.hpp"
#include "gf8_constexpr.hpp"
#include "gf8_regs.hpp"

namespace cel {
namespace ax {

using cx::add_mod8;
using cx::kGf8;
using cx::sfor;
using bs::pxor;
using bs::tr8;
using bs::xrow;

// Leopard IFFT over the data coset (offset K) then FFT over the parity coset (offset 0),
// radix 2, all K shards in w[]. Skew index: IFFT K-1 + base + D, FFT base + D - 1.
// The last IFFT layer and the first FFT layer act on the same pairs (a, a + K/2):
//   y ^= x; x ^= c1*y;  then  x ^= c2*y; y ^= x   ==   y ^= x; x ^= (c1 + c2)*y; y ^= x
// so they run as one layer with one multiply by c1 + c2 (K/2 of the K log K
// butterflies lose a multiply).
constexpr uint32_t merged_lm(uint32_t s1, uint32_t s2) {
  const uint32_t c = (s1 == 255u ? 0u : (uint32_t)kGf8.exp[s1]) ^ (s2 == 255u ? 0u : (uint32_t)kGf8.exp[s2]);
  return c == 0u ? 255u : (uint32_t)kGf8.log[c];
}

// ---------------------------------------------------------------- hybrid transform
//
// Layers with D >= 8 have the same twiddle for all 8 shards of an aligned block
// {8m .. 8m+7} (the skew index depends on base = a & ~(2D-1) only), so there the block
// is bit-sliced in place: an 8x8 bit transpose in each byte lane of w[8m .. 8m+7] turns
// "4 bytes of 8 shards" into 8 bit-planes, and a butterfly between blocks m and m+D/8 is
// an 8x8 GF(2) matrix network of v_bitop3 xor3 ops (~2 per plane) instead of the v_perm
// multiply (~10 VALU per dword). Layers D = 1, 2, 4 (twiddles differ inside a block) keep
// the v_perm multiply. For K = 128: 6 v_perm layers, 7 bit-sliced layers, 32 transposes.

// Scheduling fence after every v_perm butterfly (a fence every 2 or 4 butterflies, or
// none, measured within noise: profiles/r3_gf8_fence_ab.txt).
__device__ __forceinline__ void vperm_fence() { __builtin_amdgcn_sched_barrier(0); }

template <int K>
__device__ __forceinline__ void transform_hyb(uint32_t (&w)[K]) {
  constexpr int LOGK = __builtin_ctz(K);
  static_assert(K >= 32, "hybrid transform needs bit-sliced layers");
  const uint32_t m7 = sconst<0x07070707u>(), m3 = sconst<0x03030303u>();
  // IFFT D = 1, 2, 4: v_perm multiply
  sfor<3>([&](auto lg) {
    constexpr int D = 1 << decltype(lg)::value;
    sfor<K / (2 * D)>([&](auto bi) {
      constexpr int base = decltype(bi)::value * 2 * D;
      const Mul<kGf8.skew[K - 1 + base + D]> m;
      sfor<D>([&](auto j) {
        constexpr int a = base + decltype(j)::value;
        pin(w[a], w[a + D]);
        w[a + D] ^= w[a];
        m.muladd(w[a], w[a + D], m7, m3);
        pin(w[a], w[a + D]);
        vperm_fence();
      });
    });
  });
  sfor<K / 8>([&](auto s) {
    tr8<8 * decltype(s)::value>(w);
    __builtin_amdgcn_sched_barrier(0);
  });
  // IFFT D = 8 .. K/4, bit-sliced (block pairs)
  sfor<LOGK - 4>([&](auto t) {
    constexpr int D = 8 << decltype(t)::value;
    sfor<K / (2 * D)>([&](auto bi) {
      constexpr int base = decltype(bi)::value * 2 * D;
      sfor<D / 8>([&](auto j) {
        constexpr int a = base + 8 * decltype(j)::value;
        pxor<a, a + D>(w);
        pmuladd<kGf8.skew[K - 1 + base + D], a, a + D>(w);
        __builtin_amdgcn_sched_barrier(0);
      });
    });
  });
  {  // last IFFT layer + first FFT layer, merged (see transform)
    constexpr int D = K / 2;
    sfor<D / 8>([&](auto j) {
      constexpr int a = 8 * decltype(j)::value;
      pxor<a, a + D>(w);
      pmuladd<merged_lm(kGf8.skew[K - 1 + D], kGf8.skew[D - 1]), a, a + D>(w);
      pxor<a, a + D>(w);
      __builtin_amdgcn_sched_barrier(0);
    });
  }
  // FFT D = K/4 .. 8, bit-sliced
  sfor<LOGK - 4>([&](auto t) {
    constexpr int D = K >> (decltype(t)::value + 2);
    sfor<K / (2 * D)>([&](auto bi) {
      constexpr int base = decltype(bi)::value * 2 * D;
      sfor<D / 8>([&](auto j) {
        constexpr int a = base + 8 * decltype(j)::value;
        pmuladd<kGf8.skew[base + D - 1], a, a + D>(w);
        pxor<a, a + D>(w);
        __builtin_amdgcn_sched_barrier(0);
      });
    });
  });
  sfor<K / 8>([&](auto s) {
    tr8<8 * decltype(s)::value>(w);
    __builtin_amdgcn_sched_barrier(0);
  });
  // FFT D = 4, 2, 1: v_perm multiply
  sfor<3>([&](auto t) {
    constexpr int D = 4 >> decltype(t)::value;
    sfor<K / (2 * D)>([&](auto bi) {
      constexpr int base = decltype(bi)::value * 2 * D;
      const Mul<kGf8.skew[base + D - 1]> m;
      sfor<D>([&](auto j) {
        constexpr int a = base + decltype(j)::value;
        pin(w[a], w[a + D]);
        m.muladd(w[a], w[a + D], m7, m3);
        w[a + D] ^= w[a];
        pin(w[a], w[a + D]);
        vperm_fence();
      });
    });
  });
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}

// Tile = (square z, axis x, 256-byte slice y): one wave. Loads and stores are nt
// (non-temporal): every byte is touched once per pass and a batch is far larger than the
// Infinity Cache (k=128, 256 squares: 9.35 -> 9.00 us per square against the default
// policy, profiles/r1d_rs_cache_policy_ab.txt).
template <int LOGK>
__global__ __launch_bounds__(256, 3) void k_rs_axis_gf8(RsGeom g, uint32_t nslice) {
  constexpr int K = 1 << LOGK;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t tile = __builtin_amdgcn_readfirstlane(xcd_block(blockIdx.x, gridDim.x) * 4u + (threadIdx.x >> 6));
  if (tile >= g.axes * nslice * g.nsq) return;
  const uint32_t y = tile % nslice, r = tile / nslice;
  const uint32_t x = r % g.axes, z = r / g.axes;
  const uint32_t col = y * 256u + lane * 4u;
  const bool active = col < g.len;
  const uint32_t lo = active ? lane * 4u : 0u;  // inactive lanes load (and never store) dword 0
  uint32_t w[K];
  {
    const auto rin = rsrc(g.in + (uint64_t)z * g.in_sq + (uint64_t)x * g.in_axis + (uint64_t)y * 256u);
    const uint32_t in_shard = (uint32_t)g.in_shard;
#pragma unroll
    for (int i = 0; i < K; i++) w[i] = __builtin_amdgcn_raw_buffer_load_b32(rin, lo, (uint32_t)i * in_shard, 2);
    if (g.dcopy && active) {
      const auto rdc = rsrc(g.dcopy + (uint64_t)z * g.dc_sq + (uint64_t)x * g.dc_axis + (uint64_t)y * 256u);
      const uint32_t dc_shard = (uint32_t)g.dc_shard;
#pragma unroll
      for (int i = 0; i < K; i++) __builtin_amdgcn_raw_buffer_store_b32(w[i], rdc, lo, (uint32_t)i * dc_shard, 2);
    }
  }
  transform_hyb<K>(w);
  if (active) {
    const auto rout = rsrc(g.out + (uint64_t)z * g.out_sq + (uint64_t)x * g.out_axis + (uint64_t)y * 256u);
    const uint32_t out_shard = (uint32_t)g.out_shard;
#pragma unroll
    for (int i = 0; i < K; i++) __builtin_amdgcn_raw_buffer_store_b32(w[i], rout, lo, (uint32_t)i * out_shard, 2);
  }
}

// Two geometries in one launch, tiles interleaved (square z: row tile x, column tile x,
// row tile x + 1, ...): the extension's Q0 rows -> Q1 beside its Q0 columns -> Q2. Both read
// Q0, so with the pairs adjacent in the dispatch order the second read of each Q0 line
// comes from the L2 or the Infinity Cache while the first is recent (default-policy loads
// allocate there), and the square's Q0 crosses HBM once. The Q1 columns -> Q3 follow in a
// second launch (they need every Q1 row). HBM bytes per square: Q0 once, Q1 | Q2 written,
// Q1 read back, Q3 written = 1.25x the algorithmic 2048 k^2 (the rows-then-all-columns
// order re-reads Q0 and Q1: 1.5x).
template <int LOGK>
__global__ __launch_bounds__(256, 3) void k_rs_axis_gf8_pair(RsGeom g1, RsGeom g2, uint32_t nslice) {
  constexpr int K = 1 << LOGK;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t tile = __builtin_amdgcn_readfirstlane(xcd_block(blockIdx.x, gridDim.x) * 4u + (threadIdx.x >> 6));
  const uint32_t per_sq = 2u * g1.axes * nslice;
  if (tile >= per_sq * g1.nsq) return;
  // k = 128: slice-major inside a square, so the 2k tiles of one 256-byte slice run together
  // and the Q0 bytes they share (k^2 x 256 B = 4 MiB, one XCD's L2) stay resident between
  // the row tile's read and the column tile's: Q0 is fetched once (PMC: 1.00x of Q0 against
  // 1.47x with the slices interleaved, profiles/r5_rs_slice_ab.txt). At k <= 64 both slices
  // of a square fit together and the interleaved order measured 2 % faster.
  const uint32_t z = tile / per_sq, r = tile % per_sq, second = r & 1u, rr = r >> 1;
  const uint32_t y = LOGK >= 7 ? rr / g1.axes : rr % nslice, x = LOGK >= 7 ? rr % g1.axes : rr / nslice;
  const RsGeom& g = second ? g2 : g1;
  const uint32_t col = y * 256u + lane * 4u;
  const bool active = col < g.len;
  const uint32_t lo = active ? lane * 4u : 0u;
  uint32_t w[K];
  {
    const auto rin = rsrc(g.in + (uint64_t)z * g.in_sq + (uint64_t)x * g.in_axis + (uint64_t)y * 256u);
    const uint32_t in_shard = (uint32_t)g.in_shard;
#pragma unroll
    for (int i = 0; i < K; i++) w[i] = __builtin_amdgcn_raw_buffer_load_b32(rin, lo, (uint32_t)i * in_shard, 0);
  }
  transform_hyb<K>(w);
  if (active) {
    const auto rout = rsrc(g.out + (uint64_t)z * g.out_sq + (uint64_t)x * g.out_axis + (uint64_t)y * 256u);
    const uint32_t out_shard = (uint32_t)g.out_shard;
#pragma unroll
    for (int i = 0; i < K; i++) __builtin_amdgcn_raw_buffer_store_b32(w[i], rout, lo, (uint32_t)i * out_shard, 2);
  }
}

// Same-run probe of the transform alone (cel_probe_rs_transform): the encode tile's
// instruction stream with its HBM traffic taken away. Every wave loads the same K x 256 B
// (one 32 KiB region, cache-resident) and stores only when `store` is set (never, in the
// probe: the runtime flag keeps the transform live), so the launch time is the VALU time
// of ntiles tiles.
template <int LOGK>
__global__ __launch_bounds__(256, 3) void k_probe_rs_transform(const uint32_t* src, uint32_t* dst, uint32_t ntiles,
                                                               uint32_t store) {
  constexpr int K = 1 << LOGK;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t tile = __builtin_amdgcn_readfirstlane(xcd_block(blockIdx.x, gridDim.x) * 4u + (threadIdx.x >> 6));
  if (tile >= ntiles) return;
  uint32_t w[K];
  const auto rin = rsrc(src);
#pragma unroll
  for (int i = 0; i < K; i++) w[i] = __builtin_amdgcn_raw_buffer_load_b32(rin, lane * 4u, (uint32_t)i * 256u, 0);
  transform_hyb<K>(w);
  if (store) {
    const auto rout = rsrc(dst);
#pragma unroll
    for (int i = 0; i < K; i++) __builtin_amdgcn_raw_buffer_store_b32(w[i], rout, lane * 4u, (uint32_t)i * 256u, 0);
  }
}

template <int LOGK>
hipError_t launch(const RsGeom& g, hipStream_t s) {
  const uint32_t nslice = (g.len + 255) / 256;
  const uint64_t ntiles = (uint64_t)g.axes * nslice * g.nsq;
  if (ntiles == 0) return hipSuccess;
  if (ntiles > 0xFFFFFFF0ull) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_rs_axis_gf8<LOGK>, dim3((unsigned)((ntiles + 3) / 4)), dim3(256), 0, s, g, nslice);
  return hipGetLastError();
}

template <int LOGK>
hipError_t launch_pair(const RsGeom& g1, const RsGeom& g2, hipStream_t s) {
  const uint32_t nslice = (g1.len + 255) / 256;
  const uint64_t ntiles = 2ull * g1.axes * nslice * g1.nsq;
  if (ntiles == 0) return hipSuccess;
  if (ntiles > 0xFFFFFFF0ull) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_rs_axis_gf8_pair<LOGK>, dim3((unsigned)((ntiles + 3) / 4)), dim3(256), 0, s, g1, g2, nslice);
  return hipGetLastError();
}

// Encoding check of listed axes of a resident EDS (rsmt2d verifyEncoding after a solve,
// and the sanity / orthogonal checks): tile = (listed axis a, 256-byte slice y), one wave.
// The data half (cells 0..K-1 of the axis) is encoded in registers as above and compared
// with the parity half (cells K..2K-1) as it is loaded; a mismatch sets flags[axis]. One
// launch in place of gather -> encode -> compare (no dense copy, no parity scratch).
template <int LOGK>
__global__ __launch_bounds__(256, 3) void k_rs_check_axes(const uint8_t* __restrict__ eds, uint32_t W,
                                                          const int32_t* __restrict__ idx, int is_col, uint32_t naxes,
                                                          int32_t* __restrict__ flags) {
  constexpr int K = 1 << LOGK;
  constexpr uint32_t nslice = kShare / 256;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t tile = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
  if (tile >= naxes * nslice) return;
  const uint32_t y = tile % nslice, a = tile / nslice;
  const uint32_t ax = (uint32_t)__builtin_amdgcn_readfirstlane(idx[a]);
  const uint64_t base = is_col ? (uint64_t)ax * kShare : (uint64_t)ax * W * kShare;
  const uint32_t stride = is_col ? W * kShare : kShare;
  const auto rin = rsrc(eds + base + (uint64_t)y * 256u);
  const uint32_t lo = lane * 4u;
  uint32_t w[K];
#pragma unroll
  for (int i = 0; i < K; i++) w[i] = __builtin_amdgcn_raw_buffer_load_b32(rin, lo, (uint32_t)i * stride, 0);
  transform_hyb<K>(w);
  uint32_t diff = 0;
#pragma unroll
  for (int i = 0; i < K; i++) diff |= w[i] ^ __builtin_amdgcn_raw_buffer_load_b32(rin, lo, (uint32_t)(K + i) * stride, 0);
  if (__any(diff != 0u) && lane == 0) atomicOr(flags + ax, 1);
}

}  // namespace ax

// Byte offsets must fit the 32-bit buffer offsets: (n - 1) * shard stride + len < 2 GiB.
static bool geom_ok(const RsGeom& g) {
  const uint64_t span = (uint64_t)g.n * (g.in_shard > g.out_shard ? g.in_shard : g.out_shard) + g.len;
  return span < 0x7fffffffull && !(g.dcopy && (uint64_t)g.n * g.dc_shard + g.len >= 0x7fffffffull);
}

hipError_t launch_rs_encode_axis(const RsGeom& g, hipStream_t s) {
  if (!geom_ok(g) || g.len == 0) return hipErrorInvalidValue;
  switch (g.n) {
    case 32: return ax::launch<5>(g, s);
    case 64: return ax::launch<6>(g, s);
    case 128: return ax::launch<7>(g, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_rs_encode_axis_pair(const RsGeom& g1, const RsGeom& g2, hipStream_t s) {
  if (!geom_ok(g1) || !geom_ok(g2) || g1.len == 0 || g1.dcopy || g2.dcopy || g1.n != g2.n || g1.len != g2.len ||
      g1.axes != g2.axes || g1.nsq != g2.nsq)
    return hipErrorInvalidValue;
  switch (g1.n) {
    case 32: return ax::launch_pair<5>(g1, g2, s);
    case 64: return ax::launch_pair<6>(g1, g2, s);
    case 128: return ax::launch_pair<7>(g1, g2, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_probe_rs_transform(uint32_t k, const uint32_t* src, uint32_t* dst, uint32_t ntiles, uint32_t store,
                                     hipStream_t s) {
  if (ntiles == 0) return hipSuccess;
  const dim3 grid((ntiles + 3) / 4);
  switch (k) {
    case 32: hipLaunchKernelGGL(ax::k_probe_rs_transform<5>, grid, dim3(256), 0, s, src, dst, ntiles, store); break;
    case 64: hipLaunchKernelGGL(ax::k_probe_rs_transform<6>, grid, dim3(256), 0, s, src, dst, ntiles, store); break;
    case 128: hipLaunchKernelGGL(ax::k_probe_rs_transform<7>, grid, dim3(256), 0, s, src, dst, ntiles, store); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_rs_check_axes(const uint8_t* eds, uint32_t k, const int32_t* idx, int is_col, uint32_t naxes,
                                int32_t* flags, hipStream_t s) {
  const uint32_t W = 2 * k;
  if ((uint64_t)(W - 1) * W * kShare + kShare >= 0x7fffffffull) return hipErrorInvalidValue;
  if (naxes == 0) return hipSuccess;
  const dim3 grid((naxes * (kShare / 256) + 3) / 4);
  switch (k) {
    case 32: hipLaunchKernelGGL(ax::k_rs_check_axes<5>, grid, dim3(256), 0, s, eds, W, idx, is_col, naxes, flags); break;
    case 64: hipLaunchKernelGGL(ax::k_rs_check_axes<6>, grid, dim3(256), 0, s, eds, W, idx, is_col, naxes, flags); break;
    case 128: hipLaunchKernelGGL(ax::k_rs_check_axes<7>, grid, dim3(256), 0, s, eds, W, idx, is_col, naxes, flags); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace cel
