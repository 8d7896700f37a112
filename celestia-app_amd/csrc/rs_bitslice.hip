// Bit-sliced Leopard GF(2^8) encode for gfx950 (k <= 128, the square widths of
// celestia-app: pkg/appconsts/v1/app_consts.go:5 SquareSizeUpperBound).
//
// Same transform as rs_kernels.hip (SURVEY.md Appendix A.2 in radix-2 form), but
// each lane holds 32-byte granules of its shards as 8 bit-planes (plane b = bit b of
// 32 bytes). A multiply by a twiddle c is then an 8x8 GF(2) matrix: every output plane
// is the xor of the input planes selected by one row of the matrix. The twiddles of
// every butterfly are compile-time constants here (constexpr Leopard tables), so each
// matrix becomes a straight-line network of v_bitop3 (3-input xor) ops: ~0.75 VALU op
// per byte-butterfly instead of ~3.4 for the v_perm table multiply, with every op at
// the VOP2/bitop3 rate (tools/microbench: bitop3 ~53 T, v_perm ~35 T lane-ops/s).
//
// Work layout for K = 2^LOGK shards per axis (K <= 128):
//   S = min(K, 16) shards per lane (16 x 8 planes = 128 VGPRs), G = K / S groups.
//   A workgroup = G waves; lane = one 32-byte granule column (64 per wave, spread over
//   axes x granules); wave g holds shards [16g, 16g+16) ("A"). Radix-2 layers with
//   D < 16 are lane-local and their twiddles depend on g only: each wave runs a code
//   variant specialised for its g (-6 % measured for 8 variants per workgroup).
//   Layers with D >= 16 run after an LDS exchange in arrangement "B": every lane holds
//   shards {l + 16h : h < G} for L = 16/G values of l, whose twiddles depend on h only.
//   The exchange moves two planes per round through a 64 KiB LDS image.
#include <hip/hip_runtime.h>

#include <utility>

#include "cel_internal.hpp"
#include "gf8_constexpr.hpp"

namespace cel {
namespace bs {

using cx::add_mod8;
using cx::kGf8;
using cx::mul_row;
using cx::sfor;

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// acc ^= xor of y[j] for every set bit j of ROW (two inputs per v_bitop3).
template <uint32_t ROW, int J = 0>
__device__ __forceinline__ void xor_row(uint32_t& acc, const uint32_t (&y)[8]) {
  if constexpr (J < 8) {
    if constexpr ((ROW >> J) & 1u) {
      constexpr uint32_t rest = ROW >> (J + 1);
      if constexpr (rest != 0) {
        constexpr int J2 = J + 1 + __builtin_ctz(rest);
        acc = xor3(acc, y[J], y[J2]);
        xor_row<ROW, J2 + 1>(acc, y);
      } else {
        acc ^= y[J];
      }
    } else {
      xor_row<ROW, J + 1>(acc, y);
    }
  }
}

// x ^= exp(LM) * y   (bit-sliced), LM == 255 means the zero twiddle (no-op).
template <uint32_t LM>
__device__ __forceinline__ void muladd(uint32_t (&x)[8], const uint32_t (&y)[8]) {
  if constexpr (LM != 255u) {
    sfor<8>([&](auto i) { xor_row<mul_row(LM, decltype(i)::value)>(x[decltype(i)::value], y); });
  }
}

template <int IDX>
__device__ __forceinline__ void ifft2(uint32_t (&x)[8], uint32_t (&y)[8]) {
#pragma unroll
  for (int b = 0; b < 8; b++) y[b] ^= x[b];
  muladd<kGf8.skew[IDX]>(x, y);
}

template <int IDX>
__device__ __forceinline__ void fft2(uint32_t (&x)[8], uint32_t (&y)[8]) {
  muladd<kGf8.skew[IDX]>(x, y);
#pragma unroll
  for (int b = 0; b < 8; b++) y[b] ^= x[b];
}

// 8x8 bit transpose in each byte lane of 8 dwords (an involution): planes <-> bytes.
__device__ __forceinline__ void swap_bits(uint32_t& a, uint32_t& b, int s, uint32_t m) {
  const uint32_t t = ((a >> s) ^ b) & m;
  b ^= t;
  a ^= t << s;
}
__device__ __forceinline__ void transpose8(uint32_t (&d)[8]) {
#pragma unroll
  for (int j = 0; j < 4; j++) swap_bits(d[j], d[j + 4], 4, 0x0F0F0F0Fu);
#pragma unroll
  for (int j = 0; j < 8; j += 4) {
    swap_bits(d[j], d[j + 2], 2, 0x33333333u);
    swap_bits(d[j + 1], d[j + 3], 2, 0x33333333u);
  }
#pragma unroll
  for (int j = 0; j < 8; j += 2) swap_bits(d[j], d[j + 1], 1, 0x55555555u);
}

// ------------------------------------------------------------- layer drivers

// Arrangement A, group GI: lane holds shards [S*GI, S*GI + S) in w[0..S).
template <int K, int S, int GI>
__device__ __forceinline__ void ifft_a(uint32_t (&w)[S][8]) {
  sfor<(S > 1 ? __builtin_ctz(S) : 0)>([&](auto lg) {
    constexpr int D = 1 << decltype(lg)::value;
    sfor<S / (2 * D)>([&](auto bi) {
      constexpr int base = decltype(bi)::value * 2 * D;
      sfor<D>([&](auto j) {
        constexpr int a = base + decltype(j)::value;
        ifft2<K - 1 + S * GI + base + D>(w[a], w[a + D]);
      });
      __builtin_amdgcn_sched_barrier(0);
    });
  });
}

template <int K, int S, int GI>
__device__ __forceinline__ void fft_a(uint32_t (&w)[S][8]) {
  constexpr int LOGS = S > 1 ? __builtin_ctz(S) : 0;
  sfor<LOGS>([&](auto t) {
    constexpr int D = 1 << (LOGS - 1 - decltype(t)::value);
    sfor<S / (2 * D)>([&](auto bi) {
      constexpr int base = decltype(bi)::value * 2 * D;
      sfor<D>([&](auto j) {
        constexpr int a = base + decltype(j)::value;
        fft2<S * GI + base + D - 1>(w[a], w[a + D]);
      });
      __builtin_amdgcn_sched_barrier(0);
    });
  });
}

// Arrangement B: w[h * L + lo] = shard lo_abs + S*h. Layers D = S << t.
template <int K, int S, int G>
__device__ __forceinline__ void ifft_fft_b(uint32_t (&w)[S][8]) {
  constexpr int L = S / G;
  constexpr int LOGG = __builtin_ctz(G);
  sfor<LOGG>([&](auto t) {  // IFFT: dh = 1, 2, ..
    constexpr int dh = 1 << decltype(t)::value;
    sfor<G / (2 * dh)>([&](auto hbi) {
      constexpr int hb = decltype(hbi)::value * 2 * dh;
      sfor<dh>([&](auto hj) {
        constexpr int h = hb + decltype(hj)::value;
        sfor<L>([&](auto lo) {
          ifft2<K - 1 + S * hb + S * dh>(w[h * L + decltype(lo)::value], w[(h + dh) * L + decltype(lo)::value]);
        });
        __builtin_amdgcn_sched_barrier(0);
      });
    });
  });
  sfor<LOGG>([&](auto t) {  // FFT: dh = G/2, .., 1
    constexpr int dh = G >> (decltype(t)::value + 1);
    sfor<G / (2 * dh)>([&](auto hbi) {
      constexpr int hb = decltype(hbi)::value * 2 * dh;
      sfor<dh>([&](auto hj) {
        constexpr int h = hb + decltype(hj)::value;
        sfor<L>([&](auto lo) {
          fft2<S * hb + S * dh - 1>(w[h * L + decltype(lo)::value], w[(h + dh) * L + decltype(lo)::value]);
        });
        __builtin_amdgcn_sched_barrier(0);
      });
    });
  });
}

// LDS exchange between arrangements (two planes per round, 64 KiB image [shard][lane][2]).
template <int S, int G, bool TO_B>
__device__ __forceinline__ void exchange(uint32_t (&w)[S][8], uint2* lds, int g, int lane) {
  constexpr int L = S / G;
  __builtin_amdgcn_sched_barrier(0);
  sfor<4>([&](auto rr) {
    constexpr int r = decltype(rr)::value;
    sfor<S>([&](auto ii) {
      constexpr int i = decltype(ii)::value;
      // shard held in local slot i before the exchange
      const int shard = TO_B ? (S * g + i) : (g * L + (i % L) + S * (i / L));
      lds[shard * 64 + lane] = make_uint2(w[i][2 * r], w[i][2 * r + 1]);
    });
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
    __builtin_amdgcn_sched_barrier(0);
    sfor<S>([&](auto ii) {
      constexpr int i = decltype(ii)::value;
      const int shard = TO_B ? (g * L + (i % L) + S * (i / L)) : (S * g + i);
      const uint2 v = lds[shard * 64 + lane];
      w[i][2 * r] = v.x;
      w[i][2 * r + 1] = v.y;
    });
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
    __builtin_amdgcn_sched_barrier(0);
  });
}

}  // namespace bs

// The whole per-lane program for group GI: load, transpose, A-IFFT (variant GI),
// exchange, B layers, exchange, A-FFT (variant GI), transpose, store. Each group's
// program is a separate straight-line body selected once per wave, so no register
// state crosses a variant branch (a shared body with an inner switch spilled).
typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));

// Buffer resource over [base, base + 2 GiB): a scalar base, a 32-bit per-lane offset and
// a scalar per-shard offset, so the 16 shard streams of a lane cost one address VGPR.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}

template <int K, int S, int G, int GI>
__device__ __forceinline__ void encode_lane(const RsGeom& g, uint2* lds, int lane, bool active, uint32_t axis,
                                            uint32_t gofs) {
  const __amdgpu_buffer_rsrc_t rin = rsrc(g.in + (uint64_t)blockIdx.y * g.in_sq);
  const __amdgpu_buffer_rsrc_t rout = rsrc(g.out + (uint64_t)blockIdx.y * g.out_sq);
  const uint32_t vin = axis * (uint32_t)g.in_axis + gofs;
  const uint32_t vout = axis * (uint32_t)g.out_axis + gofs;
  uint32_t w[S][8];
#pragma unroll
  for (int i = 0; i < S; i++) {
    if (active) {
      const uint32_t so = (uint32_t)((GI * S + i) * g.in_shard);
      const v4u32 a = __builtin_amdgcn_raw_buffer_load_b128(rin, vin, so, 0);
      const v4u32 b = __builtin_amdgcn_raw_buffer_load_b128(rin, vin + 16, so, 0);
      w[i][0] = a.x; w[i][1] = a.y; w[i][2] = a.z; w[i][3] = a.w;
      w[i][4] = b.x; w[i][5] = b.y; w[i][6] = b.z; w[i][7] = b.w;
    } else {
#pragma unroll
      for (int b = 0; b < 8; b++) w[i][b] = 0;
    }
  }
  if (g.dcopy && active) {
    const __amdgpu_buffer_rsrc_t rdc = rsrc(g.dcopy + (uint64_t)blockIdx.y * g.dc_sq);
    const uint32_t vdc = axis * (uint32_t)g.dc_axis + gofs;
#pragma unroll
    for (int i = 0; i < S; i++) {
      const uint32_t so = (uint32_t)((GI * S + i) * g.dc_shard);
      __builtin_amdgcn_raw_buffer_store_b128(v4u32{w[i][0], w[i][1], w[i][2], w[i][3]}, rdc, vdc, so, 0);
      __builtin_amdgcn_raw_buffer_store_b128(v4u32{w[i][4], w[i][5], w[i][6], w[i][7]}, rdc, vdc + 16, so, 0);
    }
  }
#pragma unroll
  for (int i = 0; i < S; i++) {
    bs::transpose8(w[i]);
    __builtin_amdgcn_sched_barrier(0);
  }
  bs::ifft_a<K, S, GI>(w);
  if constexpr (G > 1) {
    bs::exchange<S, G, true>(w, lds, GI, lane);
    bs::ifft_fft_b<K, S, G>(w);
    bs::exchange<S, G, false>(w, lds, GI, lane);
  }
  bs::fft_a<K, S, GI>(w);
#pragma unroll
  for (int i = 0; i < S; i++) {
    bs::transpose8(w[i]);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (active) {
#pragma unroll
    for (int i = 0; i < S; i++) {
      const uint32_t so = (uint32_t)((GI * S + i) * g.out_shard);
      __builtin_amdgcn_raw_buffer_store_b128(v4u32{w[i][0], w[i][1], w[i][2], w[i][3]}, rout, vout, so, 0);
      __builtin_amdgcn_raw_buffer_store_b128(v4u32{w[i][4], w[i][5], w[i][6], w[i][7]}, rout, vout + 16, so, 0);
    }
  }
}

// grid: x = block of 64 granule columns (axes x granules-per-shard), y = square.
template <int LOGK>
__global__ __launch_bounds__(64 * ((LOGK > 4) ? (1 << (LOGK - 4)) : 1)) void k_rs_encode_bs(RsGeom g) {
  constexpr int K = 1 << LOGK;
  constexpr int S = K < 16 ? K : 16;
  constexpr int G = K / S;
  __shared__ uint2 lds[G > 1 ? K * 64 : 1];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t U = g.len / 32;  // granules per shard
  const uint32_t slot = blockIdx.x * 64u + lane;
  const uint32_t axis = slot / U, u = slot % U;
  const bool active = axis < g.axes;
  const uint32_t gofs = u * 32;
  if constexpr (G == 1) {
    encode_lane<K, S, G, 0>(g, lds, lane, active, axis, gofs);
  } else {
    bs::sfor<G>([&](auto gi) {
      if (wv == decltype(gi)::value) encode_lane<K, S, G, decltype(gi)::value>(g, lds, lane, active, axis, gofs);
    });
  }
}

template <int LOGK>
static hipError_t launch_bs(const RsGeom& g, hipStream_t s) {
  constexpr int threads = 64 * ((LOGK > 4) ? (1 << (LOGK - 4)) : 1);
  const uint64_t slots = (uint64_t)g.axes * (g.len / 32);
  dim3 grid((unsigned)((slots + 63) / 64), g.nsq);
  hipLaunchKernelGGL(k_rs_encode_bs<LOGK>, grid, dim3(threads), 0, s, g);
  return hipGetLastError();
}

hipError_t launch_rs_encode_bitslice(const RsGeom& g, hipStream_t s) {
  switch (g.n) {
    case 1: return launch_bs<0>(g, s);
    case 2: return launch_bs<1>(g, s);
    case 4: return launch_bs<2>(g, s);
    case 8: return launch_bs<3>(g, s);
    case 16: return launch_bs<4>(g, s);
    case 32: return launch_bs<5>(g, s);
    case 64: return launch_bs<6>(g, s);
    case 128: return launch_bs<7>(g, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace cel
