// Leopard GF(2^8) erasure decode, register-resident, for axes of n = 32 .. 256 points
// (the repair's row and column solves, cel_dev_decode / cel_dev_repair).
//
// The algorithm is the one k_rs_decode (rs_kernels.hip) runs out of LDS (SURVEY.md
// Appendix A.3; Leopard ff8 ReedSolomonDecode as rsmt2d's LeoRSCodec.Decode calls it,
// rsmt2d/leopard.go): error locator err[] by FWHT, work = shard * exp(err) on the present
// points (0 on the erased ones), IFFT (skew offset 0), formal derivative, FFT, erased
// point = work * exp(-err). Here the transforms run in registers, as the encoder's:
//   - a workgroup owns one axis and up to four 128-byte column slices, one per wave; its
//     256 threads compute the error locator in LDS once (FWHT) and stage one v_perm product
//     table per point for the two scalings, while the waves' shard loads are in flight;
//   - point p of the axis lives in lane half h = p & 1 (lanes 0-31 / 32-63), register
//     r = p >> 1, so a lane holds n/2 points of one dword column. With the half taken
//     from the LOW point bit every butterfly's twiddle is the same in both halves (the
//     skew index depends on base = a & ~(2D-1), which clears bit 0 for D >= 2): the
//     twiddles stay compile-time constants. Only layer D = 1 pairs the halves; it runs
//     on v_permlane32_swap, which hands every lane both points of its pair;
//   - layers D = 2, 4, 8 (register distance 1, 2, 4, twiddles differ inside an 8-register
//     block) use the compile-time v_perm multiply; the 8-register blocks are then bit-
//     sliced (bs::tr8) and layers D >= 16 and the formal derivative run on bit planes
//     (xor networks, no multiplies in the derivative);
//   - only erased points are stored.
#include <hip/hip_runtime.h>

#include "cel_internal.hpp"
#include "bitslice8.hpp"
#include "gf8_constexpr.hpp"
#include "gf8_regs.hpp"

namespace cel {
namespace dx {

using ax::Mul;
using ax::pin;
using ax::pmuladd;
using ax::sconst;
using bs::pxor;
using bs::tr8;
using cx::kGf8;
using cx::sfor;

__constant__ cx::Gf8Tables c_t8 = cx::kGf8;

// y * c with c's product tables {t0l, t0h, t1l, t1h} in a and t2 in t4 (rs_kernels.hip gf8_mul4)
__device__ __forceinline__ uint32_t perm_mul(uint32_t y, uint4 a, uint32_t t4) {
  const uint32_t s0 = y & 0x07070707u;
  const uint32_t s1 = (y >> 3) & 0x07070707u;
  const uint32_t s2 = (y >> 6) & 0x03030303u;
  return __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_perm(a.y, a.x, s0), __builtin_amdgcn_perm(a.w, a.z, s1),
                                     __builtin_amdgcn_perm(0u, t4, s2), 0x96);
}

// f(r, table of register r) for r = 0 .. R-1, the LDS tables read LA registers ahead of
// their use (a table per point: register r of this lane half is at t + 16 r dwords)
template <int R, int LA, class F>
__device__ __forceinline__ void with_tables(const uint32_t* t, F&& f) {
  uint4 ta[LA];
  uint32_t tb[LA];
  sfor<LA>([&](auto i) {
    constexpr int r = decltype(i)::value;
    ta[r] = *reinterpret_cast<const uint4*>(t + 16 * r);
    tb[r] = t[16 * r + 4];
  });
  sfor<R>([&](auto ri) {
    constexpr int r = decltype(ri)::value;
    const uint4 a = ta[r % LA];
    const uint32_t b = tb[r % LA];
    if constexpr (r + LA < R) {
      ta[r % LA] = *reinterpret_cast<const uint4*>(t + 16 * (r + LA));
      tb[r % LA] = t[16 * (r + LA) + 4];
    }
    f(std::integral_constant<int, r>{}, a, b);
    __builtin_amdgcn_sched_barrier(0);
  });
}

// Layer D = 1 (pairs (2r, 2r+1) = register r of the two lane halves). After the swap
// p[0] holds the lower half's point and p[1] the upper half's, in every lane.
template <uint32_t LM>
__device__ __forceinline__ void cross_ifft(uint32_t& v, bool hi, uint32_t m7, uint32_t m3) {
  const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  const uint32_t y = p[0] ^ p[1];  // y ^= x
  uint32_t x = p[0];
  const Mul<LM> m;
  m.muladd(x, y, m7, m3);  // x ^= c*y
  v = hi ? y : x;
}
template <uint32_t LM>
__device__ __forceinline__ void cross_fft(uint32_t& v, bool hi, uint32_t m7, uint32_t m3) {
  const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  uint32_t x = p[0];
  const Mul<LM> m;
  m.muladd(x, p[1], m7, m3);  // x ^= c*y
  v = hi ? (p[1] ^ x) : x;    // y ^= x
}

// Axis a (blockIdx.x) is either dense (idx == nullptr: shards + a * N * len, shard stride
// len, presence present[a * N ..]) or axis idx[a] of a W x W square of len-byte cells at
// `shards` (a row if !is_col, else a column: shard stride len or W * len) with its
// presence in the square's mask `present`; in-square decodes store the erased cells
// straight into the square and mark the axis present (the repair's gather and scatter).
template <int LOGN>
__global__ __launch_bounds__(256, 2) void k_rs_decode_axis(uint8_t* __restrict__ shards,
                                                           uint8_t* __restrict__ present, uint32_t len,
                                                           const uint32_t* __restrict__ mul8,
                                                           const int32_t* __restrict__ idx, uint32_t W, int is_col) {
  constexpr int N = 1 << LOGN, R = N / 2, M = N / 2, NB = R / 8, NW = (R + 31) / 32;
  static_assert(LOGN >= 5 && LOGN <= 8, "register decode covers 32..256 points");
  __shared__ __attribute__((aligned(16))) uint32_t ltab[2][N][8];  // [scale in / out][point][table]
  __shared__ uint32_t s_err[N], s_tl[N];
  __shared__ uint32_t s_miss[2][NW];  // erased bits by lane half, register
  __shared__ uint8_t s_pres[N];
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t h = lane >> 5;
  const bool hi = h != 0;
  const uint32_t slice = blockIdx.y * 4u + (tid >> 6);
  const uint32_t col = slice * 128u + (lane & 31u) * 4u;
  const bool active = col < len;
  uint8_t* axis;
  uint8_t* pa;
  uint32_t sst, pst;  // shard stride (bytes), presence stride
  if (idx) {
    // is_col < 0: each entry names its own direction (bit 30 set = column)
    const uint32_t e = (uint32_t)idx[blockIdx.x];
    const uint32_t ax = e & 0x3FFFFFFFu;
    if (is_col < 0) is_col = (int)((e >> 30) & 1u);
    axis = shards + (is_col ? (uint64_t)ax * len : (uint64_t)ax * W * len);
    sst = is_col ? W * len : len;
    pa = present + (is_col ? (uint64_t)ax : (uint64_t)ax * W);
    pst = is_col ? W : 1u;
  } else {
    axis = shards + (uint64_t)blockIdx.x * N * len;
    sst = len;
    pa = present + (uint64_t)blockIdx.x * N;
    pst = 1u;
  }
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(axis, 0, 0x7fffffff, 0x00020000);
  // point p = 2r + h is shard p ^ M (rsmt2d order: data, then parity; Leopard order:
  // parity, then data), at byte (p ^ M) * sst = (2r ^ M) * sst + h * sst
  const uint32_t vo = h * sst + (active ? col : 0u);
  uint32_t w[R];
#pragma unroll
  for (int r = 0; r < R; r++) w[r] = __builtin_amdgcn_raw_buffer_load_b32(rs, vo, (uint32_t)((2 * r) ^ M) * sst, 2);

  // error locator (the shard loads are in flight): err[i] = sum over erased e of
  // log(i ^ e) mod 255, an XOR convolution, by FWHT (as k_rs_decode)
  if (tid < N) {
    const uint32_t pr = pa[(tid ^ M) * pst] ? 1u : 0u;
    s_pres[tid] = (uint8_t)pr;
    s_err[tid] = 1u - pr;
    s_tl[tid] = tid == 0 ? 0u : (uint32_t)c_t8.log[tid];
  }
  __syncthreads();
  // in-square: the axis is complete once decoded (every presence read is above the barrier;
  // the slice-0 workgroup of the axis marks it)
  if (idx && blockIdx.y == 0 && tid < N) pa[tid * pst] = 1;
  auto fwht = [&](bool both) {
#pragma unroll
    for (int lh = 0; lh < LOGN; lh++) {
      const uint32_t hh = 1u << lh;
      if (tid < N / 2) {
        const uint32_t a = ((tid >> lh) << (lh + 1)) | (tid & (hh - 1)), b = a + hh;
        uint32_t x = s_err[a], y = s_err[b];
        s_err[a] = (x + y >= 255u) ? x + y - 255u : x + y;
        s_err[b] = (x >= y) ? x - y : x + 255u - y;
        if (both) {
          x = s_tl[a];
          y = s_tl[b];
          s_tl[a] = (x + y >= 255u) ? x + y - 255u : x + y;
          s_tl[b] = (x >= y) ? x - y : x + 255u - y;
        }
      }
      __syncthreads();
    }
  };
  fwht(true);
  if (tid < N) s_err[tid] = (s_err[tid] * s_tl[tid]) % 255u;
  __syncthreads();
  fwht(false);
  if (tid < N) {
    const uint32_t e = (s_err[tid] * ((1u << (8 - LOGN)) % 255u)) % 255u;  // 1/N = 2^(8 - LOGN)
    const bool pr = s_pres[tid] != 0;
    const uint4* in = reinterpret_cast<const uint4*>(mul8 + e * 8);
    const uint4* out = reinterpret_cast<const uint4*>(mul8 + ((255u - e) % 255u) * 8);
    const uint4 z{0, 0, 0, 0};
    uint4* ti = reinterpret_cast<uint4*>(ltab[0][tid]);
    uint4* to = reinterpret_cast<uint4*>(ltab[1][tid]);
    ti[0] = pr ? in[0] : z;
    ti[1] = pr ? in[1] : z;
    to[0] = out[0];
    to[1] = out[1];
  }
  if (tid < 2 * (uint32_t)NW) {  // s_pres is visible since the first barrier
    const uint32_t hh = tid & 1, word = tid >> 1;
    uint32_t bits = 0;
#pragma unroll
    for (uint32_t b = 0; b < 32; b++) {
      const uint32_t r = word * 32 + b;
      if (r < (uint32_t)R) bits |= (s_pres[2 * r + hh] ? 0u : 1u) << b;
    }
    s_miss[hh][word] = bits;
  }
  __syncthreads();
  if (slice * 128u >= len) return;  // no barrier below

  const uint32_t m7 = sconst<0x07070707u>(), m3 = sconst<0x03030303u>();
  // scale in: work = shard * exp(err) on present points, 0 on erased ones
  with_tables<R, 8>(ltab[0][h], [&](auto ri, uint4 a, uint32_t b) {
    constexpr int r = decltype(ri)::value;
    w[r] = perm_mul(w[r], a, b);
  });
  // IFFT, skew index base + D - 1
  sfor<R>([&](auto ri) {
    constexpr int r = decltype(ri)::value;
    cross_ifft<kGf8.skew[2 * r]>(w[r], hi, m7, m3);
    __builtin_amdgcn_sched_barrier(0);
  });
  sfor<3>([&](auto lg) {
    constexpr int d = 1 << decltype(lg)::value, D = 2 * d;  // register distance d
    sfor<R / (2 * d)>([&](auto bi) {
      constexpr int rb = decltype(bi)::value * 2 * d;
      const Mul<kGf8.skew[2 * rb + D - 1]> m;
      sfor<d>([&](auto j) {
        constexpr int a = rb + decltype(j)::value;
        pin(w[a], w[a + d]);
        w[a + d] ^= w[a];
        m.muladd(w[a], w[a + d], m7, m3);
        pin(w[a], w[a + d]);
        __builtin_amdgcn_sched_barrier(0);
      });
    });
  });
  sfor<NB>([&](auto s) {
    tr8<8 * decltype(s)::value>(w);
    __builtin_amdgcn_sched_barrier(0);
  });
  sfor<LOGN - 4>([&](auto t) {
    constexpr int bd = 1 << decltype(t)::value, D = 16 * bd;  // block distance bd
    sfor<NB / (2 * bd)>([&](auto bi) {
      constexpr int mb = decltype(bi)::value * 2 * bd;
      sfor<bd>([&](auto j) {
        constexpr int a = 8 * (mb + decltype(j)::value), b = a + 8 * bd;
        pxor<a, b>(w);
        pmuladd<kGf8.skew[16 * mb + D - 1], a, b>(w);
        __builtin_amdgcn_sched_barrier(0);
      });
    });
  });
  // formal derivative: new[x] = old[x] ^ xor over t with bit t of x clear of old[x + 2^t].
  // Point x = 16m + 2i + h is bit i of every byte of block m's planes: t = 0 is the other
  // lane half, t = 1..3 are bit shifts inside a plane, t >= 4 are whole blocks. Blocks in
  // ascending order, so the blocks above m that block m reads are still old.
  {
    const uint32_t lomask = hi ? 0u : 0xFFFFFFFFu;
    const uint32_t k55 = sconst<0x55555555u>(), k33 = sconst<0x33333333u>(), k0f = sconst<0x0F0F0F0Fu>();
    sfor<NB>([&](auto mi) {
      constexpr int m = decltype(mi)::value;
      sfor<8>([&](auto bi) {
        constexpr int q = 8 * m + decltype(bi)::value;
        const uint32_t o = w[q];
        const auto p = __builtin_amdgcn_permlane32_swap(o, o, false, false);
        uint32_t acc = __builtin_amdgcn_bitop3_b32(o, o >> 1, k55, 0x78);  // o ^ (o>>1 & k55)
        acc = __builtin_amdgcn_bitop3_b32(acc, o >> 2, k33, 0x78);
        acc = __builtin_amdgcn_bitop3_b32(acc, o >> 4, k0f, 0x78);
        acc = __builtin_amdgcn_bitop3_b32(acc, p[1], lomask, 0x78);
        sfor<LOGN - 4>([&](auto t) {
          constexpr int bd = 1 << decltype(t)::value;
          if constexpr (!(m & bd)) acc ^= w[q + 8 * bd];
        });
        w[q] = acc;
        __builtin_amdgcn_sched_barrier(0);
      });
    });
  }
  // FFT, skew index base + D - 1
  sfor<LOGN - 4>([&](auto t) {
    constexpr int bd = (NB / 2) >> decltype(t)::value, D = 16 * bd;
    sfor<NB / (2 * bd)>([&](auto bi) {
      constexpr int mb = decltype(bi)::value * 2 * bd;
      sfor<bd>([&](auto j) {
        constexpr int a = 8 * (mb + decltype(j)::value), b = a + 8 * bd;
        pmuladd<kGf8.skew[16 * mb + D - 1], a, b>(w);
        pxor<a, b>(w);
        __builtin_amdgcn_sched_barrier(0);
      });
    });
  });
  sfor<NB>([&](auto s) {
    tr8<8 * decltype(s)::value>(w);
    __builtin_amdgcn_sched_barrier(0);
  });
  sfor<3>([&](auto lg) {
    constexpr int d = 4 >> decltype(lg)::value, D = 2 * d;
    sfor<R / (2 * d)>([&](auto bi) {
      constexpr int rb = decltype(bi)::value * 2 * d;
      const Mul<kGf8.skew[2 * rb + D - 1]> m;
      sfor<d>([&](auto j) {
        constexpr int a = rb + decltype(j)::value;
        pin(w[a], w[a + d]);
        m.muladd(w[a], w[a + d], m7, m3);
        w[a + d] ^= w[a];
        pin(w[a], w[a + d]);
        __builtin_amdgcn_sched_barrier(0);
      });
    });
  });
  sfor<R>([&](auto ri) {
    constexpr int r = decltype(ri)::value;
    cross_fft<kGf8.skew[2 * r]>(w[r], hi, m7, m3);
    asm volatile("" : "+v"(w[r]));  // computed here, not sunk into the conditional stores
    __builtin_amdgcn_sched_barrier(0);
  });
  // scale out and store the erased points: shard = work * exp(-err)
  if (!active) return;
  uint32_t slen = sst;  // recomputed shard offsets below (not 128 SGPRs live from the loads)
  asm volatile("" : "+s"(slen));
  uint32_t miss[NW];
  sfor<NW>([&](auto i) { miss[decltype(i)::value] = s_miss[h][decltype(i)::value]; });
  with_tables<R, 8>(ltab[1][h], [&](auto ri, uint4 a, uint32_t b) {
    constexpr int r = decltype(ri)::value;
    const uint32_t v = perm_mul(w[r], a, b);
    if ((miss[r / 32] >> (r & 31)) & 1u)
      __builtin_amdgcn_raw_buffer_store_b32(v, rs, vo, (uint32_t)((2 * r) ^ M) * slen, 2);
  });
}

template <int LOGN>
hipError_t launch(uint8_t* shards, uint8_t* present, uint32_t naxes, uint32_t len, const uint32_t* mul8,
                  const int32_t* idx, uint32_t W, int is_col, hipStream_t s) {
  const uint32_t nslice = (len + 127) / 128;
  hipLaunchKernelGGL(k_rs_decode_axis<LOGN>, dim3(naxes, (nslice + 3) / 4), dim3(256), 0, s, shards, present, len,
                     mul8, idx, W, is_col);
  return hipGetLastError();
}

}  // namespace dx

bool rs_decode_axis_supported(uint32_t n, uint32_t len) {
  return n >= 32 && n <= 256 && (n & (n - 1)) == 0 && len > 0 && len % 64 == 0 && (uint64_t)n * len < 0x7fffffffull;
}

static hipError_t decode_axes(uint8_t* shards, uint8_t* present, uint32_t naxes, uint32_t n, uint32_t len,
                              const uint32_t* mul8, const int32_t* idx, uint32_t W, int is_col, hipStream_t s) {
  switch (n) {
    case 32: return dx::launch<5>(shards, present, naxes, len, mul8, idx, W, is_col, s);
    case 64: return dx::launch<6>(shards, present, naxes, len, mul8, idx, W, is_col, s);
    case 128: return dx::launch<7>(shards, present, naxes, len, mul8, idx, W, is_col, s);
    case 256: return dx::launch<8>(shards, present, naxes, len, mul8, idx, W, is_col, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_rs_decode_axis(uint8_t* shards, const uint8_t* present, uint32_t naxes, uint32_t n, uint32_t len,
                                 const uint32_t* mul8, hipStream_t s) {
  if (!rs_decode_axis_supported(n, len)) return hipErrorInvalidValue;
  if (naxes == 0) return hipSuccess;
  // dense mode never writes the presence bytes
  return decode_axes(shards, const_cast<uint8_t*>(present), naxes, n, len, mul8, nullptr, 0, 0, s);
}

hipError_t launch_rs_decode_in_square(uint8_t* eds, uint8_t* mask, uint32_t W, const int32_t* idx, int is_col,
                                      uint32_t naxes, const uint32_t* mul8, hipStream_t s) {
  // One workgroup (blockIdx.y == 0) per axis reads and marks its presence: a cell wider
  // than 4 slices of 128 B would add y-blocks whose presence reads race that mark.
  static_assert(kShare <= 4 * 128, "in-square decode: one y-block per axis");
  if (!rs_decode_axis_supported(W, kShare) || (uint64_t)W * W * kShare >= 0x7fffffffull) return hipErrorInvalidValue;
  if (naxes == 0) return hipSuccess;
  return decode_axes(eds, mask, naxes, W, kShare, mul8, idx, W, is_col, s);
}

}  // namespace cel
