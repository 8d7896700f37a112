// Leopard GF(2^16) erasure decode (2m = 512, 1024, 2048 points) and the codec encoder of
// 1024/2048 data shards, in bit planes.
//
// Replaces klauspost/reedsolomon v1.12.1 leopard.go Reconstruct (catid/leopard's
// ReedSolomonDecode) as rsmt2d v0.14.0 LeoRSCodec.Decode drives it above 256 shards
// (pkg/appconsts/global_consts.go:92). Same decoder as
// rs_kernels.hip's header: error locator by FWHT, scale, IFFT over all n points at offset
// 0, formal derivative, FFT, unscale the erased points.
//
// Products. A 64-byte Leopard block holds 32 symbols, lo bytes in dwords 0-7 and hi bytes
// in dwords 8-15. An 8x8 bit transpose in each byte lane (bs::tr8) turns each half into 8
// bit planes: plane i (i < 8 from the lo half, 8 + (i - 8) from the hi half) holds bit i
// of the 32 symbols' Cantor representations. Multiplying by a constant c is GF(2)-linear:
// plane j of c*y is the xor of the planes i of y whose basis product P_i = c*b_i has
// coordinate j set, masked xors of one v_bfe + one v_bitop3 each (one v_bitop3 and an
// s_bfe where the twiddle is wave-uniform).
//
// Tower basis. Inside the transform the planes hold coordinates in the basis b_i = prod of
// gamma_k = beta_{2^k} over the set bits k of i (beta: the Cantor basis). The twiddles of a
// layer with block bases below 2^r lie in the subfield GF(2^(2^J)), J = decode16_level(r),
// and a product by such an element maps every block of 2^J consecutive coordinates onto
// itself: 16 * 2^J masked xors instead of 256 (n = 1024: 256, 256, 128 x 4, 64, 64, 32, 16
// over the ten layers). The change of basis rides on the per-point scales, which are
// general products anyway: present points are scaled from Cantor planes into tower
// planes, erased ones unscaled from tower planes back to Cantor planes. Twiddle products
// come from a 128 KiB table built on the host (DeviceTables::tw16), the scales' from the
// exp/log tables, once per chunk. tests/test_gf16_planes.py checks both statements against
// the field on the CPU.
//
// The previous LDS decoder looked every symbol's log and exp up in the 128 KiB global
// tables (two gathers per product): k=512 repair's 1024-axis row pass took 16.2 ms,
// L2-bound on the gathers (profiles/r3_bench_repair_k512.json).
//
// Layout: one workgroup per (axis, chunk set), n/2 threads (one butterfly each per layer),
// the chunk's 16 planes of every point in LDS plane-major (plane j of point p at
// [j * n + swz(p)]: consecutive lanes read consecutive words).
#include <hip/hip_runtime.h>

#include "bitslice8.hpp"
#include "cel_internal.hpp"
#include "leopard_field.hpp"

namespace cel {

namespace {

constexpr uint32_t kMod16 = 65535u;

// x ^= c*y (32 symbols, bit planes); pk[i / 2] half i % 2 holds P_i = c * b_i. J: c lies
// in GF(2^(2^J)), so P_i only reaches the coordinates of its own block of 2^J.
template <int J>
__device__ __forceinline__ void mul_acc(uint32_t (&x)[16], const uint32_t (&y)[16], const uint32_t (&pk)[8]) {
#pragma unroll
  for (int i = 0; i < 16; i++) {
#pragma unroll
    for (int j = 0; j < 16; j++) {
      if ((i >> J) != (j >> J)) continue;
      const uint32_t msk = (uint32_t)__builtin_amdgcn_sbfe((int)pk[i >> 1], 16 * (i & 1) + j, 1);
      x[j] = __builtin_amdgcn_bitop3_b32(x[j], msk, y[i], 0x78);  // x ^ (msk & y)
    }
  }
}

__device__ __forceinline__ void load_tw(uint32_t (&pk)[8], const uint32_t* __restrict__ tw, uint32_t s) {
  const uint4 a = reinterpret_cast<const uint4*>(tw)[2 * s];
  const uint4 b = reinterpret_cast<const uint4*>(tw)[2 * s + 1];
  pk[0] = a.x; pk[1] = a.y; pk[2] = a.z; pk[3] = a.w;
  pk[4] = b.x; pk[5] = b.y; pk[6] = b.z; pk[7] = b.w;
}

// Per-point products. Scale (present points, Cantor planes in, tower planes out):
// P_i = T(exp(e) * (1 << i)); unscale (erased points, tower in, Cantor out):
// P_i = exp(e) * b_i. exp(e) * a = exp[log a + e] (e < 65535; a partial reduction may give
// 65535, and exp[65535] = exp[0]). tower: T by lo and hi byte, then b_i (DeviceTables).
__device__ __forceinline__ uint32_t exp_mul(uint32_t la, uint32_t e, const uint16_t* __restrict__ gexp) {
  uint32_t s = la + e;
  s = (s + (s >> 16)) & kMod16;
  return gexp[s];
}

__device__ __forceinline__ void scale_products(uint32_t (&pk)[8], uint32_t e, bool in, const uint16_t* __restrict__ gexp,
                                               const uint16_t* __restrict__ glog, const uint16_t* __restrict__ tower) {
#pragma unroll
  for (int b = 0; b < 16; b += 2) {
    uint32_t p[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      if (in) {
        const uint32_t c = exp_mul(glog[1u << (b + h)], e, gexp);
        p[h] = (uint32_t)tower[c & 255] ^ (uint32_t)tower[256 + (c >> 8)];
      } else {
        p[h] = exp_mul(glog[tower[512 + b + h]], e, gexp);
      }
    }
    pk[b >> 1] = p[0] | (p[1] << 16);
  }
}

// One radix-2 layer, one butterfly per thread. UNI: D >= 64, so the 64 lanes of a wave share
// the block base and the twiddle (its masks go to SGPRs).
// LDS word of point p in a plane: p with its low 5 bits flipped when bit 5 is set. A
// layer's x (or y) points seen by 32 lanes of a ds_read_b32 group differ in 5 of the bits
// 0-5 of p, so they fall on 32 distinct banks ((word mod 32)) for every D: without the
// flip D = 1..16 were 2-way conflicts.
__device__ __forceinline__ uint32_t swz(uint32_t p) { return p ^ ((0u - ((p >> 5) & 1u)) & 31u); }

template <int LGN, bool IFFT, int J, bool UNI>
__device__ __forceinline__ void layer(uint32_t* planes, const uint32_t* __restrict__ tw, uint32_t t, uint32_t ld,
                                      uint32_t off) {
  constexpr uint32_t n = 1u << LGN;
  const uint32_t D = 1u << ld;
  const uint32_t base = (t >> ld) << (ld + 1), a = base + (t & (D - 1));
  const uint32_t sa = swz(a), sb = swz(a + D);
  uint32_t x[16], y[16], pk[8];
  uint32_t sk = off + base + D - 1;
  if (UNI) sk = __builtin_amdgcn_readfirstlane(sk);
  load_tw(pk, tw, sk);
#pragma unroll
  for (int j = 0; j < 16; j++) {
    x[j] = planes[j * n + sa];
    y[j] = planes[j * n + sb];
  }
  if (IFFT) {
#pragma unroll
    for (int j = 0; j < 16; j++) y[j] ^= x[j];
    mul_acc<J>(x, y, pk);
  } else {
    mul_acc<J>(x, y, pk);
#pragma unroll
    for (int j = 0; j < 16; j++) y[j] ^= x[j];
  }
#pragma unroll
  for (int j = 0; j < 16; j++) {
    planes[j * n + sa] = x[j];
    planes[j * n + sb] = y[j];
  }
  __syncthreads();
}

// IFFT: layers 0 .. LGN-1; FFT: LGN-1 .. 0, over n = 2^LGN points at offset `off` (a
// multiple of n). The twiddle of layer ld has Cantor representation (off + block base) >> ld,
// below 2^(RB - ld) with RB = log2(off + n), so it lies in GF(2^(2^J)) with J =
// decode16_level(RB - ld) (upload_tables checks every twiddle the kernels use). The decoder
// runs both at offset 0 (RB = LGN); the encoder's IFFT runs at offset n (RB = LGN + 1).
template <int LGN, bool IFFT, int RB = LGN>
__device__ __forceinline__ void transform(uint32_t* planes, const uint32_t* __restrict__ tw, uint32_t t,
                                          uint32_t off = 0) {
  static_assert(RB >= 9 && RB <= 12, "levels: J >= 2 below layer 6, J <= 3 from it");
#pragma unroll 1
  for (uint32_t i = 0; i < (uint32_t)LGN; i++) {
    const uint32_t ld = IFFT ? i : LGN - 1 - i;
    const uint32_t J = decode16_level(RB - ld);
    if (ld >= 6) {  // D >= 64: wave-uniform twiddle
      switch (J) {
        case 0: layer<LGN, IFFT, 0, true>(planes, tw, t, ld, off); break;
        case 1: layer<LGN, IFFT, 1, true>(planes, tw, t, ld, off); break;
        case 2: layer<LGN, IFFT, 2, true>(planes, tw, t, ld, off); break;
        default: layer<LGN, IFFT, 3, true>(planes, tw, t, ld, off); break;
      }
    } else {
      switch (J) {
        case 2: layer<LGN, IFFT, 2, false>(planes, tw, t, ld, off); break;
        case 3: layer<LGN, IFFT, 3, false>(planes, tw, t, ld, off); break;
        default: layer<LGN, IFFT, 4, false>(planes, tw, t, ld, off); break;
      }
    }
  }
}

// LDS: planes [16][n] | err [n] | present [n] bytes | point order [n] u16. 71 KiB at
// n = 1024: two workgroups per CU. (Keeping the per-point products in LDS, computed once
// per workgroup instead of once per chunk, takes 101 KiB and one workgroup per CU:
// 17 % slower, profiles/r3_decode_gf16_ab.txt.)
// The per-point products of a thread's first present and first erased point stay in
// registers across its chunks instead of being recomputed per chunk: k=512 decode 1.30 ->
// 1.10 ms (profiles/r3_decode_gf16_preg_ab.txt).
template <int LGN>
constexpr size_t decode_gf16_lds() {
  constexpr size_t n = size_t(1) << LGN;
  return n * 64 + n * 4 + n + n * 2;
}

// grid: x = axis, y = chunk set (chunks blockIdx.y, blockIdx.y + gridDim.y, ...).
// shards: [naxes][n][len] in rsmt2d order (data then parity); present: [naxes][n].
template <int LGN>
__global__ __launch_bounds__(1 << (LGN - 1)) void k_rs_decode_gf16(uint8_t* __restrict__ shards,
                                                                    const uint8_t* __restrict__ present, uint32_t len,
                                                                    const uint16_t* __restrict__ gexp,
                                                                    const uint16_t* __restrict__ glog,
                                                                    const uint32_t* __restrict__ tw,
                                                                    const uint16_t* __restrict__ tower) {
  constexpr uint32_t n = 1u << LGN, m = n / 2, NT = n / 2;
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  __shared__ uint32_t s_cnt[n / 64];
  uint32_t* planes = lds;
  uint32_t* err = planes + 16 * n;
  uint8_t* pres = reinterpret_cast<uint8_t*>(err + n);
  uint16_t* order = reinterpret_cast<uint16_t*>(pres + n);  // present points, then erased ones
  uint32_t* tl = planes;  // error-locator scratch, before the first chunk
  const uint32_t t = threadIdx.x, lane = t & 63;
  uint8_t* axis = shards + (uint64_t)blockIdx.x * n * len;
  const uint8_t* pa = present + (uint64_t)blockIdx.x * n;
  // point p in Leopard order: p < m -> parity shard p (rsmt2d index m + p); else data p - m
  uint64_t bal[2];
#pragma unroll
  for (uint32_t h = 0; h < 2; h++) {
    const uint32_t p = t + h * NT;
    const bool pr = pa[p < m ? m + p : p - m] != 0;
    pres[p] = pr ? 1 : 0;
    bal[h] = __ballot(pr);
    if (lane == 0) s_cnt[p >> 6] = (uint32_t)__popcll(bal[h]);
  }
  __syncthreads();
  // the present points in ascending order, then the erased ones: the scale and unscale
  // passes take one point per thread with divergence only at the boundary
  uint32_t np = 0;
#pragma unroll 1
  for (uint32_t g = 0; g < n / 64; g++) np += s_cnt[g];
#pragma unroll
  for (uint32_t h = 0; h < 2; h++) {
    const uint32_t p = t + h * NT;
    uint32_t before = (uint32_t)__popcll(bal[h] & ((1ull << lane) - 1));
#pragma unroll 1
    for (uint32_t g = 0; g < (p >> 6); g++) before += s_cnt[g];
    order[pres[p] ? before : np + p - before] = (uint16_t)p;
  }
  // err[i] = sum_{e erased} log0[i ^ e] mod 65535: FWHT of the erasure indicator and of
  // log0, pointwise product, FWHT back, times 1/n = 2^(16 - LGN) (as k_rs_decode)
  for (uint32_t i = t; i < n; i += NT) {
    err[i] = pres[i] ? 0u : 1u;
    tl[i] = i == 0 ? 0u : (uint32_t)glog[i];
  }
  __syncthreads();
  auto fwht = [&](uint32_t* v0, uint32_t* v1) {
#pragma unroll 1
    for (uint32_t lh = 0; lh < (uint32_t)LGN; lh++) {
      const uint32_t h = 1u << lh;
      const uint32_t a = ((t >> lh) << (lh + 1)) | (t & (h - 1)), b = a + h;
      uint32_t x = v0[a], y = v0[b];
      v0[a] = (x + y >= kMod16) ? x + y - kMod16 : x + y;
      v0[b] = (x >= y) ? x - y : x + kMod16 - y;
      if (v1) {
        x = v1[a];
        y = v1[b];
        v1[a] = (x + y >= kMod16) ? x + y - kMod16 : x + y;
        v1[b] = (x >= y) ? x - y : x + kMod16 - y;
      }
      __syncthreads();
    }
  };
  fwht(err, tl);
  for (uint32_t i = t; i < n; i += NT) err[i] = (err[i] * tl[i]) % kMod16;
  __syncthreads();
  fwht(err, nullptr);
  constexpr uint32_t inv_n = (1u << (16 - LGN)) % kMod16;
  for (uint32_t i = t; i < n; i += NT) {
    const uint32_t e = (err[i] * inv_n) % kMod16;
    // present points are scaled by exp(err), erased ones unscaled by exp(-err)
    err[i] = pres[i] ? e : (kMod16 - e) % kMod16;
  }
  // the first present and the first erased point of this thread keep their products in
  // registers across the chunks (the others, if any, look theirs up per chunk); not at
  // n = 2048, whose 1024-thread workgroups have 128 VGPRs and would spill them
  constexpr bool PREG = LGN <= 10;
  uint32_t pre0[8], post0[8];
  if constexpr (PREG) {
    __syncthreads();
    if (t < np) scale_products(pre0, err[order[t]], true, gexp, glog, tower);
    if (np + t < n) scale_products(post0, err[order[np + t]], false, gexp, glog, tower);
  }
  for (uint32_t chunk = blockIdx.y; chunk < len / 64u; chunk += gridDim.y) {
    const uint32_t coff = chunk * 64u;
    __syncthreads();  // the previous chunk's stores (and the setup) are done with the LDS
#pragma unroll
    for (uint32_t h = 0; h < 2; h++) {
      const uint32_t idx = t + h * NT, p = order[idx];
      uint32_t out[16];
#pragma unroll
      for (int j = 0; j < 16; j++) out[j] = 0;
      // erased points enter the transform as zero, whatever bytes the buffer holds there
      if (idx < np) {
        const uint4* src = reinterpret_cast<const uint4*>(axis + (uint64_t)(p < m ? m + p : p - m) * len + coff);
        uint32_t w[16], pk[8];
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const uint4 v = src[q];
          w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
        }
        bs::tr8<0>(w);
        bs::tr8<8>(w);
        if (PREG && h == 0) {
#pragma unroll
          for (int q = 0; q < 8; q++) {  // opaque: else the masks are hoisted out of the loop
            pk[q] = pre0[q];
            asm volatile("" : "+v"(pk[q]));
          }
        } else {
          scale_products(pk, err[p], true, gexp, glog, tower);
        }
        mul_acc<4>(out, w, pk);
      }
#pragma unroll
      for (int j = 0; j < 16; j++) planes[j * n + swz(p)] = out[j];
    }
    __syncthreads();
    transform<LGN, true>(planes, tw, t);
    {  // formal derivative: new[x] = old[x] ^ xor_{s: bit s of x clear, x + 2^s < n} old[x + 2^s]
      // (a thread takes points t and t + n/2 in all 16 planes: one address per (point, s))
      uint32_t acc[2][16];
#pragma unroll
      for (uint32_t h = 0; h < 2; h++) {
        const uint32_t x = t + h * NT;
#pragma unroll
        for (int u = 0; u < 16; u++) acc[h][u] = 0;
#pragma unroll
        for (uint32_t s = 1; s < n; s <<= 1) {
          if ((x & s) == 0) {
            const uint32_t a = swz(x + s);
#pragma unroll
            for (int u = 0; u < 16; u++) acc[h][u] ^= planes[u * n + a];
          }
        }
      }
      __syncthreads();
#pragma unroll
      for (uint32_t h = 0; h < 2; h++) {
        const uint32_t a = swz(t + h * NT);
#pragma unroll
        for (int u = 0; u < 16; u++) planes[u * n + a] ^= acc[h][u];
      }
      __syncthreads();
    }
    transform<LGN, false>(planes, tw, t);
#pragma unroll
    for (uint32_t h = 0; h < 2; h++) {  // (h = 1 only when fewer than half are present)
      const uint32_t idx = np + t + h * NT;
      if (idx >= n) continue;
      const uint32_t p = order[idx];
      uint32_t w[16], pk[8], out[16];
#pragma unroll
      for (int j = 0; j < 16; j++) {
        w[j] = planes[j * n + swz(p)];
        out[j] = 0;
      }
      if (PREG && h == 0) {
#pragma unroll
        for (int q = 0; q < 8; q++) {
          pk[q] = post0[q];
          asm volatile("" : "+v"(pk[q]));
        }
      } else {
        scale_products(pk, err[p], false, gexp, glog, tower);
      }
      mul_acc<4>(out, w, pk);
      bs::tr8<0>(out);
      bs::tr8<8>(out);
      uint4* dst = reinterpret_cast<uint4*>(axis + (uint64_t)(p < m ? m + p : p - m) * len + coff);
#pragma unroll
      for (int q = 0; q < 4; q++) dst[q] = uint4{out[4 * q], out[4 * q + 1], out[4 * q + 2], out[4 * q + 3]};
    }
  }
}

// Encoder for 1024 and 2048 data shards (the codec API; squares stop at k = 512, which
// the register kernel rs_gf16x.hip takes): the data shards are scaled by 1 into tower
// planes, IFFT over the m points at offset m, FFT at offset 0, back to Cantor planes.
// grid: x = axis, y = chunk set, z = square; m / 2 threads; LDS: m 64-byte chunks.
template <int LGM>
__global__ __launch_bounds__(1 << (LGM - 1)) void k_rs_encode_gf16p(RsGeom g, const uint16_t* __restrict__ gexp,
                                                                     const uint16_t* __restrict__ glog,
                                                                     const uint32_t* __restrict__ tw,
                                                                     const uint16_t* __restrict__ tower) {
  constexpr uint32_t m = 1u << LGM, NT = m / 2;
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t* planes = lds;
  const uint32_t t = threadIdx.x;
  const uint8_t* in = g.in + (uint64_t)blockIdx.z * g.in_sq + (uint64_t)blockIdx.x * g.in_axis;
  uint8_t* out = g.out + (uint64_t)blockIdx.z * g.out_sq + (uint64_t)blockIdx.x * g.out_axis;
  uint32_t to_tower[8], to_cantor[8];  // the change of basis as products by 1
  scale_products(to_tower, 0, true, gexp, glog, tower);
  scale_products(to_cantor, 0, false, gexp, glog, tower);
  for (uint32_t chunk = blockIdx.y; chunk < g.len / 64u; chunk += gridDim.y) {
    const uint32_t coff = chunk * 64u;
    __syncthreads();
#pragma unroll
    for (uint32_t h = 0; h < 2; h++) {
      const uint32_t p = t + h * NT;
      const uint4* src = reinterpret_cast<const uint4*>(in + (uint64_t)p * g.in_shard + coff);
      uint32_t w[16], o[16];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint4 v = src[q];
        w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
      }
      bs::tr8<0>(w);
      bs::tr8<8>(w);
#pragma unroll
      for (int j = 0; j < 16; j++) o[j] = 0;
      uint32_t pk[8];
#pragma unroll
      for (int q = 0; q < 8; q++) {  // opaque per use: else all 256 masks are hoisted and held
        pk[q] = __builtin_amdgcn_readfirstlane(to_tower[q]);
        asm volatile("" : "+s"(pk[q]));
      }
      mul_acc<4>(o, w, pk);
#pragma unroll
      for (int j = 0; j < 16; j++) planes[j * m + swz(p)] = o[j];
    }
    __syncthreads();
    transform<LGM, true, LGM + 1>(planes, tw, t, m);
    transform<LGM, false>(planes, tw, t);
#pragma unroll
    for (uint32_t h = 0; h < 2; h++) {
      const uint32_t p = t + h * NT;
      uint32_t w[16], o[16];
#pragma unroll
      for (int j = 0; j < 16; j++) {
        w[j] = planes[j * m + swz(p)];
        o[j] = 0;
      }
      uint32_t pk[8];
#pragma unroll
      for (int q = 0; q < 8; q++) {
        pk[q] = __builtin_amdgcn_readfirstlane(to_cantor[q]);
        asm volatile("" : "+s"(pk[q]));
      }
      mul_acc<4>(o, w, pk);
      bs::tr8<0>(o);
      bs::tr8<8>(o);
      uint4* dst = reinterpret_cast<uint4*>(out + (uint64_t)p * g.out_shard + coff);
#pragma unroll
      for (int q = 0; q < 4; q++) dst[q] = uint4{o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]};
    }
  }
}

}  // namespace

bool rs_decode_gf16_supported(uint32_t n) { return n == 512 || n == 1024 || n == 2048; }

hipError_t launch_rs_decode_gf16(uint8_t* shards, const uint8_t* present, uint32_t naxes, uint32_t n, uint32_t len,
                                 const DeviceTables& t, hipStream_t s) {
  if (!naxes) return hipSuccess;
  if (!rs_decode_gf16_supported(n) || len == 0 || len % 64 || !t.tw16 || !t.tower16) return hipErrorInvalidValue;
  const uint32_t nch = len / 64;
  // enough workgroups to fill the chip; each one computes its axis's error locator once
  // for all the chunks it takes
  uint32_t sets = (512 + naxes - 1) / naxes;
  sets = sets < 1 ? 1 : (sets > nch ? nch : sets);
  const dim3 grid(naxes, sets);
  auto go = [&](auto kern, size_t lds) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, grid, dim3(n / 2), lds, s, shards, present, len, t.exp16, t.log16, t.tw16,
                       t.tower16);
  };
  switch (n) {
    case 512: go(k_rs_decode_gf16<9>, decode_gf16_lds<9>()); break;
    case 1024: go(k_rs_decode_gf16<10>, decode_gf16_lds<10>()); break;
    default: go(k_rs_decode_gf16<11>, decode_gf16_lds<11>()); break;
  }
  return hipGetLastError();
}

}  // namespace cel

namespace cel {

hipError_t launch_rs_encode_gf16p(const RsGeom& g, const DeviceTables& t, hipStream_t s) {
  if ((g.n != 1024 && g.n != 2048) || g.len == 0 || g.len % 64 || g.dcopy || g.blk_log || g.chk_flags || !t.tw16 ||
      !t.tower16)
    return hipErrorInvalidValue;
  const uint32_t nch = g.len / 64;
  const uint64_t tiles = (uint64_t)g.axes * g.nsq;
  uint32_t sets = (uint32_t)((512 + tiles - 1) / tiles);
  sets = sets < 1 ? 1 : (sets > nch ? nch : sets);
  const dim3 grid(g.axes, sets, g.nsq);
  auto go = [&](auto kern, size_t lds) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, grid, dim3(g.n / 2), lds, s, g, t.exp16, t.log16, t.tw16, t.tower16);
  };
  if (g.n == 1024)
    go(k_rs_encode_gf16p<10>, (size_t)1024 * 64);
  else
    go(k_rs_encode_gf16p<11>, (size_t)2048 * 64);
  return hipGetLastError();
}

}  // namespace cel
