// Leopard Reed-Solomon on gfx950: encode (GF(2^8), GF(2^16)) and erasure decode.
//
// Replaces klauspost/reedsolomon v1.12.1 leopard8.go / leopard.go Encode and
// Reconstruct as driven by rsmt2d v0.14.0 LeoRSCodec (DefaultCodec,
// pkg/appconsts/global_consts.go:92). Algorithm: SURVEY.md Appendix A.2/A.3,
// written here in radix-2 form:
//   IFFT over the data coset (offset m): for D = 1, 2, .., m/2, every pair
//     (a, a+D) with base = a & ~(2D-1):  y ^= x; x ^= y * exp(skew[m-1 + base + D])
//   FFT over the parity coset (offset 0): for D = m/2, .., 1:
//     x ^= y * exp(skew[base + D - 1]); y ^= x
// A skew value equal to the field modulus means "multiply by zero" (the xor-only
// butterfly of the reference).
//
// GF(2^8) encode keeps one 32-bit column of every shard of an axis in VGPRs
// (k <= 128 dwords per lane): the whole transform is lane-local, with no LDS and
// no barriers. A multiply by the (wave-uniform) twiddle c splits each byte into
// 3+3+2 bits and looks each piece up with one v_perm_b32 in an 8/8/4-entry
// product table held in SGPRs: 10-12 VALU ops per 4 bytes.
//
// GF(2^16) (k >= 256) and the decoder stage a 64-byte chunk of every shard of
// an axis in LDS (k <= 2048 -> <= 128 KiB) and run radix-2 layers with a
// barrier per layer.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <string>
#include <vector>

#include "cel_internal.hpp"
#include "leopard_field.hpp"

namespace cel {

// ------------------------------------------------------------------ tables

// Product tables for the v_perm multiply: for constant c = exp(lm):
//   T0[n] = c*n (n<8), T1[n] = c*(n<<3) (n<8), T2[n] = c*(n<<6) (n<4)
// packed as {T0[0..3], T0[4..7], T1[0..3], T1[4..7], T2[0..3], 0, 0, 0}.
// lm == 255 (the "zero twiddle" sentinel) gives all-zero tables.
static void perm_table8(const LeoField& f, uint32_t lm, uint32_t out[8]) {
  for (int i = 0; i < 8; i++) out[i] = 0;
  if (lm == f.mod) return;
  auto mul = [&](uint32_t a) { return f.mul_log(a, lm) & 0xFF; };
  for (uint32_t n = 0; n < 8; n++) {
    out[n >> 2] |= mul(n) << (8 * (n & 3));
    out[2 + (n >> 2)] |= mul(n << 3) << (8 * (n & 3));
  }
  for (uint32_t n = 0; n < 4; n++) out[4] |= mul(n << 6) << (8 * n);
}

// GF(2^16) product tables for the v_perm multiply by c = exp(lm): the 16-bit input
// symbol splits into six fields (lo byte bits 0-2, 3-5, 6-7; hi byte likewise);
// for each field a table of the low and of the high product byte, as v_perm
// operands (8 entries = 2 dwords, 4 entries = 1 dword). Layout (dwords):
//   [0,1] lo0->L  [2,3] lo0->H  [4,5] lo3->L  [6,7] lo3->H  [8] lo6->L  [9] lo6->H
//   [10..19] the same for the hi byte.  lm == 65535 (zero twiddle) gives zeros.
static void perm_table16(const LeoField& f, uint32_t lm, uint32_t out[kTw16Words]) {
  for (uint32_t i = 0; i < kTw16Words; i++) out[i] = 0;
  if (lm == f.mod) return;
  for (int half = 0; half < 2; half++) {
    uint32_t* o = out + 10 * half;
    for (uint32_t n = 0; n < 8; n++) {
      const uint32_t p0 = f.mul_log(n << (8 * half), lm), p1 = f.mul_log(n << (8 * half + 3), lm);
      o[0 + (n >> 2)] |= (p0 & 0xFF) << (8 * (n & 3));
      o[2 + (n >> 2)] |= (p0 >> 8) << (8 * (n & 3));
      o[4 + (n >> 2)] |= (p1 & 0xFF) << (8 * (n & 3));
      o[6 + (n >> 2)] |= (p1 >> 8) << (8 * (n & 3));
    }
    for (uint32_t n = 0; n < 4; n++) {
      const uint32_t p2 = f.mul_log(n << (8 * half + 6), lm);
      o[8] |= (p2 & 0xFF) << (8 * n);
      o[9] |= (p2 >> 8) << (8 * n);
    }
  }
}

hipError_t upload_tables(DeviceTables* t) {
  const LeoField& f8 = leo_gf8();
  const LeoField& f16 = leo_gf16();
  std::vector<uint32_t> tw(255 * 8), mul8(256 * 8), tw16((size_t)kTw16Count * kTw16Words);
  for (uint32_t i = 0; i < kTw16Count; i++) perm_table16(f16, f16.skew[i], &tw16[(size_t)i * kTw16Words]);
  for (uint32_t i = 0; i < 255; i++) perm_table8(f8, f8.skew[i], &tw[i * 8]);
  for (uint32_t lm = 0; lm < 256; lm++) perm_table8(f8, lm == 255 ? 0 : lm, &mul8[lm * 8]);
  // mul8[255] is "multiply by exp(255) = 1" (a real log value, not the skew sentinel)
  {
    uint32_t one[8];
    for (int i = 0; i < 8; i++) one[i] = 0;
    for (uint32_t n = 0; n < 8; n++) {
      one[n >> 2] |= n << (8 * (n & 3));
      one[2 + (n >> 2)] |= (n << 3) << (8 * (n & 3));
    }
    for (uint32_t n = 0; n < 4; n++) one[4] |= (n << 6) << (8 * n);
    for (int i = 0; i < 8; i++) mul8[255 * 8 + i] = one[i];
  }
  hipError_t e;
  if ((e = hipMalloc(&t->tw8, tw.size() * 4)) != hipSuccess) return e;
  if ((e = hipMalloc(&t->tw16, tw16.size() * 4)) != hipSuccess) return e;
  if ((e = hipMemcpy(t->tw16, tw16.data(), tw16.size() * 4, hipMemcpyHostToDevice)) != hipSuccess) return e;
  if ((e = hipMalloc(&t->mul8, mul8.size() * 4)) != hipSuccess) return e;
  if ((e = hipMalloc(&t->exp16, 65536 * 2)) != hipSuccess) return e;
  if ((e = hipMalloc(&t->log16, 65536 * 2)) != hipSuccess) return e;
  if ((e = hipMalloc(&t->skew16, 65535 * 2)) != hipSuccess) return e;
  if ((e = hipMemcpy(t->tw8, tw.data(), tw.size() * 4, hipMemcpyHostToDevice)) != hipSuccess) return e;
  if ((e = hipMemcpy(t->mul8, mul8.data(), mul8.size() * 4, hipMemcpyHostToDevice)) != hipSuccess) return e;
  if ((e = hipMemcpy(t->exp16, f16.exp.data(), 65536 * 2, hipMemcpyHostToDevice)) != hipSuccess) return e;
  if ((e = hipMemcpy(t->log16, f16.log.data(), 65536 * 2, hipMemcpyHostToDevice)) != hipSuccess) return e;
  return hipMemcpy(t->skew16, f16.skew.data(), 65535 * 2, hipMemcpyHostToDevice);
}

void free_tables(DeviceTables* t) {
  (void)hipFree(t->tw8);
  (void)hipFree(t->tw16);
  (void)hipFree(t->mul8);
  (void)hipFree(t->exp16);
  (void)hipFree(t->log16);
  (void)hipFree(t->skew16);
  *t = DeviceTables{};
}

// GF(2^8) tables for the LDS kernels (exp/log, 256 entries each).
struct Gf8Small {
  uint8_t exp[256];
  uint8_t log[256];
  uint8_t skew[256];
};
__constant__ Gf8Small c_gf8;
static bool g_gf8_const_ready = false;

static hipError_t ensure_gf8_const() {
  if (g_gf8_const_ready) return hipSuccess;
  const LeoField& f = leo_gf8();
  Gf8Small h;
  for (int i = 0; i < 256; i++) {
    h.exp[i] = (uint8_t)f.exp[i];
    h.log[i] = (uint8_t)f.log[i];
    h.skew[i] = i < 255 ? (uint8_t)f.skew[i] : 0;
  }
  hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(c_gf8), &h, sizeof(h));
  if (e == hipSuccess) g_gf8_const_ready = true;
  return e;
}

// ------------------------------------------------ GF(2^8) register encode

struct PermTab {
  uint32_t t0l, t0h, t1l, t1h, t2;
};

__device__ __forceinline__ PermTab load_tab(const uint32_t* __restrict__ tw, int idx) {
  const uint32_t* p = tw + idx * 8;
  return PermTab{p[0], p[1], p[2], p[3], p[4]};
}

// 4 parallel GF(2^8) products y*c with c given by its product tables.
__device__ __forceinline__ uint32_t gf8_mul4(uint32_t y, const PermTab& t) {
  const uint32_t s0 = y & 0x07070707u;
  const uint32_t s1 = (y >> 3) & 0x07070707u;
  const uint32_t s2 = (y >> 6) & 0x03030303u;
  // v_bitop3 0x96 = three-input xor (gfx950)
  return __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_perm(t.t0h, t.t0l, s0), __builtin_amdgcn_perm(t.t1h, t.t1l, s1),
                                     __builtin_amdgcn_perm(0u, t.t2, s2), 0x96);
}

// GF(2^8) encode, workgroup = G waves covering one 256-byte column slice of one
// axis (lane = one dword column). K = 2^LOGK shards are split into G groups of
// S = min(K, 32); wave g holds shards [S*g, S*g + S) in VGPRs ("arrangement A").
//  - radix-2 layers with D < S are lane-local; their twiddle index depends on g
//    only, so the product tables are scalar loads (wave-uniform);
//  - for D >= S (only when G > 1) the group transposes through LDS so that every
//    lane holds shards {l + S*h : h < G} for L = S/G values of l ("arrangement B");
//    the twiddle index then depends on h only: uniform across the whole workgroup.
// IFFT: A layers up, transpose, B layers up; FFT: B layers down, transpose back,
// A layers down. LDS image [shard][lane] dwords: conflict-free (lane-contiguous).
template <int LOGK>
__global__ __launch_bounds__(64 * ((LOGK > 5) ? (1 << (LOGK - 5)) : 1)) void k_rs_encode_gf8(
    RsGeom g, const uint32_t* __restrict__ tw) {
  constexpr int K = 1 << LOGK;
  constexpr int LOGS = LOGK < 5 ? LOGK : 5;
  constexpr int S = 1 << LOGS;
  constexpr int G = K / S;
  constexpr int L = S / G;
  __shared__ uint32_t lds[G > 1 ? K * 64 : 1];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t col = blockIdx.y * 256u + (uint32_t)lane * 4u;
  const bool active = col < g.len;
  const uint8_t* src = g.in + (uint64_t)blockIdx.z * g.in_sq + (uint64_t)blockIdx.x * g.in_axis + col;
  uint8_t* dst = g.out + (uint64_t)blockIdx.z * g.out_sq + (uint64_t)blockIdx.x * g.out_axis + col;
  uint32_t w[S];
#pragma unroll
  for (int i = 0; i < S; i++)
    w[i] = active ? *reinterpret_cast<const uint32_t*>(src + (uint64_t)(wv * S + i) * g.in_shard) : 0u;
  if (g.dcopy && active) {
    uint8_t* dc = g.dcopy + (uint64_t)blockIdx.z * g.dc_sq + (uint64_t)blockIdx.x * g.dc_axis + col;
#pragma unroll
    for (int i = 0; i < S; i++) *reinterpret_cast<uint32_t*>(dc + (uint64_t)(wv * S + i) * g.dc_shard) = w[i];
  }
  // IFFT, arrangement A (D < S)
#pragma unroll
  for (int lg = 0; lg < LOGS; lg++) {
    const int D = 1 << lg;
#pragma unroll
    for (int base = 0; base < S; base += 2 * D) {
      const PermTab t = load_tab(tw, K - 1 + wv * S + base + D);
#pragma unroll
      for (int j = 0; j < D; j++) {
        w[base + j + D] ^= w[base + j];
        w[base + j] ^= gf8_mul4(w[base + j + D], t);
      }
    }
  }
  if constexpr (G > 1) {
#pragma unroll
    for (int i = 0; i < S; i++) lds[(wv * S + i) * 64 + lane] = w[i];
    __syncthreads();
#pragma unroll
    for (int h = 0; h < G; h++)
#pragma unroll
      for (int lo = 0; lo < L; lo++) w[h * L + lo] = lds[(wv * L + lo + S * h) * 64 + lane];
    // IFFT, arrangement B (D = S << t): pairs (h, h + 2^t), twiddle from h only
#pragma unroll
    for (int t = 0; (1 << t) < G; t++) {
      const int dh = 1 << t;
#pragma unroll
      for (int hb = 0; hb < G; hb += 2 * dh) {
        const PermTab tb = load_tab(tw, K - 1 + S * hb + S * dh);
#pragma unroll
        for (int h = hb; h < hb + dh; h++)
#pragma unroll
          for (int lo = 0; lo < L; lo++) {
            w[(h + dh) * L + lo] ^= w[h * L + lo];
            w[h * L + lo] ^= gf8_mul4(w[(h + dh) * L + lo], tb);
          }
      }
    }
    // FFT, arrangement B
#pragma unroll
    for (int t = 0; (1 << t) < G; t++) {
      const int dh = G >> (t + 1);
#pragma unroll
      for (int hb = 0; hb < G; hb += 2 * dh) {
        const PermTab tb = load_tab(tw, S * hb + S * dh - 1);
#pragma unroll
        for (int h = hb; h < hb + dh; h++)
#pragma unroll
          for (int lo = 0; lo < L; lo++) {
            w[h * L + lo] ^= gf8_mul4(w[(h + dh) * L + lo], tb);
            w[(h + dh) * L + lo] ^= w[h * L + lo];
          }
      }
    }
#pragma unroll
    for (int h = 0; h < G; h++)
#pragma unroll
      for (int lo = 0; lo < L; lo++) lds[(wv * L + lo + S * h) * 64 + lane] = w[h * L + lo];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < S; i++) w[i] = lds[(wv * S + i) * 64 + lane];
  } else {
    // single group: the IFFT high layers are the remaining A layers (none when K == S)
  }
  // FFT, arrangement A (D < S)
#pragma unroll
  for (int lg = LOGS - 1; lg >= 0; lg--) {
    const int D = 1 << lg;
#pragma unroll
    for (int base = 0; base < S; base += 2 * D) {
      const PermTab t = load_tab(tw, wv * S + base + D - 1);
#pragma unroll
      for (int j = 0; j < D; j++) {
        w[base + j] ^= gf8_mul4(w[base + j + D], t);
        w[base + j + D] ^= w[base + j];
      }
    }
  }
  if (active) {
#pragma unroll
    for (int i = 0; i < S; i++) *reinterpret_cast<uint32_t*>(dst + (uint64_t)(wv * S + i) * g.out_shard) = w[i];
  }
}


// ------------------------------------------------ GF(2^16) register encode
//
// Same schedule as k_rs_encode_gf8 (wave g owns shards [32g, 32g+32) in VGPRs, layers
// with D < 32 lane-local with wave-uniform twiddles, layers D >= 32 after an LDS
// transpose with workgroup-uniform twiddles) but a lane holds 4 GF(2^16) symbols per
// shard: the lo-byte dword and the matching hi-byte dword of Leopard's 64-byte
// lo/hi block layout (sym[j] = b[j] | b[j+32] << 8). Lane l covers
// block l/8, dword l%8, so one workgroup (K/32 waves) is exactly one 512-byte slice of
// one axis. The multiply is twelve v_perm lookups (3+3+2-bit fields of both bytes,
// low and high product byte) in SGPR-resident product tables.
struct Perm16 {
  uint32_t t[kTw16Words];
};

// Cache policy of the data loads and stores (2 = nt: every byte is touched once per pass).
#ifndef CEL_GF16_CP
#define CEL_GF16_CP 2
#endif
constexpr int kGf16Cp = CEL_GF16_CP;

// One product table from LDS (wave-uniform address: a broadcast read, ~LDS latency instead
// of an L2 round trip per twiddle group).
__device__ __forceinline__ Perm16 lds_tab16(const uint32_t* p) {
  Perm16 r;
#pragma unroll
  for (int i = 0; i < (int)kTw16Words / 4; i++) {
    const uint4 v = reinterpret_cast<const uint4*>(p)[i];
    r.t[4 * i] = v.x;
    r.t[4 * i + 1] = v.y;
    r.t[4 * i + 2] = v.z;
    r.t[4 * i + 3] = v.w;
  }
  return r;
}

// Materialise a value: stops the combiner from folding "(a ^ b) & mask" of the next
// layer's field extraction into v_bitop3 of the un-xored inputs, which keeps both
// inputs of every butterfly alive across layers and spills.
// asm volatile statements keep their order, so pinning the inputs of every butterfly
// (pin2) and its outputs (opaque) sequences the butterflies: the SelectionDAG
// scheduler otherwise interleaves the field extraction of all butterflies of a layer.
__device__ __forceinline__ void opaque(uint32_t& v) { asm volatile("" : "+v"(v)); }
__device__ __forceinline__ void pin2(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d) {
  asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
}

// x ^= y * c for 4 symbols held as (lo dword, hi dword).
__device__ __forceinline__ void gf16_muladd4(uint32_t& xl, uint32_t& xh, uint32_t yl, uint32_t yh, const Perm16& T) {
  const uint32_t a0 = yl & 0x07070707u, a1 = (yl >> 3) & 0x07070707u, a2 = (yl >> 6) & 0x03030303u;
  const uint32_t b0 = yh & 0x07070707u, b1 = (yh >> 3) & 0x07070707u, b2 = (yh >> 6) & 0x03030303u;
  const uint32_t* t = T.t;
  const uint32_t l0 = __builtin_amdgcn_perm(t[1], t[0], a0), l1 = __builtin_amdgcn_perm(t[5], t[4], a1);
  const uint32_t l2 = __builtin_amdgcn_perm(0u, t[8], a2), l3 = __builtin_amdgcn_perm(t[11], t[10], b0);
  const uint32_t l4 = __builtin_amdgcn_perm(t[15], t[14], b1), l5 = __builtin_amdgcn_perm(0u, t[18], b2);
  const uint32_t h0 = __builtin_amdgcn_perm(t[3], t[2], a0), h1 = __builtin_amdgcn_perm(t[7], t[6], a1);
  const uint32_t h2 = __builtin_amdgcn_perm(0u, t[9], a2), h3 = __builtin_amdgcn_perm(t[13], t[12], b0);
  const uint32_t h4 = __builtin_amdgcn_perm(t[17], t[16], b1), h5 = __builtin_amdgcn_perm(0u, t[19], b2);
  xl = __builtin_amdgcn_bitop3_b32(xl, __builtin_amdgcn_bitop3_b32(l0, l1, l2, 0x96),
                                   __builtin_amdgcn_bitop3_b32(l3, l4, l5, 0x96), 0x96);
  xh = __builtin_amdgcn_bitop3_b32(xh, __builtin_amdgcn_bitop3_b32(h0, h1, h2, 0x96),
                                   __builtin_amdgcn_bitop3_b32(h3, h4, h5, 0x96), 0x96);
}

template <int LOGK>
__global__ __launch_bounds__(64 * (1 << (LOGK - 5))) void k_rs_encode_gf16p(RsGeom g, const uint32_t* __restrict__ tw) {
  constexpr int K = 1 << LOGK;
  constexpr int S = 32;
  constexpr int LOGS = 5;
  constexpr int G = K / S;
  constexpr int L = S / G;
  // LDS: [K][64] dwords = one half (lo or hi) of the exchange image, then the 2(G-1)
  // product tables of the B layers. While the image is not in use (before the first
  // exchange, after the second) its space holds each wave's 31 A-layer tables, staged
  // with one bulk load: table reads in the A layers cost an LDS round trip, not a
  // dependent L2 load per twiddle group (which left the kernel 43 % memory-wait bound).
  extern __shared__ uint32_t lds[];
  constexpr int TW = (int)kTw16Words;
  uint32_t* const btab = lds + K * 64;  // [2][G-1][TW]
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t* const atab = lds + wv * 31 * TW;  // this wave's A tables, table m - 1 for m = 1..31
  // stage: A tables of the IFFT (skew K-1 + wv*S + m) and all B tables
  for (int i = lane; i < 31 * TW; i += 64) atab[i] = tw[(K - 1 + wv * S + 1) * TW + i];
  for (int i = threadIdx.x; i < 2 * (G - 1) * TW; i += blockDim.x) {
    const int tb = i / TW, dir = tb / (G - 1), m = tb % (G - 1) + 1;
    btab[i] = tw[(dir == 0 ? K - 1 + S * m : S * m - 1) * TW + i % TW];
  }
  // every lane is active: the launcher requires len % 512 == 0
  const uint32_t col = blockIdx.y * 512u + (uint32_t)(lane >> 3) * 64u + (uint32_t)(lane & 7) * 4u;
  // buffer resources: scalar base per (square, axis), 32-bit lane offset, scalar shard offset
  const __amdgpu_buffer_rsrc_t rin =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(g.in + (uint64_t)blockIdx.z * g.in_sq +
                                                             (uint64_t)blockIdx.x * g.in_axis),
                                        0, 0x7fffffff, 0x00020000);
  const uint32_t in_shard = (uint32_t)g.in_shard, out_shard = (uint32_t)g.out_shard;
  uint32_t wl[S], wh[S];
#pragma unroll
  for (int i = 0; i < S; i++) {
    const uint32_t so = (uint32_t)(wv * S + i) * in_shard;
    wl[i] = __builtin_amdgcn_raw_buffer_load_b32(rin, col, so, kGf16Cp);
    wh[i] = __builtin_amdgcn_raw_buffer_load_b32(rin, col + 32, so, kGf16Cp);
  }
  // shard j -> byte offset, linear or blocked (see RsGeom::blk_log)
  const uint32_t blk_mask = g.blk_log ? (1u << g.blk_log) - 1u : 0xFFFFFFFFu;
  const uint32_t blk_shift = g.blk_log ? g.blk_log : 31u;
  auto place = [&](uint32_t j, uint32_t shard, uint32_t blk) { return (j >> blk_shift) * blk + (j & blk_mask) * shard; };
  if (g.dcopy) {
    const __amdgpu_buffer_rsrc_t rdc = __builtin_amdgcn_make_buffer_rsrc(
        g.dcopy + (uint64_t)blockIdx.z * g.dc_sq + (uint64_t)blockIdx.x * g.dc_axis, 0, 0x7fffffff, 0x00020000);
    const uint32_t dc_shard = (uint32_t)g.dc_shard, dc_blk = (uint32_t)g.dc_blk;
#pragma unroll
    for (int i = 0; i < S; i++) {
      const uint32_t so = place((uint32_t)(wv * S + i), dc_shard, dc_blk);
      __builtin_amdgcn_raw_buffer_store_b32(wl[i], rdc, col, so, 0);
      __builtin_amdgcn_raw_buffer_store_b32(wh[i], rdc, col + 32, so, 0);
    }
  }
  __syncthreads();  // staged tables visible
  // IFFT, arrangement A (D < S): twiddle from the wave's group only
#pragma unroll
  for (int lg = 0; lg < LOGS; lg++) {
    const int D = 1 << lg;
#pragma unroll
    for (int base = 0; base < S; base += 2 * D) {
      const Perm16 t = lds_tab16(atab + (base + D - 1) * TW);
#pragma unroll
      for (int j = 0; j < D; j++) {
        pin2(wl[base + j], wh[base + j], wl[base + j + D], wh[base + j + D]);
        wl[base + j + D] ^= wl[base + j];
        wh[base + j + D] ^= wh[base + j];
        gf16_muladd4(wl[base + j], wh[base + j], wl[base + j + D], wh[base + j + D], t);
        opaque(wl[base + j]);
        opaque(wh[base + j]);
        __builtin_amdgcn_sched_barrier(0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // A -> B: lane holds shards {lo_abs + S*h : h < G} for L values lo_abs = wv*L + lo
  auto exchange = [&](bool to_b) {
#pragma unroll
    for (int half = 0; half < 2; half++) {
      uint32_t* w = half ? wh : wl;
#pragma unroll
      for (int i = 0; i < S; i++) {
        const int shard = to_b ? (wv * S + i) : (wv * L + (i % L) + S * (i / L));
        lds[shard * 64 + lane] = w[i];
      }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < S; i++) {
        const int shard = to_b ? (wv * L + (i % L) + S * (i / L)) : (wv * S + i);
        w[i] = lds[shard * 64 + lane];
      }
      __syncthreads();
    }
  };
  __syncthreads();  // every wave done with its A tables before the image overwrites them
  exchange(true);
  // IFFT, arrangement B (D = S << t): pairs (h, h + 2^t), twiddle from h only
#pragma unroll
  for (int t = 0; (1 << t) < G; t++) {
    const int dh = 1 << t;
#pragma unroll
    for (int hb = 0; hb < G; hb += 2 * dh) {
      const Perm16 tb = lds_tab16(btab + (hb + dh - 1) * TW);
#pragma unroll
      for (int h = hb; h < hb + dh; h++)
#pragma unroll
        for (int lo = 0; lo < L; lo++) {
          const int x = h * L + lo, y = (h + dh) * L + lo;
          pin2(wl[x], wh[x], wl[y], wh[y]);
          wl[y] ^= wl[x];
          wh[y] ^= wh[x];
          gf16_muladd4(wl[x], wh[x], wl[y], wh[y], tb);
          opaque(wl[x]);
          opaque(wh[x]);
          __builtin_amdgcn_sched_barrier(0);
        }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // FFT, arrangement B. The group at hb = 0 has skew index S*dh - 1 = 2^m - 1, whose
  // skew is 0 (log = modulus: Leopard's FFT_DIT2 skips the multiply), so those
  // butterflies are y ^= x only: the whole first layer and 1/2, 1/4, ... of the next.
#pragma unroll
  for (int t = 0; (1 << t) < G; t++) {
    const int dh = G >> (t + 1);
#pragma unroll
    for (int hb = 0; hb < G; hb += 2 * dh) {
      const Perm16 tb = lds_tab16(btab + ((G - 1) + hb + dh - 1) * TW);
#pragma unroll
      for (int h = hb; h < hb + dh; h++)
#pragma unroll
        for (int lo = 0; lo < L; lo++) {
          const int x = h * L + lo, y = (h + dh) * L + lo;
          pin2(wl[x], wh[x], wl[y], wh[y]);
          if (hb != 0) gf16_muladd4(wl[x], wh[x], wl[y], wh[y], tb);
          opaque(wl[x]);
          opaque(wh[x]);
          wl[y] ^= wl[x];
          wh[y] ^= wh[x];
          opaque(wl[y]);
          opaque(wh[y]);
          __builtin_amdgcn_sched_barrier(0);
        }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  exchange(false);  // ends with a barrier: the image space is free again
  for (int i = lane; i < 31 * TW; i += 64) atab[i] = tw[(wv * S) * TW + i];  // FFT A: skew wv*S + m - 1
  __syncthreads();
  // FFT, arrangement A (wave 0, base 0: skew index D - 1 = 2^m - 1, multiply by zero)
#pragma unroll
  for (int lg = LOGS - 1; lg >= 0; lg--) {
    const int D = 1 << lg;
#pragma unroll
    for (int base = 0; base < S; base += 2 * D) {
      const Perm16 t = lds_tab16(atab + (base + D - 1) * TW);
      const bool zero_tw = base == 0 && wv == 0;  // wave-uniform
#pragma unroll
      for (int j = 0; j < D; j++) {
        pin2(wl[base + j], wh[base + j], wl[base + j + D], wh[base + j + D]);
        if (!zero_tw) gf16_muladd4(wl[base + j], wh[base + j], wl[base + j + D], wh[base + j + D], t);
        opaque(wl[base + j]);
        opaque(wh[base + j]);
        wl[base + j + D] ^= wl[base + j];
        wh[base + j + D] ^= wh[base + j];
        opaque(wl[base + j + D]);
        opaque(wh[base + j + D]);
        __builtin_amdgcn_sched_barrier(0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  const __amdgpu_buffer_rsrc_t rout = __builtin_amdgcn_make_buffer_rsrc(
      g.out + (uint64_t)blockIdx.z * g.out_sq + (uint64_t)blockIdx.x * g.out_axis, 0, 0x7fffffff, 0x00020000);
  const uint32_t out_blk = (uint32_t)g.out_blk;
#pragma unroll
  for (int i = 0; i < S; i++) {
    const uint32_t so = place((uint32_t)(wv * S + i), out_shard, out_blk);
    __builtin_amdgcn_raw_buffer_store_b32(wl[i], rout, col, so, kGf16Cp);
    __builtin_amdgcn_raw_buffer_store_b32(wh[i], rout, col + 32, so, kGf16Cp);
  }
}

template <int LOGK>
static hipError_t launch_gf16p(const RsGeom& g, const DeviceTables& t, hipStream_t s) {
  constexpr int K = 1 << LOGK;
  constexpr int threads = 64 * (K / 32);
  const size_t lds = ((size_t)K * 64 + 2 * (K / 32 - 1) * kTw16Words) * 4;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)k_rs_encode_gf16p<LOGK>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    attr = true;
  }
  dim3 grid(g.axes, (g.len + 511) / 512, g.nsq);
  hipLaunchKernelGGL(k_rs_encode_gf16p<LOGK>, grid, dim3(threads), lds, s, g, t.tw16);
  return hipGetLastError();
}

// ------------------------------------------------- LDS transform kernels

// Field ops for the LDS kernels. A "unit" is one dword of 4 GF(2^8) symbols, or
// a GF(2^16) quad: lo-byte dword j and hi-byte dword j+8 of a 64-byte chunk.
struct Gf8Ops {
  static constexpr uint32_t MOD = 255;
  static constexpr int UNITS = 16;  // dwords per 64-byte chunk
  const uint8_t* lexp;
  const uint8_t* llog;
  __device__ uint32_t mul_log1(uint32_t a, uint32_t lm) const {
    if (!a) return 0;
    uint32_t s = llog[a] + lm;
    s = (s + (s >> 8)) & 255u;
    return lexp[s];
  }
  __device__ void muladd(uint32_t* chunk_x, const uint32_t* chunk_y, int u, uint32_t lm) const {
    const uint32_t y = chunk_y[u];
    uint32_t p = 0;
#pragma unroll
    for (int b = 0; b < 4; b++) p |= mul_log1((y >> (8 * b)) & 0xFF, lm) << (8 * b);
    chunk_x[u] ^= p;
  }
  __device__ void xorin(uint32_t* chunk_y, const uint32_t* chunk_x, int u) const { chunk_y[u] ^= chunk_x[u]; }
  __device__ void scale(uint32_t* chunk, int u, uint32_t lm) const {
    uint32_t y = chunk[u], p = 0;
#pragma unroll
    for (int b = 0; b < 4; b++) p |= mul_log1((y >> (8 * b)) & 0xFF, lm) << (8 * b);
    chunk[u] = p;
  }
};

struct Gf16Ops {
  static constexpr uint32_t MOD = 65535;
  static constexpr int UNITS = 8;  // quads per 64-byte chunk
  const uint16_t* __restrict__ gexp;
  const uint16_t* __restrict__ glog;
  __device__ uint32_t mul_log1(uint32_t a, uint32_t lm) const {
    if (!a) return 0;
    uint32_t s = glog[a] + lm;
    s = (s + (s >> 16)) & 65535u;
    return gexp[s];
  }
  __device__ void muladd(uint32_t* cx, const uint32_t* cy, int u, uint32_t lm) const {
    const uint32_t lo = cy[u], hi = cy[u + 8];
    uint32_t plo = 0, phi = 0;
#pragma unroll
    for (int b = 0; b < 4; b++) {
      const uint32_t s = ((lo >> (8 * b)) & 0xFF) | (((hi >> (8 * b)) & 0xFF) << 8);
      const uint32_t p = mul_log1(s, lm);
      plo |= (p & 0xFF) << (8 * b);
      phi |= (p >> 8) << (8 * b);
    }
    cx[u] ^= plo;
    cx[u + 8] ^= phi;
  }
  __device__ void xorin(uint32_t* cy, const uint32_t* cx, int u) const {
    cy[u] ^= cx[u];
    cy[u + 8] ^= cx[u + 8];
  }
  __device__ void scale(uint32_t* c, int u, uint32_t lm) const {
    const uint32_t lo = c[u], hi = c[u + 8];
    uint32_t plo = 0, phi = 0;
#pragma unroll
    for (int b = 0; b < 4; b++) {
      const uint32_t s = ((lo >> (8 * b)) & 0xFF) | (((hi >> (8 * b)) & 0xFF) << 8);
      const uint32_t p = mul_log1(s, lm);
      plo |= (p & 0xFF) << (8 * b);
      phi |= (p >> 8) << (8 * b);
    }
    c[u] = plo;
    c[u + 8] = phi;
  }
};

// Radix-2 transform layers over `npts` chunks of 16 dwords in LDS.
// ifft: D ascending, constant skew[off + base + D - 1]; y ^= x; x ^= y*c
// fft:  D descending, constant skew[base + D - 1];      x ^= y*c; y ^= x
template <class Ops, class SkewFn>
__device__ void lds_ifft(const Ops& ops, uint32_t* lds, uint32_t npts, uint32_t off, SkewFn skew) {
  const uint32_t items = (npts / 2) * Ops::UNITS;
  for (uint32_t D = 1; D < npts; D <<= 1) {
    for (uint32_t it = threadIdx.x; it < items; it += blockDim.x) {
      const uint32_t pair = it / Ops::UNITS, u = it % Ops::UNITS;
      const uint32_t base = (pair / D) * 2 * D, a = base + pair % D;
      uint32_t* x = lds + a * 16;
      uint32_t* y = lds + (a + D) * 16;
      const uint32_t lm = skew(off + base + D - 1);
      ops.xorin(y, x, u);
      if (lm != Ops::MOD) ops.muladd(x, y, u, lm);
    }
    __syncthreads();
  }
}

template <class Ops, class SkewFn>
__device__ void lds_fft(const Ops& ops, uint32_t* lds, uint32_t npts, SkewFn skew) {
  const uint32_t items = (npts / 2) * Ops::UNITS;
  for (uint32_t D = npts >> 1; D >= 1; D >>= 1) {
    for (uint32_t it = threadIdx.x; it < items; it += blockDim.x) {
      const uint32_t pair = it / Ops::UNITS, u = it % Ops::UNITS;
      const uint32_t base = (pair / D) * 2 * D, a = base + pair % D;
      uint32_t* x = lds + a * 16;
      uint32_t* y = lds + (a + D) * 16;
      const uint32_t lm = skew(base + D - 1);
      if (lm != Ops::MOD) ops.muladd(x, y, u, lm);
      ops.xorin(y, x, u);
    }
    __syncthreads();
  }
}

// GF(2^16) encode: grid x = axis, y = 64-byte chunk, z = square. LDS: n * 64 B.
__global__ __launch_bounds__(256) void k_rs_encode_gf16(RsGeom g, const uint16_t* __restrict__ gexp,
                                                        const uint16_t* __restrict__ glog,
                                                        const uint16_t* __restrict__ gskew) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const uint32_t n = g.n;
  const uint32_t coff = blockIdx.y * 64u;
  const uint8_t* src = g.in + (uint64_t)blockIdx.z * g.in_sq + (uint64_t)blockIdx.x * g.in_axis + coff;
  uint8_t* dst = g.out + (uint64_t)blockIdx.z * g.out_sq + (uint64_t)blockIdx.x * g.out_axis + coff;
  for (uint32_t it = threadIdx.x; it < n * 4; it += blockDim.x) {
    const uint32_t i = it >> 2, q = it & 3;
    const uint4 v = reinterpret_cast<const uint4*>(src + (uint64_t)i * g.in_shard)[q];
    reinterpret_cast<uint4*>(lds)[it] = v;
    if (g.dcopy)
      reinterpret_cast<uint4*>(g.dcopy + (uint64_t)blockIdx.z * g.dc_sq + (uint64_t)blockIdx.x * g.dc_axis + coff +
                               (uint64_t)i * g.dc_shard)[q] = v;
  }
  __syncthreads();
  Gf16Ops ops{gexp, glog};
  auto skew = [&](uint32_t i) { return (uint32_t)gskew[i]; };
  lds_ifft(ops, lds, n, n, skew);
  lds_fft(ops, lds, n, skew);
  for (uint32_t it = threadIdx.x; it < n * 4; it += blockDim.x) {
    const uint32_t i = it >> 2, q = it & 3;
    reinterpret_cast<uint4*>(dst + (uint64_t)i * g.out_shard)[q] = reinterpret_cast<const uint4*>(lds)[it];
  }
}

template <int LOGK>
static void launch_gf8(const RsGeom& g, const DeviceTables& t, hipStream_t s) {
  constexpr int threads = 64 * ((LOGK > 5) ? (1 << (LOGK - 5)) : 1);
  dim3 grid(g.axes, (g.len + 255) / 256, g.nsq);
  hipLaunchKernelGGL(k_rs_encode_gf8<LOGK>, grid, dim3(threads), 0, s, g, t.tw8);
}

// GF(2^8) implementation. Bit-sliced for n <= 16 (one shard group per lane: 172 VGPRs,
// no LDS exchange); v_perm tables for n >= 32, where the bit-sliced kernel needs the
// whole 256 KiB granule set of a workgroup in registers (256 VGPRs, one workgroup per
// CU) and its load/compute/store phases stop overlapping (profiles/r1_rs_impl_ab.txt).
// CEL_RS_IMPL=perm|bitslice|axis forces one implementation for every n.
static int gf8_impl_override() {
  static const int v = [] {
    const char* e = getenv("CEL_RS_IMPL");
    if (!e) return 0;
    if (std::string(e) == "perm") return 1;
    if (std::string(e) == "bitslice") return 2;
    if (std::string(e) == "axis") return 3;
    return 0;
  }();
  return v;
}
static bool use_perm_gf8(uint32_t n) {
  const int o = gf8_impl_override();
  if (o) return o != 2;
  return n >= 32;
}
// Wave-per-axis kernel (rs_axis.hip) for n >= 32: compile-time twiddles, no LDS.
// k = 128, 32 squares (profiles/r1_axis_ab.txt): 15.2 us/square against 18.1 for
// k_rs_encode_gf8 (CEL_RS_IMPL=perm).
static bool use_axis_gf8(uint32_t n) {
  const int o = gf8_impl_override();
  if (o) return o == 3;
  return n >= 32;
}

hipError_t launch_rs_encode(const RsGeom& g, const DeviceTables& t, hipStream_t s) {
  if (g.axes == 0 || g.nsq == 0) return hipSuccess;
  if (g.blk_log && !((g.n == 256 || g.n == 512) && g.len % 512 == 0)) return hipErrorInvalidValue;
  if (2 * g.n <= 256 && !use_perm_gf8(g.n) && g.len % 32 == 0) return launch_rs_encode_bitslice(g, s);
  if (2 * g.n <= 256 && use_axis_gf8(g.n)) return launch_rs_encode_axis(g, s);
  if (2 * g.n <= 256) {
    switch (g.n) {
      case 1: launch_gf8<0>(g, t, s); break;
      case 2: launch_gf8<1>(g, t, s); break;
      case 4: launch_gf8<2>(g, t, s); break;
      case 8: launch_gf8<3>(g, t, s); break;
      case 16: launch_gf8<4>(g, t, s); break;
      case 32: launch_gf8<5>(g, t, s); break;
      case 64: launch_gf8<6>(g, t, s); break;
      case 128: launch_gf8<7>(g, t, s); break;
      default: return hipErrorInvalidValue;
    }
  } else {
    if (g.n > kMaxGf16Width) return hipErrorInvalidValue;
    static const bool lds_only = [] {
      const char* e = getenv("CEL_GF16_IMPL");  // "lds": force the LDS/gather kernel (A/B runs)
      return e && std::string(e) == "lds";
    }();
    const bool reg = !lds_only || g.blk_log;
    if (reg && (g.n == 256 || g.n == 512) && g.len % 64 == 0) return launch_rs_encode_gf16x(g, s);
    dim3 grid(g.axes, g.len / 64, g.nsq);
    const size_t lds = (size_t)g.n * 64;
    if (lds > 64 * 1024)
      (void)hipFuncSetAttribute((const void*)k_rs_encode_gf16, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k_rs_encode_gf16, grid, dim3(256), lds, s, g, t.exp16, t.log16, t.skew16);
  }
  return hipGetLastError();
}

// Squares per pipeline chunk of the wave-per-axis extension (CEL_RS_CHUNK, default 0 =
// two launches over the whole batch: rows(Q0) -> Q1, then all 2k columns).
// The chunked schedule (launch_extend_axis) re-reads Q0 and Q1 from the Infinity
// Cache and cuts the memory-only time 9.57 -> 8.68 us per k=128 square, but with the
// transform on it is slower (chunk 6: 14.9, chunk 8/12: 13.7 vs 12.3 us): the kernel
// is VALU-bound and every small launch pays a full wave lifetime of tail
// (profiles/r1_rs_chunk_ab.txt). Kept for A/B runs.
static uint32_t rs_chunk(uint32_t) {
  static const int env = [] {
    const char* e = getenv("CEL_RS_CHUNK");
    return e ? atoi(e) : 0;
  }();
  return env > 0 ? (uint32_t)env : 0u;
}

// Geometries of the extension of nsq squares starting at square `first`.
//   rows(Q0) -> Q1, cols(Q0) -> Q2, cols(Q1) -> Q3
// (Q2 = C*Q0 and Q3 = C*Q1 are exactly the reference's column pass over [Q0|Q1],
// SURVEY A.4.) Q0 is read from `ods` (and copied into the EDS by the row pass) when
// ods != nullptr, else from the EDS itself.
struct ExtGeoms {
  RsGeom rows, cols0, cols1;
};
static ExtGeoms ext_geoms(const uint8_t* ods, uint8_t* eds, uint32_t k, uint32_t first, uint32_t nsq) {
  const uint64_t row = (uint64_t)2 * k * kShare;  // bytes per EDS row
  const uint64_t sq_eds = (uint64_t)4 * k * k * kShare;
  const uint64_t sq_ods = (uint64_t)k * k * kShare;
  eds += first * sq_eds;
  if (ods) ods += first * sq_ods;
  ExtGeoms x{};
  RsGeom& r = x.rows;
  r.in = ods ? ods : eds;
  r.in_sq = ods ? sq_ods : sq_eds;
  r.in_axis = ods ? (uint64_t)k * kShare : row;
  r.in_shard = kShare;
  if (ods) {
    r.dcopy = eds;
    r.dc_sq = sq_eds;
    r.dc_axis = row;
    r.dc_shard = kShare;
  }
  r.out = eds + (uint64_t)k * kShare;
  r.out_sq = sq_eds;
  r.out_axis = row;
  r.out_shard = kShare;
  r.n = k;
  r.len = kShare;
  r.axes = k;
  r.nsq = nsq;
  RsGeom& c0 = x.cols0;
  c0.in = ods ? ods : eds;
  c0.in_sq = ods ? sq_ods : sq_eds;
  c0.in_axis = kShare;
  c0.in_shard = ods ? (uint64_t)k * kShare : row;
  c0.out = eds + (uint64_t)k * row;
  c0.out_sq = sq_eds;
  c0.out_axis = kShare;
  c0.out_shard = row;
  c0.n = k;
  c0.len = kShare;
  c0.axes = k;
  c0.nsq = nsq;
  RsGeom& c1 = x.cols1;
  c1 = c0;
  c1.in = eds + (uint64_t)k * kShare;
  c1.in_sq = sq_eds;
  c1.in_shard = row;
  c1.out = eds + (uint64_t)k * row + (uint64_t)k * kShare;
  return x;
}

// Chunked schedule of the wave-per-axis kernel: launch j runs cols(Q1) of chunk j-1
// beside rows(Q0) and cols(Q0) of chunk j. Every Q0 tile is read by a row tile and a
// column tile of the same launch (the second read hits the Infinity Cache), and the
// Q1 tiles that chunk j-1 wrote are re-read one launch later, still cache-resident.
// The kernel boundary orders cols(Q1) after rows(Q0) of its chunk.
static hipError_t launch_extend_axis(const uint8_t* ods, uint8_t* eds, uint32_t k, uint32_t nsq, uint32_t chunk,
                                     hipStream_t s) {
  const uint32_t nch = (nsq + chunk - 1) / chunk;
  for (uint32_t j = 0; j <= nch; j++) {
    RsGeom gs[kMaxSegs];
    uint32_t ns = 0;
    if (j > 0) {
      const uint32_t f = (j - 1) * chunk, n = (f + chunk <= nsq) ? chunk : nsq - f;
      gs[ns++] = ext_geoms(ods, eds, k, f, n).cols1;
    }
    if (j < nch) {
      const uint32_t f = j * chunk, n = (f + chunk <= nsq) ? chunk : nsq - f;
      const ExtGeoms x = ext_geoms(ods, eds, k, f, n);
      gs[ns++] = x.rows;
      gs[ns++] = x.cols0;
    }
    const hipError_t e = launch_rs_encode_axis_segs(gs, ns, s);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// Chunks of the two-stream extension (CEL_RS_OVERLAP; 0 or 1 = off).
uint32_t extend_overlap_chunks() {
  static const int v = [] {
    const char* e = getenv("CEL_RS_OVERLAP");
    return e ? atoi(e) : 0;
  }();
  return v > 1 ? (uint32_t)v : 0u;
}

hipError_t launch_extend_2s(const uint8_t* ods, uint8_t* eds, uint32_t k, uint32_t nsq, uint32_t m,
                            const DeviceTables& t, hipStream_t s0, hipStream_t s1, hipEvent_t* ev) {
  if (m > nsq) m = nsq;
  if (m < 2) return launch_extend(ods, eds, k, nsq, t, s0);
  const uint32_t chunk = (nsq + m - 1) / m;
  m = (nsq + chunk - 1) / chunk;
  hipError_t e;
  if ((e = hipEventRecord(ev[m], s0)) != hipSuccess || (e = hipStreamWaitEvent(s1, ev[m], 0)) != hipSuccess) return e;
  for (uint32_t c = 0; c < m; c++) {
    const uint32_t first = c * chunk, n = (first + chunk <= nsq) ? chunk : nsq - first;
    hipStream_t sc = (c & 1) ? s1 : s0;
    // rows(c) starts once rows(c - 1) is done, i.e. beside cols(c - 1) on the other stream
    if (c > 0 && (e = hipStreamWaitEvent(sc, ev[c - 1], 0)) != hipSuccess) return e;
    const ExtGeoms x = ext_geoms(ods, eds, k, first, n);
    if ((e = launch_rs_encode(x.rows, t, sc)) != hipSuccess) return e;
    if ((e = hipEventRecord(ev[c], sc)) != hipSuccess) return e;
    RsGeom cols = x.cols0;  // all 2k columns of [Q0|Q1] in one geometry (in place)
    cols.in = eds + (uint64_t)first * 4 * k * k * kShare;
    cols.in_sq = (uint64_t)4 * k * k * kShare;
    cols.in_shard = (uint64_t)2 * k * kShare;
    cols.axes = 2 * k;
    if ((e = launch_rs_encode(cols, t, sc)) != hipSuccess) return e;
  }
  if ((e = hipEventRecord(ev[m], s1)) != hipSuccess) return e;
  return hipStreamWaitEvent(s0, ev[m], 0);
}

hipError_t launch_extend(const uint8_t* ods, uint8_t* eds, uint32_t k, uint32_t nsq, const DeviceTables& t,
                         hipStream_t s) {
  if (nsq == 0) return hipSuccess;
  if (k >= 32 && k <= 128 && use_axis_gf8(k)) {
    const uint32_t chunk = rs_chunk(k);
    if (chunk) return launch_extend_axis(ods, eds, k, nsq, chunk, s);
  }
  const uint64_t row = (uint64_t)2 * k * kShare;  // bytes per EDS row
  const uint64_t sq_eds = (uint64_t)4 * k * k * kShare;
  hipError_t e;
  // Q0 rows -> Q1 (reading the ODS and writing Q0 into the EDS on the way when ods != nullptr)
  const ExtGeoms x = ext_geoms(ods, eds, k, 0, nsq);
  if ((e = launch_rs_encode(x.rows, t, s)) != hipSuccess) return e;
  // columns of [Q0|Q1] -> [Q2|Q3]
  RsGeom cols{};
  cols.in = eds;
  cols.in_sq = sq_eds;
  cols.in_axis = kShare;
  cols.in_shard = row;
  cols.out = eds + (uint64_t)k * row;
  cols.out_sq = sq_eds;
  cols.out_axis = kShare;
  cols.out_shard = row;
  cols.n = k;
  cols.len = kShare;
  cols.axes = 2 * k;
  cols.nsq = nsq;
  return launch_rs_encode(cols, t, s);
}

// ------------------------------------------------------------------ decode
//
// Leopard's error-locator erasure decoder (catid/leopard ReedSolomonDecode as used
// by klauspost Reconstruct), over the n = 2m point domain with the recovery
// (parity) shards at positions [0, m) and the original (data) shards at [m, 2m):
//   err[i]   = sum_{e erased} log0[i ^ e]   (mod field modulus; log0 = log with log0[0] = 0)
//              = log prod_{e erased, e != i} (w_i + w_e)
//   work[i]  = present ? shard_i * exp(err[i]) : 0
//   IFFT over all n points (offset 0), formal derivative, FFT over all n points
//   erased i: shard_i = work[i] * exp(-err[i])
// Erased parity shards are revealed by the same formula (the codeword is unique).

template <class Ops, class SkewFn>
__device__ void decode_chunk(const Ops& ops, uint32_t* lds, uint32_t* err, const uint8_t* pres, uint32_t m,
                             SkewFn skew) {
  const uint32_t n = 2 * m;
  // work <- present * exp(err)
  for (uint32_t it = threadIdx.x; it < n * Ops::UNITS; it += blockDim.x) {
    const uint32_t i = it / Ops::UNITS, u = it % Ops::UNITS;
    if (pres[i]) ops.scale(lds + i * 16, u, err[i]);
  }
  __syncthreads();
  lds_ifft(ops, lds, n, 0, skew);
  // formal derivative: new[x] = old[x] ^ xor_{t: bit t of x clear, x + 2^t < n} old[x + 2^t].
  // Sources are never modified before being read in the sequential reference loop,
  // so processing x in descending order of blocks is unnecessary: read old values
  // for all targets first (per lane, a unit at a time), then write.
  for (uint32_t base = 0; base < n * Ops::UNITS; base += blockDim.x) {
    const uint32_t it = base + threadIdx.x;
    uint32_t acc[2] = {0, 0};
    const bool active = it < n * Ops::UNITS;
    uint32_t x = 0, u = 0;
    if (active) {
      x = it / Ops::UNITS;
      u = it % Ops::UNITS;
      for (uint32_t t = 1; t < n; t <<= 1) {
        if ((x & t) == 0 && x + t < n) {
          acc[0] ^= lds[(x + t) * 16 + u];
          if (Ops::UNITS == 8) acc[1] ^= lds[(x + t) * 16 + u + 8];
        }
      }
    }
    __syncthreads();
    if (active) {
      lds[x * 16 + u] ^= acc[0];
      if (Ops::UNITS == 8) lds[x * 16 + u + 8] ^= acc[1];
    }
    __syncthreads();
  }
  lds_fft(ops, lds, n, skew);
  for (uint32_t it = threadIdx.x; it < n * Ops::UNITS; it += blockDim.x) {
    const uint32_t i = it / Ops::UNITS, u = it % Ops::UNITS;
    if (!pres[i]) ops.scale(lds + i * 16, u, (Ops::MOD - err[i]) % Ops::MOD);
  }
  __syncthreads();
}

// GF(2^8) decode of one 64-byte chunk with v_perm product tables staged in LDS
// (ltw: twiddle tables by skew index, lmul: tables by log value; 5 dwords each) in
// place of the per-byte log/exp lookups of Gf8Ops: same transform as decode_chunk.
// Layers go two at a time (radix 4: a thread owns one dword of four points, half the
// LDS round trips and barriers of radix 2); the formal derivative reads every source
// before one barrier and writes after it.
__device__ void decode_chunk_gf8p(uint32_t* lds, const uint32_t* err, const uint8_t* pres, uint32_t m,
                                  const uint32_t* ltw, const uint32_t* lmul) {
  const uint32_t n = 2 * m;
  const uint32_t lgn = 31u - __builtin_clz(n);
  constexpr uint32_t U = 16;  // dwords per 64-byte chunk
  auto tab = [](const uint32_t* t) { return PermTab{t[0], t[1], t[2], t[3], t[4]}; };
  // x ^= c(idx) * y, skipped for the zero twiddle
  auto mad = [&](uint32_t& x, uint32_t y, uint32_t idx) {
    if (c_gf8.skew[idx] != 255u) x ^= gf8_mul4(y, tab(ltw + idx * 5));
  };
  for (uint32_t it = threadIdx.x; it < n * U; it += blockDim.x) {
    const uint32_t i = it / U, u = it % U;
    if (pres[i]) lds[i * 16 + u] = gf8_mul4(lds[i * 16 + u], tab(lmul + err[i] * 5));
  }
  __syncthreads();
  // IFFT (offset 0): layers D = 1, 2, 4, ...; butterfly y ^= x; x ^= c*y
  uint32_t lD = 0;
  for (; lD + 1 < lgn; lD += 2) {
    const uint32_t D = 1u << lD;
    for (uint32_t it = threadIdx.x; it < (n / 4) * U; it += blockDim.x) {
      const uint32_t q = it / U, u = it % U;
      const uint32_t b4 = (q >> lD) << (lD + 2), a = b4 + (q & (D - 1));
      uint32_t* p = lds + a * 16 + u;
      uint32_t v0 = p[0], v1 = p[D * 16], v2 = p[2 * D * 16], v3 = p[3 * D * 16];
      v1 ^= v0; mad(v0, v1, b4 + D - 1);
      v3 ^= v2; mad(v2, v3, b4 + 3 * D - 1);
      v2 ^= v0; mad(v0, v2, b4 + 2 * D - 1);
      v3 ^= v1; mad(v1, v3, b4 + 2 * D - 1);
      p[0] = v0; p[D * 16] = v1; p[2 * D * 16] = v2; p[3 * D * 16] = v3;
    }
    __syncthreads();
  }
  if (lD < lgn) {  // odd log2(n): one radix-2 layer left
    const uint32_t D = 1u << lD;
    for (uint32_t it = threadIdx.x; it < (n / 2) * U; it += blockDim.x) {
      const uint32_t pair = it / U, u = it % U;
      const uint32_t base = (pair >> lD) << (lD + 1), a = base + (pair & (D - 1));
      uint32_t x = lds[a * 16 + u], y = lds[(a + D) * 16 + u];
      y ^= x;
      mad(x, y, base + D - 1);
      lds[a * 16 + u] = x;
      lds[(a + D) * 16 + u] = y;
    }
    __syncthreads();
  }
  {  // formal derivative: new[x] = old[x] ^ xor_{t: bit t of x clear, x + 2^t < n} old[x + 2^t]
    constexpr uint32_t kMaxItems = 256 * 16 / 256;  // GF(2^8): n <= 256 points, 256 threads
    uint32_t acc[kMaxItems];
#pragma unroll
    for (uint32_t r = 0; r < kMaxItems; r++) {
      const uint32_t it = threadIdx.x + r * 256u;
      acc[r] = 0;
      if (it < n * U) {
        const uint32_t x = it / U, u = it % U;
        for (uint32_t t = 1; t < n; t <<= 1)
          if ((x & t) == 0 && x + t < n) acc[r] ^= lds[(x + t) * 16 + u];
      }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t r = 0; r < kMaxItems; r++) {
      const uint32_t it = threadIdx.x + r * 256u;
      if (it < n * U) lds[(it / U) * 16 + it % U] ^= acc[r];
    }
    __syncthreads();
  }
  // FFT: layers D = n/2, ..., 1; butterfly x ^= c*y; y ^= x
  lD = lgn;
  if (lgn & 1) {  // odd log2(n): the top layer alone
    lD = lgn - 1;
    const uint32_t D = 1u << lD;
    for (uint32_t it = threadIdx.x; it < (n / 2) * U; it += blockDim.x) {
      const uint32_t pair = it / U, u = it % U;
      const uint32_t base = (pair >> lD) << (lD + 1), a = base + (pair & (D - 1));
      uint32_t x = lds[a * 16 + u], y = lds[(a + D) * 16 + u];
      mad(x, y, base + D - 1);
      y ^= x;
      lds[a * 16 + u] = x;
      lds[(a + D) * 16 + u] = y;
    }
    __syncthreads();
  }
  while (lD >= 2) {
    lD -= 2;  // layers 2D then D
    const uint32_t D = 1u << lD;
    for (uint32_t it = threadIdx.x; it < (n / 4) * U; it += blockDim.x) {
      const uint32_t q = it / U, u = it % U;
      const uint32_t b4 = (q >> lD) << (lD + 2), a = b4 + (q & (D - 1));
      uint32_t* p = lds + a * 16 + u;
      uint32_t v0 = p[0], v1 = p[D * 16], v2 = p[2 * D * 16], v3 = p[3 * D * 16];
      mad(v0, v2, b4 + 2 * D - 1); v2 ^= v0;
      mad(v1, v3, b4 + 2 * D - 1); v3 ^= v1;
      mad(v0, v1, b4 + D - 1); v1 ^= v0;
      mad(v2, v3, b4 + 3 * D - 1); v3 ^= v2;
      p[0] = v0; p[D * 16] = v1; p[2 * D * 16] = v2; p[3 * D * 16] = v3;
    }
    __syncthreads();
  }
  for (uint32_t it = threadIdx.x; it < n * U; it += blockDim.x) {
    const uint32_t i = it / U, u = it % U;
    if (!pres[i]) lds[i * 16 + u] = gf8_mul4(lds[i * 16 + u], tab(lmul + ((255u - err[i]) % 255u) * 5));
  }
  __syncthreads();
}

// grid: x = axis, y = 64-byte chunk. shards: [naxes][2m][len] in rsmt2d order
// (data then parity); present: [naxes][2m].
template <bool GF16>
__global__ __launch_bounds__(256) void k_rs_decode(uint8_t* shards, const uint8_t* present, uint32_t m,
                                                   uint32_t len, const uint16_t* __restrict__ gexp,
                                                   const uint16_t* __restrict__ glog,
                                                   const uint16_t* __restrict__ gskew,
                                                   const uint32_t* __restrict__ tw8,
                                                   const uint32_t* __restrict__ mul8) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const uint32_t n = 2 * m;
  uint32_t* err = lds + n * 16;
  uint32_t* ltw = err + 2 * n;      // (err + n: n words of error-locator scratch)
  uint32_t* lmul = ltw + 255 * 5;   // GF(2^8): [255][5] twiddle tables, [256][5] by log value
  uint8_t* pres = reinterpret_cast<uint8_t*>(GF16 ? ltw : lmul + 256 * 5);
  if (!GF16) {
    for (uint32_t i = threadIdx.x; i < 255 * 5; i += blockDim.x) ltw[i] = tw8[(i / 5) * 8 + i % 5];
    for (uint32_t i = threadIdx.x; i < 256 * 5; i += blockDim.x) lmul[i] = mul8[(i / 5) * 8 + i % 5];
  }
  __shared__ uint8_t s_log[256];
  uint8_t* axis = shards + (uint64_t)blockIdx.x * n * len;
  const uint8_t* pa = present + (uint64_t)blockIdx.x * n;
  // position p in Leopard order: p < m -> parity shard p (rsmt2d index m + p); else data p - m.
  for (uint32_t p = threadIdx.x; p < n; p += blockDim.x) pres[p] = pa[p < m ? m + p : p - m] ? 1 : 0;
  if (!GF16) {
    for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) {
      s_log[i] = c_gf8.log[i];
    }
  }
  __syncthreads();
  // Error locator err[i] = sum_{e erased} log0[i ^ e] (mod MOD), an XOR convolution of
  // the erasure indicator with log0: FWHT both, multiply pointwise, FWHT back and scale
  // by 1/n = 2^(bits - log2 n) (2^bits = 1 mod MOD) - Leopard's own FWHT route, O(n log n)
  // instead of the O(n^2) direct sum.
  {
    constexpr uint32_t MOD = GF16 ? 65535u : 255u;
    constexpr uint32_t BITS = GF16 ? 16u : 8u;
    uint32_t* tl = err + n;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
      err[i] = pres[i] ? 0u : 1u;
      tl[i] = i == 0 ? 0u : (GF16 ? (uint32_t)glog[i] : (uint32_t)s_log[i]);
    }
    __syncthreads();
    const uint32_t lgn = 31u - __builtin_clz(n);
    auto fwht = [&](uint32_t* v0, uint32_t* v1) {
      for (uint32_t lh = 0; lh < lgn; lh++) {
        const uint32_t h = 1u << lh;
        for (uint32_t j = threadIdx.x; j < n / 2; j += blockDim.x) {
          const uint32_t a = ((j >> lh) << (lh + 1)) | (j & (h - 1)), b = a + h;
          uint32_t x = v0[a], y = v0[b];
          v0[a] = (x + y >= MOD) ? x + y - MOD : x + y;
          v0[b] = (x >= y) ? x - y : x + MOD - y;
          if (v1) {
            x = v1[a];
            y = v1[b];
            v1[a] = (x + y >= MOD) ? x + y - MOD : x + y;
            v1[b] = (x >= y) ? x - y : x + MOD - y;
          }
        }
        __syncthreads();
      }
    };
    fwht(err, tl);
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) err[i] = (err[i] * tl[i]) % MOD;
    __syncthreads();
    fwht(err, nullptr);
    const uint32_t inv_n = (1u << (BITS - lgn)) % MOD;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) err[i] = (err[i] * inv_n) % MOD;
  }
  // the error locator and the staged tables serve every 64-byte chunk of the axis this
  // workgroup takes (chunks blockIdx.y, blockIdx.y + gridDim.y, ...)
  for (uint32_t chunk = blockIdx.y; chunk < len / 64u; chunk += gridDim.y) {
    const uint32_t coff = chunk * 64u;
    __syncthreads();  // the previous chunk's stores have read the LDS image
    for (uint32_t it = threadIdx.x; it < n * 4; it += blockDim.x) {
      const uint32_t p = it >> 2, q = it & 3;
      const uint32_t r = p < m ? m + p : p - m;
      reinterpret_cast<uint4*>(lds)[it] = reinterpret_cast<const uint4*>(axis + (uint64_t)r * len + coff)[q];
    }
    __syncthreads();
    if (GF16) {
      Gf16Ops ops{gexp, glog};
      decode_chunk(ops, lds, err, pres, m, [&](uint32_t i) { return (uint32_t)gskew[i]; });
    } else {
      decode_chunk_gf8p(lds, err, pres, m, ltw, lmul);
    }
    for (uint32_t it = threadIdx.x; it < n * 4; it += blockDim.x) {
      const uint32_t p = it >> 2, q = it & 3;
      if (pres[p]) continue;
      const uint32_t r = p < m ? m + p : p - m;
      reinterpret_cast<uint4*>(axis + (uint64_t)r * len + coff)[q] = reinterpret_cast<const uint4*>(lds)[it];
    }
  }
}

size_t decode_workspace_size(uint32_t, uint32_t) { return 0; }

hipError_t launch_rs_decode(uint8_t* shards, const uint8_t* present, uint32_t naxes, uint32_t m, uint32_t len,
                            const DeviceTables& t, void*, hipStream_t s) {
  if (!naxes) return hipSuccess;
  hipError_t e = ensure_gf8_const();
  if (e != hipSuccess) return e;
  const uint32_t n = 2 * m;
  const size_t lds = (size_t)n * 64 + (size_t)n * 8 + n + (2 * m <= 256 ? (255 + 256) * 5 * 4 : 0);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  // chunks per workgroup (CEL_DEC_CPW, default 2): the per-axis setup (error locator,
  // table staging) is shared by that many 64-byte chunks
  static const uint32_t cpw = [] {
    const char* e = getenv("CEL_DEC_CPW");
    const int v = e ? atoi(e) : 2;
    return (uint32_t)(v < 1 ? 1 : v);
  }();
  const uint32_t nch = len / 64;
  dim3 grid(naxes, (nch + cpw - 1) / cpw);
  if (lds > 64 * 1024) {
    (void)hipFuncSetAttribute((const void*)k_rs_decode<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)hipFuncSetAttribute((const void*)k_rs_decode<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  }
  if (2 * m <= 256)
    hipLaunchKernelGGL(k_rs_decode<false>, grid, dim3(256), lds, s, shards, present, m, len, t.exp16, t.log16,
                       t.skew16, t.tw8, t.mul8);
  else
    hipLaunchKernelGGL(k_rs_decode<true>, grid, dim3(256), lds, s, shards, present, m, len, t.exp16, t.log16,
                       t.skew16, t.tw8, t.mul8);
  return hipGetLastError();
}

}  // namespace cel
