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
// GF(2^16) runs in rs_gf16x.hip (encode, 256/512 data shards) and rs_decode_gf16.hip
// (decode; encode of 1024/2048 shards). The GF(2^8) LDS decoder below takes the axes the
// register decoder (rs_decode_axis.hip) does not.
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

hipError_t upload_tables(DeviceTables* t) {
  const LeoField& f8 = leo_gf8();
  const LeoField& f16 = leo_gf16();
  std::vector<uint32_t> tw(255 * 8), mul8(256 * 8);
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
  // GF(2^16) decoder (rs_decode_gf16.hip): products in the tower basis b_i = prod over the
  // set bits k of i of gamma_k = beta_{2^k} (Cantor basis elements), in which a product by
  // an element of the subfield GF(2^(2^J)) = span(beta_0 .. beta_{2^J - 1}) maps each
  // block of 2^J consecutive coordinates onto itself. v[i]: Cantor representation of b_i;
  // tinv: Cantor representation -> tower coordinates.
  std::vector<uint16_t> v(16), tinv(65536), tower(512 + 16);
  for (uint32_t i = 0; i < 16; i++) {
    uint32_t x = 1;
    for (uint32_t k = 0; k < 4; k++)
      if (i >> k & 1) x = f16.mul(x, 1u << (1u << k));
    v[i] = (uint16_t)x;
  }
  {
    std::vector<uint8_t> seen(65536, 0);
    for (uint32_t c = 0; c < 65536; c++) {
      uint32_t r = 0;
      for (uint32_t i = 0; i < 16; i++)
        if (c >> i & 1) r ^= v[i];
      if (seen[r]) return hipErrorInvalidValue;  // not a basis
      seen[r] = 1;
      tinv[r] = (uint16_t)c;
    }
  }
  for (uint32_t u = 0; u < 256; u++) {
    tower[u] = tinv[u];
    tower[256 + u] = tinv[u << 8];
  }
  for (uint32_t i = 0; i < 16; i++) tower[512 + i] = v[i];
  // twiddle skew[s] (s < 4095: decoder n <= 2048 points at offset 0, encoder m <= 2048 at
  // offset m): P_i = c * b_i in tower coordinates, two per dword; the zero-twiddle sentinel
  // gives zeros
  constexpr uint32_t kTw16 = 4095;
  std::vector<uint32_t> tw16(kTw16 * 8, 0);
  for (uint32_t i = 0; i < kTw16; i++)
    for (uint32_t b = 0; b < 16; b++)
      if (f16.skew[i] != f16.mod) tw16[i * 8 + b / 2] |= (uint32_t)tinv[f16.mul_log(v[b], f16.skew[i])] << (16 * (b & 1));
  // the kernels run layer ld of a 2^lgn-point transform at offset off with blocks of 2^J
  // coordinates, J = decode16_level(log2(off + 2^lgn) - ld): every such twiddle must keep
  // its blocks. (lgn, offset): decoder (9..11, 0); encoder IFFT (10..11, 2^lgn), FFT (10..11, 0).
  struct Tr {
    uint32_t lgn, off;
  };
  const Tr trs[] = {{9, 0}, {10, 0}, {11, 0}, {10, 1024}, {11, 2048}};
  for (const Tr& tr : trs) {
    const uint32_t rb = tr.off ? tr.lgn + 1 : tr.lgn;
    for (uint32_t ld = 0; ld < tr.lgn; ld++) {
      const uint32_t J = decode16_level(rb - ld);
      for (uint32_t base = 0; base < (1u << tr.lgn); base += 2u << ld) {
        const uint32_t s = tr.off + base + (1u << ld) - 1;
        for (uint32_t b = 0; b < 16; b++) {
          const uint32_t blk = ((1u << (1u << J)) - 1) << ((b >> J) << J);
          if ((tw16[s * 8 + b / 2] >> (16 * (b & 1)) & 0xFFFF) & ~blk) return hipErrorInvalidValue;
        }
      }
    }
  }
  hipError_t e;
  if ((e = hipMalloc(&t->tw16, tw16.size() * 4)) != hipSuccess) return e;
  if ((e = hipMemcpy(t->tw16, tw16.data(), tw16.size() * 4, hipMemcpyHostToDevice)) != hipSuccess) return e;
  if ((e = hipMalloc(&t->tower16, tower.size() * 2)) != hipSuccess) return e;
  if ((e = hipMemcpy(t->tower16, tower.data(), tower.size() * 2, hipMemcpyHostToDevice)) != hipSuccess) return e;
  if ((e = hipMalloc(&t->tw8, tw.size() * 4)) != hipSuccess) return e;
  if ((e = hipMalloc(&t->mul8, mul8.size() * 4)) != hipSuccess) return e;
  if ((e = hipMalloc(&t->exp16, 65536 * 2)) != hipSuccess) return e;
  if ((e = hipMalloc(&t->log16, 65536 * 2)) != hipSuccess) return e;
  if ((e = hipMemcpy(t->tw8, tw.data(), tw.size() * 4, hipMemcpyHostToDevice)) != hipSuccess) return e;
  if ((e = hipMemcpy(t->mul8, mul8.data(), mul8.size() * 4, hipMemcpyHostToDevice)) != hipSuccess) return e;
  if ((e = hipMemcpy(t->exp16, f16.exp.data(), 65536 * 2, hipMemcpyHostToDevice)) != hipSuccess) return e;
  if ((e = hipMemcpy(t->log16, f16.log.data(), 65536 * 2, hipMemcpyHostToDevice)) != hipSuccess) return e;
  return hipSuccess;
}

void free_tables(DeviceTables* t) {
  (void)hipFree(t->tw8);
  (void)hipFree(t->mul8);
  (void)hipFree(t->exp16);
  (void)hipFree(t->log16);
  (void)hipFree(t->tw16);
  (void)hipFree(t->tower16);
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

// 4 parallel GF(2^8) products y*c with c given by its product tables.
__device__ __forceinline__ uint32_t gf8_mul4(uint32_t y, const PermTab& t) {
  const uint32_t s0 = y & 0x07070707u;
  const uint32_t s1 = (y >> 3) & 0x07070707u;
  const uint32_t s2 = (y >> 6) & 0x03030303u;
  // v_bitop3 0x96 = three-input xor (gfx950)
  return __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_perm(t.t0h, t.t0l, s0), __builtin_amdgcn_perm(t.t1h, t.t1l, s1),
                                     __builtin_amdgcn_perm(0u, t.t2, s2), 0x96);
}

// GF(2^8) (2n <= 256): bit-sliced for n <= 16 (rs_bitslice.hip), one wave per axis slice
// for n >= 32 (rs_axis.hip: k = 128, 32 squares, 15.2 us/square against 18.1 for the
// workgroup-per-slice v_perm kernel this replaced, profiles/r1_axis_ab.txt).
// GF(2^16): the constant-twiddle register kernel for n = 256, 512 (rs_gf16x.hip); the
// bit-plane kernel for n = 1024, 2048 (rs_decode_gf16.hip; codec API only: squares stop at
// k = 512).
hipError_t launch_rs_encode(const RsGeom& g, const DeviceTables& t, hipStream_t s) {
  if (g.axes == 0 || g.nsq == 0) return hipSuccess;
  if (g.blk_log && !((g.n == 256 || g.n == 512) && g.len % 512 == 0)) return hipErrorInvalidValue;
  if (2 * g.n <= 256) {
    if (g.chk_flags) return hipErrorInvalidValue;
    return g.n <= 16 ? launch_rs_encode_bitslice(g, s) : launch_rs_encode_axis(g, s);
  }
  if (g.n > kMaxGf16Width || g.len % 64 != 0) return hipErrorInvalidValue;
  if (g.n == 256 || g.n == 512) return launch_rs_encode_gf16x(g, s);
  if (g.chk_flags) return hipErrorInvalidValue;  // check mode: the register kernel only
  return launch_rs_encode_gf16p(g, t, s);  // n = 1024, 2048 (no data copy, linear placement)
}

// Row pass of the extension, Q0 rows -> Q1. Q0 is read from `ods` (and copied into the
// EDS by the row pass) when ods != nullptr, else from the EDS itself.
static RsGeom row_geom(const uint8_t* ods, uint8_t* eds, uint32_t k, uint32_t nsq) {
  const uint64_t row = (uint64_t)2 * k * kShare;  // bytes per EDS row
  const uint64_t sq_eds = (uint64_t)4 * k * k * kShare;
  const uint64_t sq_ods = (uint64_t)k * k * kShare;
  RsGeom r{};
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
  return r;
}

// columns of [Q0|Q1] -> [Q2|Q3] (all 2k columns, after every row)
static RsGeom col_geom(uint8_t* eds, uint32_t k, uint32_t nsq) {
  const uint64_t row = (uint64_t)2 * k * kShare;  // bytes per EDS row
  RsGeom cols{};
  cols.in = eds;
  cols.in_sq = (uint64_t)4 * k * k * kShare;
  cols.in_axis = kShare;
  cols.in_shard = row;
  cols.out = eds + (uint64_t)k * row;
  cols.out_sq = cols.in_sq;
  cols.out_axis = kShare;
  cols.out_shard = row;
  cols.n = k;
  cols.len = kShare;
  cols.axes = 2 * k;
  cols.nsq = nsq;
  return cols;
}

hipError_t launch_extend(const uint8_t* ods, uint8_t* eds, uint32_t k, uint32_t nsq, const DeviceTables& t,
                         hipStream_t s) {
  if (nsq == 0) return hipSuccess;
  hipError_t e;
  if (!ods && k >= 32 && k <= kMaxGf8Width) {
    // GF(2^8) in place: Q0 rows -> Q1 beside Q0 columns -> Q2 (one launch, each Q0 line read
    // from HBM once), then Q1 columns -> Q3 (rs_axis.hip, k_rs_axis_gf8_pair)
    const uint64_t half = (uint64_t)k * kShare;
    RsGeom c0 = col_geom(eds, k, nsq), c1 = c0;
    c0.axes = c1.axes = k;
    c1.in += half;
    c1.out += half;
    {
      const Range r("rs.rows+q0cols");
      if ((e = launch_rs_encode_axis_pair(row_geom(nullptr, eds, k, nsq), c0, s)) != hipSuccess) return e;
    }
    const Range r("rs.q1cols");
    return launch_rs_encode(c1, t, s);
  }
  // Q0 rows -> Q1 (reading the ODS and writing Q0 into the EDS on the way when ods != nullptr)
  {
    const Range r("rs.rows");
    if ((e = launch_rs_encode(row_geom(ods, eds, k, nsq), t, s)) != hipSuccess) return e;
  }
  const Range r("rs.cols");
  return launch_rs_encode(col_geom(eds, k, nsq), t, s);
}

hipError_t launch_extend_rows(uint8_t* eds, uint32_t k, uint32_t row0, uint32_t row1, const DeviceTables& t,
                              hipStream_t s, const uint8_t* ods) {
  RsGeom g = row_geom(ods, eds, k, 1);
  const uint64_t off = (uint64_t)row0 * 2 * k * kShare;
  g.in += ods ? (uint64_t)row0 * k * kShare : off;
  if (ods) g.dcopy += off;
  g.out += off;
  g.axes = row1 - row0;
  const Range r("rs.rows");
  return launch_rs_encode(g, t, s);
}

hipError_t launch_extend_cols(uint8_t* eds, uint32_t k, uint32_t nsq, const DeviceTables& t, hipStream_t s) {
  const Range r("rs.cols");
  return launch_rs_encode(col_geom(eds, k, nsq), t, s);
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

// GF(2^8) decode of one 64-byte chunk with v_perm product tables staged in LDS
// (ltw: twiddle tables by skew index, lmul: tables by log value; 5 dwords each): the
// transform above.
// Layers go two at a time (radix 4: a thread owns one dword of four points, half the
// LDS round trips and barriers of radix 2); the formal derivative reads every source
// before one barrier and writes after it.
// Compile-time loop: f(std::integral_constant<uint32_t, 0>) .. f(..., N - 1>).
template <uint32_t N, uint32_t I = 0, class F>
__device__ __forceinline__ void sfor_u(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<uint32_t, I>{});
    sfor_u<N, I + 1>(f);
  }
}

// Items [0, C) of a 256-thread workgroup, unrolled (C compile-time): item it goes to
// thread it % 256. A fixed trip count lets the compiler issue all of a thread's LDS loads
// of a layer before its multiplies (the decode is latency-bound: barriered layers).
template <uint32_t C, class F>
__device__ __forceinline__ void for_items(F&& f) {
#pragma unroll
  for (uint32_t r = 0; r < (C + 255) / 256; r++) {
    const uint32_t it = threadIdx.x + 256u * r;
    if (C % 256 == 0 || it < C) f(it);
  }
}

template <uint32_t N>
__device__ void decode_chunk_gf8p(uint32_t* lds, const uint32_t* err, const uint8_t* pres, const uint32_t* ltw,
                                  const uint32_t* lmul) {
  constexpr uint32_t n = N;
  constexpr uint32_t lgn = __builtin_ctz(N);
  constexpr uint32_t U = 16;  // dwords per 64-byte chunk
  // a table is 8 dwords in LDS (5 used): one ds_read_b128 + one ds_read_b32
  auto tab = [](const uint32_t* t) {
    const uint4 a = *reinterpret_cast<const uint4*>(t);
    return PermTab{a.x, a.y, a.z, a.w, t[4]};
  };
  // x ^= c(idx) * y; the zero twiddle's table is all zeros, so no branch
  auto mad = [&](uint32_t& x, uint32_t y, uint32_t idx) { x ^= gf8_mul4(y, tab(ltw + idx * 8)); };
  for_items<n * U>([&](uint32_t it) {
    const uint32_t i = it / U, u = it % U;
    if (pres[i]) lds[i * 16 + u] = gf8_mul4(lds[i * 16 + u], tab(lmul + err[i] * 8));
  });
  __syncthreads();
  // IFFT (offset 0): layers D = 1, 2, 4, ...; butterfly y ^= x; x ^= c*y
  sfor_u<lgn / 2>([&](auto li) {
    constexpr uint32_t lD = 2 * decltype(li)::value, D = 1u << lD;
    for_items<(n / 4) * U>([&](uint32_t it) {
      const uint32_t q = it / U, u = it % U;
      const uint32_t b4 = (q >> lD) << (lD + 2), a = b4 + (q & (D - 1));
      uint32_t* p = lds + a * 16 + u;
      uint32_t v0 = p[0], v1 = p[D * 16], v2 = p[2 * D * 16], v3 = p[3 * D * 16];
      v1 ^= v0; mad(v0, v1, b4 + D - 1);
      v3 ^= v2; mad(v2, v3, b4 + 3 * D - 1);
      v2 ^= v0; mad(v0, v2, b4 + 2 * D - 1);
      v3 ^= v1; mad(v1, v3, b4 + 2 * D - 1);
      p[0] = v0; p[D * 16] = v1; p[2 * D * 16] = v2; p[3 * D * 16] = v3;
    });
    __syncthreads();
  });
  if constexpr (lgn & 1) {  // odd log2(n): one radix-2 layer left
    constexpr uint32_t lD = lgn - 1, D = 1u << lD;
    for_items<(n / 2) * U>([&](uint32_t it) {
      const uint32_t pair = it / U, u = it % U;
      const uint32_t base = (pair >> lD) << (lD + 1), a = base + (pair & (D - 1));
      uint32_t x = lds[a * 16 + u], y = lds[(a + D) * 16 + u];
      y ^= x;
      mad(x, y, base + D - 1);
      lds[a * 16 + u] = x;
      lds[(a + D) * 16 + u] = y;
    });
    __syncthreads();
  }
  {  // formal derivative: new[x] = old[x] ^ xor_{t: bit t of x clear, x + 2^t < n} old[x + 2^t]
    constexpr uint32_t kItems = (n * U + 255) / 256;
    uint32_t acc[kItems];
#pragma unroll
    for (uint32_t r = 0; r < kItems; r++) {
      const uint32_t it = threadIdx.x + r * 256u;
      acc[r] = 0;
      if ((n * U) % 256 == 0 || it < n * U) {
        const uint32_t x = it / U, u = it % U;
#pragma unroll
        for (uint32_t t = 1; t < n; t <<= 1)
          if ((x & t) == 0 && x + t < n) acc[r] ^= lds[(x + t) * 16 + u];
      }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t r = 0; r < kItems; r++) {
      const uint32_t it = threadIdx.x + r * 256u;
      if ((n * U) % 256 == 0 || it < n * U) lds[(it / U) * 16 + it % U] ^= acc[r];
    }
    __syncthreads();
  }
  // FFT: layers D = n/2, ..., 1; butterfly x ^= c*y; y ^= x
  if constexpr (lgn & 1) {  // odd log2(n): the top layer alone
    constexpr uint32_t lD = lgn - 1, D = 1u << lD;
    for_items<(n / 2) * U>([&](uint32_t it) {
      const uint32_t pair = it / U, u = it % U;
      const uint32_t base = (pair >> lD) << (lD + 1), a = base + (pair & (D - 1));
      uint32_t x = lds[a * 16 + u], y = lds[(a + D) * 16 + u];
      mad(x, y, base + D - 1);
      y ^= x;
      lds[a * 16 + u] = x;
      lds[(a + D) * 16 + u] = y;
    });
    __syncthreads();
  }
  sfor_u<lgn / 2>([&](auto li) {
    constexpr uint32_t lD = 2 * (lgn / 2 - 1 - decltype(li)::value), D = 1u << lD;  // layers 2D then D
    for_items<(n / 4) * U>([&](uint32_t it) {
      const uint32_t q = it / U, u = it % U;
      const uint32_t b4 = (q >> lD) << (lD + 2), a = b4 + (q & (D - 1));
      uint32_t* p = lds + a * 16 + u;
      uint32_t v0 = p[0], v1 = p[D * 16], v2 = p[2 * D * 16], v3 = p[3 * D * 16];
      mad(v0, v2, b4 + 2 * D - 1); v2 ^= v0;
      mad(v1, v3, b4 + 2 * D - 1); v3 ^= v1;
      mad(v0, v1, b4 + D - 1); v1 ^= v0;
      mad(v2, v3, b4 + 3 * D - 1); v3 ^= v2;
      p[0] = v0; p[D * 16] = v1; p[2 * D * 16] = v2; p[3 * D * 16] = v3;
    });
    __syncthreads();
  });
  for_items<n * U>([&](uint32_t it) {
    const uint32_t i = it / U, u = it % U;
    if (!pres[i]) lds[i * 16 + u] = gf8_mul4(lds[i * 16 + u], tab(lmul + ((255u - err[i]) % 255u) * 8));
  });
  __syncthreads();
}

// grid: x = axis, y = 64-byte chunk. shards: [naxes][2m][len] in rsmt2d order
// (data then parity); present: [naxes][2m].
// GF(2^8) axes the register decoder does not take (2m = 2..256 points; m < 16 or a chunk
// tail). GF(2^16): rs_decode_gf16.hip.
template <uint32_t N8>
__global__ __launch_bounds__(256) void k_rs_decode(uint8_t* shards, const uint8_t* present, uint32_t m,
                                                   uint32_t len, const uint32_t* __restrict__ tw8,
                                                   const uint32_t* __restrict__ mul8) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const uint32_t n = 2 * m;
  uint32_t* err = lds + n * 16;
  uint32_t* ltw = err + 2 * n;      // (err + n: n words of error-locator scratch)
  uint32_t* lmul = ltw + 256 * 8;   // GF(2^8): [255][8] twiddle tables, [256][8] by log value (16-B aligned)
  uint8_t* pres = reinterpret_cast<uint8_t*>(lmul + 256 * 8);
  for (uint32_t i = threadIdx.x; i < 255 * 2; i += blockDim.x)
    reinterpret_cast<uint4*>(ltw)[i] = reinterpret_cast<const uint4*>(tw8)[i];
  for (uint32_t i = threadIdx.x; i < 256 * 2; i += blockDim.x)
    reinterpret_cast<uint4*>(lmul)[i] = reinterpret_cast<const uint4*>(mul8)[i];
  __shared__ uint8_t s_log[256];
  uint8_t* axis = shards + (uint64_t)blockIdx.x * n * len;
  const uint8_t* pa = present + (uint64_t)blockIdx.x * n;
  // position p in Leopard order: p < m -> parity shard p (rsmt2d index m + p); else data p - m.
  for (uint32_t p = threadIdx.x; p < n; p += blockDim.x) pres[p] = pa[p < m ? m + p : p - m] ? 1 : 0;
  for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) s_log[i] = c_gf8.log[i];
  __syncthreads();
  // Error locator err[i] = sum_{e erased} log0[i ^ e] (mod MOD), an XOR convolution of
  // the erasure indicator with log0: FWHT both, multiply pointwise, FWHT back and scale
  // by 1/n = 2^(bits - log2 n) (2^bits = 1 mod MOD) - Leopard's own FWHT route, O(n log n)
  // instead of the O(n^2) direct sum.
  {
    constexpr uint32_t MOD = 255u;
    constexpr uint32_t BITS = 8u;
    uint32_t* tl = err + n;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
      err[i] = pres[i] ? 0u : 1u;
      tl[i] = i == 0 ? 0u : (uint32_t)s_log[i];
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
    // erased points enter the transform as zero (work[i] = 0), whatever bytes the
    // caller's buffer holds there ("missing cells may hold anything")
    for (uint32_t it = threadIdx.x; it < n * 4; it += blockDim.x) {
      const uint32_t p = it >> 2, q = it & 3;
      const uint32_t r = p < m ? m + p : p - m;
      reinterpret_cast<uint4*>(lds)[it] =
          pres[p] ? reinterpret_cast<const uint4*>(axis + (uint64_t)r * len + coff)[q] : uint4{0, 0, 0, 0};
    }
    __syncthreads();
    decode_chunk_gf8p<N8>(lds, err, pres, ltw, lmul);
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
  const uint32_t n = 2 * m;
  if (rs_decode_axis_supported(n, len)) return launch_rs_decode_axis(shards, present, naxes, n, len, t.mul8, s);
  if (rs_decode_gf16_supported(n)) return launch_rs_decode_gf16(shards, present, naxes, n, len, t, s);
  if (n > 256 || len == 0 || len % 64) return hipErrorInvalidValue;
  hipError_t e = ensure_gf8_const();
  if (e != hipSuccess) return e;
  const size_t lds = (size_t)n * 64 + (size_t)n * 8 + n + (256 + 256) * 8 * 4;
  // 2 chunks per workgroup: the per-axis setup (error locator, table staging) is shared
  // by both 64-byte chunks (1 and 4 measured slower, profiles/r1j_repair_cpw_ab.txt)
  constexpr uint32_t cpw = 2;
  const uint32_t nch = len / 64;
  dim3 grid(naxes, (nch + cpw - 1) / cpw);
  auto go = [&](auto kern) {
    if (lds > 64 * 1024)
      (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, grid, dim3(256), lds, s, shards, present, m, len, t.tw8, t.mul8);
  };
  switch (n) {  // the point count is a template constant (unrolled layers)
    case 2: go(k_rs_decode<2>); break;
    case 4: go(k_rs_decode<4>); break;
    case 8: go(k_rs_decode<8>); break;
    case 16: go(k_rs_decode<16>); break;
    case 32: go(k_rs_decode<32>); break;
    case 64: go(k_rs_decode<64>); break;
    case 128: go(k_rs_decode<128>); break;
    default: go(k_rs_decode<256>); break;
  }
  return hipGetLastError();
}

}  // namespace cel
