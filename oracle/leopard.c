/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.h). Never linked by the product.
 *
 * CPU restatement of Leopard Reed-Solomon as used by the reference:
 *   rsmt2d v0.14.0 LeoRSCodec (pkg/appconsts/global_consts.go:92 DefaultCodec)
 *   -> klauspost/reedsolomon v1.12.1 New(k, k, WithLeopardGF(true))
 *      leopard8.go  (GF(2^8),  total shards <= 256)   [dep, not in /root/reference]
 *      leopard.go   (GF(2^16), total shards  > 256)   [dep, not in /root/reference]
 * The algorithm text followed is SURVEY.md Appendix A.2 / A.3 (restated from the
 * pinned dependency and verified there against mainnet block 408's data root).
 *
 * Decoding restates Leopard's error-locator decoder (klauspost reconstruct with
 * recoverAll), so it matches klauspost Reconstruct also on shards that are not a
 * codeword (byzantine squares), where decoders of the same code differ.
 */
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#if defined(__x86_64__)
#include <immintrin.h>
#endif
#include "oracle.h"
#include "oracle_internal.h"

/* ---------------------------------------------------------------- tables */

static const uint16_t kCantor8[8] = {1, 214, 152, 146, 86, 200, 88, 230};
static const uint16_t kCantor16[16] = {0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E,
                                       0x914C, 0x4012, 0x6C98, 0x10D8, 0x6A72, 0xB900,
                                       0xFDB8, 0xFB34, 0xFF38, 0x991E};

gf_t g_gf8, g_gf16;
static int g_inited = 0;
int g_simd = 0;

static inline uint32_t add_mod(const gf_t* f, uint32_t a, uint32_t b) {
  /* klauspost addMod: partial reduction, result may equal MOD (== 0 mod MOD). */
  uint32_t s = a + b;
  return (s + (s >> f->bits)) & f->mod;
}

uint32_t gf_mul_log(const gf_t* f, uint32_t a, uint32_t log_b) {
  if (a == 0) return 0;
  return f->exp[add_mod(f, f->log[a], log_b)];
}

static void gf_build(gf_t* f, int bits, uint32_t poly, const uint16_t* cantor) {
  f->bits = bits;
  f->order = 1u << bits;
  f->mod = f->order - 1;
  f->exp = (uint16_t*)calloc(f->order, sizeof(uint16_t));
  f->log = (uint16_t*)calloc(f->order, sizeof(uint16_t));
  f->skew = (uint16_t*)calloc(f->mod, sizeof(uint16_t));
  uint16_t* exp = f->exp;
  uint16_t* lg = f->log;
  /* LFSR table: exp temporarily holds logs of polynomial-basis elements. */
  uint32_t st = 1;
  for (uint32_t i = 0; i < f->mod; i++) {
    exp[st] = (uint16_t)i;
    st <<= 1;
    if (st >= f->order) st ^= poly;
  }
  exp[0] = (uint16_t)f->mod;
  /* Cantor basis conversion. */
  lg[0] = 0;
  for (int i = 0; i < bits; i++) {
    uint32_t w = 1u << i;
    for (uint32_t j = 0; j < w; j++) lg[j + w] = lg[j] ^ cantor[i];
  }
  for (uint32_t i = 0; i < f->order; i++) lg[i] = exp[lg[i]];
  for (uint32_t i = 0; i < f->order; i++) exp[lg[i]] = (uint16_t)i;
  exp[f->mod] = exp[0];

  /* FFT skew factors. */
  uint32_t temp[16];
  for (int i = 1; i < bits; i++) temp[i - 1] = 1u << i;
  uint16_t* skew = f->skew;
  for (int m = 0; m < bits - 1; m++) {
    uint32_t step = 1u << (m + 1);
    skew[(1u << m) - 1] = 0;
    for (int i = m; i < bits - 1; i++) {
      uint32_t s = 1u << (i + 1);
      for (uint32_t j = (1u << m) - 1; j < s; j += step) skew[j + s] = skew[j] ^ (uint16_t)temp[i];
    }
    temp[m] = f->mod - lg[gf_mul_log(f, temp[m], lg[temp[m] ^ 1])];
    for (int i = m + 1; i < bits - 1; i++) {
      uint32_t sum = add_mod(f, lg[temp[i] ^ 1], temp[m]);
      temp[i] = gf_mul_log(f, temp[i], sum);
    }
  }
  for (uint32_t i = 0; i < f->mod; i++) skew[i] = lg[skew[i]];
}

/* Nibble product tables for the SIMD (baseline) path. */
static uint8_t (*g_lut8)[2][16];   /* [256 log][lo/hi][16] */
/* GF2P8AFFINEQB matrices of y -> y * exp(lm): a product by a constant is GF(2)-linear on
 * the 8 bits of y in any representation (Leopard's Cantor basis included), so one affine
 * instruction multiplies 64 bytes (klauspost's GFNI kernels do the same). */
static uint64_t g_aff8[256];
static int g_gfni = 0;
static uint8_t (*g_lut16)[8][16];  /* [65536 log][q*2 + outbyte][16] */

static void build_aff8(void) {
  for (uint32_t lm = 0; lm < 256; lm++) {
    uint64_t a = 0;
    for (int i = 0; i < 8; i++) { /* row of output bit i lives in byte 7 - i */
      uint32_t row = 0;
      for (int b = 0; b < 8; b++) row |= ((gf_mul_log(&g_gf8, 1u << b, lm) >> i) & 1u) << b;
      a |= (uint64_t)row << (8 * (7 - i));
    }
    g_aff8[lm] = a;
  }
}

static void build_lut8(void) {
  g_lut8 = malloc(sizeof(*g_lut8) * 256);
  for (uint32_t lm = 0; lm < 256; lm++)
    for (uint32_t n = 0; n < 16; n++) {
      g_lut8[lm][0][n] = (uint8_t)gf_mul_log(&g_gf8, n, lm);
      g_lut8[lm][1][n] = (uint8_t)gf_mul_log(&g_gf8, n << 4, lm);
    }
}

static void build_lut16(void) {
  uint8_t (*t)[8][16] = malloc(sizeof(*t) * 65536);
#pragma omp parallel for schedule(static)
  for (int lm = 0; lm < 65536; lm++)
    for (int q = 0; q < 4; q++)
      for (uint32_t n = 0; n < 16; n++) {
        uint32_t p = gf_mul_log(&g_gf16, n << (4 * q), (uint32_t)lm);
        t[lm][q * 2 + 0][n] = (uint8_t)(p & 0xFF);
        t[lm][q * 2 + 1][n] = (uint8_t)(p >> 8);
      }
  g_lut16 = t;
}

void orc_init(void) {
  if (g_inited) return;
  gf_build(&g_gf8, 8, 0x11D, kCantor8);
  gf_build(&g_gf16, 16, 0x1002D, kCantor16);
  build_lut8();
  build_aff8();
#if defined(__x86_64__)
  __builtin_cpu_init();
  g_gfni = __builtin_cpu_supports("gfni") && __builtin_cpu_supports("avx512bw") && __builtin_cpu_supports("avx512f");
#endif
  g_inited = 1;
}

int orc_simd_available(void) {
#if defined(__x86_64__)
  __builtin_cpu_init();
  return __builtin_cpu_supports("avx2") ? 1 : 0;
#else
  return 0;
#endif
}

void orc_set_simd(int on) { g_simd = on && orc_simd_available(); }

void orc_set_threads(int n) {
#ifdef _OPENMP
  if (n > 0) omp_set_num_threads(n);
#else
  (void)n;
#endif
}

int orc_get_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

int orc_gf_exp(int field, int i) { orc_init(); return (field == 8 ? g_gf8 : g_gf16).exp[i]; }
int orc_gf_log(int field, int i) { orc_init(); return (field == 8 ? g_gf8 : g_gf16).log[i]; }
int orc_gf_skew(int field, int i) { orc_init(); return (field == 8 ? g_gf8 : g_gf16).skew[i]; }

uint32_t gf_mul(const gf_t* f, uint32_t a, uint32_t b) {
  if (a == 0 || b == 0) return 0;
  return f->exp[(f->log[a] + (uint32_t)f->log[b]) % f->mod];
}

uint32_t gf_inv(const gf_t* f, uint32_t a) { return f->exp[(f->mod - f->log[a]) % f->mod]; }

int orc_gf_mul(int field, int a, int b) {
  orc_init();
  return (int)gf_mul(field == 8 ? &g_gf8 : &g_gf16, (uint32_t)a, (uint32_t)b);
}

/* ------------------------------------------------------- shard operations */

static void xor_shard(uint8_t* restrict dst, const uint8_t* restrict src, size_t len) {
  for (size_t i = 0; i < len; i++) dst[i] ^= src[i];
}

#if defined(__x86_64__)
__attribute__((target("avx2"))) static void muladd8_avx2(uint8_t* x, const uint8_t* y,
                                                          uint32_t lm, size_t len) {
  const __m256i tlo = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i*)g_lut8[lm][0]));
  const __m256i thi = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i*)g_lut8[lm][1]));
  const __m256i mask = _mm256_set1_epi8(0x0F);
  size_t i = 0;
  for (; i + 32 <= len; i += 32) {
    __m256i v = _mm256_loadu_si256((const __m256i*)(y + i));
    __m256i l = _mm256_and_si256(v, mask);
    __m256i h = _mm256_and_si256(_mm256_srli_epi64(v, 4), mask);
    __m256i p = _mm256_xor_si256(_mm256_shuffle_epi8(tlo, l), _mm256_shuffle_epi8(thi, h));
    __m256i o = _mm256_loadu_si256((const __m256i*)(x + i));
    _mm256_storeu_si256((__m256i*)(x + i), _mm256_xor_si256(o, p));
  }
  for (; i < len; i++) x[i] ^= (uint8_t)gf_mul_log(&g_gf8, y[i], lm);
}

__attribute__((target("avx512f,avx512bw,gfni"))) static void muladd8_gfni(uint8_t* x, const uint8_t* y,
                                                                          uint32_t lm, size_t len) {
  const __m512i a = _mm512_set1_epi64((long long)g_aff8[lm]);
  size_t i = 0;
  for (; i + 64 <= len; i += 64) {
    const __m512i p = _mm512_gf2p8affine_epi64_epi8(_mm512_loadu_si512((const void*)(y + i)), a, 0);
    _mm512_storeu_si512((void*)(x + i), _mm512_xor_si512(_mm512_loadu_si512((const void*)(x + i)), p));
  }
  for (; i < len; i++) x[i] ^= (uint8_t)gf_mul_log(&g_gf8, y[i], lm);
}

__attribute__((target("avx2"))) static void muladd16_avx2(uint8_t* x, const uint8_t* y,
                                                           uint32_t lm, size_t len) {
  const uint8_t (*t)[16] = g_lut16[lm];
  __m256i T[8];
  for (int q = 0; q < 8; q++) T[q] = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i*)t[q]));
  const __m256i mask = _mm256_set1_epi8(0x0F);
  for (size_t c = 0; c < len; c += 64) {
    __m256i lo = _mm256_loadu_si256((const __m256i*)(y + c));
    __m256i hi = _mm256_loadu_si256((const __m256i*)(y + c + 32));
    __m256i n0 = _mm256_and_si256(lo, mask);
    __m256i n1 = _mm256_and_si256(_mm256_srli_epi64(lo, 4), mask);
    __m256i n2 = _mm256_and_si256(hi, mask);
    __m256i n3 = _mm256_and_si256(_mm256_srli_epi64(hi, 4), mask);
    __m256i plo = _mm256_xor_si256(
        _mm256_xor_si256(_mm256_shuffle_epi8(T[0], n0), _mm256_shuffle_epi8(T[2], n1)),
        _mm256_xor_si256(_mm256_shuffle_epi8(T[4], n2), _mm256_shuffle_epi8(T[6], n3)));
    __m256i phi = _mm256_xor_si256(
        _mm256_xor_si256(_mm256_shuffle_epi8(T[1], n0), _mm256_shuffle_epi8(T[3], n1)),
        _mm256_xor_si256(_mm256_shuffle_epi8(T[5], n2), _mm256_shuffle_epi8(T[7], n3)));
    __m256i xl = _mm256_loadu_si256((const __m256i*)(x + c));
    __m256i xh = _mm256_loadu_si256((const __m256i*)(x + c + 32));
    _mm256_storeu_si256((__m256i*)(x + c), _mm256_xor_si256(xl, plo));
    _mm256_storeu_si256((__m256i*)(x + c + 32), _mm256_xor_si256(xh, phi));
  }
}
#endif

/* x ^= y * exp(lm), symbol-wise. GF16 shards use the 64-byte lo/hi split layout:
 * sym[j] = b[j] | b[j+32] << 8 inside every 64-byte chunk (klauspost refMulAdd). */
static void muladd_shard(const gf_t* f, uint8_t* x, const uint8_t* y, uint32_t lm, size_t len) {
  if (f->bits == 8) {
#if defined(__x86_64__)
    if (g_simd && g_gfni) { muladd8_gfni(x, y, lm, len); return; }
    if (g_simd) { muladd8_avx2(x, y, lm, len); return; }
#endif
    for (size_t i = 0; i < len; i++) x[i] ^= (uint8_t)gf_mul_log(f, y[i], lm);
  } else {
#if defined(__x86_64__)
    if (g_simd && g_lut16 && (len % 64) == 0) { muladd16_avx2(x, y, lm, len); return; }
#endif
    for (size_t c = 0; c < len; c += 64)
      for (int j = 0; j < 32; j++) {
        uint32_t s = (uint32_t)y[c + j] | ((uint32_t)y[c + 32 + j] << 8);
        uint32_t p = gf_mul_log(f, s, lm);
        x[c + j] ^= (uint8_t)(p & 0xFF);
        x[c + 32 + j] ^= (uint8_t)(p >> 8);
      }
  }
}

/* Leopard butterflies (Appendix A.2). "log_m == MOD => xor only" is mandatory. */
static void ifft2(const gf_t* f, uint8_t* x, uint8_t* y, uint32_t lm, size_t len) {
  xor_shard(y, x, len);
  if (lm != f->mod) muladd_shard(f, x, y, lm, len);
}

static void fft2(const gf_t* f, uint8_t* x, uint8_t* y, uint32_t lm, size_t len) {
  if (lm != f->mod) muladd_shard(f, x, y, lm, len);
  xor_shard(y, x, len);
}

#if defined(__x86_64__)
/* Radix-4 butterflies of one 64-byte column of four shards at distance d, GFNI + AVX-512
 * (klauspost's ifftDIT48 / fftDIT48 GFNI kernels: two layers per pass over memory).
 * A zero matrix stands for log_m == MOD (the butterfly's multiply is skipped). */
static inline uint64_t aff8(uint32_t lm) { return lm == 255u ? 0ull : g_aff8[lm]; }

__attribute__((target("avx512f,avx512bw,gfni"))) static void ifft4_gfni(uint8_t** w, uint32_t i, uint32_t d,
                                                                        uint32_t l01, uint32_t l23, uint32_t l02,
                                                                        size_t len) {
  const __m512i a01 = _mm512_set1_epi64((long long)aff8(l01)), a23 = _mm512_set1_epi64((long long)aff8(l23)),
                a02 = _mm512_set1_epi64((long long)aff8(l02));
  uint8_t *p0 = w[i], *p1 = w[i + d], *p2 = w[i + 2 * d], *p3 = w[i + 3 * d];
  for (size_t c = 0; c < len; c += 64) {
    __m512i v0 = _mm512_loadu_si512(p0 + c), v1 = _mm512_loadu_si512(p1 + c);
    __m512i v2 = _mm512_loadu_si512(p2 + c), v3 = _mm512_loadu_si512(p3 + c);
    v1 = _mm512_xor_si512(v1, v0);
    v0 = _mm512_xor_si512(v0, _mm512_gf2p8affine_epi64_epi8(v1, a01, 0));
    v3 = _mm512_xor_si512(v3, v2);
    v2 = _mm512_xor_si512(v2, _mm512_gf2p8affine_epi64_epi8(v3, a23, 0));
    v2 = _mm512_xor_si512(v2, v0);
    v0 = _mm512_xor_si512(v0, _mm512_gf2p8affine_epi64_epi8(v2, a02, 0));
    v3 = _mm512_xor_si512(v3, v1);
    v1 = _mm512_xor_si512(v1, _mm512_gf2p8affine_epi64_epi8(v3, a02, 0));
    _mm512_storeu_si512(p0 + c, v0);
    _mm512_storeu_si512(p1 + c, v1);
    _mm512_storeu_si512(p2 + c, v2);
    _mm512_storeu_si512(p3 + c, v3);
  }
}

__attribute__((target("avx512f,avx512bw,gfni"))) static void fft4_gfni(uint8_t** w, uint32_t i, uint32_t d,
                                                                       uint32_t l01, uint32_t l23, uint32_t l02,
                                                                       size_t len) {
  const __m512i a01 = _mm512_set1_epi64((long long)aff8(l01)), a23 = _mm512_set1_epi64((long long)aff8(l23)),
                a02 = _mm512_set1_epi64((long long)aff8(l02));
  uint8_t *p0 = w[i], *p1 = w[i + d], *p2 = w[i + 2 * d], *p3 = w[i + 3 * d];
  for (size_t c = 0; c < len; c += 64) {
    __m512i v0 = _mm512_loadu_si512(p0 + c), v1 = _mm512_loadu_si512(p1 + c);
    __m512i v2 = _mm512_loadu_si512(p2 + c), v3 = _mm512_loadu_si512(p3 + c);
    v0 = _mm512_xor_si512(v0, _mm512_gf2p8affine_epi64_epi8(v2, a02, 0));
    v2 = _mm512_xor_si512(v2, v0);
    v1 = _mm512_xor_si512(v1, _mm512_gf2p8affine_epi64_epi8(v3, a02, 0));
    v3 = _mm512_xor_si512(v3, v1);
    v0 = _mm512_xor_si512(v0, _mm512_gf2p8affine_epi64_epi8(v1, a01, 0));
    v1 = _mm512_xor_si512(v1, v0);
    v2 = _mm512_xor_si512(v2, _mm512_gf2p8affine_epi64_epi8(v3, a23, 0));
    v3 = _mm512_xor_si512(v3, v2);
    _mm512_storeu_si512(p0 + c, v0);
    _mm512_storeu_si512(p1 + c, v1);
    _mm512_storeu_si512(p2 + c, v2);
    _mm512_storeu_si512(p3 + c, v3);
  }
}
#endif

/* In-place Leopard encode: work[0..m) holds the m data shards on entry and the m
 * parity shards on exit (klauspost ifftDITEncoder + fftDIT with mtrunc = m). */
void leo_encode_inplace(const gf_t* f, uint32_t m, uint8_t** w, size_t len) {
#if defined(__x86_64__)
  const int fused = f->bits == 8 && g_simd && g_gfni && len % 64 == 0;
#else
  const int fused = 0;
#endif
  const uint16_t* skew = f->skew;
  const uint16_t* sk = skew + (m - 1); /* skewLUT = fftSkew[m-1:] */
  /* IFFT, decimation in time, two layers at a time. */
  uint32_t dist = 1, dist4 = 4;
  while (dist4 <= m) {
    for (uint32_t r = 0; r < m; r += dist4) {
      uint32_t ie = r + dist;
      uint32_t l01 = sk[ie], l02 = sk[ie + dist], l23 = sk[ie + 2 * dist];
#if defined(__x86_64__)
      if (fused) {
        for (uint32_t i = r; i < ie; i++) ifft4_gfni(w, i, dist, l01, l23, l02, len);
        continue;
      }
#endif
      for (uint32_t i = r; i < ie; i++) {
        ifft2(f, w[i], w[i + dist], l01, len);
        ifft2(f, w[i + 2 * dist], w[i + 3 * dist], l23, len);
        ifft2(f, w[i], w[i + 2 * dist], l02, len);
        ifft2(f, w[i + dist], w[i + 3 * dist], l02, len);
      }
    }
    dist = dist4;
    dist4 <<= 2;
  }
  if (dist < m) { /* one layer left, dist == m/2 */
    uint32_t lm = sk[dist];
    for (uint32_t i = 0; i < dist; i++) ifft2(f, w[i], w[i + dist], lm, len);
  }
  /* FFT, decimation in time, two layers at a time. */
  dist4 = m;
  dist = m >> 2;
  while (dist != 0) {
    for (uint32_t r = 0; r < m; r += dist4) {
      uint32_t ie = r + dist;
      uint32_t l01 = skew[ie - 1], l02 = skew[ie + dist - 1], l23 = skew[ie + 2 * dist - 1];
#if defined(__x86_64__)
      if (fused) {
        for (uint32_t i = r; i < ie; i++) fft4_gfni(w, i, dist, l01, l23, l02, len);
        continue;
      }
#endif
      for (uint32_t i = r; i < ie; i++) {
        fft2(f, w[i], w[i + 2 * dist], l02, len);
        fft2(f, w[i + dist], w[i + 3 * dist], l02, len);
        fft2(f, w[i], w[i + dist], l01, len);
        fft2(f, w[i + 2 * dist], w[i + 3 * dist], l23, len);
      }
    }
    dist4 = dist;
    dist >>= 2;
  }
  if (dist4 == 2) {
    for (uint32_t r = 0; r < m; r += 2) fft2(f, w[r], w[r + 1], skew[r], len);
  }
}

const gf_t* field_for(uint32_t n) { return (2 * n <= 256) ? &g_gf8 : &g_gf16; }

static int is_pow2(uint32_t n) { return n && !(n & (n - 1)); }

int orc_rs_encode(uint32_t n, size_t len, const uint8_t* data, uint8_t* parity) {
  orc_init();
  if (!is_pow2(n) || n > 32768) return ORC_EINVAL;
  const gf_t* f = field_for(n);
  if (f->bits == 16) {
    if (len % 64) return ORC_ECHUNK;
    if (g_simd && !g_lut16) {
#pragma omp critical(orc_lut16)
      if (!g_lut16) build_lut16();
    }
  }
  uint8_t** w = (uint8_t**)malloc(sizeof(uint8_t*) * n);
  memcpy(parity, data, n * len);
  for (uint32_t i = 0; i < n; i++) w[i] = parity + (size_t)i * len;
  leo_encode_inplace(f, n, w, len);
  free(w);
  return ORC_OK;
}

/* ------------------------------------------------------------- decoding */

/* In-place Walsh-Hadamard transform mod f->mod over N points (values < mod). */
static void fwht_mod(uint32_t* a, uint32_t N, uint32_t mod) {
  for (uint32_t h = 1; h < N; h <<= 1)
    for (uint32_t i = 0; i < N; i += 2 * h)
      for (uint32_t j = i; j < i + h; j++) {
        const uint32_t x = a[j], y = a[j + h];
        a[j] = (x + y) % mod;
        a[j + h] = (x + mod - y) % mod;
      }
}

/* x = x * exp(lm), symbol-wise (tmp: len bytes of scratch). */
static void mul_shard(const gf_t* f, uint8_t* x, uint32_t lm, size_t len, uint8_t* tmp) {
  memset(tmp, 0, len);
  muladd_shard(f, tmp, x, lm, len);
  memcpy(x, tmp, len);
}

/*
 * klauspost leopard8.go / leopard.go reconstruct with recoverAll (rsmt2d LeoRSCodec.Decode
 * calls Reconstruct), the catid/leopard erasure decoder:
 *   err[i]   = sum over erased e of log(i ^ e)  mod MOD   (error locator, by FWHTs)
 *   work[i]  = present ? shard_i * exp(err[i]) : 0
 *   work     = FFT(FormalDerivative(IFFT(work)))          (skew offset 0, N = 2n points)
 *   shard_i  = work[i] * exp(-err[i])                     for every erased i, data and parity
 * Leopard position p holds rsmt2d shard p ^ n (parity first, then data). Every present
 * shard takes part, so on shards that are not a codeword the output is this formula's,
 * not that of any other decoder (byzantine squares; no reference vector covers that
 * case: parity unpinned there). O(N log N) shard operations per axis.
 */
int orc_rs_decode(uint32_t n, size_t len, uint8_t* shards, const uint8_t* present) {
  orc_init();
  if (!is_pow2(n) || n > 32768) return ORC_EINVAL;
  const gf_t* f = field_for(n);
  if (f->bits == 16) {
    if (len % 64) return ORC_ECHUNK;
    if (g_simd && !g_lut16) {
#pragma omp critical(orc_lut16)
      if (!g_lut16) build_lut16();
    }
  }
  uint32_t have = 0;
  for (uint32_t i = 0; i < 2 * n; i++) have += present[i] ? 1 : 0;
  if (have == 2 * n) return ORC_OK;
  if (have < n) return ORC_ETOOFEW;
  const uint32_t N = 2 * n, mod = f->mod;
  /* error locator: XOR convolution of the erasure flags with the log table */
  uint32_t* err = (uint32_t*)malloc(sizeof(uint32_t) * N);
  uint32_t* lg = (uint32_t*)malloc(sizeof(uint32_t) * N);
  for (uint32_t p = 0; p < N; p++) {
    err[p] = present[p ^ n] ? 0u : 1u;
    lg[p] = f->log[p] % mod; /* log(0) = MOD == 0 */
  }
  fwht_mod(err, N, mod);
  fwht_mod(lg, N, mod);
  for (uint32_t p = 0; p < N; p++) err[p] = (uint32_t)(((uint64_t)err[p] * lg[p]) % mod);
  fwht_mod(err, N, mod);
  /* 1/N = 2^(bits - log2 N) (2^bits == 1 mod MOD) */
  const uint32_t inv_n = (1u << (f->bits - __builtin_ctz(N))) % mod;
  for (uint32_t p = 0; p < N; p++) err[p] = (uint32_t)(((uint64_t)err[p] * inv_n) % mod);
  uint8_t* buf = (uint8_t*)calloc((size_t)N + 1, len);
  uint8_t* tmp = buf + (size_t)N * len;
  uint8_t** w = (uint8_t**)malloc(sizeof(uint8_t*) * N);
  for (uint32_t p = 0; p < N; p++) {
    w[p] = buf + (size_t)p * len;
    if (present[p ^ n]) {
      memcpy(w[p], shards + (size_t)(p ^ n) * len, len);
      mul_shard(f, w[p], err[p], len, tmp);
    }
  }
  const uint16_t* skew = f->skew; /* skewLUT = fftSkew - 1: block b, half d -> skew[b + d - 1] */
  for (uint32_t d = 1; d < N; d <<= 1)
    for (uint32_t b = 0; b < N; b += 2 * d)
      for (uint32_t j = 0; j < d; j++) ifft2(f, w[b + j], w[b + d + j], skew[b + d - 1], len);
  for (uint32_t i = 1; i < N; i++) { /* formal derivative */
    const uint32_t width = i & (~i + 1);
    for (uint32_t j = 0; j < width; j++) xor_shard(w[i - width + j], w[i + j], len);
  }
  for (uint32_t d = N >> 1; d >= 1; d >>= 1)
    for (uint32_t b = 0; b < N; b += 2 * d)
      for (uint32_t j = 0; j < d; j++) fft2(f, w[b + j], w[b + d + j], skew[b + d - 1], len);
  for (uint32_t p = 0; p < N; p++) {
    if (present[p ^ n]) continue;
    mul_shard(f, w[p], (mod - err[p]) % mod, len, tmp);
    memcpy(shards + (size_t)(p ^ n) * len, w[p], len);
  }
  free(w);
  free(buf);
  free(lg);
  free(err);
  return ORC_OK;
}
