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
 * Decoding here is NOT Leopard's error-locator decoder: it is plain Gauss-Jordan
 * over the field using the generator matrix obtained by encoding unit vectors.
 * The code is MDS, so the recovered codeword is unique and any correct decoder
 * is bit-exact with klauspost Reconstruct.
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
static uint8_t (*g_lut16)[8][16];  /* [65536 log][q*2 + outbyte][16] */

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

/* In-place Leopard encode: work[0..m) holds the m data shards on entry and the m
 * parity shards on exit (klauspost ifftDITEncoder + fftDIT with mtrunc = m). */
void leo_encode_inplace(const gf_t* f, uint32_t m, uint8_t** w, size_t len) {
  const uint16_t* skew = f->skew;
  const uint16_t* sk = skew + (m - 1); /* skewLUT = fftSkew[m-1:] */
  /* IFFT, decimation in time, two layers at a time. */
  uint32_t dist = 1, dist4 = 4;
  while (dist4 <= m) {
    for (uint32_t r = 0; r < m; r += dist4) {
      uint32_t ie = r + dist;
      uint32_t l01 = sk[ie], l02 = sk[ie + dist], l23 = sk[ie + 2 * dist];
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

/* Generator matrices G[i][j] = parity symbol i of encode(e_j), cached per n. */
typedef struct {
  uint32_t n;
  uint16_t* g;
} gen_cache_t;
static gen_cache_t g_gen[16];

static const uint16_t* generator(uint32_t n) {
  int slot = __builtin_ctz(n);
  const uint16_t* res = NULL;
#pragma omp critical(orc_gen)
  {
    if (!g_gen[slot].g) {
      const gf_t* f = field_for(n);
      size_t slen = f->bits == 8 ? 1 : 64;
      uint16_t* g = (uint16_t*)malloc(sizeof(uint16_t) * n * n);
      uint8_t* buf = (uint8_t*)calloc((size_t)n * slen, 1);
      uint8_t** w = (uint8_t**)malloc(sizeof(uint8_t*) * n);
      int simd = g_simd;
      g_simd = 0;
      for (uint32_t j = 0; j < n; j++) {
        memset(buf, 0, (size_t)n * slen);
        buf[(size_t)j * slen] = 1; /* symbol value 1 at position 0 */
        for (uint32_t i = 0; i < n; i++) w[i] = buf + (size_t)i * slen;
        leo_encode_inplace(f, n, w, slen);
        for (uint32_t i = 0; i < n; i++) {
          uint32_t s = buf[(size_t)i * slen];
          if (f->bits == 16) s |= (uint32_t)buf[(size_t)i * slen + 32] << 8;
          g[(size_t)i * n + j] = (uint16_t)s;
        }
      }
      g_simd = simd;
      free(w);
      free(buf);
      g_gen[slot].n = n;
      g_gen[slot].g = g;
    }
    res = g_gen[slot].g;
  }
  return res;
}

static inline uint32_t get_sym(const gf_t* f, const uint8_t* s, size_t idx) {
  if (f->bits == 8) return s[idx];
  size_t c = (idx / 32) * 64, j = idx % 32;
  return (uint32_t)s[c + j] | ((uint32_t)s[c + 32 + j] << 8);
}

static inline void put_sym(const gf_t* f, uint8_t* s, size_t idx, uint32_t v) {
  if (f->bits == 8) { s[idx] = (uint8_t)v; return; }
  size_t c = (idx / 32) * 64, j = idx % 32;
  s[c + j] = (uint8_t)(v & 0xFF);
  s[c + 32 + j] = (uint8_t)(v >> 8);
}

int orc_rs_decode(uint32_t n, size_t len, uint8_t* shards, const uint8_t* present) {
  orc_init();
  if (!is_pow2(n) || n > 32768) return ORC_EINVAL;
  const gf_t* f = field_for(n);
  if (f->bits == 16 && len % 64) return ORC_ECHUNK;
  uint32_t have = 0;
  for (uint32_t i = 0; i < 2 * n; i++) have += present[i] ? 1 : 0;
  if (have == 2 * n) return ORC_OK;
  if (have < n) return ORC_ETOOFEW;
  int data_complete = 1;
  for (uint32_t i = 0; i < n; i++) data_complete &= present[i] ? 1 : 0;
  if (!data_complete) {
    const uint16_t* G = generator(n);
    uint32_t* rows = (uint32_t*)malloc(sizeof(uint32_t) * n);
    uint32_t cnt = 0;
    for (uint32_t i = 0; i < 2 * n && cnt < n; i++)
      if (present[i]) rows[cnt++] = i;
    /* A (n x n) | I -> Gauss-Jordan -> A^-1 */
    uint16_t* a = (uint16_t*)calloc((size_t)n * 2 * n, sizeof(uint16_t));
    for (uint32_t r = 0; r < n; r++) {
      uint32_t p = rows[r];
      uint16_t* row = a + (size_t)r * 2 * n;
      if (p < n) row[p] = 1;
      else memcpy(row, G + (size_t)(p - n) * n, sizeof(uint16_t) * n);
      row[n + r] = 1;
    }
    for (uint32_t col = 0; col < n; col++) {
      uint32_t piv = col;
      while (piv < n && a[(size_t)piv * 2 * n + col] == 0) piv++;
      if (piv == n) { free(a); free(rows); return ORC_EINVAL; } /* cannot happen for MDS */
      if (piv != col)
        for (uint32_t c = 0; c < 2 * n; c++) {
          uint16_t t = a[(size_t)piv * 2 * n + c];
          a[(size_t)piv * 2 * n + c] = a[(size_t)col * 2 * n + c];
          a[(size_t)col * 2 * n + c] = t;
        }
      uint16_t* prow = a + (size_t)col * 2 * n;
      uint32_t inv = gf_inv(f, prow[col]);
      for (uint32_t c = 0; c < 2 * n; c++) prow[c] = (uint16_t)gf_mul(f, prow[c], inv);
      for (uint32_t r = 0; r < n; r++) {
        if (r == col) continue;
        uint16_t* row = a + (size_t)r * 2 * n;
        uint32_t fac = row[col];
        if (!fac) continue;
        for (uint32_t c = 0; c < 2 * n; c++) row[c] ^= (uint16_t)gf_mul(f, prow[c], fac);
      }
    }
    /* data[i] = sum_r inv[i][r] * known[rows[r]] */
    size_t nsym = f->bits == 8 ? len : len / 2;
    uint8_t* out = (uint8_t*)malloc((size_t)n * len);
    for (uint32_t i = 0; i < n; i++) {
      const uint16_t* ir = a + (size_t)i * 2 * n + n;
      for (size_t s = 0; s < nsym; s++) {
        uint32_t acc = 0;
        for (uint32_t r = 0; r < n; r++) {
          if (!ir[r]) continue;
          acc ^= gf_mul(f, ir[r], get_sym(f, shards + (size_t)rows[r] * len, s));
        }
        put_sym(f, out + (size_t)i * len, s, acc);
      }
    }
    for (uint32_t i = 0; i < n; i++)
      if (!present[i]) memcpy(shards + (size_t)i * len, out + (size_t)i * len, len);
    free(out);
    free(a);
    free(rows);
  }
  /* Re-encode the parity half. */
  uint8_t* par = (uint8_t*)malloc((size_t)n * len);
  orc_rs_encode(n, len, shards, par);
  for (uint32_t i = 0; i < n; i++)
    if (!present[n + i]) memcpy(shards + (size_t)(n + i) * len, par + (size_t)i * len, len);
  free(par);
  return ORC_OK;
}
