/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * SHA-256 per FIPS 180-4. The reference reaches it through
 * appconsts.NewBaseHashFunc (pkg/appconsts/global_consts.go:86) -> Go crypto/sha256,
 * whose amd64 block function uses SHA-NI; the optional SHA-NI path here plays the
 * same role for the CPU baseline (selected with orc_set_simd, checked against the
 * scalar path in tests).
 */
#include <string.h>
#if defined(__x86_64__)
#include <immintrin.h>
#endif
#include "oracle.h"
#include "oracle_internal.h"

static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

static const uint32_t H0[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                               0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};

#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

static void compress_scalar(uint32_t st[8], const uint8_t* blk) {
  uint32_t w[64];
  for (int i = 0; i < 16; i++)
    w[i] = ((uint32_t)blk[4 * i] << 24) | ((uint32_t)blk[4 * i + 1] << 16) |
           ((uint32_t)blk[4 * i + 2] << 8) | blk[4 * i + 3];
  for (int i = 16; i < 64; i++) {
    uint32_t s0 = ROR(w[i - 15], 7) ^ ROR(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = ROR(w[i - 2], 17) ^ ROR(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
  for (int i = 0; i < 64; i++) {
    uint32_t S1 = ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25);
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = h + S1 + ch + K256[i] + w[i];
    uint32_t S0 = ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22);
    uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint32_t t2 = S0 + mj;
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d;
  st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

#if defined(__x86_64__)
/* SHA-NI block function (Intel SHA extensions, standard two-lane state layout). */
__attribute__((target("sha,sse4.1"))) static void compress_shani(uint32_t st[8], const uint8_t* blk,
                                                                 size_t nblk) {
  const __m128i MASK = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
  __m128i tmp = _mm_loadu_si128((const __m128i*)&st[0]);
  __m128i s1 = _mm_loadu_si128((const __m128i*)&st[4]);
  tmp = _mm_shuffle_epi32(tmp, 0xB1);        /* CDAB */
  s1 = _mm_shuffle_epi32(s1, 0x1B);          /* EFGH */
  __m128i s0 = _mm_alignr_epi8(tmp, s1, 8);  /* ABEF */
  s1 = _mm_blend_epi16(s1, tmp, 0xF0);       /* CDGH */
  for (size_t b = 0; b < nblk; b++, blk += 64) {
    __m128i a0 = s0, c0 = s1, msg, t;
    __m128i m[4];
#pragma GCC unroll 16
    for (int j = 0; j < 16; j++) {
      if (j < 4) {
        m[j] = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(blk + 16 * j)), MASK);
      } else {
        /* M_j = msg2(msg1(M_{j-4}, M_{j-3}) + alignr(M_{j-1}, M_{j-2}, 4), M_{j-1}) */
        t = _mm_sha256msg1_epu32(m[j & 3], m[(j + 1) & 3]);
        t = _mm_add_epi32(t, _mm_alignr_epi8(m[(j + 3) & 3], m[(j + 2) & 3], 4));
        m[j & 3] = _mm_sha256msg2_epu32(t, m[(j + 3) & 3]);
      }
      msg = _mm_add_epi32(m[j & 3], _mm_loadu_si128((const __m128i*)&K256[4 * j]));
      s1 = _mm_sha256rnds2_epu32(s1, s0, msg);
      msg = _mm_shuffle_epi32(msg, 0x0E);
      s0 = _mm_sha256rnds2_epu32(s0, s1, msg);
    }
    s0 = _mm_add_epi32(s0, a0);
    s1 = _mm_add_epi32(s1, c0);
  }
  tmp = _mm_shuffle_epi32(s0, 0x1B);        /* FEBA */
  s1 = _mm_shuffle_epi32(s1, 0xB1);         /* DCHG */
  s0 = _mm_blend_epi16(tmp, s1, 0xF0);      /* DCBA */
  s1 = _mm_alignr_epi8(s1, tmp, 8);         /* ABEF */
  _mm_storeu_si128((__m128i*)&st[0], s0);
  _mm_storeu_si128((__m128i*)&st[4], s1);
}

static int g_has_shani = -1;
static int has_shani(void) {
  if (g_has_shani < 0) {
    __builtin_cpu_init();
    unsigned a, b, c, d;
    __asm__("cpuid" : "=a"(a), "=b"(b), "=c"(c), "=d"(d) : "a"(7), "c"(0));
    g_has_shani = ((b >> 29) & 1) && __builtin_cpu_supports("sse4.1");
  }
  return g_has_shani;
}
#endif

static void compress(uint32_t st[8], const uint8_t* blk, size_t nblk) {
#if defined(__x86_64__)
  if (g_simd && has_shani()) { compress_shani(st, blk, nblk); return; }
#endif
  for (size_t i = 0; i < nblk; i++) compress_scalar(st, blk + 64 * i);
}

void sha256_3(const uint8_t* a, size_t la, const uint8_t* b, size_t lb, const uint8_t* c,
              size_t lc, uint8_t out[32]) {
  uint32_t st[8];
  memcpy(st, H0, sizeof(st));
  uint8_t buf[128];
  size_t fill = 0;
  const uint8_t* parts[3] = {a, b, c};
  size_t lens[3] = {la, lb, lc};
  uint64_t total = (uint64_t)la + lb + lc;
  for (int p = 0; p < 3; p++) {
    const uint8_t* s = parts[p];
    size_t l = lens[p];
    if (!l) continue;
    if (fill) {
      size_t take = 64 - fill < l ? 64 - fill : l;
      memcpy(buf + fill, s, take);
      fill += take; s += take; l -= take;
      if (fill == 64) { compress(st, buf, 1); fill = 0; }
    }
    if (l >= 64) {
      size_t nb = l / 64;
      compress(st, s, nb);
      s += nb * 64; l -= nb * 64;
    }
    if (l) { memcpy(buf, s, l); fill = l; }
  }
  buf[fill++] = 0x80;
  if (fill > 56) {
    memset(buf + fill, 0, 128 - fill);
    fill = 128;
  } else {
    memset(buf + fill, 0, 64 - fill);
    fill = 64;
  }
  uint64_t bits = total * 8;
  for (int i = 0; i < 8; i++) buf[fill - 1 - i] = (uint8_t)(bits >> (8 * i));
  compress(st, buf, fill / 64);
  for (int i = 0; i < 8; i++) {
    out[4 * i] = (uint8_t)(st[i] >> 24);
    out[4 * i + 1] = (uint8_t)(st[i] >> 16);
    out[4 * i + 2] = (uint8_t)(st[i] >> 8);
    out[4 * i + 3] = (uint8_t)st[i];
  }
}

/* One message already laid out with its padding in nblk whole blocks (the NMT's fixed
 * 542-byte leaf and 181-byte node messages): one block-function call, no buffering. */
void sha256_blocks(const uint8_t* blocks, size_t nblk, uint8_t out[32]) {
  uint32_t st[8];
  memcpy(st, H0, sizeof(st));
  compress(st, blocks, nblk);
  for (int i = 0; i < 8; i++) {
    const uint32_t v = __builtin_bswap32(st[i]);
    memcpy(out + 4 * i, &v, 4);
  }
}

/* Pad a message of len bytes sitting at the start of buf (capacity >= the padded size):
 * returns the number of 64-byte blocks. */
size_t sha256_pad(uint8_t* buf, size_t len) {
  const size_t nblk = (len + 8) / 64 + 1;
  buf[len] = 0x80;
  memset(buf + len + 1, 0, nblk * 64 - len - 1);
  const uint64_t bits = (uint64_t)len * 8;
  for (int i = 0; i < 8; i++) buf[nblk * 64 - 1 - i] = (uint8_t)(bits >> (8 * i));
  return nblk;
}

void orc_sha256(const uint8_t* msg, size_t len, uint8_t out[32]) {
  sha256_3(msg, len, NULL, 0, NULL, 0, out);
}
