// Host check of celestia-app_amd/csrc/gf16_constexpr.hpp against the oracle's
// table-driven Leopard GF(2^16) (oracle/leopard.c). Built and run by
// tests/test_gf16_constexpr.py; prints "ok" or the first mismatch.
#include <cstdio>
#include <cstdlib>

#include "../celestia-app_amd/csrc/gf16_constexpr.hpp"

extern "C" {
int orc_gf_exp(int field, int i);
int orc_gf_skew(int field, int i);
int orc_gf_mul(int field, int a, int b);
void orc_init(void);
}

using namespace cel::g16c;

static_assert(amap(0) == 0, "A is linear");
static_assert(mul(1, 0x1234) == 0x1234, "one is the identity");

int main() {
  orc_init();
  unsigned x = 12345;
  auto rnd = [&]() { x = x * 1103515245u + 12345u; return (x >> 8) & 0xFFFFu; };
  for (int t = 0; t < 200000; t++) {
    const unsigned a = rnd(), b = rnd();
    if (mul(a, b) != (unsigned)orc_gf_mul(16, (int)a, (int)b)) {
      printf("mul(%u,%u) = %u, oracle %d\n", a, b, mul(a, b), orc_gf_mul(16, (int)a, (int)b));
      return 1;
    }
  }
  // skew entry 2^m - 1 + B (B a multiple of 2^(m+1)) is the element with representation B >> m
  for (int m = 0; m < 15; m++)
    for (unsigned B = 0; (1u << m) - 1 + B < 65535; B += 2u << m) {
      const int s = orc_gf_skew(16, (int)((1u << m) - 1 + B));
      const unsigned v = s == 65535 ? 0u : (unsigned)orc_gf_exp(16, s);
      if (v != (B >> m)) {
        printf("skew m=%d B=%u: %u != %u\n", m, B, v, B >> m);
        return 1;
      }
    }
  // GF(2^8) subfield, (a, b) coordinates, gamma^2 = p + q gamma
  for (unsigned c = 0; c < 256; c++)
    for (unsigned d = 0; d < 256; d++)
      if (mul(c, d) >= 256) { printf("subfield %u %u\n", c, d); return 1; }
  for (unsigned hi = 0; hi < 256; hi++)
    if (amap(hi) >= 256) { printf("amap %u\n", hi); return 1; }
  for (int t = 0; t < 100000; t++) {
    const unsigned y = rnd(), a = coord_a(y), b = coord_b(y);
    if ((a ^ mul(b, kGamma)) != y) { printf("coords %u\n", y); return 1; }
    // general product in coordinates: (ca + cb g)(a + b g) = (ca a + cb p b) + (cb a + (ca + cb q) b) g
    const unsigned c = rnd(), ca = coord_a(c), cb = coord_b(c);
    const unsigned na = mul(ca, a) ^ mul(mul(cb, kP), b), nb = mul(cb, a) ^ mul(ca ^ mul(cb, kQ), b);
    const unsigned p = mul(c, y);
    if (coord_a(p) != na || coord_b(p) != nb) { printf("general product %u %u\n", c, y); return 1; }
  }
  // v_perm tables: byte product through the 3+3+2 split
  for (unsigned c = 0; c < 256; c++) {
    const Tab8 t = tab8(c);
    for (unsigned y = 0; y < 256; y++) {
      const unsigned n0 = y & 7, n1 = (y >> 3) & 7, n2 = y >> 6;
      const unsigned p0 = ((n0 < 4 ? t.t0l : t.t0h) >> (8 * (n0 & 3))) & 0xFF;
      const unsigned p1 = ((n1 < 4 ? t.t1l : t.t1h) >> (8 * (n1 & 3))) & 0xFF;
      const unsigned p2 = (t.t2 >> (8 * n2)) & 0xFF;
      if ((p0 ^ p1 ^ p2) != mul(c, y)) { printf("tab8 %u %u\n", c, y); return 1; }
      unsigned bits = 0;
      for (int i = 0; i < 8; i++) {
        unsigned r = mul_row8(c, i), v = 0;
        for (int j = 0; j < 8; j++) v ^= ((r >> j) & 1u) & ((y >> j) & 1u);
        bits |= v << i;
      }
      if (bits != mul(c, y)) { printf("mul_row8 %u %u\n", c, y); return 1; }
    }
  }
  // rs_gf16x layer_p (layers 2-4, arrangement A): the encoder's twiddle of a butterfly whose
  // group base s has lane bits L (shard bits 5-7) is ca ^ L << (5 - m), ca the twiddle of the
  // same base with L = 0, all in GF(2^8) (coord_b 0); so x ^= c*y is ca*y plus the lane bits'
  // products. Checked against the oracle's skew table and field for K = 256, 512, both the
  // IFFT (block base K + s) and the FFT (base s).
  for (unsigned K = 256; K <= 512; K *= 2)
    for (int m = 2; m <= 4; m++)
      for (int fft = 0; fft < 2; fft++)
        for (unsigned s = 0; s < K; s += 2u << m) {
          const unsigned B = fft ? s : K + s, B0 = fft ? (s & ~0xE0u) : K + (s & ~0xE0u), L = (s >> 5) & 7u;
          const int e = orc_gf_skew(16, (int)((1u << m) - 1 + B)), e0 = orc_gf_skew(16, (int)((1u << m) - 1 + B0));
          const unsigned c = e == 65535 ? 0u : (unsigned)orc_gf_exp(16, e);
          const unsigned c0 = e0 == 65535 ? 0u : (unsigned)orc_gf_exp(16, e0);
          if (coord_b(c) != 0 || c != (c0 ^ (L << (5 - m)))) {
            printf("layer_p twiddle K=%u m=%d fft=%d s=%u: %u vs %u ^ lane\n", K, m, fft, s, c, c0);
            return 1;
          }
          for (int t = 0; t < 8; t++) {
            const unsigned y = rnd();
            unsigned v = (unsigned)orc_gf_mul(16, (int)c0, (int)y);
            for (int j = 0; j < 3; j++)
              if ((L >> j) & 1u) v ^= (unsigned)orc_gf_mul(16, (int)((1u << j) << (5 - m)), (int)y);
            if (v != (unsigned)orc_gf_mul(16, (int)c, (int)y)) {
              printf("layer_p lane product K=%u m=%d s=%u\n", K, m, s);
              return 1;
            }
          }
        }
  printf("ok p=%u q=%u\n", kP, kQ);
  return 0;
}
