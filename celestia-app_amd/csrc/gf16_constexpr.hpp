// Compile-time Leopard GF(2^16) arithmetic (klauspost/reedsolomon v1.12.1 leopard.go,
// SURVEY.md Appendix A.3) for kernels whose twiddles are template constants
// (rs_gf16x.hip). Plain C++17: the host test tests/gf16_constexpr_check.cpp includes it
// too and compares it with the oracle's table-driven field.
//
// Leopard represents an element by its coordinates in the Cantor basis beta_0..beta_15
// (kCantor16 gives each beta_i in the polynomial basis of GF(2)[x] / 0x1002D), so the
// product of two representations is  rep(poly(a) * poly(b) mod 0x1002D).
//
// Two facts the kernel is built on (both checked by the host test):
//  - FFT twiddles: the skew entry used by the butterfly layer of half-distance 2^m at
//    block base B (skew index 2^m - 1 + B, B a multiple of 2^(m+1)) is the element whose
//    representation is B >> m. The Leopard encoder's IFFT uses B = K + base, its FFT
//    B = base (rs_kernels.hip header), so every twiddle is known from the indices alone.
//  - span(beta_0..beta_7) (representations < 256) is the subfield GF(2^8), and with
//    gamma = beta_8 every element is a + b*gamma, a, b in GF(2^8), where b = hi byte and
//    a = lo byte ^ A(hi byte) for a fixed GF(2)-linear map A. A twiddle c in GF(2^8)
//    multiplies a and b separately: GF(2^16) butterflies with such twiddles are GF(2^8)
//    butterflies on bytes.
#pragma once
#include <cstdint>

namespace cel {
namespace g16c {

constexpr uint32_t kPoly16 = 0x1002D;
constexpr uint16_t kCantor16[16] = {0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E, 0x914C, 0x4012,
                                    0x6C98, 0x10D8, 0x6A72, 0xB900, 0xFDB8, 0xFB34, 0xFF38, 0x991E};

constexpr uint32_t to_poly(uint32_t rep) {
  uint32_t p = 0;
  for (int i = 0; i < 16; i++)
    if ((rep >> i) & 1u) p ^= kCantor16[i];
  return p;
}

constexpr uint32_t poly_mul(uint32_t a, uint32_t b) {
  uint32_t r = 0;
  for (int i = 0; i < 16; i++)
    if ((b >> i) & 1u) r ^= a << i;
  for (int i = 31; i >= 16; i--)
    if ((r >> i) & 1u) r ^= kPoly16 << (i - 16);
  return r;
}

// Inverse of to_poly: column i = the representation of x^i (Gauss-Jordan over GF(2)).
struct InvCantor {
  uint16_t col[16];
};
constexpr InvCantor make_inv_cantor() {
  // rows: [poly(beta_i) | e_i]; reduce the poly halves to the identity
  uint32_t rows[16] = {};
  for (int i = 0; i < 16; i++) rows[i] = (uint32_t)kCantor16[i] | (1u << (16 + i));
  for (int bit = 0; bit < 16; bit++) {
    int piv = bit;
    while (piv < 16 && !((rows[piv] >> bit) & 1u)) piv++;
    const uint32_t t = rows[piv];
    rows[piv] = rows[bit];
    rows[bit] = t;
    for (int r = 0; r < 16; r++)
      if (r != bit && ((rows[r] >> bit) & 1u)) rows[r] ^= rows[bit];
  }
  InvCantor inv{};
  for (int i = 0; i < 16; i++) inv.col[i] = (uint16_t)(rows[i] >> 16);  // rep of x^i
  return inv;
}
inline constexpr InvCantor kInvCantor = make_inv_cantor();

constexpr uint32_t from_poly(uint32_t p) {
  uint32_t rep = 0;
  for (int i = 0; i < 16; i++)
    if ((p >> i) & 1u) rep ^= kInvCantor.col[i];
  return rep;
}

// Field product in Leopard representation.
constexpr uint32_t mul(uint32_t a, uint32_t b) { return from_poly(poly_mul(to_poly(a), to_poly(b))); }

// (lo, hi) <-> (a, b) coordinates: a = lo ^ A(hi), b = hi.
constexpr uint32_t kGamma = 0x100;  // beta_8
constexpr uint32_t amap(uint32_t hi) {
  uint32_t r = 0;
  for (int k = 0; k < 8; k++)
    if ((hi >> k) & 1u) r ^= (1u << (8 + k)) ^ mul(1u << k, kGamma);
  return r;
}
// gamma^2 = p + q*gamma
constexpr uint32_t kGammaSq = mul(kGamma, kGamma);
constexpr uint32_t kP = (kGammaSq & 0xFFu) ^ amap(kGammaSq >> 8);
constexpr uint32_t kQ = kGammaSq >> 8;

// a-coordinate / b-coordinate of an element given by its representation
constexpr uint32_t coord_a(uint32_t rep) { return (rep & 0xFFu) ^ amap(rep >> 8); }
constexpr uint32_t coord_b(uint32_t rep) { return rep >> 8; }

// v_perm product tables of "multiply by c" for c in GF(2^8) (c < 256) acting on a byte
// split 3 + 3 + 2 bits: T0[n] = c*n, T1[n] = c*(n << 3) (n < 8), T2[n] = c*(n << 6)
// (n < 4), packed as {T0[0..3], T0[4..7], T1[0..3], T1[4..7], T2[0..3]}. Linear in c.
struct Tab8 {
  uint32_t t0l, t0h, t1l, t1h, t2;
};
constexpr Tab8 tab8(uint32_t c) {
  Tab8 t{0, 0, 0, 0, 0};
  for (uint32_t n = 0; n < 4; n++) {
    t.t0l |= mul(c, n) << (8 * n);
    t.t0h |= mul(c, n + 4) << (8 * n);
    t.t1l |= mul(c, n << 3) << (8 * n);
    t.t1h |= mul(c, (n + 4) << 3) << (8 * n);
    t.t2 |= mul(c, n << 6) << (8 * n);
  }
  return t;
}
// The same tables for the GF(2)-linear map A (the (lo, hi) -> (a, b) conversion).
constexpr Tab8 tab_amap() {
  Tab8 t{0, 0, 0, 0, 0};
  for (uint32_t n = 0; n < 4; n++) {
    t.t0l |= amap(n) << (8 * n);
    t.t0h |= amap(n + 4) << (8 * n);
    t.t1l |= amap(n << 3) << (8 * n);
    t.t1h |= amap((n + 4) << 3) << (8 * n);
    t.t2 |= amap(n << 6) << (8 * n);
  }
  return t;
}

// Row i of the 8x8 GF(2) matrix of "multiply by c" (c < 256) on a byte: bit j set if
// bit i of c * (1 << j) is set.
constexpr uint32_t mul_row8(uint32_t c, int i) {
  uint32_t r = 0;
  for (int j = 0; j < 8; j++) r |= ((mul(c, 1u << j) >> i) & 1u) << j;
  return r;
}

// Encoder twiddle (representation) of the radix-2 layer of half-distance 2^m at the
// block base `base` (a multiple of 2^(m+1)) for K data shards.
constexpr uint32_t ifft_tw(uint32_t K, uint32_t m, uint32_t base) { return (K + base) >> m; }
constexpr uint32_t fft_tw(uint32_t m, uint32_t base) { return base >> m; }

}  // namespace g16c
}  // namespace cel
