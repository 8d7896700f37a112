// Leopard-RS field tables (GF(2^8) and GF(2^16) in the Cantor-basis representation).
//
// The reference reaches this arithmetic through rsmt2d v0.14.0 LeoRSCodec
// (pkg/appconsts/global_consts.go:92) -> klauspost/reedsolomon v1.12.1
// leopard8.go / leopard.go (initLUTs, initFFTSkew; [dep], restated in SURVEY.md
// Appendix A.2/A.3). The tables are built once on the host and shipped to the
// device as twiddle / product tables; they are tiny (<= 256 KiB).
#pragma once
#include <cstdint>
#include <vector>

namespace cel {

struct LeoField {
  int bits = 0;
  uint32_t order = 0, mod = 0;
  std::vector<uint16_t> exp, log, skew;

  uint32_t add_mod(uint32_t a, uint32_t b) const {
    uint32_t s = a + b;  // partial reduction: result may equal mod (== 0 mod mod)
    return (s + (s >> bits)) & mod;
  }
  uint32_t mul_log(uint32_t a, uint32_t log_b) const {
    return a == 0 ? 0u : exp[add_mod(log[a], log_b)];
  }
  // Field product of two elements (used by the decoder's error locator only).
  uint32_t mul(uint32_t a, uint32_t b) const {
    if (a == 0 || b == 0) return 0;
    return exp[(log[a] + (uint32_t)log[b]) % mod];
  }

  void build(int nbits, uint32_t poly, const uint16_t* cantor) {
    bits = nbits;
    order = 1u << bits;
    mod = order - 1;
    exp.assign(order, 0);
    log.assign(order, 0);
    skew.assign(mod, 0);
    uint32_t st = 1;
    for (uint32_t i = 0; i < mod; i++) {  // LFSR: exp[] temporarily holds logs
      exp[st] = (uint16_t)i;
      st <<= 1;
      if (st >= order) st ^= poly;
    }
    exp[0] = (uint16_t)mod;
    log[0] = 0;
    for (int i = 0; i < bits; i++) {  // Cantor basis -> polynomial basis
      const uint32_t w = 1u << i;
      for (uint32_t j = 0; j < w; j++) log[j + w] = log[j] ^ cantor[i];
    }
    for (uint32_t i = 0; i < order; i++) log[i] = exp[log[i]];
    for (uint32_t i = 0; i < order; i++) exp[log[i]] = (uint16_t)i;
    exp[mod] = exp[0];

    uint32_t temp[16];
    for (int i = 1; i < bits; i++) temp[i - 1] = 1u << i;
    for (int m = 0; m < bits - 1; m++) {
      const uint32_t step = 1u << (m + 1);
      skew[(1u << m) - 1] = 0;
      for (int i = m; i < bits - 1; i++) {
        const uint32_t s = 1u << (i + 1);
        for (uint32_t j = (1u << m) - 1; j < s; j += step) skew[j + s] = skew[j] ^ (uint16_t)temp[i];
      }
      temp[m] = mod - log[mul_log(temp[m], log[temp[m] ^ 1])];
      for (int i = m + 1; i < bits - 1; i++) temp[i] = mul_log(temp[i], add_mod(log[temp[i] ^ 1], temp[m]));
    }
    for (uint32_t i = 0; i < mod; i++) skew[i] = log[skew[i]];
  }
};

inline const LeoField& leo_gf8() {
  static const LeoField f = [] {
    static const uint16_t cantor[8] = {1, 214, 152, 146, 86, 200, 88, 230};
    LeoField x;
    x.build(8, 0x11D, cantor);
    return x;
  }();
  return f;
}

inline const LeoField& leo_gf16() {
  static const LeoField f = [] {
    static const uint16_t cantor[16] = {0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E, 0x914C, 0x4012,
                                        0x6C98, 0x10D8, 0x6A72, 0xB900, 0xFDB8, 0xFB34, 0xFF38, 0x991E};
    LeoField x;
    x.build(16, 0x1002D, cantor);
    return x;
  }();
  return f;
}

}  // namespace cel
