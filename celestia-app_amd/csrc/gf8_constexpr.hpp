// Compile-time Leopard GF(2^8) tables (klauspost/reedsolomon v1.12.1 leopard8.go
// initLUTs8 / initFFTSkew8) and compile-time loop helpers,
// shared by the kernels whose butterfly twiddles are template constants
// (rs_bitslice.hip, rs_axis.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <utility>

namespace cel {
namespace cx {


struct Gf8Tables {
  uint8_t exp[256];
  uint8_t log[256];
  uint8_t skew[256];
};

constexpr uint32_t add_mod8(uint32_t a, uint32_t b) {
  const uint32_t s = a + b;
  return (s + (s >> 8)) & 255u;
}

constexpr Gf8Tables make_gf8() {
  Gf8Tables t{};
  uint32_t expv[256] = {};
  uint32_t logv[256] = {};
  const uint32_t cantor[8] = {1, 214, 152, 146, 86, 200, 88, 230};
  uint32_t st = 1;
  for (uint32_t i = 0; i < 255; i++) {
    expv[st] = i;
    st <<= 1;
    if (st >= 256) st ^= 0x11D;
  }
  expv[0] = 255;
  logv[0] = 0;
  for (int i = 0; i < 8; i++) {
    const uint32_t w = 1u << i;
    for (uint32_t j = 0; j < w; j++) logv[j + w] = logv[j] ^ cantor[i];
  }
  for (uint32_t i = 0; i < 256; i++) logv[i] = expv[logv[i]];
  for (uint32_t i = 0; i < 256; i++) expv[logv[i]] = i;
  expv[255] = expv[0];
  uint32_t skew[256] = {};
  uint32_t temp[8] = {};
  for (int i = 1; i < 8; i++) temp[i - 1] = 1u << i;
  auto mul_log = [&](uint32_t a, uint32_t lb) -> uint32_t { return a == 0 ? 0u : expv[add_mod8(logv[a], lb)]; };
  for (int m = 0; m < 7; m++) {
    const uint32_t step = 1u << (m + 1);
    skew[(1u << m) - 1] = 0;
    for (int i = m; i < 7; i++) {
      const uint32_t s = 1u << (i + 1);
      for (uint32_t j = (1u << m) - 1; j < s; j += step) skew[j + s] = skew[j] ^ temp[i];
    }
    temp[m] = 255 - logv[mul_log(temp[m], logv[temp[m] ^ 1])];
    for (int i = m + 1; i < 7; i++) temp[i] = mul_log(temp[i], add_mod8(logv[temp[i] ^ 1], temp[m]));
  }
  for (uint32_t i = 0; i < 255; i++) skew[i] = logv[skew[i]];
  for (int i = 0; i < 256; i++) {
    t.exp[i] = (uint8_t)expv[i];
    t.log[i] = (uint8_t)logv[i];
    t.skew[i] = (uint8_t)skew[i];
  }
  return t;
}

inline constexpr Gf8Tables kGf8 = make_gf8();

// Row i of the bit matrix of "multiply by exp(lm)": bit j set if bit i of c*(1<<j) is set.
constexpr uint32_t mul_row(uint32_t lm, int i) {
  uint32_t r = 0;
  for (int j = 0; j < 8; j++) {
    const uint32_t p = kGf8.exp[add_mod8(kGf8.log[1u << j], lm)];
    r |= ((p >> i) & 1u) << j;
  }
  return r;
}

// ------------------------------------------------------------ compile-time loops

template <typename F, int... I>
__device__ __forceinline__ void sfor_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  sfor_impl(f, std::make_integer_sequence<int, N>{});
}

}  // namespace cx
}  // namespace cel
