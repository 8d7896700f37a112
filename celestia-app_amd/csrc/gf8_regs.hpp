// Register-resident GF(2^8) multiply helpers shared by the axis kernels (rs_axis.hip encode,
// rs_decode_axis.hip decode): compile-time v_perm product tables per twiddle and the
// bit-sliced multiply of 8 bit planes by a compile-time constant.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "bitslice8.hpp"
#include "gf8_constexpr.hpp"

namespace cel {
namespace ax {

using cx::add_mod8;
using cx::kGf8;
using cx::sfor;
using bs::xrow;

struct Tab {
  uint32_t t0l, t0h, t1l, t1h, t2;
};

constexpr uint32_t cmul(uint32_t a, uint32_t lm) { return a == 0 ? 0u : kGf8.exp[add_mod8(kGf8.log[a], lm)]; }

// Product tables of c = exp(lm): T0[n] = c*n, T1[n] = c*(n << 3) (n < 8), T2[n] = c*(n << 6) (n < 4).
constexpr Tab make_tab(uint32_t lm) {
  Tab t{0, 0, 0, 0, 0};
  for (uint32_t n = 0; n < 4; n++) {
    t.t0l |= cmul(n, lm) << (8 * n);
    t.t0h |= cmul(n + 4, lm) << (8 * n);
    t.t1l |= cmul(n << 3, lm) << (8 * n);
    t.t1h |= cmul((n + 4) << 3, lm) << (8 * n);
    t.t2 |= cmul(n << 6, lm) << (8 * n);
  }
  return t;
}

// Constants materialised where they are used (volatile asm: the compiler would
// otherwise CSE the table constants of all twiddles into VGPRs live across the whole
// transform). gfx950 VOP3 takes no literal and reads one SGPR, so each 8-entry
// product table has one dword in an SGPR (s_mov on the scalar unit) and one in a VGPR.
template <uint32_t C>
__device__ __forceinline__ uint32_t sconst() {
  uint32_t r;
  asm volatile("s_mov_b32 %0, %1" : "=s"(r) : "i"(C));
  return r;
}
template <uint32_t C>
__device__ __forceinline__ uint32_t vconst() {
  uint32_t r;
  asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "i"(C));
  return r;
}

// Multiplier by c = exp(LM), tables materialised once per butterfly group.
// LM == 255 is the zero twiddle (nothing to add), c == 1 is a plain xor.
template <uint32_t LM>
struct Mul {
  static constexpr bool kZero = LM == 255u;
  static constexpr bool kOne = !kZero && cmul(1, LM) == 1u;
  static constexpr Tab t = make_tab(kZero ? 0u : LM);
  uint32_t t0l, t0h, t1l, t1h, t2;
  __device__ __forceinline__ Mul() {
    if constexpr (!kZero && !kOne) {
      t0h = sconst<t.t0h>();
      t1h = sconst<t.t1h>();
      t2 = sconst<t.t2>();
      t0l = vconst<t.t0l>();
      t1l = vconst<t.t1l>();
    }
  }
  // x ^= c * y on 4 bytes; m7 = 0x07070707, m3 = 0x03030303 held in SGPRs (a VOP2
  // with an SGPR operand is 4 bytes against 8 with a literal: the unrolled transform
  // is ~60 KiB of code, at the size of the instruction cache)
  __device__ __forceinline__ void muladd(uint32_t& x, uint32_t y, uint32_t m7, uint32_t m3) const {
    if constexpr (kOne) {
      x ^= y;
    } else if constexpr (!kZero) {
      const uint32_t s0 = y & m7;
      const uint32_t s1 = (y >> 3) & m7;
      const uint32_t s2 = (y >> 6) & m3;
      const uint32_t p0 = __builtin_amdgcn_perm(t0h, t0l, s0);
      const uint32_t p1 = __builtin_amdgcn_perm(t1h, t1l, s1);
      const uint32_t p2 = __builtin_amdgcn_perm(0u, t2, s2);
      x = __builtin_amdgcn_bitop3_b32(x, p0, p1, 0x96) ^ p2;
    }
  }
};

// Pins a butterfly's pair (asm volatile keeps the order): stops the combiner from
// folding xor chains across butterflies, which keeps extra values alive and spills.
__device__ __forceinline__ void pin(uint32_t& a, uint32_t& b) { asm volatile("" : "+v"(a), "+v"(b)); }

// planes w[XO..XO+8) ^= exp(LM) * planes w[YO..YO+8); LM == 255 is the zero twiddle.
template <uint32_t LM, int XO, int YO, int K>
__device__ __forceinline__ void pmuladd(uint32_t (&w)[K]) {
  if constexpr (LM != 255u) {
    sfor<8>([&](auto r) { xrow<cx::mul_row(LM, decltype(r)::value), YO, 0>(w[XO + decltype(r)::value], w); });
  }
}

}  // namespace ax
}  // namespace cel
