// Bit-slice helpers shared by the register-resident RS kernels (rs_axis.hip GF(2^8),
// rs_gf16x.hip GF(2^16) in GF(2^8)-coordinates): an 8x8 bit transpose in each byte lane of
// 8 dwords (bytes -> bit planes and back), and the XOR networks of a GF(2) bit matrix with
// compile-time rows.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace cel {
namespace bs {

// 8x8 bit transpose in each byte lane of w[O .. O+8) (an involution): dword j <-> plane j.
// Bit-field inserts (v_bfi_b32 / v_bitop3 0xCA): shift + insert for each side, 4 VALU.
template <int A, int B, int S, uint32_t M, int K>
__device__ __forceinline__ void swapb(uint32_t (&w)[K]) {
  const uint32_t a = w[A], b = w[B];
  constexpr uint32_t MH = M << S;
  w[B] = __builtin_amdgcn_bitop3_b32(M, a >> S, b, 0xCA);
  w[A] = __builtin_amdgcn_bitop3_b32(MH, b << S, a, 0xCA);
}
template <int O, int K>
__device__ __forceinline__ void tr8(uint32_t (&w)[K]) {
  swapb<O + 0, O + 4, 4, 0x0F0F0F0Fu>(w);
  swapb<O + 1, O + 5, 4, 0x0F0F0F0Fu>(w);
  swapb<O + 2, O + 6, 4, 0x0F0F0F0Fu>(w);
  swapb<O + 3, O + 7, 4, 0x0F0F0F0Fu>(w);
  swapb<O + 0, O + 2, 2, 0x33333333u>(w);
  swapb<O + 1, O + 3, 2, 0x33333333u>(w);
  swapb<O + 4, O + 6, 2, 0x33333333u>(w);
  swapb<O + 5, O + 7, 2, 0x33333333u>(w);
  swapb<O + 0, O + 1, 1, 0x55555555u>(w);
  swapb<O + 2, O + 3, 1, 0x55555555u>(w);
  swapb<O + 4, O + 5, 1, 0x55555555u>(w);
  swapb<O + 6, O + 7, 1, 0x55555555u>(w);
}

// acc ^= xor of w[YO + j] for every set bit j of ROW (two inputs per v_bitop3).
template <uint32_t ROW, int YO, int J, int K>
__device__ __forceinline__ void xrow(uint32_t& acc, const uint32_t (&w)[K]) {
  if constexpr (J < 8) {
    if constexpr ((ROW >> J) & 1u) {
      constexpr uint32_t rest = ROW >> (J + 1);
      if constexpr (rest != 0) {
        constexpr int J2 = J + 1 + __builtin_ctz(rest);
        acc = __builtin_amdgcn_bitop3_b32(acc, w[YO + J], w[YO + J2], 0x96);
        xrow<ROW, YO, J2 + 1>(acc, w);
      } else {
        acc ^= w[YO + J];
      }
    } else {
      xrow<ROW, YO, J + 1>(acc, w);
    }
  }
}

template <int XO, int YO, int K>
__device__ __forceinline__ void pxor(uint32_t (&w)[K]) {
#pragma unroll
  for (int b = 0; b < 8; b++) w[YO + b] ^= w[XO + b];
}

}  // namespace bs
}  // namespace cel
