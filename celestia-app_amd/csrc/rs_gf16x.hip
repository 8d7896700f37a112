// Leopard GF(2^16) encode (k = 256, 512: 2k > 256 shards), one wave per
// (square, axis, 64-byte column), no LDS, no barrier.
//
// Replaces klauspost/reedsolomon v1.12.1 leopard.go Encode as rsmt2d v0.14.0's
// LeoRSCodec drives it for more than 256 shards (pkg/appconsts/global_consts.go:92;
// SURVEY.md Appendix A.3): IFFT of the K data shards over the coset at K, then FFT over
// the coset at 0, radix 2 (the transform of rs_kernels.hip's header).
//
// Layout. A wave holds one 64-byte Leopard block (32 symbols) of every one of the K
// shards of an axis in VGPRs: lane l = j + 8L takes dword j of the lo half and dword j
// of the hi half of the block (4 symbols), so 8 lanes cover a block and L (3 bits) is
// part of the shard index; each lane holds NR = K/8 shards, 2 dwords each (K = 512:
// 128 VGPRs). Waves never talk to each other; 3 per SIMD overlap memory with compute.
//
// Arithmetic (gf16_constexpr.hpp). Symbols are kept in (a, b) coordinates over GF(2^8):
// y = a + b*gamma. Every twiddle's representation is its block base >> layer, so every
// twiddle is known from indices alone, and all but the lowest layers' twiddles lie in
// the subfield GF(2^8), where a butterfly is a GF(2^8) butterfly on each byte.
//
// Two arrangements of the shard index s (K = 512; K = 256 drops bit 8):
//   A: register r bits 0-4 = s bits 0-4, r bit 5 = s bit 8, lane L = s bits 5-7.
//      Layers 0-4 (IFFT up, FFT down). Twiddle = compile-time part (register bits) XOR
//      L << (5 - layer) (lane part, in GF(2^8)). Layers 0-1 (partners inside a block of
//      4 registers): v_perm product tables per lane, built by XORing the compile-time
//      table with the lane's table of the layer. Layers 2-4 (partners in different
//      blocks, twiddles in GF(2^8)): on bit planes, as in B, the lane part added as
//      XOR networks under lane masks (layer_p).
//   B: register r bits 0-1 = s bits 0-1, r bits 2.. = s bits 5.., lane L = s bits 2-4.
//      Layers 5..log2(K)-1 have compile-time twiddles in GF(2^8): four shards x 4
//      symbols x (a, b) = 32 bytes share every twiddle, so each 8-dword block (turned
//      into 8 bit planes by an 8x8 bit transpose before layer 2) is a butterfly of 8
//      xors plus an 8x8 GF(2) matrix network of xor3 ops.
//   A <-> B swaps register bits 2, 3, 4 with lane bits 3, 4, 5: DPP row_ror:8,
//   v_permlane16_swap and v_permlane32_swap (a 2x2 transpose per register pair each).
#include <hip/hip_runtime.h>

#include "bitslice8.hpp"
#include "cel_internal.hpp"
#include "gf16_constexpr.hpp"
#include "gf8_constexpr.hpp"

namespace cel {
namespace g16 {

using bs::pxor;
using bs::tr8;
using bs::xrow;
using cx::sfor;
using namespace g16c;

// Constants materialised where used (volatile: keeps the compiler from hoisting every
// twiddle's table into registers live across the transform). A VOP3 reads one SGPR.
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
__device__ __forceinline__ void pin(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d) {
  asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
}

// 3+3+2-bit selector fields of the 4 bytes of y (m7 = 0x07070707, m3 = 0x03030303).
struct Sel {
  uint32_t f0, f1, f2;
};
__device__ __forceinline__ Sel sel(uint32_t y, uint32_t m7, uint32_t m3) { return {y & m7, (y >> 3) & m7, (y >> 6) & m3}; }

// A product table in registers (VGPR or SGPR operands).
struct Tb {
  uint32_t t0l, t0h, t1l, t1h, t2;
};
// x ^= the 4 byte products of the selectors by the table
__device__ __forceinline__ uint32_t madd(uint32_t x, const Sel& s, const Tb& t) {
  const uint32_t p0 = __builtin_amdgcn_perm(t.t0h, t.t0l, s.f0);
  const uint32_t p1 = __builtin_amdgcn_perm(t.t1h, t.t1l, s.f1);
  const uint32_t p2 = __builtin_amdgcn_perm(0u, t.t2, s.f2);
  return __builtin_amdgcn_bitop3_b32(x, p0, p1, 0x96) ^ p2;
}
__device__ __forceinline__ uint32_t madd2(uint32_t x, const Sel& s, const Tb& t, const Sel& u, const Tb& v) {
  const uint32_t p0 = __builtin_amdgcn_perm(t.t0h, t.t0l, s.f0);
  const uint32_t p1 = __builtin_amdgcn_perm(t.t1h, t.t1l, s.f1);
  const uint32_t p2 = __builtin_amdgcn_perm(0u, t.t2, s.f2);
  const uint32_t q0 = __builtin_amdgcn_perm(v.t0h, v.t0l, u.f0);
  const uint32_t q1 = __builtin_amdgcn_perm(v.t1h, v.t1l, u.f1);
  const uint32_t q2 = __builtin_amdgcn_perm(0u, v.t2, u.f2);
  return __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(x, p0, p1, 0x96), __builtin_amdgcn_bitop3_b32(p2, q0, q1, 0x96),
                                     q2, 0x96);
}

// Compile-time table of "multiply by C" (C < 256): high halves in SGPRs, low in VGPRs.
template <uint32_t C>
__device__ __forceinline__ Tb ctab() {
  constexpr Tab8 t = tab8(C);
  return Tb{vconst<t.t0l>(), sconst<t.t0h>(), vconst<t.t1l>(), sconst<t.t1h>(), sconst<t.t2>()};
}
// x ^ C as one volatile instruction: each group's table is built where the group starts
// (plain XORs would be hoisted to the top of the transform, or CSE'd between layers, and
// held in VGPRs), straight from the layer's lane table, with no copy.
template <uint32_t C>
__device__ __forceinline__ uint32_t vxor(uint32_t v) {
  if constexpr (C == 0) {
    return v;
  } else {
    uint32_t r;
    asm volatile("v_xor_b32 %0, %1, %2" : "=v"(r) : "i"(C), "v"(v));
    return r;
  }
}
// Per-lane table: compile-time table of C XOR the lane's table g.
template <uint32_t C>
__device__ __forceinline__ Tb rtab(const Tb& g) {
  constexpr Tab8 t = tab8(C);
  return Tb{vxor<t.t0l>(g.t0l), vxor<t.t0h>(g.t0h), vxor<t.t1l>(g.t1l), vxor<t.t1h>(g.t1h), vxor<t.t2>(g.t2)};
}

// The lane's table of c_g = L << S (S = 5 - layer): linear in c, so the XOR of the tables
// of the bits of L, each selected by a lane mask (all ones where bit i of L is set).
template <int S>
__device__ __forceinline__ Tb lane_tab(uint32_t m0, uint32_t m1, uint32_t m2) {
  constexpr Tab8 a = tab8(1u << S), b = tab8(2u << S), c = tab8(4u << S);
  asm volatile("" : "+v"(m0), "+v"(m1), "+v"(m2));  // built where the layer starts
  auto f = [&](uint32_t x, uint32_t y, uint32_t z) {
    return (m0 & x) ^ (m1 & y) ^ (m2 & z);
  };
  return Tb{f(a.t0l, b.t0l, c.t0l), f(a.t0h, b.t0h, c.t0h), f(a.t1l, b.t1l, c.t1l), f(a.t1h, b.t1h, c.t1h),
            f(a.t2, b.t2, c.t2)};
}

// lane_tab of this lane, its masks recomputed from the lane id where the layer starts (three
// lane masks live across the whole transform pushed the k = 512 kernel into scratch spills)
template <int S>
__device__ __forceinline__ Tb lane_tab_here() {
  uint32_t l = threadIdx.x;
  asm volatile("" : "+v"(l));
  const uint32_t L = (l & 63u) >> 3;
  return lane_tab<S>(0u - (L & 1u), 0u - ((L >> 1) & 1u), 0u - ((L >> 2) & 1u));
}

// Register index r (arrangement A) -> the register-held bits of the shard index.
template <int LOGK>
constexpr uint32_t shard_bits_a(uint32_t r) {
  return (r & 31u) | ((r >> 5) << 8);
}

// One radix-2 layer of arrangement A on bytes (layer D_LOG in 0..1 as shipped; 0..4 valid)
// over w[2r] (a), w[2r+1] (b).
// Groups run in two halves by register bit 5 (shard bit 8): the twiddle's gamma
// coordinate cb is constant over a half (it only sees shard bit 8 and K), so the
// lane-independent tables of cb and cb*p are built once per half. HS >= 0: half HS only.
template <int LOGK, int D_LOG, bool IFFT, int HS, int NW>
__device__ __forceinline__ void layer_a(uint32_t (&w)[NW], const Tb& g, uint32_t m7, uint32_t m3) {
  constexpr uint32_t K = 1u << LOGK;
  constexpr int NR = NW / 2;
  constexpr int D = 1 << D_LOG;
  constexpr int NH = NR / 32;      // halves (1 for K = 256)
  constexpr int GPH = 32 / (2 * D);  // groups per half
  auto tw = [](int r0) constexpr { return IFFT ? ifft_tw(K, D_LOG, shard_bits_a<LOGK>((uint32_t)r0))
                                               : fft_tw(D_LOG, shard_bits_a<LOGK>((uint32_t)r0)); };
  sfor<NH>([&](auto hi) {
    constexpr int h = decltype(hi)::value;
    constexpr uint32_t cb = coord_b(tw(32 * h));
    if constexpr (HS >= 0 && h != HS) {
      // the other half: not in this call
    } else if constexpr (cb == 0) {
      sfor<GPH>([&](auto gi) {
        constexpr int r0 = 32 * h + decltype(gi)::value * 2 * D;  // bit D_LOG clear, bits below zero
        constexpr uint32_t c = tw(r0);  // lane part added per lane
        static_assert(coord_b(c) == cb, "gamma coordinate varies inside a half");
        const Tb t = rtab<coord_a(c)>(g);
        sfor<D>([&](auto ji) {
          constexpr int x = r0 + decltype(ji)::value, y = x + D;
          pin(w[2 * x], w[2 * x + 1], w[2 * y], w[2 * y + 1]);
          if constexpr (IFFT) {
            w[2 * y] ^= w[2 * x];
            w[2 * y + 1] ^= w[2 * x + 1];
            w[2 * x] = madd(w[2 * x], sel(w[2 * y], m7, m3), t);
            w[2 * x + 1] = madd(w[2 * x + 1], sel(w[2 * y + 1], m7, m3), t);
          } else {
            w[2 * x] = madd(w[2 * x], sel(w[2 * y], m7, m3), t);
            w[2 * x + 1] = madd(w[2 * x + 1], sel(w[2 * y + 1], m7, m3), t);
            w[2 * y] ^= w[2 * x];
            w[2 * y + 1] ^= w[2 * x + 1];
          }
          pin(w[2 * x], w[2 * x + 1], w[2 * y], w[2 * y + 1]);
          __builtin_amdgcn_sched_barrier(0);
        });
      });
    } else {
      // c = ca + cb*gamma (cb compile-time, ca = compile-time part ^ lane part):
      //   x_a ^= ca*y_a + (cb p)*y_b,  x_b ^= cb*y_a + (ca + cb q)*y_b
      const Tb tcbp = ctab<mul(cb, kP)>();
      const Tb tcb = ctab<cb>();
      sfor<GPH>([&](auto gi) {
        constexpr int r0 = 32 * h + decltype(gi)::value * 2 * D;
        constexpr uint32_t c = tw(r0);
        static_assert(coord_b(c) == cb, "gamma coordinate varies inside a half");
        constexpr uint32_t ca = coord_a(c);
        const Tb tca = rtab<ca>(g);
        const Tb tq = rtab<ca ^ mul(cb, kQ)>(g);
        sfor<D>([&](auto ji) {
          constexpr int x = r0 + decltype(ji)::value, y = x + D;
          pin(w[2 * x], w[2 * x + 1], w[2 * y], w[2 * y + 1]);
          if constexpr (IFFT) {
            w[2 * y] ^= w[2 * x];
            w[2 * y + 1] ^= w[2 * x + 1];
          }
          const Sel sa = sel(w[2 * y], m7, m3), sb = sel(w[2 * y + 1], m7, m3);
          w[2 * x] = madd2(w[2 * x], sa, tca, sb, tcbp);
          w[2 * x + 1] = madd2(w[2 * x + 1], sa, tcb, sb, tq);
          if constexpr (!IFFT) {
            w[2 * y] ^= w[2 * x];
            w[2 * y + 1] ^= w[2 * x + 1];
          }
          pin(w[2 * x], w[2 * x + 1], w[2 * y], w[2 * y + 1]);
          __builtin_amdgcn_sched_barrier(0);
        });
      });
    }
  });
}

// The lane's masks of the bits of L (all ones where the bit is set), from the lane id
__device__ __forceinline__ void lane_masks(uint32_t& m0, uint32_t& m1, uint32_t& m2) {
  uint32_t l = threadIdx.x;
  asm volatile("" : "+v"(l));
  const uint32_t L = (l & 63u) >> 3;
  m0 = 0u - (L & 1u);
  m1 = 0u - ((L >> 1) & 1u);
  m2 = 0u - ((L >> 2) & 1u);
}

// Row R of x ^= (CA + lane part) * y, the lane part sum_j L_j * (1 << (S + j)): the
// coefficient of plane y_k is c0 ^ parity(L & J) (c0 = bit k of CA's row, J = the e_j whose
// rows have bit k). g[R][key] = the planes k whose (J, c0) is (key >> 1, key & 1). One table
// per (CA, S), evaluated once (a static constexpr member), so the compile stays short.
struct LaneGroupTab {
  uint32_t g[8][16];
};
constexpr LaneGroupTab make_lane_groups(uint32_t CA, int S) {
  LaneGroupTab t{};
  for (int R = 0; R < 8; R++) {
    const uint32_t rc = mul_row8(CA, R);
    const uint32_t r0 = mul_row8(1u << S, R), r1 = mul_row8(2u << S, R), r2 = mul_row8(4u << S, R);
    for (int k = 0; k < 8; k++) {
      const uint32_t J = ((r0 >> k) & 1u) | (((r1 >> k) & 1u) << 1) | (((r2 >> k) & 1u) << 2);
      t.g[R][J * 2 + ((rc >> k) & 1u)] |= 1u << k;
    }
  }
  return t;
}
// The classes rebuild "multiply by CA + lane part" for every lane value L (mul_row8 is
// linear in c; checked at compile time for each (CA, S) the kernel uses).
constexpr bool lane_groups_ok(const LaneGroupTab& t, uint32_t CA, int S) {
  for (uint32_t L = 0; L < 8; L++) {
    const uint32_t c = CA ^ ((L & 1u) << S) ^ ((L & 2u) << S) ^ ((L & 4u) << S);
    for (int R = 0; R < 8; R++) {
      uint32_t row = 0;
      for (int key = 1; key < 16; key++)
        if (((uint32_t)key & 1u) ^ (__builtin_popcount(L & ((uint32_t)key >> 1)) & 1u)) row |= t.g[R][key];
      if (row != mul_row8(c, R)) return false;
    }
  }
  return true;
}
template <uint32_t CA, int S>
struct LaneGroups {
  static constexpr LaneGroupTab tab = make_lane_groups(CA, S);
  static_assert(lane_groups_ok(tab, CA, S), "coefficient classes do not rebuild the product");
};

// planes w[XO..XO+8) ^= (CA + lane part) * planes w[YO..YO+8): per row, the planes of one
// coefficient class are XORed together and added under that class's lane mask M[J] (or its
// complement when c0 is set) by one v_bitop3; the class (J = 0, c0 = 1) is added plainly.
template <uint32_t CA, int S, int XO, int YO, int NW>
__device__ __forceinline__ void pmuladd_lane(uint32_t (&w)[NW], const uint32_t (&M)[8]) {
  sfor<8>([&](auto ri) {
    constexpr int r = decltype(ri)::value;
    sfor<16>([&](auto ki) {
      constexpr int key = decltype(ki)::value;
      constexpr uint32_t g = LaneGroups<CA, S>::tab.g[r][key];
      if constexpr (key == 1 && g != 0) {
        xrow<g, YO, 0>(w[XO + r], w);
      } else if constexpr (key > 1 && g != 0) {
        constexpr int k0 = __builtin_ctz(g);
        uint32_t q = w[YO + k0];
        xrow<g & ~(1u << k0), YO, 0>(q, w);
        if constexpr (key & 1) {
          w[XO + r] = __builtin_amdgcn_bitop3_b32(w[XO + r], M[key >> 1], q, 0xD2);  // x ^ (~m & q)
        } else {
          w[XO + r] = __builtin_amdgcn_bitop3_b32(w[XO + r], M[key >> 1], q, 0x78);  // x ^ (m & q)
        }
      }
    });
  });
}

// planes w[XO..XO+8) ^= C * planes w[YO..YO+8) (C < 256; C == 0 adds nothing)
template <uint32_t C, int XO, int YO, int NW>
__device__ __forceinline__ void pmuladd(uint32_t (&w)[NW]) {
  if constexpr (C != 0) {
    sfor<8>([&](auto r) { xrow<mul_row8(C, decltype(r)::value), YO, 0>(w[XO + decltype(r)::value], w); });
  }
}

template <int HS, int B>
constexpr bool in_half() { return HS < 0 || (B >> 3) == HS; }

// Layers 2-4 of arrangement A on bit planes. Their twiddles lie in GF(2^8) (coord_b 0):
// c = ca (register bits, compile-time) + L0*e0 + L1*e1 + L2*e2 with e_j = 1 << (S + j),
// S = 5 - layer (the lane part, linear in L's bits), so x ^= c*y is the compile-time network
// of ca plus the three networks of e_j, each row added under lane mask j. The shards of a
// block (register bits 0-1) share the twiddle and the butterfly pairs whole blocks (D >= 4
// registers), so each block w[8b..8b+8) is 8 planes (tr8) as in arrangement B.
template <int LOGK, int D_LOG, bool IFFT, int HS, int NW>
__device__ __forceinline__ void layer_p(uint32_t (&w)[NW], const uint32_t (&M)[8]) {
  static_assert(D_LOG >= 2 && D_LOG <= 4, "plane layers are 2-4");
  constexpr uint32_t K = 1u << LOGK;
  constexpr int NB = NW / 8;
  constexpr int DB = 1 << (D_LOG - 2);  // block distance
  constexpr int S = 5 - D_LOG;
  sfor<NB / (2 * DB)>([&](auto gi) {
    constexpr int b0 = decltype(gi)::value * 2 * DB;
    if constexpr (in_half<HS, b0>()) {
      constexpr uint32_t sb = shard_bits_a<LOGK>(4u * b0);
      constexpr uint32_t c = IFFT ? ifft_tw(K, D_LOG, sb) : fft_tw(D_LOG, sb);
      static_assert(coord_b(c) == 0, "plane layers need twiddles in GF(2^8)");
      sfor<DB>([&](auto ji) {
        constexpr int x = 8 * (b0 + decltype(ji)::value), y = x + 8 * DB;
        if constexpr (IFFT) pxor<x, y>(w);
        pmuladd_lane<coord_a(c), S, x, y>(w, M);
        if constexpr (!IFFT) pxor<x, y>(w);
        __builtin_amdgcn_sched_barrier(0);
      });
    }
  });
}

// bytes <-> bit planes for every block of half HS (all if HS < 0)
template <int HS, int NW>
__device__ __forceinline__ void tr_blocks(uint32_t (&w)[NW]) {
  sfor<NW / 8>([&](auto b) {
    if constexpr (in_half<HS, decltype(b)::value>()) {
      tr8<8 * decltype(b)::value>(w);
      __builtin_amdgcn_sched_barrier(0);
    }
  });
}

// Register bit RB (2, 3, 4) <-> lane bit RB + 1 (8, 16, 32 lanes apart): a 2x2 transpose
// of every register pair (r, r | 1 << RB), for both coordinates. An involution. HS >= 0:
// the registers of half HS (register bit 5) only.
template <int RB, int HS, int NW>
__device__ __forceinline__ void swap_bit(uint32_t (&w)[NW]) {
  constexpr int NR = NW / 2;
  sfor<NR>([&](auto ri) {
    constexpr int r = decltype(ri)::value;
    if constexpr (!((r >> RB) & 1) && (HS < 0 || (r >> 5) == HS)) {
      constexpr int r1 = r | (1 << RB);
      sfor<2>([&](auto ci) {
        constexpr int u = 2 * r + decltype(ci)::value, v = 2 * r1 + decltype(ci)::value;
        if constexpr (RB == 4) {
          const auto p = __builtin_amdgcn_permlane32_swap(w[u], w[v], false, false);
          w[u] = p[0];
          w[v] = p[1];
        } else if constexpr (RB == 3) {
          const auto p = __builtin_amdgcn_permlane16_swap(w[u], w[v], false, false);
          w[u] = p[0];
          w[v] = p[1];
        } else {
          // row_ror:8 reads lane l ^ 8; banks 2-3 (lane bit 3 set) take the partner's w[v]
          // into w[u], banks 0-1 the partner's w[u] into w[v]
          const uint32_t nu = __builtin_amdgcn_update_dpp(w[u], w[v], 0x128, 0xF, 0xC, false);
          const uint32_t nv = __builtin_amdgcn_update_dpp(w[v], w[u], 0x128, 0xF, 0x3, false);
          w[u] = nu;
          w[v] = nv;
        }
      });
    }
  });
}

// Arrangement B: block b = registers 4b..4b+3 = w[8b..8b+8), shard bits 5.. = b; block b
// lies in half b >> 3 (register bit 5); the blocks are already bit planes (tr_blocks before
// layer 2). stage_b_in: the IFFT layers 5 .. LOGK-2 (block groups of at most 8, inside one
// half), for half HS (all if HS < 0); stage_b_mid: the merged last-IFFT / first-FFT layer
// (K = 512: across the halves); stage_b_out: the FFT layers LOGK-2 .. 5, for half HS.
template <int LOGK, int HS, int NW>
__device__ __forceinline__ void stage_b_in(uint32_t (&w)[NW]) {
  constexpr uint32_t K = 1u << LOGK;
  constexpr int NB = NW / 8;
  // IFFT layers 5 .. LOGK-2
  sfor<LOGK - 6>([&](auto t) {
    constexpr int d = 5 + decltype(t)::value;
    constexpr int DB = 1 << (d - 5);  // block distance
    sfor<NB / (2 * DB)>([&](auto gi) {
      constexpr int b0 = decltype(gi)::value * 2 * DB;
      if constexpr (in_half<HS, b0>()) {
        constexpr uint32_t c = ifft_tw(K, d, (uint32_t)b0 << 5);
        sfor<DB>([&](auto ji) {
          constexpr int x = 8 * (b0 + decltype(ji)::value), y = x + 8 * DB;
          pxor<x, y>(w);
          pmuladd<c, x, y>(w);
          __builtin_amdgcn_sched_barrier(0);
        });
      }
    });
  });
}

template <int LOGK, int NW>
__device__ __forceinline__ void stage_b_mid(uint32_t (&w)[NW]) {
  // last IFFT layer and first FFT layer act on the same pairs: one multiply by c1 + c2
  constexpr uint32_t K = 1u << LOGK;
  constexpr int d = LOGK - 1;
  constexpr int DB = 1 << (d - 5);
  constexpr uint32_t c = ifft_tw(K, d, 0) ^ fft_tw(d, 0);
  sfor<DB>([&](auto ji) {
    constexpr int x = 8 * decltype(ji)::value, y = x + 8 * DB;
    pxor<x, y>(w);
    pmuladd<c, x, y>(w);
    pxor<x, y>(w);
    __builtin_amdgcn_sched_barrier(0);
  });
}

template <int LOGK, int HS, int NW>
__device__ __forceinline__ void stage_b_out(uint32_t (&w)[NW]) {
  constexpr int NB = NW / 8;
  // FFT layers LOGK-2 .. 5
  sfor<LOGK - 6>([&](auto t) {
    constexpr int d = LOGK - 2 - decltype(t)::value;
    constexpr int DB = 1 << (d - 5);
    sfor<NB / (2 * DB)>([&](auto gi) {
      constexpr int b0 = decltype(gi)::value * 2 * DB;
      if constexpr (in_half<HS, b0>()) {
        constexpr uint32_t c = fft_tw(d, (uint32_t)b0 << 5);
        sfor<DB>([&](auto ji) {
          constexpr int x = 8 * (b0 + decltype(ji)::value), y = x + 8 * DB;
          pmuladd<c, x, y>(w);
          pxor<x, y>(w);
          __builtin_amdgcn_sched_barrier(0);
        });
      }
    });
  });
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}

// (lo, hi) -> (a, b): a = lo ^ A(hi), b = hi; the inverse is the same map. One table
// materialisation for the whole array, one register's conversion at a time.
template <int HS, int NW>
__device__ __forceinline__ void convert(uint32_t (&w)[NW], uint32_t m7, uint32_t m3) {
  constexpr Tab8 t = tab_amap();
  const Tb tb{vconst<t.t0l>(), sconst<t.t0h>(), vconst<t.t1l>(), sconst<t.t1h>(), sconst<t.t2>()};
  sfor<NW / 2>([&](auto ri) {
    constexpr int i = decltype(ri)::value;
    if constexpr (HS < 0 || (i >> 5) == HS) {
      w[2 * i] = madd(w[2 * i], sel(w[2 * i + 1], m7, m3), tb);
      __builtin_amdgcn_sched_barrier(0);
    }
  });
}

typedef uint32_t D2 __attribute__((ext_vector_type(2)));

// Memory <-> register layout. A wave moves a block with 8-byte accesses, 8 lanes per
// shard (one 64-byte segment per shard per instruction: dword-wide accesses, 8 x 32-byte
// segments per instruction, ran the column pass at 1.9 TB/s without any transform,
// tools/microbench/gf16_mem.hip), so lane bit 2 first holds the lo/hi half of the block
// and the two dwords of an access are neighbours in the half. One exchange across lane
// bit 2 (a 2x2 transpose of every register pair, DPP row_ror:4 / row_ror:12 in alternate
// 4-lane banks) turns each pair into (lo dword, hi dword) of the same 4 symbols and lane
// bit 2 into a column bit; it is an involution, so the same exchange undoes it before
// the stores.
template <int HS, int NW>
__device__ __forceinline__ void pair_lo_hi(uint32_t (&w)[NW]) {
  sfor<NW / 2>([&](auto ri) {
    constexpr int i = decltype(ri)::value;
    if constexpr (HS >= 0 && (i >> 5) != HS) return;
    // banks 1, 3 (lane bit 2 set) take the partner's second dword into the first;
    // banks 0, 2 take the partner's first dword into the second
    const uint32_t lo = __builtin_amdgcn_update_dpp(w[2 * i], w[2 * i + 1], 0x124, 0xF, 0xA, false);
    const uint32_t hi = __builtin_amdgcn_update_dpp(w[2 * i + 1], w[2 * i], 0x12C, 0xF, 0x5, false);
    w[2 * i] = lo;
    w[2 * i + 1] = hi;
  });
}

// Tile = (square z, axis x, 64-byte column cb): one wave. Shard j of the axis sits at
// in + z*in_sq + x*in_axis + place(j) + 64*cb (see RsGeom; blocked placement for the
// output and the data copy when blk_log != 0).
// PROBE (cel_probe_rs_transform): the same tile with its stores aimed past the buffer's
// range (dropped by the buffer range check, so the transform stays live and nothing reaches
// HBM); its geometry points every load at one cache-resident 512-byte block.
template <int LOGK, bool CHECK = false, bool PROBE = false>
__global__ __launch_bounds__(256, LOGK == 9 ? 3 : 4) void k_rs_gf16x(RsGeom g) {
  constexpr int K = 1 << LOGK;
  constexpr int NR = K / 8;
  constexpr int NW = 2 * NR;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t tile = __builtin_amdgcn_readfirstlane(xcd_block(blockIdx.x, gridDim.x) * 4u + (threadIdx.x >> 6));
  const uint32_t nblk = g.len / 64u;
  if (tile >= (uint32_t)g.axes * nblk * g.nsq) return;
  const uint32_t cb = tile % nblk, r = tile / nblk;
  const uint32_t x = r % g.axes, z = r / g.axes;
  const uint32_t xa = CHECK && g.chk_axes ? (uint32_t)g.chk_axes[x] : x;  // the axis addressed
  const uint32_t L = lane >> 3;
  const uint32_t col = cb * 64u + (lane & 7u) * 8u;  // 8 lanes x 8 B = one 64-byte block
  const uint32_t m7 = sconst<0x07070707u>(), m3 = sconst<0x03030303u>();
  const uint32_t blk_mask = g.blk_log ? (1u << g.blk_log) - 1u : 0xFFFFFFFFu;
  const uint32_t blk_shift = g.blk_log ? g.blk_log : 31u;
  // Shard index in arrangement A = a register part (register bits 0-4 -> shard bits 0-4,
  // bit 5 -> shard bit 8) plus a lane part (L -> shard bits 5-7). The two occupy disjoint
  // bits, so every placement below (linear or blocked) is the sum of a wave-uniform
  // register term (the buffer instruction's SGPR offset) and a lane term (its VGPR
  // offset): no per-register address VGPRs.
  // (the shift and mask go through an opaque copy at each use site: otherwise the data
  // copy's and the output's offsets share their scalar subterms, which stay live across
  // the whole transform and spill)
  auto place = [&](uint32_t s, uint32_t shard, uint32_t blk) {
    uint32_t sh = blk_shift, mk = blk_mask;
    asm volatile("" : "+s"(sh), "+s"(mk));
    return (s >> sh) * blk + (s & mk) * shard;
  };
  auto reg_bits = [](uint32_t i) { return (i & 31u) | ((i >> 5) << 8); };
  const uint32_t lane_bits = L << 5;
  uint32_t w[NW];
  {
    const auto rin = rsrc(g.in + (uint64_t)z * g.in_sq + (uint64_t)xa * g.in_axis);
    const uint32_t in_shard = (uint32_t)g.in_shard;
    const uint32_t vin = lane_bits * in_shard + col;
#pragma unroll
    for (int i = 0; i < NR; i++) {
      const uint32_t so = __builtin_amdgcn_readfirstlane(reg_bits((uint32_t)i) * in_shard);
      const auto v = __builtin_amdgcn_raw_buffer_load_b64(rin, vin, so, 0);
      w[2 * i] = v[0];
      w[2 * i + 1] = v[1];
    }
    if (g.dcopy) {
      const auto rdc = rsrc(g.dcopy + (uint64_t)z * g.dc_sq + (uint64_t)x * g.dc_axis);
      const uint32_t dc_shard = (uint32_t)g.dc_shard, dc_blk = (uint32_t)g.dc_blk;
      const uint32_t vdc = place(lane_bits, dc_shard, dc_blk) + col;
#pragma unroll
      for (int i = 0; i < NR; i++) {
        const uint32_t so = __builtin_amdgcn_readfirstlane(place(reg_bits((uint32_t)i), dc_shard, dc_blk));
        __builtin_amdgcn_raw_buffer_store_b64(D2{w[2 * i], w[2 * i + 1]}, rdc, vdc, so, 0);
      }
    }
  }
  // The transform. K = 512 runs half by half (register bit 5 = shard bit 8) where it can: both
  // halves' loads are issued above, half 0 goes through the IFFT layers 0-7 while half 1's
  // loads land, the merged layer 8 joins them, and half 0's FFT ends with its stores before
  // half 1's FFT starts, so loads and stores overlap this wave's own arithmetic instead of
  // bracketing it. K = 256 (one half) keeps the whole-array order.
  constexpr int NHALF = LOGK == 9 ? 2 : 1;
  auto front = [&](auto hs) {
    constexpr int HS = decltype(hs)::value;
    pair_lo_hi<HS>(w);
    convert<HS>(w, m7, m3);  // -> (a, b)
    // IFFT, arrangement A
    layer_a<LOGK, 0, true, HS>(w, lane_tab_here<5>(), m7, m3);
    layer_a<LOGK, 1, true, HS>(w, lane_tab_here<4>(), m7, m3);
    tr_blocks<HS>(w);  // -> bit planes
    uint32_t m0, m1, m2;
    lane_masks(m0, m1, m2);
    const uint32_t M[8] = {0u, m0, m1, m0 ^ m1, m2, m0 ^ m2, m1 ^ m2, m0 ^ m1 ^ m2};  // M[J]: parity of L & J
    layer_p<LOGK, 2, true, HS>(w, M);
    layer_p<LOGK, 3, true, HS>(w, M);
    layer_p<LOGK, 4, true, HS>(w, M);
    swap_bit<2, HS>(w);
    swap_bit<3, HS>(w);
    swap_bit<4, HS>(w);
    stage_b_in<LOGK, HS>(w);
  };
  const auto rout = rsrc(g.out + (uint64_t)z * g.out_sq + (uint64_t)xa * g.out_axis);
  const uint32_t out_shard = (uint32_t)g.out_shard, out_blk = (uint32_t)g.out_blk;
  uint32_t diff = 0;
  auto back = [&](auto hs) {
    constexpr int HS = decltype(hs)::value;
    stage_b_out<LOGK, HS>(w);
    swap_bit<2, HS>(w);
    swap_bit<3, HS>(w);
    swap_bit<4, HS>(w);
    // FFT, arrangement A
    uint32_t m0, m1, m2;
    lane_masks(m0, m1, m2);
    const uint32_t M[8] = {0u, m0, m1, m0 ^ m1, m2, m0 ^ m2, m1 ^ m2, m0 ^ m1 ^ m2};  // M[J]: parity of L & J
    layer_p<LOGK, 4, false, HS>(w, M);
    layer_p<LOGK, 3, false, HS>(w, M);
    layer_p<LOGK, 2, false, HS>(w, M);
    tr_blocks<HS>(w);  // -> bytes
    layer_a<LOGK, 1, false, HS>(w, lane_tab_here<4>(), m7, m3);
    layer_a<LOGK, 0, false, HS>(w, lane_tab_here<5>(), m7, m3);
    convert<HS>(w, m7, m3);  // -> (lo, hi)
    pair_lo_hi<HS>(w);
    // the lane's output offset from the lane id again: col and lane_bits held across the
    // transform would cost two more VGPRs at the 168 the kernel runs at
    uint32_t ln = threadIdx.x;
    asm volatile("" : "+v"(ln));
    ln &= 63u;
    const uint32_t vout = place((ln >> 3) << 5, out_shard, out_blk) + cb * 64u + (ln & 7u) * 8u;
    constexpr int i0 = HS < 0 ? 0 : 32 * HS, i1 = HS < 0 ? NR : 32 * HS + 32;
    if constexpr (CHECK) {  // repair's encoding check: compare with the parity in place
#pragma unroll
      for (int i = i0; i < i1; i++) {
        const uint32_t so = __builtin_amdgcn_readfirstlane(place(reg_bits((uint32_t)i), out_shard, out_blk));
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(rout, vout, so, 0);
        diff |= (v[0] ^ w[2 * i]) | (v[1] ^ w[2 * i + 1]);
      }
      asm volatile("" : "+v"(diff));
    } else {
      // PROBE: the same stores aimed past the buffer's range (offset >= num_records: dropped),
      // so the probe runs the encode's instruction stream without writing HBM
      const uint32_t vo = PROBE ? 0x80000000u : vout;
#pragma unroll
      for (int i = i0; i < i1; i++) {
        const uint32_t so = __builtin_amdgcn_readfirstlane(place(reg_bits((uint32_t)i), out_shard, out_blk));
        __builtin_amdgcn_raw_buffer_store_b64(D2{w[2 * i], w[2 * i + 1]}, rout, vo, so, 0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  if constexpr (NHALF == 2) {
    front(std::integral_constant<int, 0>{});
    front(std::integral_constant<int, 1>{});
    stage_b_mid<LOGK>(w);
    back(std::integral_constant<int, 0>{});
    back(std::integral_constant<int, 1>{});
  } else {
    front(std::integral_constant<int, -1>{});
    stage_b_mid<LOGK>(w);
    back(std::integral_constant<int, -1>{});
  }
  if constexpr (CHECK) {
    if (__any(diff != 0) && lane == 0) atomicOr(g.chk_flags + (g.chk_idx ? g.chk_idx[x] : (int32_t)x), 1);
  }
}

// The transform alone for cel_probe_rs_transform: ntiles tiles, every load from the 512
// bytes at src, nothing stored.
template <int LOGK>
static hipError_t launch_probe(const uint8_t* src, uint8_t* dst, uint32_t ntiles, hipStream_t s) {
  RsGeom g{};
  g.in = src;
  g.out = dst;
  g.n = 1u << LOGK;
  g.len = 512;
  g.axes = (ntiles + 7) / 8;
  g.nsq = 1;
  hipLaunchKernelGGL((k_rs_gf16x<LOGK, false, true>), dim3((g.axes * 8 + 3) / 4), dim3(256), 0, s, g);
  return hipGetLastError();
}

template <int LOGK>
static hipError_t launch(const RsGeom& g, hipStream_t s) {
  const uint64_t tiles = (uint64_t)g.axes * (g.len / 64u) * g.nsq;
  if (tiles == 0) return hipSuccess;
  if (tiles > 0xFFFFFFF0ull) return hipErrorInvalidValue;
  if (g.chk_flags) {
    if (g.nsq != 1 || g.dcopy) return hipErrorInvalidValue;
    hipLaunchKernelGGL((k_rs_gf16x<LOGK, true>), dim3((unsigned)((tiles + 3) / 4)), dim3(256), 0, s, g);
  } else {
    hipLaunchKernelGGL((k_rs_gf16x<LOGK, false>), dim3((unsigned)((tiles + 3) / 4)), dim3(256), 0, s, g);
  }
  return hipGetLastError();
}

}  // namespace g16

// Byte offsets must fit the 32-bit buffer offsets.
static bool gf16x_geom_ok(const RsGeom& g) {
  auto span = [&](uint64_t shard, uint64_t blk) {
    return g.blk_log ? ((uint64_t)(g.n >> g.blk_log) * blk + (uint64_t)(1u << g.blk_log) * shard + g.len)
                     : (uint64_t)g.n * shard + g.len;
  };
  return g.len % 64 == 0 && g.len > 0 && (uint64_t)g.n * g.in_shard + g.len < 0x7fffffffull &&
         span(g.out_shard, g.out_blk) < 0x7fffffffull && (!g.dcopy || span(g.dc_shard, g.dc_blk) < 0x7fffffffull);
}

hipError_t launch_probe_rs_transform_gf16(uint32_t k, const uint8_t* src, uint8_t* dst, uint32_t ntiles,
                                          hipStream_t s) {
  switch (k) {
    case 256: return g16::launch_probe<8>(src, dst, ntiles, s);
    case 512: return g16::launch_probe<9>(src, dst, ntiles, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_rs_encode_gf16x(const RsGeom& g, hipStream_t s) {
  if (!gf16x_geom_ok(g)) return hipErrorInvalidValue;
  switch (g.n) {
    case 256: return g16::launch<8>(g, s);
    case 512: return g16::launch<9>(g, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace cel
