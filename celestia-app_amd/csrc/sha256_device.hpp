// SHA-256 (FIPS 180-4) compression for one message per lane on gfx950.
//
// Replaces Go crypto/sha256 (reached through appconsts.NewBaseHashFunc,
// pkg/appconsts/global_consts.go:86) for the NMT and RFC-6962 hashing of the DAH.
// Everything lives in VGPRs: rotates are v_alignbit_b32, Ch/Maj are v_bfi_b32,
// the round sums fold into v_add3_u32. The 16-word message window is rolled in
// place; callers feed message words already in big-endian word order.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace cel {

__device__ __forceinline__ uint32_t rotr32(uint32_t x, uint32_t n) { return __builtin_amdgcn_alignbit(x, x, n); }
// gfx950 v_bitop3_b32: any boolean function of three inputs in one VALU op.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t maj3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
}

// byte swap of a dword via one v_perm_b32
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_amdgcn_perm(0u, x, 0x00010203u); }

struct Sha256 {
  uint32_t h[8];
  __device__ __forceinline__ void init() {
    h[0] = 0x6a09e667u; h[1] = 0xbb67ae85u; h[2] = 0x3c6ef372u; h[3] = 0xa54ff53au;
    h[4] = 0x510e527fu; h[5] = 0x9b05688cu; h[6] = 0x1f83d9abu; h[7] = 0x5be0cd19u;
  }
};

__constant__ const uint32_t kSha256K[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

struct ShaRegs {
  uint32_t a, b, c, d, e, f, g, h;
};

__device__ __forceinline__ void sha_round(ShaRegs& r, uint32_t kw) {
  const uint32_t S1 = xor3(rotr32(r.e, 6), rotr32(r.e, 11), rotr32(r.e, 25));
  const uint32_t ch = (r.e & r.f) | (~r.e & r.g);  // v_bfi_b32 / v_bitop3
  const uint32_t t1 = r.h + S1 + ch + kw;
  const uint32_t S0 = xor3(rotr32(r.a, 2), rotr32(r.a, 13), rotr32(r.a, 22));
  const uint32_t t2 = S0 + maj3(r.a, r.b, r.c);
  r.h = r.g; r.g = r.f; r.f = r.e; r.e = r.d + t1; r.d = r.c; r.c = r.b; r.b = r.a; r.a = t1 + t2;
}

// Rounds [START, 64) of one compression of the 16-word block w into st, with r0 the
// working variables after round START - 1. START > 0 skips the rounds of a message
// prefix that is the same for every lane (precomputed by sha_midstate at compile time);
// w must still hold the prefix words, the message schedule reads them. Rounds run as
// four unrolled 16-round bodies inside a rolled loop: the scheduler's window stays one
// body wide, which keeps the state + 16-word window near 40 VGPRs instead of letting it
// hoist the whole message schedule (200+ VGPRs, occupancy 2).
template <int START>
__device__ __forceinline__ void sha256_compress_from(uint32_t (&st)[8], const ShaRegs& r0, uint32_t (&w)[16]) {
  ShaRegs r = r0;
#pragma unroll
  for (int i = START; i < 16; i++) sha_round(r, w[i] + kSha256K[i]);
#pragma unroll 1
  for (int base = 16; base < 64; base += 16) {
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const uint32_t w15 = w[(j + 1) & 15], w2 = w[(j + 14) & 15];
      const uint32_t s0 = xor3(rotr32(w15, 7), rotr32(w15, 18), w15 >> 3);
      const uint32_t s1 = xor3(rotr32(w2, 17), rotr32(w2, 19), w2 >> 10);
      const uint32_t wi = w[j] + s0 + w[(j + 9) & 15] + s1;
      w[j] = wi;
      sha_round(r, wi + kSha256K[base + j]);
    }
  }
  st[0] += r.a; st[1] += r.b; st[2] += r.c; st[3] += r.d;
  st[4] += r.e; st[5] += r.f; st[6] += r.g; st[7] += r.h;
}

__device__ __forceinline__ void sha256_compress(uint32_t (&st)[8], uint32_t (&w)[16]) {
  sha256_compress_from<0>(st, ShaRegs{st[0], st[1], st[2], st[3], st[4], st[5], st[6], st[7]}, w);
}

// The same compression with all 64 rounds unrolled: for latency-bound kernels (one wave
// per SIMD, a serial chain of compressions), where a rolled loop's overhead is on the
// chain and message words known at compile time (padding blocks) fold into the schedule.
__device__ __forceinline__ void sha256_compress_unrolled(uint32_t (&st)[8], uint32_t (&w)[16]) {
  ShaRegs r{st[0], st[1], st[2], st[3], st[4], st[5], st[6], st[7]};
#pragma unroll
  for (int i = 0; i < 16; i++) sha_round(r, w[i] + kSha256K[i]);
#pragma unroll
  for (int i = 16; i < 64; i++) {
    const int j = i & 15;
    const uint32_t w15 = w[(j + 1) & 15], w2 = w[(j + 14) & 15];
    const uint32_t s0 = xor3(rotr32(w15, 7), rotr32(w15, 18), w15 >> 3);
    const uint32_t s1 = xor3(rotr32(w2, 17), rotr32(w2, 19), w2 >> 10);
    const uint32_t wi = w[j] + s0 + w[(j + 9) & 15] + s1;
    w[j] = wi;
    sha_round(r, wi + kSha256K[i]);
  }
  st[0] += r.a; st[1] += r.b; st[2] += r.c; st[3] += r.d;
  st[4] += r.e; st[5] += r.f; st[6] += r.g; st[7] += r.h;
}

// Compile-time SHA-256: working variables after the first n rounds of a first block
// (chaining value = IV) whose words w[0..n) are constants. Used for the constant
// prefixes of parity leaves (0x00 || 0xFF*27...) and parity inner nodes (0x01 || 0xFF*55).
struct ShaMid {
  uint32_t v[8];
};
constexpr uint32_t kShaKc[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u};
constexpr uint32_t c_rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
constexpr ShaMid sha_midstate(const uint32_t* w, int n) {
  uint32_t a = 0x6a09e667u, b = 0xbb67ae85u, c = 0x3c6ef372u, d = 0xa54ff53au;
  uint32_t e = 0x510e527fu, f = 0x9b05688cu, g = 0x1f83d9abu, h = 0x5be0cd19u;
  for (int i = 0; i < n; i++) {
    const uint32_t t1 = h + (c_rotr(e, 6) ^ c_rotr(e, 11) ^ c_rotr(e, 25)) + ((e & f) ^ (~e & g)) + kShaKc[i] + w[i];
    const uint32_t t2 = (c_rotr(a, 2) ^ c_rotr(a, 13) ^ c_rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  return ShaMid{{a, b, c, d, e, f, g, h}};
}
__device__ __forceinline__ ShaRegs mid_regs(const ShaMid& m) {
  return ShaRegs{m.v[0], m.v[1], m.v[2], m.v[3], m.v[4], m.v[5], m.v[6], m.v[7]};
}

__device__ __forceinline__ void sha256_init(uint32_t (&st)[8]) {
  st[0] = 0x6a09e667u; st[1] = 0xbb67ae85u; st[2] = 0x3c6ef372u; st[3] = 0xa54ff53au;
  st[4] = 0x510e527fu; st[5] = 0x9b05688cu; st[6] = 0x1f83d9abu; st[7] = 0x5be0cd19u;
}

// v_perm_b32 byte select: result byte b = sel byte b picks from {S0:S1} (0-3 = S1 bytes,
// 4-7 = S0 bytes, 12 = 0x00). perm(a, b, sel) with little-endian dwords a (high) and b (low).
__device__ __forceinline__ uint32_t perm(uint32_t s0, uint32_t s1, uint32_t sel) {
  return __builtin_amdgcn_perm(s0, s1, sel);
}

}  // namespace cel
