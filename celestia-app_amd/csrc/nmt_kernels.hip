// Namespaced Merkle tree roots and the DataAvailabilityHeader hash on gfx950.
//
// Replaces, for the 4k axes of a 2k x 2k EDS:
//   rsmt2d RowRoots/ColRoots [dep] -> wrapper.ErasuredNamespacedMerkleTree.Push/Root
//   (pkg/wrapper/nmt_wrapper.go:93-124) -> nmt v0.22.0 HashLeaf / HashNode with
//   IgnoreMaxNamespace (text copy: test/util/malicious/hasher.go:196-310), and
//   DataAvailabilityHeader.Hash (pkg/da/data_availability_header.go:92-108) ->
//   go-square/merkle RFC-6962.
//
// Work decomposition (one message per lane everywhere):
//   k_leaf   : one lane per EDS cell. A cell's row leaf and column leaf are the same
//              bytes (the Q0 test of nmt_wrapper.go:138-140 is symmetric), so each
//              leaf is hashed once: 4k^2 x 9 compressions instead of the reference's
//              8k^2 x 9. Also checks the honest push order on Q0.
//   k_level  : one lane per inner node of one tree level, all 4k trees at once.
//   k_dah    : one workgroup per square, RFC-6962 over the 4k roots.
// Nodes live on the device as 96-byte records (90 B node + 6 zero bytes) = 24 dwords.
#include <hip/hip_runtime.h>

#include <climits>

#include "cel_internal.hpp"
#include "sha256_device.hpp"

namespace cel {

struct Node {
  uint32_t d[kNodeWords];
};

__device__ __forceinline__ void load_node(const uint32_t* p, uint32_t (&n)[kNodeWords]) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
  for (int i = 0; i < 6; i++) {
    const uint4 v = q[i];
    n[4 * i] = v.x; n[4 * i + 1] = v.y; n[4 * i + 2] = v.z; n[4 * i + 3] = v.w;
  }
}

__device__ __forceinline__ void store_node(uint32_t* p, const uint32_t (&n)[kNodeWords]) {
  uint4* q = reinterpret_cast<uint4*>(p);
#pragma unroll
  for (int i = 0; i < 6; i++) q[i] = make_uint4(n[4 * i], n[4 * i + 1], n[4 * i + 2], n[4 * i + 3]);
}

// Node dwords 14..23 from the 8 big-endian digest words (digest = node bytes 58..89).
// nd14 keeps its low 16 bits (the last two max-namespace bytes).
__device__ __forceinline__ void put_digest(uint32_t (&nd)[kNodeWords], const uint32_t (&st)[8]) {
  uint32_t sw[8];
#pragma unroll
  for (int i = 0; i < 8; i++) sw[i] = bswap32(st[i]);
  nd[14] = (nd[14] & 0xFFFFu) | (sw[0] << 16);
#pragma unroll
  for (int i = 15; i <= 21; i++) nd[i] = __builtin_amdgcn_alignbyte(sw[i - 14], sw[i - 15], 2);
  nd[22] = sw[7] >> 16;
  nd[23] = 0;
}

// --------------------------------------------------------------------- leaves

// Leaf message: 0x00 || ns(29) || share(512) = 542 B -> 9 blocks.
// sh = the share's little-endian dwords; ns = share[0:29] for Q0 cells, 0xFF*29 else.
// Message word at byte p >= 32 is share bytes q..q+3 with q = p - 30 (q = 2 mod 4):
// bytes 2,3 of dword (q-2)/4 and bytes 0,1 of the next -> one v_perm_b32 (and the
// byte swap to big-endian comes for free in the same select).
// Parity cells: message bytes 0..27 are 0x00 || 0xFF*27 (ns = 0xFF*29 continues into w7).
constexpr uint32_t kLeafParPrefix[7] = {0x00FFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu,
                                        0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
constexpr ShaMid kLeafParMid = sha_midstate(kLeafParPrefix, 7);

// PF (prefetch): the next block's words are loaded while the current block is compressed.
// At one or two waves per SIMD (a single square's commit, a rank's slab) nothing else
// covers a block's load latency, which the plain form exposes nine times per leaf; at
// batch occupancy other waves cover it and the 17 extra VGPRs cost 1.5-3 %
// (profiles/r2_nmt_leaf_prefetch_ab.txt), so the batch keeps PF = false.
template <bool PF>
__device__ __forceinline__ void leaf_hash(uint32_t (&st)[8], const uint32_t* __restrict__ sh, bool q0) {
  sha256_init(st);
  uint32_t w[16];
  uint32_t nx[17];  // PF: the next block's share dwords
  auto load17 = [&](int b) {  // share bytes [64b-30, 64b+34) for block b = 1..7
    const uint32_t* base = sh + 16 * b - 8;
    const uint4* p4 = reinterpret_cast<const uint4*>(base);
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const uint4 v = p4[i];
      nx[4 * i] = v.x; nx[4 * i + 1] = v.y; nx[4 * i + 2] = v.z; nx[4 * i + 3] = v.w;
    }
    nx[16] = base[16];
  };
  {  // block 0: 0x00 || ns || share[0:34]
    uint32_t s[9];
    const uint4* p4 = reinterpret_cast<const uint4*>(sh);
    const uint4 v0 = p4[0], v1 = p4[1];
    s[0] = v0.x; s[1] = v0.y; s[2] = v0.z; s[3] = v0.w; s[4] = v1.x; s[5] = v1.y; s[6] = v1.z; s[7] = v1.w;
    s[8] = sh[8];
    if (PF) load17(1);
#pragma unroll
    for (int i = 8; i < 16; i++) w[i] = perm(s[i - 8], s[i - 7], 0x06070001u);
    if (__all(!q0)) {  // wave-uniform parity cells: rounds 0..6 are one constant
#pragma unroll
      for (int i = 0; i < 7; i++) w[i] = kLeafParPrefix[i];
      w[7] = 0xFFFF0000u | perm(0u, s[0], 0x0C0C0001u);
      sha256_compress_from<7>(st, mid_regs(kLeafParMid), w);
    } else {
      if (q0) {
        w[0] = perm(0u, s[0], 0x0C000102u);
#pragma unroll
        for (int i = 1; i < 7; i++) w[i] = perm(s[i - 1], s[i], 0x07000102u);
        w[7] = perm(s[6], s[7], 0x07000C0Cu) | perm(0u, s[0], 0x0C0C0001u);
      } else {
#pragma unroll
        for (int i = 0; i < 7; i++) w[i] = kLeafParPrefix[i];
        w[7] = 0xFFFF0000u | perm(0u, s[0], 0x0C0C0001u);
      }
      sha256_compress(st, w);
    }
  }
#pragma unroll 1
  for (int b = 1; b < 8; b++) {  // blocks 1..7: share bytes [64b-30, 64b+34)
    if (!PF) load17(b);
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = perm(nx[i], nx[i + 1], 0x06070001u);
    if (PF) {
      if (b < 7) {
        load17(b + 1);
      } else {  // the last block's 8 dwords
        const uint4* p4 = reinterpret_cast<const uint4*>(sh + 120);
        const uint4 v0 = p4[0], v1 = p4[1];
        nx[0] = v0.x; nx[1] = v0.y; nx[2] = v0.z; nx[3] = v0.w; nx[4] = v1.x; nx[5] = v1.y; nx[6] = v1.z; nx[7] = v1.w;
      }
    }
    sha256_compress(st, w);
  }
  {  // block 8: share[482:512] || 0x80 || 0... || len
    if (!PF) {
      const uint4* p4 = reinterpret_cast<const uint4*>(sh + 120);
      const uint4 v0 = p4[0], v1 = p4[1];
      nx[0] = v0.x; nx[1] = v0.y; nx[2] = v0.z; nx[3] = v0.w; nx[4] = v1.x; nx[5] = v1.y; nx[6] = v1.z; nx[7] = v1.w;
    }
#pragma unroll
    for (int i = 0; i < 7; i++) w[i] = perm(nx[i], nx[i + 1], 0x06070001u);
    w[7] = perm(nx[7], 0x80u, 0x0607000Cu);
#pragma unroll
    for (int i = 8; i < 15; i++) w[i] = 0u;
    w[15] = 542u * 8u;
    sha256_compress(st, w);
  }
}

// Namespace order: is ns(a) < ns(b)? (29-byte lexicographic compare of share prefixes)
__device__ __forceinline__ bool ns_less(const uint32_t* __restrict__ a, const uint32_t* __restrict__ b) {
  const uint4* pa = reinterpret_cast<const uint4*>(a);
  const uint4* pb = reinterpret_cast<const uint4*>(b);
  uint32_t x[8], y[8];
#pragma unroll
  for (int i = 0; i < 2; i++) {
    const uint4 u = pa[i], v = pb[i];
    x[4 * i] = u.x; x[4 * i + 1] = u.y; x[4 * i + 2] = u.z; x[4 * i + 3] = u.w;
    y[4 * i] = v.x; y[4 * i + 1] = v.y; y[4 * i + 2] = v.z; y[4 * i + 3] = v.w;
  }
  int res = 0;  // -1 a<b, 1 a>b
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint32_t xa = bswap32(x[i]), yb = bswap32(y[i]);
    if (i == 7) { xa &= 0xFF000000u; yb &= 0xFF000000u; }
    if (res == 0 && xa != yb) res = xa < yb ? -1 : 1;
  }
  return res < 0;
}

// Leaf node of one EDS cell: ns || ns || SHA256(0x00 || ns || share), ns = share[0:29]
// for Q0 cells and 0xFF*29 (parity namespace) otherwise.
template <bool PF>
__device__ __forceinline__ void make_leaf_node(const uint32_t* __restrict__ sh, bool q0, uint32_t (&nd)[kNodeWords]) {
  uint32_t st[8];
  leaf_hash<PF>(st, sh, q0);
  if (q0) {
    const uint4* p4 = reinterpret_cast<const uint4*>(sh);
    uint32_t s[8];
    const uint4 v0 = p4[0], v1 = p4[1];
    s[0] = v0.x; s[1] = v0.y; s[2] = v0.z; s[3] = v0.w; s[4] = v1.x; s[5] = v1.y; s[6] = v1.z; s[7] = v1.w;
#pragma unroll
    for (int i = 0; i < 7; i++) nd[i] = s[i];
    nd[7] = (s[7] & 0xFFu) | (s[0] << 8);
#pragma unroll
    for (int i = 0; i < 6; i++) nd[8 + i] = __builtin_amdgcn_alignbyte(s[i + 1], s[i], 3);
    nd[14] = (s[6] >> 24) | ((s[7] & 0xFFu) << 8);
  } else {
#pragma unroll
    for (int i = 0; i < 14; i++) nd[i] = 0xFFFFFFFFu;
    nd[14] = 0xFFFFu;
  }
  put_digest(nd, st);
}

// grid: x = cell block (256 cells from cell0), y = square. Writes leaf nodes [sq][W*W][24]
// of cells [cell0, cell1).
template <bool ORDER, bool PF>
__global__ __launch_bounds__(256) void k_leaf(const uint8_t* __restrict__ eds, uint32_t k, uint32_t* __restrict__ leaves,
                                              int32_t* __restrict__ bad_axis, uint32_t cell0, uint32_t cell1) {
  const uint32_t W = 2 * k;
  const uint32_t cell = cell0 + blockIdx.x * 256u + threadIdx.x;
  if (cell >= cell1) return;
  const uint32_t r = cell / W, c = cell % W;
  const uint64_t sq_eds = (uint64_t)W * W * kShare;
  const uint32_t* sh = reinterpret_cast<const uint32_t*>(eds + blockIdx.y * sq_eds + (uint64_t)cell * kShare);
  const bool q0 = (r < k) && (c < k);
  {
    uint32_t nd[kNodeWords];
    make_leaf_node<PF>(sh, q0, nd);
    store_node(leaves + ((uint64_t)blockIdx.y * W * W + cell) * kNodeWords, nd);
  }
  // The push-order check runs after the hash: done first, its share prefixes stay live
  // across the nine compressions (103 VGPRs, 4 waves/SIMD, against 52 and 8).
  __builtin_amdgcn_sched_barrier(0);
  if (ORDER && q0) {
    if (c > 0 && ns_less(sh, sh - kShare / 4)) atomicMin(bad_axis + blockIdx.y, (int32_t)r);
    if (r > 0 && ns_less(sh, sh - (uint64_t)W * kShare / 4)) atomicMin(bad_axis + blockIdx.y, (int32_t)(W + c));
  }
}

// ---------------------------------------------------------------- inner nodes

// HashNode(L, R): message 0x01 || L(90) || R(90) = 181 B -> 3 blocks.
// minNs = L.min; maxNs = (R.min == 0xFF*29) ? L.max : R.max  (IgnoreMaxNamespace).
// Parity left child (min = max = 0xFF*29, nodes of Q1-Q3): message bytes 0..55 are
// 0x01 || 0xFF*55 for every such node, so rounds 0..13 of block 0 are one constant.
constexpr uint32_t kNodeParPrefix[14] = {0x01FFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu,
                                         0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu,
                                         0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
constexpr ShaMid kNodeParMid = sha_midstate(kNodeParPrefix, 14);

__device__ __forceinline__ uint32_t node_word(const uint32_t (&L)[kNodeWords], const uint32_t (&R)[kNodeWords], int q) {
  if (q == 0) return perm(1u, L[0], 0x04000102u);
  if (q <= 21) return perm(L[q - 1], L[q], 0x07000102u);
  if (q == 22) return perm(L[21], L[22], 0x0700010Cu) | (R[0] & 0xFFu);
  if (q <= 44) return perm(R[q - 23], R[q - 22], 0x05060700u);
  if (q == 45) return perm(R[22], 0x80u, 0x05000C0Cu);
  if (q == 47) return 181u * 8u;
  return 0u;
}

__device__ __forceinline__ void hash_node(const uint32_t (&L)[kNodeWords], const uint32_t (&R)[kNodeWords],
                                          uint32_t (&out)[kNodeWords]) {
  uint32_t st[8];
  sha256_init(st);
  bool lpar = (L[14] & 0xFFFFu) == 0xFFFFu;
#pragma unroll
  for (int i = 0; i < 14; i++) lpar = lpar && (L[i] == 0xFFFFFFFFu);
  {
    uint32_t w[16];
    if (__all(lpar)) {  // wave-uniform: the whole wave starts block 0 at round 14
#pragma unroll
      for (int wi = 0; wi < 14; wi++) w[wi] = kNodeParPrefix[wi];
      w[14] = node_word(L, R, 14);
      w[15] = node_word(L, R, 15);
      sha256_compress_from<14>(st, mid_regs(kNodeParMid), w);
    } else {
#pragma unroll
      for (int wi = 0; wi < 16; wi++) w[wi] = node_word(L, R, wi);
      sha256_compress(st, w);
    }
  }
#pragma unroll
  for (int b = 1; b < 3; b++) {
    uint32_t w[16];
#pragma unroll
    for (int wi = 0; wi < 16; wi++) w[wi] = node_word(L, R, 16 * b + wi);
    sha256_compress(st, w);
  }
  bool rpar = (R[7] & 0xFFu) == 0xFFu;
#pragma unroll
  for (int i = 0; i < 7; i++) rpar = rpar && (R[i] == 0xFFFFFFFFu);
  // out: min from L (bytes 0..28), max from L or R (bytes 29..57)
#pragma unroll
  for (int i = 0; i < 7; i++) out[i] = L[i];
  const uint32_t X7 = rpar ? L[7] : R[7];
  out[7] = (L[7] & 0xFFu) | (X7 & 0xFFFFFF00u);
#pragma unroll
  for (int i = 8; i < 14; i++) out[i] = rpar ? L[i] : R[i];
  out[14] = (rpar ? L[14] : R[14]) & 0xFFFFu;
  put_digest(out, st);
}

// One tree level for all trees. Input addressing:
//   FROM_LEAVES: tree t < W is row t (children leaves (t, 2j), (t, 2j+1));
//                tree t >= W is column t-W (children (2j, c), (2j+1, c)).
//   otherwise  : in[sq][t][2j], in[sq][t][2j+1] with `nin` nodes per tree.
__device__ __forceinline__ void rfc_leaf90(const uint32_t (&R)[kNodeWords], uint32_t (&st)[8]);

// One tree level for all trees. At the root level the lane writes its root, packed to
// 90 bytes, straight into the caller's row_out / col_out ([nsq][W][90]); with
// leafd != nullptr it also hashes the root as an RFC-6962 leaf of the DAH tree
// (2 compressions) so the per-square DAH kernel starts from leaf digests.
template <bool FROM_LEAVES>
__global__ __launch_bounds__(256) void k_level(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, uint32_t W,
                                               uint32_t nin, uint32_t trees, uint32_t* __restrict__ leafd,
                                               uint8_t* __restrict__ row_out, uint8_t* __restrict__ col_out) {
  const uint32_t nout = nin / 2;
  const uint32_t idx = blockIdx.x * 256u + threadIdx.x;
  if (idx >= trees * nout) return;
  const uint32_t t = idx / nout, j = idx % nout;
  uint64_t li, ri;
  if (FROM_LEAVES) {
    const uint64_t sq = (uint64_t)blockIdx.y * W * W;
    if (t < W) { li = sq + (uint64_t)t * W + 2 * j; ri = li + 1; }
    else { li = sq + (uint64_t)(2 * j) * W + (t - W); ri = li + W; }
  } else {
    const uint64_t sq = (uint64_t)blockIdx.y * trees * nin;
    li = sq + (uint64_t)t * nin + 2 * j;
    ri = li + 1;
  }
  uint32_t L[kNodeWords], R[kNodeWords], o[kNodeWords];
  load_node(in + li * kNodeWords, L);
  load_node(in + ri * kNodeWords, R);
  hash_node(L, R, o);
  const uint64_t oi = (uint64_t)blockIdx.y * trees * nout + idx;
  store_node(out + oi * kNodeWords, o);
  if (row_out) {
    {  // 90-byte record at a 2-byte aligned address: 45 halfword stores
      uint8_t* r = (t < W ? row_out + ((uint64_t)blockIdx.y * W + t) * kNode
                          : col_out + ((uint64_t)blockIdx.y * W + (t - W)) * kNode);
      uint16_t* r16 = reinterpret_cast<uint16_t*>(r);
#pragma unroll
      for (int i = 0; i < 45; i++) r16[i] = (uint16_t)(o[i / 2] >> (16 * (i & 1)));
    }
  }
  if (leafd) {
    uint32_t st[8];
    rfc_leaf90(o, st);
    uint4* d = reinterpret_cast<uint4*>(leafd + oi * 8);
    d[0] = make_uint4(st[0], st[1], st[2], st[3]);
    d[1] = make_uint4(st[4], st[5], st[6], st[7]);
  }
}

// ------------------------------------------------------------------ RFC-6962

// leafHash = SHA256(0x00 || item) for a 90-byte item (2 blocks).
__device__ __forceinline__ void rfc_leaf90(const uint32_t (&R)[kNodeWords], uint32_t (&st)[8]) {
  sha256_init(st);
#pragma unroll
  for (int b = 0; b < 2; b++) {
    uint32_t w[16];
#pragma unroll
    for (int wi = 0; wi < 16; wi++) {
      const int q = 16 * b + wi;
      uint32_t x;
      if (q == 0) x = perm(0u, R[0], 0x0C000102u);
      else if (q <= 21) x = perm(R[q - 1], R[q], 0x07000102u);
      else if (q == 22) x = perm(R[21], R[22], 0x0700010Cu) | 0x80u;
      else if (q == 31) x = 91u * 8u;
      else x = 0u;
      w[wi] = x;
    }
    sha256_compress(st, w);
  }
}

// innerHash = SHA256(0x01 || l(32) || r(32)) (2 blocks). The DAH tree hashes its levels
// one after the other in one workgroup (a latency chain), so both compressions are
// unrolled; the second block's 15 constant words fold into its schedule.
__device__ __forceinline__ void rfc_inner(const uint32_t* l, const uint32_t* r, uint32_t (&st)[8]) {
  uint32_t w[16];
  w[0] = 0x01000000u | (l[0] >> 8);
#pragma unroll
  for (int i = 1; i < 8; i++) w[i] = __builtin_amdgcn_alignbit(l[i - 1], l[i], 8);
  w[8] = __builtin_amdgcn_alignbit(l[7], r[0], 8);
#pragma unroll
  for (int i = 9; i < 16; i++) w[i] = __builtin_amdgcn_alignbit(r[i - 9], r[i - 8], 8);
  sha256_init(st);
  uint32_t w2[16];
  w2[0] = (r[7] << 24) | 0x00800000u;
#pragma unroll
  for (int i = 1; i < 15; i++) w2[i] = 0;
  w2[15] = 65u * 8u;
  sha256_compress(st, w);
  sha256_compress(st, w2);
}

// SHA256 of the empty string (RFC-6962 empty tree).
__device__ __forceinline__ void sha_empty(uint32_t (&st)[8]) {
  uint32_t w[16];
  w[0] = 0x80000000u;
#pragma unroll
  for (int i = 1; i < 16; i++) w[i] = 0;
  sha256_init(st);
  sha256_compress(st, w);
}

// One workgroup per item list: items[g][n] 96-byte records -> 32-byte root (BE words in
// out[g*8..]). Also packs the first n items into 90-byte outputs (row/col roots) if given.
// out_src / host_out (one square, optional): after the DAH, the workgroup copies out_bytes
// (a multiple of 16) from out_src (roots | dah | status, written before the copy) to host_out,
// page-locked host memory, with 16-byte stores: the results cross PCIe inside this launch
// instead of in a separate copy after it.
// row_out, col_out, dah and status may all lie inside [out_src, out_src + out_bytes) (the
// one-square path copies that block out to host_out after writing it), so none of the four
// nor out_src is __restrict__: the copy-out loads must see thread 0's dah / status stores.
__global__ __launch_bounds__(1024) void k_merkle(const uint32_t* __restrict__ items, const uint32_t* __restrict__ leafd,
                                                uint32_t n, uint8_t* dah, uint8_t* row_out, uint8_t* col_out,
                                                const int32_t* __restrict__ bad_axis, int32_t* status,
                                                const uint8_t* out_src = nullptr, uint8_t* __restrict__ host_out = nullptr,
                                                uint32_t out_bytes = 0) {
  extern __shared__ __attribute__((aligned(16))) uint32_t hs[];  // n * 8 words
  const uint32_t g = blockIdx.x;
  const uint32_t* it = items + (uint64_t)g * n * kNodeWords;
  if (leafd) {
    for (uint32_t i = threadIdx.x; i < n * 8; i += blockDim.x) hs[i] = leafd[(uint64_t)g * n * 8 + i];
  } else {
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
      uint32_t R[kNodeWords], st[8];
      load_node(it + (uint64_t)i * kNodeWords, R);
      rfc_leaf90(R, st);
#pragma unroll
      for (int j = 0; j < 8; j++) hs[i * 8 + j] = st[j];
    }
  }
  // pack 90-byte roots (first half rows, second half columns)
  if (row_out) {
    const uint32_t half = n / 2;
    for (uint32_t b = threadIdx.x; b < n * kNode; b += blockDim.x) {
      const uint32_t i = b / kNode, o = b % kNode;
      const uint8_t v = reinterpret_cast<const uint8_t*>(it + (uint64_t)i * kNodeWords)[o];
      if (i < half) row_out[((uint64_t)g * half + i) * kNode + o] = v;
      else col_out[((uint64_t)g * half + (i - half)) * kNode + o] = v;
    }
  }
  __syncthreads();
  uint32_t cnt = n;
  while (cnt > 1) {
    const uint32_t half = cnt / 2;
    uint32_t st[8];
    for (uint32_t base = 0; base < half; base += blockDim.x) {
      const uint32_t i = base + threadIdx.x;
      if (i < half) rfc_inner(hs + (2 * i) * 8, hs + (2 * i + 1) * 8, st);
      __syncthreads();
      if (i < half) {
#pragma unroll
        for (int j = 0; j < 8; j++) hs[i * 8 + j] = st[j];
      }
      __syncthreads();
    }
    if (cnt & 1) {
      if (threadIdx.x < 8) hs[half * 8 + threadIdx.x] = hs[(cnt - 1) * 8 + threadIdx.x];
      __syncthreads();
    }
    cnt = half + (cnt & 1);
  }
  if (threadIdx.x == 0) {
    uint32_t st[8];
    if (n == 0) sha_empty(st);
    else
      for (int j = 0; j < 8; j++) st[j] = hs[j];
    for (int j = 0; j < 8; j++) {
      dah[g * 32 + 4 * j] = (uint8_t)(st[j] >> 24);
      dah[g * 32 + 4 * j + 1] = (uint8_t)(st[j] >> 16);
      dah[g * 32 + 4 * j + 2] = (uint8_t)(st[j] >> 8);
      dah[g * 32 + 4 * j + 3] = (uint8_t)st[j];
    }
    if (status) status[g] = (bad_axis && bad_axis[g] != INT_MAX) ? CEL_EORDER : CEL_OK;
  }
  if (host_out) {
    __threadfence();  // thread 0's dah / status stores before the workgroup reads them back
    __syncthreads();
    const uint4* src = reinterpret_cast<const uint4*>(out_src);
    uint4* dst = reinterpret_cast<uint4*>(host_out);
    for (uint32_t i = threadIdx.x; i < out_bytes / 16; i += blockDim.x) dst[i] = src[i];
  }
}

// Threads of a k_merkle workgroup: one per pair of the widest level (each level is one
// round of 2-compression hashes then), 64..1024.
static uint32_t merkle_block(uint32_t n) {
  const uint32_t pairs = ((n / 2 + 63) / 64) * 64;
  return pairs < 64 ? 64u : (pairs > 1024 ? 1024u : pairs);
}

// RFC-6962 leaf digests of n node records, one lane each (k_merkle then starts from them),
// and the records packed to 90 bytes: the first n/2 into row_out, the rest into col_out.
__global__ __launch_bounds__(256) void k_dah_leaves(const uint32_t* __restrict__ items, uint32_t n,
                                                    uint32_t* __restrict__ leafd, uint8_t* __restrict__ row_out,
                                                    uint8_t* __restrict__ col_out) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  uint32_t R[kNodeWords], st[8];
  load_node(items + (uint64_t)i * kNodeWords, R);
  rfc_leaf90(R, st);
  uint4* d = reinterpret_cast<uint4*>(leafd + (uint64_t)i * 8);
  d[0] = make_uint4(st[0], st[1], st[2], st[3]);
  d[1] = make_uint4(st[4], st[5], st[6], st[7]);
  const uint32_t half = n / 2;
  uint16_t* r16 = reinterpret_cast<uint16_t*>(i < half ? row_out + (uint64_t)i * kNode : col_out + (uint64_t)(i - half) * kNode);
#pragma unroll
  for (int j = 0; j < 45; j++) r16[j] = (uint16_t)(R[j / 2] >> (16 * (j & 1)));
}

__global__ void k_fill_i32(int32_t* p, uint32_t n, int32_t v) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

// ----------------------------------------------------------------- launchers

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// A leaf launch of this many lanes leaves at most two waves per SIMD (1024 SIMDs): load
// latency is then exposed and the prefetching leaf hash (leaf_hash<true>) pays.
static bool latency_bound(uint64_t lanes) { return lanes <= 2ull * 1024 * 64; }

// Workspace: leaves [nsq][W*W] nodes | ping [nsq][2W][W/2] | pong [nsq][2W][W/4] |
//            roots [nsq][2W] nodes | bad_axis [nsq] int32 | DAH leaf digests [nsq][2W][8]
size_t nmt_workspace_size(uint32_t k, uint32_t nsq) {
  const size_t W = 2 * (size_t)k, nb = kNodeWords * 4;
  return align256(nsq * W * W * nb) + align256(nsq * 2 * W * (W / 2 + 1) * nb) +
         align256(nsq * 2 * W * (W / 4 + 1) * nb) + align256(nsq * 2 * W * nb) + align256(nsq * 4 + 4) +
         align256(nsq * 2 * W * 32);
}

struct CommitWork {
  uint32_t *leaves, *ping, *pong, *roots, *leafd;
  int32_t* bad;
};

static CommitWork commit_work(void* work, uint32_t k, uint32_t nsq) {
  const uint32_t W = 2 * k;
  const size_t nb = kNodeWords * 4;
  uint8_t* base = static_cast<uint8_t*>(work);
  CommitWork w;
  w.leaves = reinterpret_cast<uint32_t*>(base);
  base += align256((size_t)nsq * W * W * nb);
  w.ping = reinterpret_cast<uint32_t*>(base);
  base += align256((size_t)nsq * 2 * W * (W / 2 + 1) * nb);
  w.pong = reinterpret_cast<uint32_t*>(base);
  base += align256((size_t)nsq * 2 * W * (W / 4 + 1) * nb);
  w.roots = reinterpret_cast<uint32_t*>(base);
  base += align256((size_t)nsq * 2 * W * nb);
  w.bad = reinterpret_cast<int32_t*>(base);
  base += align256((size_t)nsq * 4 + 4);
  w.leafd = reinterpret_cast<uint32_t*>(base);
  return w;
}

hipError_t launch_commit_leaves(const uint8_t* eds, uint32_t k, uint32_t nsq, void* work, bool order_check,
                                uint32_t row0, uint32_t row1, bool init_bad, hipStream_t s) {
  const uint32_t W = 2 * k;
  const CommitWork w = commit_work(work, k, nsq);
  const Range r("nmt.leaf");
  if (init_bad) hipLaunchKernelGGL(k_fill_i32, dim3((nsq + 255) / 256), dim3(256), 0, s, w.bad, nsq, INT_MAX);
  const uint32_t c0 = row0 * W, c1 = row1 * W;
  if (c1 <= c0) return hipGetLastError();
  dim3 gl((c1 - c0 + 255) / 256, nsq);
  if (latency_bound((uint64_t)(c1 - c0) * nsq)) {
    if (order_check) hipLaunchKernelGGL((k_leaf<true, true>), gl, dim3(256), 0, s, eds, k, w.leaves, w.bad, c0, c1);
    else hipLaunchKernelGGL((k_leaf<false, true>), gl, dim3(256), 0, s, eds, k, w.leaves, w.bad, c0, c1);
  } else {
    if (order_check) hipLaunchKernelGGL((k_leaf<true, false>), gl, dim3(256), 0, s, eds, k, w.leaves, w.bad, c0, c1);
    else hipLaunchKernelGGL((k_leaf<false, false>), gl, dim3(256), 0, s, eds, k, w.leaves, w.bad, c0, c1);
  }
  return hipGetLastError();
}

hipError_t launch_commit_trees(uint32_t k, uint32_t nsq, uint8_t* row_roots, uint8_t* col_roots, uint8_t* dah,
                               int32_t* status, void* work, hipStream_t s, uint8_t* host_out, uint32_t out_bytes) {
  const uint32_t W = 2 * k;
  const CommitWork w = commit_work(work, k, nsq);
  // One launch per tree level, all 4k trees of all squares at once: every lane hashes
  // one node, no idle lanes. The last level writes the root records.
  const uint32_t trees = 2 * W;
  uint32_t nin = W;
  const uint32_t* src = w.leaves;
  uint32_t* dst = w.ping;
  bool first = true;
  roctxRangePushA("nmt.levels");
  while (nin > 1) {
    const uint32_t nout = nin / 2;
    uint32_t* out = (nout == 1) ? w.roots : dst;
    uint32_t* ld = (nout == 1 && dah) ? w.leafd : nullptr;  // dah == nullptr: roots only
    dim3 g((trees * nout + 255) / 256, nsq);
    uint8_t* ro = (nout == 1) ? row_roots : nullptr;
    uint8_t* co = (nout == 1) ? col_roots : nullptr;
    if (first) hipLaunchKernelGGL(k_level<true>, g, dim3(256), 0, s, src, out, W, nin, trees, ld, ro, co);
    else hipLaunchKernelGGL(k_level<false>, g, dim3(256), 0, s, src, out, W, nin, trees, ld, ro, co);
    first = false;
    src = out;
    dst = (dst == w.ping) ? w.pong : w.ping;
    nin = nout;
  }
  roctxRangePop();
  const size_t lds = (size_t)trees * 8 * 4;
  // roots already packed into row_roots / col_roots by the root level
  const Range r("dah");
  if (dah)
    hipLaunchKernelGGL(k_merkle, dim3(nsq), dim3(merkle_block(trees)), lds, s, w.roots, w.leafd, trees, dah, nullptr,
                       nullptr, w.bad, status, host_out ? row_roots : nullptr, host_out, out_bytes);
  return hipGetLastError();
}

hipError_t launch_commit(const uint8_t* eds, uint32_t k, uint32_t nsq, uint8_t* row_roots, uint8_t* col_roots,
                         uint8_t* dah, int32_t* status, void* work, bool order_check, hipStream_t s) {
  hipError_t e = launch_commit_leaves(eds, k, nsq, work, order_check, 0, 2 * k, true, s);
  if (e == hipSuccess) e = launch_commit_trees(k, nsq, row_roots, col_roots, dah, status, work, s);
  return e;
}


// ------------------------------------------------------- row-sharded mode (§8e)
//
// A rank holds a column slab of one EDS: slab[i][j] = cell (i, c0 + j), i < 2k, j < w,
// w = 2k / nranks. It hashes the slab's leaves once, builds its w column trees in full
// and, for every row, the subtree root over its w-wide slice (an aligned power-of-two
// range, hence a subtree of the row's perfect tree). Rank-ordered subtree roots are
// combined into the row roots after an all-gather.

template <bool ORDER, bool PF>
__global__ __launch_bounds__(256) void k_slab_leaf(const uint8_t* __restrict__ slab, uint32_t k, uint32_t c0, uint32_t w,
                                            uint32_t cell0, uint32_t cell1, uint32_t* __restrict__ leaves,
                                            int32_t* __restrict__ bad_axis) {
  const uint32_t W = 2 * k;
  const uint32_t cell = cell0 + blockIdx.x * 256u + threadIdx.x;
  if (cell >= cell1) return;
  const uint32_t i = cell / w, j = cell % w, c = c0 + j;
  const uint32_t* sh = reinterpret_cast<const uint32_t*>(slab + (uint64_t)cell * kShare);
  const bool q0 = (i < k) && (c < k);
  if (ORDER && q0) {
    if (j > 0 && ns_less(sh, sh - kShare / 4)) atomicMin(bad_axis, (int32_t)i);
    if (i > 0 && ns_less(sh, sh - (uint64_t)w * kShare / 4)) atomicMin(bad_axis, (int32_t)(W + c));
  }
  uint32_t nd[kNodeWords];
  make_leaf_node<PF>(sh, q0, nd);
  store_node(leaves + (uint64_t)cell * kNodeWords, nd);
}

// First tree level over a strided node grid: tree t's leaf l is in[t * tstride + l * lstride].
// Output compact: out[t][nin / 2].
__global__ __launch_bounds__(256) void k_level_grid(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, uint32_t nin,
                                              uint32_t trees, uint32_t tstride, uint32_t lstride) {
  const uint32_t nout = nin / 2;
  const uint32_t idx = blockIdx.x * 256u + threadIdx.x;
  if (idx >= trees * nout) return;
  const uint32_t t = idx / nout, j = idx % nout;
  const uint64_t li = (uint64_t)t * tstride + (uint64_t)(2 * j) * lstride, ri = li + lstride;
  uint32_t L[kNodeWords], R[kNodeWords], o[kNodeWords];
  load_node(in + li * kNodeWords, L);
  load_node(in + ri * kNodeWords, R);
  hash_node(L, R, o);
  store_node(out + (uint64_t)idx * kNodeWords, o);
}

// One level of two independent tree sets in one launch (the slab's column trees and row
// subtrees): job j reduces trees_j trees of nin_j nodes, tree t's node l at
// in_j[t * tstride_j + l * lstride_j], into out_j[t][nin_j / 2] (compact).
struct LevelJob {
  const uint32_t* in;
  uint32_t* out;
  uint32_t nin, trees, tstride, lstride;
};

__global__ __launch_bounds__(256) void k_level_pair(LevelJob a, LevelJob b) {
  uint32_t idx = blockIdx.x * 256u + threadIdx.x;
  const uint32_t na = a.nin > 1 ? a.trees * (a.nin / 2) : 0u;
  const uint32_t nb = b.nin > 1 ? b.trees * (b.nin / 2) : 0u;
  if (idx >= na + nb) return;
  const LevelJob& j = idx < na ? a : b;
  if (idx >= na) idx -= na;
  const uint32_t nout = j.nin / 2;
  const uint32_t t = idx / nout, l = idx % nout;
  const uint64_t li = (uint64_t)t * j.tstride + (uint64_t)(2 * l) * j.lstride, ri = li + j.lstride;
  uint32_t L[kNodeWords], R[kNodeWords], o[kNodeWords];
  load_node(j.in + li * kNodeWords, L);
  load_node(j.in + ri * kNodeWords, R);
  hash_node(L, R, o);
  store_node(j.out + (uint64_t)idx * kNodeWords, o);
}

// Namespace compare of two node records: is R's minNs (bytes 0..28) below L's maxNs
// (bytes 29..57)? Big-endian words: 7 full words, then the 29th byte.
__device__ __forceinline__ bool min_below_max(const uint32_t* __restrict__ R, const uint32_t* __restrict__ L) {
  uint32_t r[8], l[16];
#pragma unroll
  for (int q = 0; q < 2; q++) {
    const uint4 v = reinterpret_cast<const uint4*>(R)[q];
    r[4 * q] = v.x; r[4 * q + 1] = v.y; r[4 * q + 2] = v.z; r[4 * q + 3] = v.w;
  }
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const uint4 v = reinterpret_cast<const uint4*>(L)[q];
    l[4 * q] = v.x; l[4 * q + 1] = v.y; l[4 * q + 2] = v.z; l[4 * q + 3] = v.w;
  }
#pragma unroll
  for (int q = 0; q < 7; q++) {
    const uint32_t a = bswap32(r[q]), b = bswap32(__builtin_amdgcn_alignbyte(l[8 + q], l[7 + q], 1));
    if (a != b) return a < b;
  }
  return (r[7] & 0xFFu) < ((l[14] >> 8) & 0xFFu);
}

// The finish's status in one workgroup: the max over ranks of the gathered step-2 status
// (first int32 of record r * stride + at), or CEL_EORDER when the push order breaks
// across a slab boundary in a row of Q0 (rank r's first leaf namespace below rank r-1's
// last: the subtrees' minNs / maxNs; subs: rank r's 2k row-subtree records at
// subs[r * stride]).
__global__ __launch_bounds__(256) void k_shard_status(const uint32_t* __restrict__ subs, uint32_t stride, uint32_t at,
                                                      uint32_t k, uint32_t w, uint32_t nranks, int order_check,
                                                      int32_t* __restrict__ status) {
  __shared__ int bad;
  if (threadIdx.x == 0) bad = 0;
  __syncthreads();
  if (order_check) {
    int mine = 0;
    for (uint32_t i = threadIdx.x; i < k; i += blockDim.x)
      for (uint32_t r = 1; r < nranks && r * w < k; r++)
        mine |= min_below_max(subs + ((uint64_t)r * stride + i) * kNodeWords,
                              subs + ((uint64_t)(r - 1) * stride + i) * kNodeWords);
    if (mine) atomicOr(&bad, 1);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int32_t m = 0;
    for (uint32_t r = 0; r < nranks; r++) {
      const int32_t v = (int32_t)subs[((uint64_t)r * stride + at) * kNodeWords];
      m = v > m ? v : m;
    }
    *status = bad ? CEL_EORDER : m;
  }
}

__global__ void k_status_from_bad(const int32_t* __restrict__ bad_axis, int32_t* __restrict__ status) {
  if (threadIdx.x == 0) *status = *bad_axis != INT_MAX ? CEL_EORDER : CEL_OK;
}

__global__ void k_pack_records(const uint32_t* __restrict__ rec, uint32_t n, uint8_t* __restrict__ out) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n * kNode) return;
  out[b] = reinterpret_cast<const uint8_t*>(rec + (uint64_t)(b / kNode) * kNodeWords)[b % kNode];
}

// Reduce `trees` trees of nin nodes each (first level strided, then compact) to one
// record per tree in `roots`. ping/pong hold trees * nin / 2 records each.
static void reduce_grid(const uint32_t* in, uint32_t nin, uint32_t trees, uint32_t tstride, uint32_t lstride,
                        uint32_t* ping, uint32_t* pong, uint32_t* roots, hipStream_t s) {
  if (nin < 2) return;  // callers copy single-leaf trees themselves
  uint32_t nout = nin / 2;
  uint32_t* out = (nout == 1) ? roots : ping;
  hipLaunchKernelGGL(k_level_grid, dim3((trees * nout + 255) / 256), dim3(256), 0, s, in, out, nin, trees, tstride,
                     lstride);
  const uint32_t* src = out;
  uint32_t* dst = pong;
  nin = nout;
  while (nin > 1) {
    nout = nin / 2;
    out = (nout == 1) ? roots : dst;
    hipLaunchKernelGGL(k_level<false>, dim3((trees * nout + 255) / 256, 1), dim3(256), 0, s, src, out, 0u, nin, trees,
                       nullptr, nullptr, nullptr);
    src = out;
    dst = (dst == ping) ? pong : ping;
    nin = nout;
  }
}

// Two tree sets reduced level by level in lockstep, one k_level_pair launch per level:
// set j has trees_j trees of nin_j leaves (first level strided as in k_level_grid, then
// compact in its own ping / pong buffers); each set's last level writes roots_j.
static void reduce_grid_pair(LevelJob a, uint32_t* ping_a, uint32_t* pong_a, uint32_t* roots_a, LevelJob b,
                             uint32_t* ping_b, uint32_t* pong_b, uint32_t* roots_b, hipStream_t s) {
  uint32_t* dst_a = ping_a;
  uint32_t* dst_b = ping_b;
  while (a.nin > 1 || b.nin > 1) {
    if (a.nin > 1) a.out = a.nin == 2 ? roots_a : dst_a;
    if (b.nin > 1) b.out = b.nin == 2 ? roots_b : dst_b;
    const uint32_t n = (a.nin > 1 ? a.trees * (a.nin / 2) : 0u) + (b.nin > 1 ? b.trees * (b.nin / 2) : 0u);
    hipLaunchKernelGGL(k_level_pair, dim3((n + 255) / 256), dim3(256), 0, s, a, b);
    if (a.nin > 1) {
      a.in = a.out;
      a.nin /= 2;
      a.tstride = a.nin;
      a.lstride = 1;
      dst_a = dst_a == ping_a ? pong_a : ping_a;
    }
    if (b.nin > 1) {
      b.in = b.out;
      b.nin /= 2;
      b.tstride = b.nin;
      b.lstride = 1;
      dst_b = dst_b == ping_b ? pong_b : ping_b;
    }
  }
}

// Workspace: leaves [2k*w] | ping, pong of the column trees [k*w] | roots area (unused) |
//            bad int32 | ping, pong of the row subtrees [k*w]
size_t slab_workspace_size(uint32_t k, uint32_t w) {
  const size_t nb = kNodeWords * 4, W = 2 * (size_t)k;
  return align256(W * w * nb) + 4 * align256((size_t)k * w * nb + nb) + align256(W * 2 * nb) + 256;
}

// The slab commit's workspace: leaves, the column trees' ping / pong, the roots area, the
// order flag, the row subtrees' ping / pong.
struct SlabWork {
  uint32_t *leaves, *ping, *pong, *ping2, *pong2;
  int32_t* bad;
};
static SlabWork slab_work(void* work, uint32_t k, uint32_t w) {
  const uint32_t W = 2 * k;
  const size_t nb = kNodeWords * 4;
  uint8_t* base = static_cast<uint8_t*>(work);
  SlabWork sw;
  sw.leaves = reinterpret_cast<uint32_t*>(base);
  base += align256((size_t)W * w * nb);
  sw.ping = reinterpret_cast<uint32_t*>(base);
  base += align256((size_t)k * w * nb + nb);
  sw.pong = reinterpret_cast<uint32_t*>(base);
  base += align256((size_t)k * w * nb + nb);
  base += align256((size_t)W * 2 * nb);
  sw.bad = reinterpret_cast<int32_t*>(base);
  base += 256;
  sw.ping2 = reinterpret_cast<uint32_t*>(base);
  base += align256((size_t)k * w * nb + nb);
  sw.pong2 = reinterpret_cast<uint32_t*>(base);
  return sw;
}

// Leaves of slab rows [row0, row1) (2k rows of w cells). The half holding rows < k checks
// the push order and must come first in stream order after the flag is reset (init_bad).
hipError_t launch_slab_leaves(const uint8_t* slab, uint32_t k, uint32_t c0, uint32_t w, uint32_t row0, uint32_t row1,
                              void* work, bool order_check, bool init_bad, hipStream_t s) {
  const SlabWork sw = slab_work(work, k, w);
  if (init_bad) hipLaunchKernelGGL(k_fill_i32, dim3(1), dim3(64), 0, s, sw.bad, 1u, INT_MAX);
  const uint32_t cell0 = row0 * w, cell1 = row1 * w;
  if (cell1 <= cell0) return hipGetLastError();
  dim3 gl((cell1 - cell0 + 255) / 256);
  if (latency_bound(2ull * k * w)) {
    if (order_check)
      hipLaunchKernelGGL((k_slab_leaf<true, true>), gl, dim3(256), 0, s, slab, k, c0, w, cell0, cell1, sw.leaves, sw.bad);
    else
      hipLaunchKernelGGL((k_slab_leaf<false, true>), gl, dim3(256), 0, s, slab, k, c0, w, cell0, cell1, sw.leaves, sw.bad);
  } else {
    if (order_check)
      hipLaunchKernelGGL((k_slab_leaf<true, false>), gl, dim3(256), 0, s, slab, k, c0, w, cell0, cell1, sw.leaves, sw.bad);
    else
      hipLaunchKernelGGL((k_slab_leaf<false, false>), gl, dim3(256), 0, s, slab, k, c0, w, cell0, cell1, sw.leaves,
                         sw.bad);
  }
  return hipGetLastError();
}

// After every leaf of the slab: w column trees of 2k leaves (leaf i of column j at
// i*w + j) and 2k row subtrees of w leaves (leaf j of row i at i*w + j), both sets one
// level per launch, then the status.
hipError_t launch_slab_trees(uint32_t k, uint32_t w, uint32_t* col_rec, uint32_t* row_sub, int32_t* status,
                             void* work, hipStream_t s) {
  const uint32_t W = 2 * k;
  const size_t nb = kNodeWords * 4;
  const SlabWork sw = slab_work(work, k, w);
  if (w == 1) {
    const hipError_t e = hipMemcpyAsync(row_sub, sw.leaves, (size_t)W * nb, hipMemcpyDeviceToDevice, s);
    if (e != hipSuccess) return e;
  }
  const LevelJob cols{sw.leaves, nullptr, W, w, 1, w};
  const LevelJob rows{sw.leaves, nullptr, w, W, w, 1};
  reduce_grid_pair(cols, sw.ping, sw.pong, col_rec, rows, sw.ping2, sw.pong2, row_sub, s);
  hipLaunchKernelGGL(k_status_from_bad, dim3(1), dim3(64), 0, s, sw.bad, status);
  return hipGetLastError();
}

// Workspace: ping/pong [2k * nranks / 2] | items [4k] | (256 B unused) | DAH leaf digests [4k][8]
size_t shard_finish_workspace_size(uint32_t k, uint32_t nranks) {
  const size_t nb = kNodeWords * 4, W = 2 * (size_t)k;
  return 2 * align256(W * (nranks / 2 + 1) * nb) + align256(2 * W * nb) + 256 + align256(2 * W * 32);
}

hipError_t launch_shard_finish(const uint32_t* gathered, uint32_t k, uint32_t nranks, uint8_t* row_roots,
                               uint8_t* col_roots, uint8_t* dah, int32_t* status, void* work, bool order_check,
                               hipStream_t s) {
  const uint32_t W = 2 * k, w = W / nranks;
  const uint32_t S = W + w + 1;  // records per rank: row subtrees, column roots, status
  const uint32_t* row_subs = gathered;
  const size_t nb = kNodeWords * 4;
  uint8_t* base = static_cast<uint8_t*>(work);
  uint32_t* ping = reinterpret_cast<uint32_t*>(base);
  base += align256((size_t)W * (nranks / 2 + 1) * nb);
  uint32_t* pong = reinterpret_cast<uint32_t*>(base);
  base += align256((size_t)W * (nranks / 2 + 1) * nb);
  uint32_t* items = reinterpret_cast<uint32_t*>(base);  // [rows 2k | cols 2k]
  base += align256((size_t)2 * W * nb) + 256;
  uint32_t* leafd = reinterpret_cast<uint32_t*>(base);
  // the ranks' step-2 status (max), or EORDER across slab boundaries: one workgroup
  hipLaunchKernelGGL(k_shard_status, dim3(1), dim3(256), 0, s, gathered, S, W + w, k, w, nranks,
                     (order_check && nranks > 1) ? 1 : 0, status);
  // row i's subtree from rank r is gathered[r][i]: trees of nranks leaves, stride S
  hipError_t e = hipSuccess;
  if (nranks == 1) e = hipMemcpyAsync(items, row_subs, (size_t)W * nb, hipMemcpyDeviceToDevice, s);
  else reduce_grid(row_subs, nranks, W, 1, S, ping, pong, items, s);
  // the column roots: rank r's w records at gathered[r][W], in rank order
  if (e == hipSuccess)
    e = hipMemcpy2DAsync(items + (size_t)W * kNodeWords, (size_t)w * nb, gathered + (size_t)W * kNodeWords,
                         (size_t)S * nb, (size_t)w * nb, nranks, hipMemcpyDeviceToDevice, s);
  if (e != hipSuccess) return e;
  // the 4k RFC-6962 leaf digests and the packed roots one lane each, then the DAH tree
  // one level per round in one workgroup
  hipLaunchKernelGGL(k_dah_leaves, dim3((2 * W + 255) / 256), dim3(256), 0, s, items, 2 * W, leafd, row_roots,
                     col_roots);
  const size_t lds = (size_t)2 * W * 8 * 4;
  hipLaunchKernelGGL(k_merkle, dim3(1), dim3(merkle_block(2 * W)), lds, s, items, leafd, 2 * W, dah, nullptr, nullptr,
                     nullptr, nullptr);
  return hipGetLastError();
}

// Plain NMT over arbitrary leaves (k_leaf assumes 512-byte EDS cells, so leaves are
// hashed by a generic lane-per-leaf kernel over a byte message).
__device__ void sha_bytes(const uint8_t* __restrict__ a, uint32_t la, const uint8_t* __restrict__ b, uint32_t lb,
                          uint8_t pre, uint32_t (&st)[8]) {
  // message = pre || a || b; processed byte-wise (generic path, small inputs only)
  const uint64_t total = 1ull + la + lb;
  sha256_init(st);
  uint32_t w[16];
  uint64_t pos = 0;
  const uint64_t padded = ((total + 8) / 64 + 1) * 64;
  for (uint64_t blk = 0; blk < padded; blk += 64) {
    for (int wi = 0; wi < 16; wi++) {
      uint32_t x = 0;
      for (int j = 0; j < 4; j++) {
        const uint64_t p = blk + 4 * wi + j;
        uint32_t v;
        if (p == 0) v = pre;
        else if (p < 1 + la) v = a[p - 1];
        else if (p < total) v = b[p - 1 - la];
        else if (p == total) v = 0x80;
        else if (p >= padded - 8) v = (uint32_t)(((total * 8) >> (8 * (padded - 1 - p))) & 0xFF);
        else v = 0;
        x = (x << 8) | v;
      }
      w[wi] = x;
    }
    sha256_compress(st, w);
    pos += 64;
  }
  (void)pos;
}

__global__ __launch_bounds__(256) void k_generic_leaf(const uint8_t* __restrict__ leaves, uint32_t n, uint32_t len,
                                                      uint32_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  const uint8_t* lf = leaves + (uint64_t)i * len;
  uint32_t st[8];
  sha_bytes(lf, len, nullptr, 0, 0x00, st);
  uint32_t nd[kNodeWords];
  uint8_t* nb = reinterpret_cast<uint8_t*>(nd);
  for (int j = 0; j < 29; j++) { nb[j] = lf[j]; nb[29 + j] = lf[j]; }
  nb[58] = nb[59] = 0;
  nd[14] &= 0xFFFFu;
  put_digest(nd, st);
  store_node(out + (uint64_t)i * kNodeWords, nd);
}

// Erasured axis: cells (2k x 512 B) with the wrapper's namespace rule.
__global__ __launch_bounds__(256) void k_axis_leaf(const uint8_t* __restrict__ cells, uint32_t k, uint32_t axis,
                                                   uint32_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= 2 * k) return;
  const uint32_t* sh = reinterpret_cast<const uint32_t*>(cells + (uint64_t)i * kShare);
  const bool q0 = (i < k) && (axis < k);
  uint32_t st[8];
  leaf_hash<true>(st, sh, q0);
  uint32_t nd[kNodeWords];
  if (q0) {
    uint32_t s[8];
    for (int j = 0; j < 8; j++) s[j] = sh[j];
    for (int j = 0; j < 7; j++) nd[j] = s[j];
    nd[7] = (s[7] & 0xFFu) | (s[0] << 8);
    for (int j = 0; j < 6; j++) nd[8 + j] = __builtin_amdgcn_alignbyte(s[j + 1], s[j], 3);
    nd[14] = (s[6] >> 24) | ((s[7] & 0xFFu) << 8);
  } else {
    for (int j = 0; j < 14; j++) nd[j] = 0xFFFFFFFFu;
    nd[14] = 0xFFFFu;
  }
  put_digest(nd, st);
  store_node(out + (uint64_t)i * kNodeWords, nd);
}

// Reduce n nodes (one tree) to a root with repeated k_level-like passes, then pack.
__global__ __launch_bounds__(256) void k_reduce_pass(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                     uint32_t n) {
  const uint32_t half = n / 2;
  const uint32_t j = blockIdx.x * 256u + threadIdx.x;
  if (j < half) {
    uint32_t L[kNodeWords], R[kNodeWords], o[kNodeWords];
    load_node(in + (uint64_t)(2 * j) * kNodeWords, L);
    load_node(in + (uint64_t)(2 * j + 1) * kNodeWords, R);
    hash_node(L, R, o);
    store_node(out + (uint64_t)j * kNodeWords, o);
  } else if ((n & 1) && j == half) {
    uint32_t x[kNodeWords];
    load_node(in + (uint64_t)(n - 1) * kNodeWords, x);
    store_node(out + (uint64_t)half * kNodeWords, x);
  }
}

__global__ void k_pack_root(const uint32_t* __restrict__ node, uint32_t n, uint8_t* __restrict__ out) {
  const uint32_t i = threadIdx.x;
  if (i >= kNode) return;
  if (n == 0) {  // empty tree: 0*58 || SHA256("")
    if (i < 58) out[i] = 0;
    if (i == 0) {
      uint32_t st[8];
      sha_empty(st);
      for (int j = 0; j < 32; j++) out[58 + j] = (uint8_t)(st[j / 4] >> (24 - 8 * (j % 4)));
    }
    return;
  }
  out[i] = reinterpret_cast<const uint8_t*>(node)[i];
}

static hipError_t reduce_tree(uint32_t* a, uint32_t* b, uint32_t n, uint8_t* root, hipStream_t s) {
  uint32_t* src = a;
  uint32_t* dst = b;
  while (n > 1) {
    const uint32_t nout = n / 2 + (n & 1);
    hipLaunchKernelGGL(k_reduce_pass, dim3((nout + 255) / 256), dim3(256), 0, s, src, dst, n);
    uint32_t* t = src;
    src = dst;
    dst = t;
    n = nout;
  }
  hipLaunchKernelGGL(k_pack_root, dim3(1), dim3(128), 0, s, src, n, root);
  return hipGetLastError();
}

size_t axis_root_workspace_size(uint32_t k) { return 2 * align256((size_t)2 * k * kNodeWords * 4); }

hipError_t launch_axis_root(const uint8_t* cells, uint32_t k, uint32_t axis, uint8_t* root, void* work,
                            hipStream_t s) {
  uint32_t* a = static_cast<uint32_t*>(work);
  uint32_t* b = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(work) + align256((size_t)2 * k * kNodeWords * 4));
  hipLaunchKernelGGL(k_axis_leaf, dim3((2 * k + 255) / 256), dim3(256), 0, s, cells, k, axis, a);
  return reduce_tree(a, b, 2 * k, root, s);
}

size_t nmt_root_workspace_size(uint32_t n) { return 2 * align256((size_t)(n ? n : 1) * kNodeWords * 4); }

hipError_t launch_nmt_root(const uint8_t* leaves, uint32_t n, uint32_t len, uint8_t* root, void* work,
                           hipStream_t s) {
  uint32_t* a = static_cast<uint32_t*>(work);
  uint32_t* b = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(work) + align256((size_t)(n ? n : 1) * kNodeWords * 4));
  if (n) hipLaunchKernelGGL(k_generic_leaf, dim3((n + 255) / 256), dim3(256), 0, s, leaves, n, len, a);
  return reduce_tree(a, b, n, root, s);
}

// Roots of `naxes` erasured axes held densely as cells[a][2k][512]; axis_idx[a] is the
// row/column index that decides the Q0 namespace rule. roots: [naxes] 96-byte records.
__global__ __launch_bounds__(256) void k_axes_leaf(const uint8_t* __restrict__ cells, uint32_t k,
                                                   const int32_t* __restrict__ axis_idx, uint32_t naxes,
                                                   uint32_t* __restrict__ out) {
  const uint32_t W = 2 * k;
  const uint32_t g = blockIdx.x * 256u + threadIdx.x;
  if (g >= naxes * W) return;
  const uint32_t a = g / W, i = g % W;
  const uint32_t* sh = reinterpret_cast<const uint32_t*>(cells + (uint64_t)g * kShare);
  const bool q0 = (i < k) && ((uint32_t)axis_idx[a] < k);
  uint32_t st[8];
  leaf_hash<true>(st, sh, q0);
  uint32_t nd[kNodeWords];
  if (q0) {
    uint32_t s[8];
    for (int j = 0; j < 8; j++) s[j] = sh[j];
    for (int j = 0; j < 7; j++) nd[j] = s[j];
    nd[7] = (s[7] & 0xFFu) | (s[0] << 8);
    for (int j = 0; j < 6; j++) nd[8 + j] = __builtin_amdgcn_alignbyte(s[j + 1], s[j], 3);
    nd[14] = (s[6] >> 24) | ((s[7] & 0xFFu) << 8);
  } else {
    for (int j = 0; j < 14; j++) nd[j] = 0xFFFFFFFFu;
    nd[14] = 0xFFFFu;
  }
  put_digest(nd, st);
  store_node(out + (uint64_t)g * kNodeWords, nd);
}

size_t axes_roots_workspace_size(uint32_t k, uint32_t naxes) {
  const size_t W = 2 * (size_t)k, nb = kNodeWords * 4;
  return align256(naxes * W * nb) + align256(naxes * (W / 2 + 1) * nb) + align256(naxes * (W / 4 + 1) * nb);
}

hipError_t launch_axes_roots(const uint8_t* cells, uint32_t k, const int32_t* axis_idx, uint32_t naxes,
                             uint32_t* roots, void* work, hipStream_t s) {
  const uint32_t W = 2 * k;
  const size_t nb = kNodeWords * 4;
  uint8_t* base = static_cast<uint8_t*>(work);
  uint32_t* leaves = reinterpret_cast<uint32_t*>(base);
  base += align256((size_t)naxes * W * nb);
  uint32_t* ping = reinterpret_cast<uint32_t*>(base);
  base += align256((size_t)naxes * (W / 2 + 1) * nb);
  uint32_t* pong = reinterpret_cast<uint32_t*>(base);
  hipLaunchKernelGGL(k_axes_leaf, dim3((naxes * W + 255) / 256), dim3(256), 0, s, cells, k, axis_idx, naxes, leaves);
  uint32_t nin = W;
  const uint32_t* src = leaves;
  uint32_t* dst = ping;
  while (nin > 1) {
    const uint32_t nout = nin / 2;
    uint32_t* out = (nout == 1) ? roots : dst;
    hipLaunchKernelGGL(k_level<false>, dim3((naxes * nout + 255) / 256, 1), dim3(256), 0, s, src, out, W, nin, naxes,
                       nullptr, nullptr, nullptr);
    src = out;
    dst = (dst == ping) ? pong : ping;
    nin = nout;
  }
  return hipGetLastError();
}

size_t merkle_workspace_size(uint32_t n) { return align256((size_t)(n ? n : 1) * kNodeWords * 4); }

__global__ void k_pad_items(const uint8_t* __restrict__ items, uint32_t n, uint32_t len, uint32_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t* o = reinterpret_cast<uint8_t*>(out + (uint64_t)i * kNodeWords);
  for (uint32_t j = 0; j < kNodeWords * 4; j++) o[j] = j < len ? items[(uint64_t)i * len + j] : 0;
}

hipError_t launch_merkle_root(const uint8_t* items, uint32_t n, uint32_t item_len, uint8_t* out, void* work,
                              hipStream_t s) {
  if (item_len != kNode) return hipErrorInvalidValue;  // DAH items are NMT roots
  uint32_t* pad = static_cast<uint32_t*>(work);
  if (n) hipLaunchKernelGGL(k_pad_items, dim3((n + 255) / 256), dim3(256), 0, s, items, n, item_len, pad);
  const size_t lds = (size_t)(n ? n : 1) * 8 * 4;
  if (lds > 64 * 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_merkle, dim3(1), dim3(merkle_block(n)), lds, s, pad, nullptr, n, out, nullptr, nullptr, nullptr,
                     nullptr);
  return hipGetLastError();
}

// ---------------------------------------------------- exported trees (proofs, §8f)
//
// Every node of the NMT trees of `naxes` gathered axes (cells[a][2k][512], axis_idx[a]
// = the row/column index that decides the Q0 namespace rule), level-major:
//   nodes = level 0 [naxes][2k] | level 1 [naxes][k] | ... | level log2(2k) [naxes][1]
// 96-byte records. This is what nmt ProveRange / the subtree-root cacher read instead
// of rebuilding the trees on the CPU (pkg/proof/proof.go:151-201,
// pkg/inclusion/nmt_caching.go:96-124).
size_t axes_trees_nodes(uint32_t k, uint32_t naxes) { return (size_t)naxes * (4 * (size_t)k - 1); }

hipError_t launch_axes_trees(const uint8_t* cells, uint32_t k, const int32_t* axis_idx, uint32_t naxes,
                             uint32_t* nodes, hipStream_t s) {
  const uint32_t W = 2 * k;
  hipLaunchKernelGGL(k_axes_leaf, dim3((naxes * W + 255) / 256), dim3(256), 0, s, cells, k, axis_idx, naxes, nodes);
  uint32_t nin = W;
  uint32_t* src = nodes;
  while (nin > 1) {
    const uint32_t nout = nin / 2;
    uint32_t* out = src + (size_t)naxes * nin * kNodeWords;
    hipLaunchKernelGGL(k_level<false>, dim3((naxes * nout + 255) / 256, 1), dim3(256), 0, s, src, out, W, nin, naxes,
                       nullptr, nullptr, nullptr);
    src = out;
    nin = nout;
  }
  return hipGetLastError();
}

// RFC-6962 tree of n = 2^m items of 90 bytes (DataAvailabilityHeader.Hash over
// rowRoots || colRoots), every level: level 0 = the n leaf hashes SHA256(0x00 || item),
// then n/2 inner hashes SHA256(0x01 || l || r), ..., the root. 8 big-endian words per
// node. (merkle.ProofsFromByteSlices reads its aunts from these levels.)
__global__ void k_rfc_leaves(const uint32_t* __restrict__ items, uint32_t n, uint32_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t R[kNodeWords], st[8];
  load_node(items + (uint64_t)i * kNodeWords, R);
  rfc_leaf90(R, st);
  for (int j = 0; j < 8; j++) out[(uint64_t)i * 8 + j] = st[j];
}

__global__ void k_rfc_level(const uint32_t* __restrict__ in, uint32_t nout, uint32_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nout) return;
  uint32_t st[8];
  rfc_inner(in + (uint64_t)(2 * i) * 8, in + (uint64_t)(2 * i + 1) * 8, st);
  for (int j = 0; j < 8; j++) out[(uint64_t)i * 8 + j] = st[j];
}

hipError_t launch_rfc_tree(const uint8_t* items90, uint32_t n, uint32_t* levels, void* work, hipStream_t s) {
  if (!n || (n & (n - 1))) return hipErrorInvalidValue;
  uint32_t* pad = static_cast<uint32_t*>(work);
  hipLaunchKernelGGL(k_pad_items, dim3((n + 255) / 256), dim3(256), 0, s, items90, n, kNode, pad);
  hipLaunchKernelGGL(k_rfc_leaves, dim3((n + 255) / 256), dim3(256), 0, s, pad, n, levels);
  uint32_t* src = levels;
  for (uint32_t m = n; m > 1; m /= 2) {
    uint32_t* out = src + (size_t)m * 8;
    hipLaunchKernelGGL(k_rfc_level, dim3((m / 2 + 255) / 256), dim3(256), 0, s, src, m / 2, out);
    src = out;
  }
  return hipGetLastError();
}

// Pack selected 96-byte node records into 90-byte items: out[i] = nodes[rec[i]].
__global__ void k_gather_nodes(const uint32_t* __restrict__ nodes, const int32_t* __restrict__ rec, uint32_t n,
                               uint8_t* __restrict__ out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * kNode) return;
  const uint32_t i = t / kNode, b = t % kNode;
  out[t] = reinterpret_cast<const uint8_t*>(nodes + (uint64_t)rec[i] * kNodeWords)[b];
}

hipError_t launch_gather_nodes(const uint32_t* nodes, const int32_t* rec, uint32_t n, uint8_t* out, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_gather_nodes, dim3((n * kNode + 255) / 256), dim3(256), 0, s, nodes, rec, n, out);
  return hipGetLastError();
}

// merkle.HashFromByteSlices (tendermint crypto/merkle, RFC-6962) over n byte slices of any
// length: the DAH hash when the roots are not all 90-byte NMT roots
// (data_availability_header.go:92-108 hashes whatever RowRoots / ColumnRoots hold). Leaf
// i = SHA256(0x00 || slice i), one lane each; then one workgroup pairs adjacent nodes
// level by level, carrying an odd last node up unchanged, which is the same tree as the
// reference's split at the largest power of two below n. n == 0: SHA256("").
__global__ void k_slice_leaves(const uint8_t* __restrict__ data, const uint64_t* __restrict__ off, uint32_t n,
                               uint32_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t st[8];
  sha_bytes(data + off[i], (uint32_t)(off[i + 1] - off[i]), nullptr, 0, 0x00, st);
  for (int j = 0; j < 8; j++) out[(uint64_t)i * 8 + j] = st[j];
}

__global__ __launch_bounds__(256) void k_slice_tree(uint32_t* __restrict__ a, uint32_t* __restrict__ b, uint32_t n,
                                                    uint8_t* __restrict__ out) {
  if (n == 0) {
    if (threadIdx.x == 0) {
      uint32_t st[8], w[16];
      sha256_init(st);
      w[0] = 0x80000000u;
      for (int j = 1; j < 16; j++) w[j] = 0;
      sha256_compress(st, w);
      for (int j = 0; j < 32; j++) out[j] = (uint8_t)(st[j / 4] >> (24 - 8 * (j % 4)));
    }
    return;
  }
  uint32_t* src = a;
  uint32_t* dst = b;
  for (uint32_t m = n; m > 1; m = (m + 1) / 2) {  // ping-pong: a level reads src, writes dst
    for (uint32_t i = threadIdx.x; i < m / 2; i += blockDim.x) {
      uint32_t st[8];
      rfc_inner(src + (uint64_t)(2 * i) * 8, src + (uint64_t)(2 * i + 1) * 8, st);
      for (int j = 0; j < 8; j++) dst[(uint64_t)i * 8 + j] = st[j];
    }
    if ((m & 1) && threadIdx.x == 0)
      for (int j = 0; j < 8; j++) dst[(uint64_t)(m / 2) * 8 + j] = src[(uint64_t)(m - 1) * 8 + j];
    __syncthreads();
    uint32_t* t = src;
    src = dst;
    dst = t;
  }
  if (threadIdx.x < 32) out[threadIdx.x] = (uint8_t)(src[threadIdx.x / 4] >> (24 - 8 * (threadIdx.x % 4)));
}

size_t slices_workspace_size(uint32_t n) { return 2 * align256((size_t)(n ? n : 1) * 32); }

hipError_t launch_hash_slices(const uint8_t* data, const uint64_t* off, uint32_t n, uint8_t* out, void* work,
                              hipStream_t s) {
  uint32_t* a = static_cast<uint32_t*>(work);
  uint32_t* b = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(work) + align256((size_t)(n ? n : 1) * 32));
  if (n) hipLaunchKernelGGL(k_slice_leaves, dim3((n + 255) / 256), dim3(256), 0, s, data, off, n, a);
  hipLaunchKernelGGL(k_slice_tree, dim3(1), dim3(256), 0, s, a, b, n, out);
  return hipGetLastError();
}

}  // namespace cel
