// Leopard GF(2^8) encode, one wave per axis slice (32 <= k <= 128).
//
// The transform of SURVEY.md Appendix A.2 in radix-2 form (see the header of
// rs_kernels.hip), laid out so that nothing is shared between waves:
//   - a wave owns one tile = (square, axis, 256-byte slice); lane l holds dword l of
//     the slice of every one of the K data shards of the axis in VGPRs (K <= 128);
//   - every radix-2 layer is lane-local, so there is no LDS image and no barrier: the
//     waves of a CU drift apart and one wave's loads and stores run under the
//     butterflies of the others;
//   - the skew index of every butterfly is a compile-time constant, so the v_perm
//     product tables are immediates (no table loads), "multiply by zero" butterflies
//     (skew == 255) lose their multiply and "multiply by one" becomes an xor.
// Multiply: the byte splits into 3+3+2 bits, each looked up with one v_perm_b32 in
// an 8/8/4-entry product table (as rs_kernels.hip gf8_mul4).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "cel_internal.hpp"
#include "bitslice8.hpp"
#include "gf8_constexpr.hpp"

namespace cel {
namespace ax {

using cx::add_mod8;
using cx::kGf8;
using cx::sfor;
using bs::pxor;
using bs::tr8;
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

// Leopard IFFT over the data coset (offset K) then FFT over the parity coset (offset 0),
// radix 2, all K shards in w[]. Skew index: IFFT K-1 + base + D, FFT base + D - 1.
// The last IFFT layer and the first FFT layer act on the same pairs (a, a + K/2):
//   y ^= x; x ^= c1*y;  then  x ^= c2*y; y ^= x   ==   y ^= x; x ^= (c1 + c2)*y; y ^= x
// so they run as one layer with one multiply by c1 + c2 (K/2 of the K log K
// butterflies lose a multiply).
constexpr uint32_t merged_lm(uint32_t s1, uint32_t s2) {
  const uint32_t c = (s1 == 255u ? 0u : (uint32_t)kGf8.exp[s1]) ^ (s2 == 255u ? 0u : (uint32_t)kGf8.exp[s2]);
  return c == 0u ? 255u : (uint32_t)kGf8.log[c];
}

// ---------------------------------------------------------------- hybrid transform
//
// Layers with D >= 8 have the same twiddle for all 8 shards of an aligned block
// {8m .. 8m+7} (the skew index depends on base = a & ~(2D-1) only), so there the block
// is bit-sliced in place: an 8x8 bit transpose in each byte lane of w[8m .. 8m+7] turns
// "4 bytes of 8 shards" into 8 bit-planes, and a butterfly between blocks m and m+D/8 is
// an 8x8 GF(2) matrix network of v_bitop3 xor3 ops (~2 per plane) instead of the v_perm
// multiply (~10 VALU per dword). Layers D = 1, 2, 4 (twiddles differ inside a block) keep
// the v_perm multiply. For K = 128: 6 v_perm layers, 7 bit-sliced layers, 32 transposes.

// planes w[XO..XO+8) ^= exp(LM) * planes w[YO..YO+8); LM == 255 is the zero twiddle.
template <uint32_t LM, int XO, int YO, int K>
__device__ __forceinline__ void pmuladd(uint32_t (&w)[K]) {
  if constexpr (LM != 255u) {
    sfor<8>([&](auto r) { xrow<cx::mul_row(LM, decltype(r)::value), YO, 0>(w[XO + decltype(r)::value], w); });
  }
}

template <int K>
__device__ __forceinline__ void transform_hyb(uint32_t (&w)[K]) {
  constexpr int LOGK = __builtin_ctz(K);
  static_assert(K >= 32, "hybrid transform needs bit-sliced layers");
  const uint32_t m7 = sconst<0x07070707u>(), m3 = sconst<0x03030303u>();
  // IFFT D = 1, 2, 4: v_perm multiply
  sfor<3>([&](auto lg) {
    constexpr int D = 1 << decltype(lg)::value;
    sfor<K / (2 * D)>([&](auto bi) {
      constexpr int base = decltype(bi)::value * 2 * D;
      const Mul<kGf8.skew[K - 1 + base + D]> m;
      sfor<D>([&](auto j) {
        constexpr int a = base + decltype(j)::value;
        pin(w[a], w[a + D]);
        w[a + D] ^= w[a];
        m.muladd(w[a], w[a + D], m7, m3);
        pin(w[a], w[a + D]);
        __builtin_amdgcn_sched_barrier(0);
      });
    });
  });
  sfor<K / 8>([&](auto s) {
    tr8<8 * decltype(s)::value>(w);
    __builtin_amdgcn_sched_barrier(0);
  });
  // IFFT D = 8 .. K/4, bit-sliced (block pairs)
  sfor<LOGK - 4>([&](auto t) {
    constexpr int D = 8 << decltype(t)::value;
    sfor<K / (2 * D)>([&](auto bi) {
      constexpr int base = decltype(bi)::value * 2 * D;
      sfor<D / 8>([&](auto j) {
        constexpr int a = base + 8 * decltype(j)::value;
        pxor<a, a + D>(w);
        pmuladd<kGf8.skew[K - 1 + base + D], a, a + D>(w);
        __builtin_amdgcn_sched_barrier(0);
      });
    });
  });
  {  // last IFFT layer + first FFT layer, merged (see transform)
    constexpr int D = K / 2;
    sfor<D / 8>([&](auto j) {
      constexpr int a = 8 * decltype(j)::value;
      pxor<a, a + D>(w);
      pmuladd<merged_lm(kGf8.skew[K - 1 + D], kGf8.skew[D - 1]), a, a + D>(w);
      pxor<a, a + D>(w);
      __builtin_amdgcn_sched_barrier(0);
    });
  }
  // FFT D = K/4 .. 8, bit-sliced
  sfor<LOGK - 4>([&](auto t) {
    constexpr int D = K >> (decltype(t)::value + 2);
    sfor<K / (2 * D)>([&](auto bi) {
      constexpr int base = decltype(bi)::value * 2 * D;
      sfor<D / 8>([&](auto j) {
        constexpr int a = base + 8 * decltype(j)::value;
        pmuladd<kGf8.skew[base + D - 1], a, a + D>(w);
        pxor<a, a + D>(w);
        __builtin_amdgcn_sched_barrier(0);
      });
    });
  });
  sfor<K / 8>([&](auto s) {
    tr8<8 * decltype(s)::value>(w);
    __builtin_amdgcn_sched_barrier(0);
  });
  // FFT D = 4, 2, 1: v_perm multiply
  sfor<3>([&](auto t) {
    constexpr int D = 4 >> decltype(t)::value;
    sfor<K / (2 * D)>([&](auto bi) {
      constexpr int base = decltype(bi)::value * 2 * D;
      const Mul<kGf8.skew[base + D - 1]> m;
      sfor<D>([&](auto j) {
        constexpr int a = base + decltype(j)::value;
        pin(w[a], w[a + D]);
        m.muladd(w[a], w[a + D], m7, m3);
        w[a + D] ^= w[a];
        pin(w[a], w[a + D]);
        __builtin_amdgcn_sched_barrier(0);
      });
    });
  });
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}

// Tile = (square z, axis x, 256-byte slice y) of geometry g: one wave. LP / SP: cache
// policy of the loads / stores (2 = nt).
template <int LOGK, int LP, int SP>
__device__ __forceinline__ void axis_tile(const RsGeom& g, uint32_t nslice, uint32_t tile, uint32_t lane) {
  constexpr int K = 1 << LOGK;
  const uint32_t y = tile % nslice, r = tile / nslice;
  const uint32_t x = r % g.axes, z = r / g.axes;
  const uint32_t col = y * 256u + lane * 4u;
  const bool active = col < g.len;
  const uint32_t lo = active ? lane * 4u : 0u;  // inactive lanes load (and never store) dword 0
  uint32_t w[K];
  {
    const auto rin = rsrc(g.in + (uint64_t)z * g.in_sq + (uint64_t)x * g.in_axis + (uint64_t)y * 256u);
    const uint32_t in_shard = (uint32_t)g.in_shard;
#pragma unroll
    for (int i = 0; i < K; i++) w[i] = __builtin_amdgcn_raw_buffer_load_b32(rin, lo, (uint32_t)i * in_shard, LP);
    if (g.dcopy && active) {
      const auto rdc = rsrc(g.dcopy + (uint64_t)z * g.dc_sq + (uint64_t)x * g.dc_axis + (uint64_t)y * 256u);
      const uint32_t dc_shard = (uint32_t)g.dc_shard;
#pragma unroll
      for (int i = 0; i < K; i++) __builtin_amdgcn_raw_buffer_store_b32(w[i], rdc, lo, (uint32_t)i * dc_shard, SP);
    }
  }
  transform_hyb<K>(w);
  if (active) {
    const auto rout = rsrc(g.out + (uint64_t)z * g.out_sq + (uint64_t)x * g.out_axis + (uint64_t)y * 256u);
    const uint32_t out_shard = (uint32_t)g.out_shard;
#pragma unroll
    for (int i = 0; i < K; i++) __builtin_amdgcn_raw_buffer_store_b32(w[i], rout, lo, (uint32_t)i * out_shard, SP);
  }
}

// One pass (rows or columns) of every square of g. Loads and stores are nt (non-temporal):
// every byte is touched once per pass and a batch is far larger than the Infinity Cache
// (k=128, 256 squares: 9.35 -> 9.00 us per square against the default policy,
// profiles/r1d_rs_cache_policy_ab.txt).
template <int LOGK>
__global__ __launch_bounds__(256, 3) void k_rs_axis_gf8(RsGeom g, uint32_t nslice) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t tile = __builtin_amdgcn_readfirstlane(xcd_block(blockIdx.x, gridDim.x) * 4u + (threadIdx.x >> 6));
  if (tile >= g.axes * nslice * g.nsq) return;
  axis_tile<LOGK, 2, 2>(g, nslice, tile, lane);
}

// Both passes of the extension in one launch, as a dequeue-ordered tile queue.
//
// Every wave takes tickets from one atomic counter and runs the tile its ticket names
// until the tickets run out. Ticket order: for block j = 0, 1, ..: the row tiles of
// square j, then its Q0 column tiles, then the Q1 column tiles of square j - kLag. A Q1
// column tile (column x >= k, slice y) needs the outputs of all k row tiles of slice y of
// its square; those carry smaller tickets, so they were dequeued by waves that are
// already running and that wait on nothing. That is the forward-progress argument a
// blockIdx-ordered version lacks: there a waiting tile may hold the
// CU slot that the tile it waits on needs, because dispatch order does not guarantee
// residency. Hand-off (cdna_hip_programming.md Guideline 16, write-through form R1): the
// row tile stores its output sc1 (write-through, so no release fence: a buffer_wbl2 per
// tile flushes the whole XCD L2 and made a first version 4x slower), waits for its
// stores (s_waitcnt vmcnt(0)), then adds 1 to the (square, slice) counter at agent scope;
// the consumer polls with agent-scope atomics (wait_count) and reads every handed-off
// byte with sc1 loads, which need no acquire. A poll loop that exceeds its budget (only possible with a bug) gives up and
// raises sync[1], so every wave reaches the exit.
//
// Cache policy: the row tiles load with the default policy (their Q0 rows are read again
// by the Q0 column tiles a few hundred tickets later), the column tiles store nt.
struct FusedExt {
  RsGeom rows, cols;  // row pass (Q0 rows -> Q1) and column pass (all 2k columns)
  uint32_t* sync;     // [0] ticket, [1] poll budget exceeded, [2 + 2s + y] row tiles done
  uint32_t nsq;
  uint32_t wait_q0;   // the row pass writes Q0 (separate ODS input): Q0 column tiles wait too
};
constexpr uint32_t kLag = 4;  // squares between a square's row tiles and its Q1 column tiles
constexpr int kSc1 = 16;      // buffer aux bit of sc1

// ticket -> (square, kind, index inside the kind's 2K tiles); kind 0 rows, 1 Q0 cols, 2 Q1 cols
__device__ __forceinline__ void fused_ticket(uint32_t t, uint32_t K, uint32_t nsq, uint32_t& sq, uint32_t& kind,
                                             uint32_t& u) {
  const uint32_t lag = nsq < kLag ? nsq : kLag;
  const uint32_t head = lag * 4 * K;                  // blocks 0 .. lag-1: rows + Q0 cols
  const uint32_t body = (nsq - lag) * 6 * K;          // blocks lag .. nsq-1: + Q1 cols of j - lag
  uint32_t j, v;
  if (t < head) {
    j = t / (4 * K);
    v = t % (4 * K);
  } else if (t < head + body) {
    j = lag + (t - head) / (6 * K);
    v = (t - head) % (6 * K);
  } else {  // tail: Q1 cols of the last `lag` squares
    const uint32_t r = t - head - body;
    sq = nsq - lag + r / (2 * K);
    kind = 2;
    u = r % (2 * K);
    return;
  }
  if (v < 4 * K) {
    sq = j;
    kind = v / (2 * K);
    u = v % (2 * K);
  } else {
    sq = j - lag;
    kind = 2;
    u = v - 4 * K;
  }
}

// One lane takes the wave's ticket; every lane gets it.
__device__ __forceinline__ uint32_t next_ticket(uint32_t* ctr, uint32_t lane) {
  uint32_t v = 0;
  if (lane == 0) v = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return __builtin_amdgcn_readfirstlane(v);
}

// Waits until *ctr reaches `target`: one lane polls with relaxed agent-scope loads (sc1,
// L1 bypassed), sleeping ~1 us between polls. (Polling with atomic read-modify-writes
// queued the polls with the producers' adds on the same word and ran 4x slower.) false
// after the poll budget (sync[1] raised by the caller).
__device__ __forceinline__ bool wait_count(uint32_t* ctr, uint32_t target, uint32_t lane) {
  for (uint32_t polls = 0; polls < (1u << 16); polls++) {
    uint32_t v = 0;
    if (lane == 0) v = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (__builtin_amdgcn_readfirstlane(v) >= target) return true;
    __builtin_amdgcn_s_sleep(32);
  }
  return false;
}

template <int LOGK>
__global__ __launch_bounds__(256, 3) void k_rs_extend_fused(FusedExt f) {
  constexpr uint32_t K = 1u << LOGK;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t total = 6 * K * f.nsq;
  for (uint32_t t = next_ticket(f.sync, lane); t < total; t = next_ticket(f.sync, lane)) {
    uint32_t sq, kind, u;
    fused_ticket(t, K, f.nsq, sq, kind, u);
    const uint32_t y = u / K, x = u % K;  // slice-major: slice 0's tiles first
    uint32_t* cnt = f.sync + 2 + 2 * sq + y;
    if (kind == 0) {
      axis_tile<LOGK, 0, kSc1>(f.rows, 2, (sq * K + x) * 2 + y, lane);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every sc1 store of this wave is out
      if (lane == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      const uint32_t tile = (sq * 2 * K + (kind == 2 ? K : 0) + x) * 2 + y;
      if (kind == 2 || f.wait_q0) {
        if (!wait_count(cnt, K, lane) && lane == 0)
          __hip_atomic_store(f.sync + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the loads below the poll
        axis_tile<LOGK, kSc1, 2>(f.cols, 2, tile, lane);
      } else {
        axis_tile<LOGK, 2, 2>(f.cols, 2, tile, lane);
      }
    }
  }
}

template <int LOGK>
hipError_t launch(const RsGeom& g, hipStream_t s) {
  const uint32_t nslice = (g.len + 255) / 256;
  const uint64_t ntiles = (uint64_t)g.axes * nslice * g.nsq;
  if (ntiles == 0) return hipSuccess;
  if (ntiles > 0xFFFFFFF0ull) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_rs_axis_gf8<LOGK>, dim3((unsigned)((ntiles + 3) / 4)), dim3(256), 0, s, g, nslice);
  return hipGetLastError();
}

}  // namespace ax

// Byte offsets must fit the 32-bit buffer offsets: (n - 1) * shard stride + len < 2 GiB.
static bool geom_ok(const RsGeom& g) {
  const uint64_t span = (uint64_t)g.n * (g.in_shard > g.out_shard ? g.in_shard : g.out_shard) + g.len;
  return span < 0x7fffffffull && !(g.dcopy && (uint64_t)g.n * g.dc_shard + g.len >= 0x7fffffffull);
}

// Waves of the fused launch: three 4-wave workgroups per CU (168 VGPRs).
static uint32_t fused_workgroups() {
  static const uint32_t v = [] {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                               hipSuccess || cus <= 0)
      cus = 256;
    return (uint32_t)cus * 3u;
  }();
  return v;
}

hipError_t launch_extend_fused(const RsGeom& rows, const RsGeom& cols, uint32_t nsq, bool wait_q0, uint32_t* d_sync,
                               hipStream_t s) {
  const uint32_t k = rows.n;
  if (nsq == 0) return hipSuccess;
  if (!d_sync || nsq > kMaxFusedSquares || rows.len != 512 || cols.len != 512 || !geom_ok(rows) || !geom_ok(cols))
    return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(d_sync, 0, (2 + 2 * (size_t)nsq) * 4, s);
  if (e != hipSuccess) return e;
  ax::FusedExt f{rows, cols, d_sync, nsq, wait_q0 ? 1u : 0u};
  const uint64_t waves = (uint64_t)6 * k * nsq;
  const uint32_t wgs = (uint32_t)std::min<uint64_t>((waves + 3) / 4, fused_workgroups());
  switch (k) {
    case 32: hipLaunchKernelGGL(ax::k_rs_extend_fused<5>, dim3(wgs), dim3(256), 0, s, f); break;
    case 64: hipLaunchKernelGGL(ax::k_rs_extend_fused<6>, dim3(wgs), dim3(256), 0, s, f); break;
    case 128: hipLaunchKernelGGL(ax::k_rs_extend_fused<7>, dim3(wgs), dim3(256), 0, s, f); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_rs_encode_axis(const RsGeom& g, hipStream_t s) {
  if (!geom_ok(g) || g.len == 0) return hipErrorInvalidValue;
  switch (g.n) {
    case 32: return ax::launch<5>(g, s);
    case 64: return ax::launch<6>(g, s);
    case 128: return ax::launch<7>(g, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace cel

