// C ABI of the repair (include/celestia_eds.h): cel_repair, cel_dev_repair and their test
// hooks, split from api.cpp. Host-side control of rsmt2d's Repair over a device-resident
// EDS; every decode, re-encode, compare and root runs in the HIP kernels.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "api_common.hpp"
#include "cel_internal.hpp"

using namespace cel;
using namespace cel::abi;

extern "C" {

// ------------------------------------------------------------------- repair

// rsmt2d v0.14.0 ExtendedDataSquare.Repair [dep] (extendeddatacrossword.go), with the
// oracle's restatement (oracle/eds.c) as the checker. The crossword control loop runs on
// the host over the presence mask; decoding, re-encoding, byte comparisons and root
// computation run on the device over the EDS kept resident.
namespace {

// Axis lists of the passes of one repair: each pass gets its own slot of a page-locked
// host buffer and of the device index buffer, so its upload is asynchronous and no pass
// waits for the previous one's kernels (a pageable upload into one shared buffer
// serialised the host against the stream). Slots wrap with one stream sync.
constexpr uint32_t kIdxSlots = 64;

struct RepairBufs {
  uint32_t W;
  uint8_t* eds;
  uint8_t* mask;
  int32_t* list0;     // the first pass's axis list, right after the mask (one upload for both)
  uint8_t* dense[2];  // gathered axes of the solve passes, alternating (main stream)
  uint8_t* dmask;
  uint8_t* dchk;      // gathered axes of the check passes (side stream)
  uint8_t* dmask_chk;
  uint8_t* tmp;       // re-encoded parity halves (side stream)
  uint8_t* work;      // NMT workspace of the final verification
  uint8_t* roots;     // [2][W][90] row then column roots of the final verification, then flags
  uint8_t* hres;      // page-locked copy of roots + flags (one D2H at the end)
  size_t res_bytes;
  int32_t* idx;       // [kIdxSlots][W] device axis lists
  int32_t* hidx;      // [kIdxSlots][W] page-locked staging of the same
  uint8_t* hmask;     // [W][W] page-locked staging of the presence mask
  uint32_t slot;      // next free slot
  uint32_t solves;    // solve passes so far (which dense buffer is next)
  int32_t* flags;     // [2][W] encoding-check flags by (direction, axis), right after the roots
  // Two streams: the solve chain (gather -> decode -> scatter) runs on `main`; every
  // re-encode check (of the solved axes, the sanity and the orthogonal checks) runs on
  // `side`, off the chain's critical path: its outcome is only read at the end.
  hipStream_t main, side;
  hipEvent_t ev_main;     // the square after the main stream's latest pass
  hipEvent_t ev_side[2];  // the side stream is done with dense[i]
  hipEvent_t ev_done;     // the side stream's last check
};

// `list` into the next axis-list slot, uploaded on stream s. Every slot in flight: drain
// both streams (the side stream's compares read the lists too), then reuse.
static cel_status upload_list(cel_ctx* ctx, RepairBufs& b, const std::vector<int32_t>& list, hipStream_t s,
                              int32_t** d_list) {
  hipError_t e;
  if (b.slot == kIdxSlots) {
    if ((e = hipStreamSynchronize(b.main)) != hipSuccess || (e = hipStreamSynchronize(b.side)) != hipSuccess)
      return hip_fail(ctx, e, "sync");
    b.slot = 0;
  }
  int32_t* hidx = b.hidx + (size_t)b.slot * b.W;
  *d_list = b.idx + (size_t)b.slot * b.W;
  b.slot++;
  std::memcpy(hidx, list.data(), list.size() * 4);
  if ((e = hipMemcpyAsync(*d_list, hidx, list.size() * 4, hipMemcpyHostToDevice, s)) != hipSuccess)
    return hip_fail(ctx, e, "H2D");
  return CEL_OK;
}

// Randomised idle time in front of an enqueue point (cel_debug_schedule_fuzz; off = 0).
static cel_status fuzz(cel_ctx* ctx, hipStream_t s) {
  if (!ctx->fuzz_max_us) return CEL_OK;
  uint64_t x = (ctx->fuzz_state += 0x9E3779B97F4A7C15ull);  // splitmix64
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  x ^= x >> 31;
  const hipError_t e = launch_delay((uint32_t)(x % (ctx->fuzz_max_us + 1ull)), s);
  return e == hipSuccess ? CEL_OK : hip_fail(ctx, e, "delay");
}

// Re-encode check of na gathered axes at `dense` on stream s: the data half of each axis
// is encoded again and compared with its parity half; mismatches set flags[is_col*W + axis].
// k = 256, 512: one launch of the GF(2^16) register kernel in check mode; else encode into
// b.tmp and k_cmp.
static cel_status encode_check(cel_ctx* ctx, RepairBufs& b, uint32_t k, int is_col, uint32_t na, const uint8_t* dense,
                               const int32_t* idx, hipStream_t s) {
  const uint32_t W = 2 * k;
  RsGeom g{};
  g.in = dense;
  g.in_sq = (uint64_t)na * W * kShare;
  g.in_axis = (uint64_t)W * kShare;
  g.in_shard = kShare;
  g.out = b.tmp;
  g.out_sq = (uint64_t)na * k * kShare;
  g.out_axis = (uint64_t)k * kShare;
  g.out_shard = kShare;
  g.n = k;
  g.len = kShare;
  g.axes = na;
  g.nsq = 1;
  hipError_t e;
  if (k == 256 || k == 512) {  // GF(2^16): the register kernel compares with the parity half as it goes
    g.out = const_cast<uint8_t*>(dense) + (uint64_t)k * kShare;
    g.out_sq = g.in_sq;
    g.out_axis = g.in_axis;
    g.chk_flags = b.flags + (size_t)is_col * W;
    g.chk_idx = idx;
    if ((e = launch_rs_encode(g, ctx->tables, s)) != hipSuccess) return hip_fail(ctx, e, "encoding check");
    return CEL_OK;
  }
  if ((e = launch_rs_encode(g, ctx->tables, s)) != hipSuccess) return hip_fail(ctx, e, "re-encode");
  if ((e = launch_cmp(b.tmp, (uint64_t)k * kShare, dense + (uint64_t)k * kShare, (uint64_t)W * kShare,
                      (uint64_t)k * kShare, na, b.flags + (size_t)is_col * W, s, idx)) != hipSuccess)
    return hip_fail(ctx, e, "compare");
  return CEL_OK;
}

// Encoding check of na complete axes of the square (list idx on the device) on stream s:
// one in-place launch for k = 32..128 (k_rs_check_axes) and k = 256/512 (k_rs_gf16x in
// check mode), else gather into dchk and encode_check.
static cel_status check_in_square(cel_ctx* ctx, RepairBufs& b, uint32_t k, int is_col, uint32_t na,
                                  const int32_t* idx, hipStream_t s) {
  const uint32_t W = 2 * k;
  hipError_t e;
  if (k >= 32 && k <= kMaxGf8Width) {
    if ((e = launch_rs_check_axes(b.eds, k, idx, is_col, na, b.flags + (size_t)is_col * W, s)) != hipSuccess)
      return hip_fail(ctx, e, "encoding check");
    return CEL_OK;
  }
  if (k == 256 || k == 512) {  // the GF(2^16) register kernel in check mode, in place
    const uint64_t row = (uint64_t)W * kShare;
    RsGeom g{};
    g.in = b.eds;
    g.out = b.eds + (is_col ? (uint64_t)k * row : (uint64_t)k * kShare);
    g.in_axis = g.out_axis = is_col ? kShare : row;
    g.in_shard = g.out_shard = is_col ? row : kShare;
    g.in_sq = g.out_sq = row * W;
    g.n = k;
    g.len = kShare;
    g.axes = na;
    g.nsq = 1;
    g.chk_flags = b.flags + (size_t)is_col * W;
    g.chk_idx = idx;
    g.chk_axes = idx;
    if ((e = launch_rs_encode(g, ctx->tables, s)) != hipSuccess) return hip_fail(ctx, e, "encoding check");
    return CEL_OK;
  }
  if ((e = launch_gather_axes(b.eds, b.mask, W, idx, is_col, na, b.dchk, b.dmask_chk, s)) != hipSuccess)
    return hip_fail(ctx, e, "gather");
  return encode_check(ctx, b, k, is_col, na, b.dchk, idx, s);
}

// rsmt2d solveCrossword's decode of `list` (incomplete axes of one direction), in two
// halves so the host can put other side-stream work between them:
//   solve_issue  the decode on the main stream (in place in the square, or gather ->
//                decode -> scatter), then ev_main;
//   solve_check  the encoding check of the solved axes on the side stream, after ev_main.
// Nothing is synchronised: every flag is read back once at the end of the repair.
struct Issued {
  uint32_t na = 0;
  uint32_t d = 0;
  int32_t* idx = nullptr;
};

static cel_status solve_issue(cel_ctx* ctx, RepairBufs& b, uint32_t k, int is_col, const std::vector<int32_t>& list,
                              Issued* out, int32_t* uploaded = nullptr) {
  const Range range("repair.solve");
  const uint32_t W = 2 * k, na = (uint32_t)list.size();
  out->na = na;
  if (!na) return CEL_OK;
  const uint32_t d = out->d = b.solves++ & 1u;
  cel_status st;
  if (uploaded) out->idx = uploaded;  // `list` is already on the device there
  else if ((st = upload_list(ctx, b, list, b.main, &out->idx)) != CEL_OK) return st;
  if ((st = fuzz(ctx, b.main)) != CEL_OK) return st;
  const int32_t* idx = out->idx;
  hipError_t e;
  if (rs_decode_axis_supported(W, kShare)) {
    // register decoder in place: erased cells straight into the square (no gather /
    // scatter on the chain)
    if ((e = launch_rs_decode_in_square(b.eds, b.mask, W, idx, is_col, na, ctx->tables.mul8, b.main)) != hipSuccess ||
        (e = hipEventRecord(b.ev_main, b.main)) != hipSuccess)
      return hip_fail(ctx, e, "solve");
    return CEL_OK;
  }
  uint8_t* dense = b.dense[d];
  if ((e = hipStreamWaitEvent(b.main, b.ev_side[d], 0)) != hipSuccess ||  // the side stream is done with dense[d]
      (e = launch_gather_axes(b.eds, b.mask, W, idx, is_col, na, dense, b.dmask, b.main)) != hipSuccess ||
      (e = launch_rs_decode(dense, b.dmask, na, k, kShare, ctx->tables, nullptr, b.main)) != hipSuccess ||
      (e = launch_scatter_axes(b.eds, b.mask, W, idx, is_col, na, dense, b.main)) != hipSuccess ||
      (e = hipEventRecord(b.ev_main, b.main)) != hipSuccess)
    return hip_fail(ctx, e, "solve");
  return CEL_OK;
}

// The side half of a solve_issue, enqueued after it with ev_main that solve's record or a
// later one of the main stream (the axes it checks are final from their pass on). Dense
// path: it must be enqueued before the solve after next, which reuses dense[s.d] once
// this check has recorded ev_side[s.d].
static cel_status solve_check(cel_ctx* ctx, RepairBufs& b, uint32_t k, int is_col, const Issued& s) {
  if (!s.na) return CEL_OK;
  const uint32_t W = 2 * k;
  hipError_t e;
  if ((e = hipStreamWaitEvent(b.side, b.ev_main, 0)) != hipSuccess) return hip_fail(ctx, e, "event");
  cel_status st;
  if ((st = fuzz(ctx, b.side)) != CEL_OK) return st;
  if (rs_decode_axis_supported(W, kShare))  // the completed axes are checked in the square
    return check_in_square(ctx, b, k, is_col, s.na, s.idx, b.side);
  if ((st = encode_check(ctx, b, k, is_col, s.na, b.dense[s.d], s.idx, b.side)) != CEL_OK) return st;
  if ((e = hipEventRecord(b.ev_side[s.d], b.side)) != hipSuccess) return hip_fail(ctx, e, "event");
  return CEL_OK;
}

// Encoding check of complete axes (preRepairSanityCheck, and the orthogonal axes a solve
// completed) on the side stream. wait_main: after the main stream's latest work; without
// it the caller guarantees the axes are final in the side stream's order already (the
// orthogonal axes of a pass whose solve_check the side stream has passed).
static cel_status check_pass(cel_ctx* ctx, RepairBufs& b, uint32_t k, int is_col, const std::vector<int32_t>& list,
                             bool wait_main) {
  const Range range("repair.check");
  const uint32_t na = (uint32_t)list.size();
  if (!na) return CEL_OK;
  hipError_t e;
  if (wait_main &&
      ((e = hipEventRecord(b.ev_main, b.main)) != hipSuccess || (e = hipStreamWaitEvent(b.side, b.ev_main, 0)) != hipSuccess))
    return hip_fail(ctx, e, "event");
  int32_t* idx;
  cel_status st;
  if ((st = upload_list(ctx, b, list, b.side, &idx)) != CEL_OK || (st = fuzz(ctx, b.side)) != CEL_OK) return st;
  return check_in_square(ctx, b, k, is_col, na, idx, b.side);
}

// One check of the replay, in rsmt2d's order (oracle/eds.c orc_repair):
//   SANITY  an axis complete before the repair: root (else "bad root input"), encoding
//   SOLVE   an axis decoded by solve `solve`: encoding, root
//   ORTH    an axis that solve `solve` completed: root, encoding
struct Check {
  enum Kind { SANITY, SOLVE, ORTH } kind;
  int is_col;
  int32_t idx;
  int32_t solve;  // index into the solve log (-1 for SANITY)
};
struct Solve {
  int is_col;
  int32_t idx;
};

struct RepairOut {
  int32_t* bad_axis;
  int32_t* bad_index;
  uint8_t* byz_shares;   // nullable, W * 512
  uint8_t* byz_present;  // nullable, W
};

// a[i] bit j <-> a[j] bit i
static void transpose64(uint64_t* a) {
  uint64_t m = 0x00000000FFFFFFFFull;
  for (int j = 32; j != 0; j >>= 1, m ^= (m << j)) {
    for (int k = 0; k < 64; k = ((k | j) + 1) & ~j) {
      const uint64_t t = ((a[k] >> j) ^ a[k | j]) & m;
      a[k | j] ^= t;
      a[k] ^= t << j;
    }
  }
}

// The presence mask as bitsets by row and by column (bit j of axis i = cell j of it) with
// per-axis counts, so a solve's bookkeeping visits only the cells it fills.
struct MaskBits {
  uint32_t W, nw;
  std::vector<uint64_t> bits[2];  // [is_col][axis * nw + word]
  std::vector<uint32_t> cnt[2];
  uint64_t total = 0;
  MaskBits(const std::vector<uint8_t>& hm, uint32_t w) : W(w), nw((w + 63) / 64) {
    const uint32_t P = nw * 64;  // padded to whole 64x64 tiles for the transpose
    std::vector<uint64_t> rows((size_t)P * nw, 0), cols((size_t)P * nw, 0);
    for (uint32_t i = 0; i < W; i++) {
      const uint8_t* r = hm.data() + (size_t)i * W;
      for (uint32_t j = 0; j < W; j += 8) {
        uint64_t x = 0;
        const uint32_t n = W - j < 8 ? W - j : 8;
        std::memcpy(&x, r + j, n);  // bytes 0 / 1
        rows[(size_t)i * nw + j / 64] |= ((x * 0x0102040810204080ull) >> 56) << (j % 64);
      }
    }
    // cols = rows transposed, tile by tile
    uint64_t t[64];
    for (uint32_t bi = 0; bi < nw; bi++)
      for (uint32_t bj = 0; bj < nw; bj++) {
        for (int r = 0; r < 64; r++) t[r] = rows[(size_t)(bi * 64 + r) * nw + bj];
        transpose64(t);
        for (int r = 0; r < 64; r++) cols[(size_t)(bj * 64 + r) * nw + bi] = t[r];
      }
    rows.resize((size_t)W * nw);
    cols.resize((size_t)W * nw);
    bits[0] = std::move(rows);
    bits[1] = std::move(cols);
    for (int d = 0; d < 2; d++) {
      cnt[d].assign(W, 0);
      for (uint32_t i = 0; i < W; i++) {
        uint32_t c = 0;
        for (uint32_t q = 0; q < nw; q++) c += (uint32_t)__builtin_popcountll(bits[d][(size_t)i * nw + q]);
        cnt[d][i] = c;
      }
    }
    for (uint32_t i = 0; i < W; i++) total += cnt[0][i];
  }
  // A pass: every axis of `list` (direction is_col, ascending) gets all its cells.
  // orth[t] = the orthogonal axes that solve list[t] completes, ascending: those whose
  // missing cells all lie in listed axes, the last of them in list[t] (rsmt2d fills the
  // axes one by one in list order). Word operations over the bitsets, O(W^2 / 64).
  void fill_pass(int is_col, const std::vector<int32_t>& list, std::vector<std::vector<int32_t>>& orth) {
    std::vector<uint64_t> S(nw, 0);
    std::vector<int32_t> pos(W, -1);
    for (size_t t = 0; t < list.size(); t++) {
      S[(uint32_t)list[t] / 64] |= 1ull << ((uint32_t)list[t] % 64);
      pos[list[t]] = (int32_t)t;
    }
    orth.assign(list.size(), {});
    for (uint32_t j = 0; j < W; j++) {
      if (cnt[!is_col][j] == W) continue;
      uint64_t* a = bits[!is_col].data() + (size_t)j * nw;
      bool inside = true;
      int32_t last = -1;
      uint32_t c = 0;
      for (uint32_t q = 0; q < nw; q++) {
        const uint64_t valid = (q + 1) * 64 <= W ? ~0ull : ((1ull << (W % 64)) - 1);
        const uint64_t miss = ~a[q] & valid;
        if (miss & ~S[q]) inside = false;
        if (miss) last = (int32_t)(q * 64 + 63 - __builtin_clzll(miss));
        a[q] |= S[q];
        c += (uint32_t)__builtin_popcountll(a[q] & valid);
      }
      total += c - cnt[!is_col][j];
      cnt[!is_col][j] = c;
      if (inside && last >= 0) orth[pos[last]].push_back((int32_t)j);
    }
    for (int32_t i : list) {
      uint64_t* a = bits[is_col].data() + (size_t)i * nw;
      for (uint32_t q = 0; q < nw; q++) a[q] = (q + 1) * 64 <= W ? ~0ull : ((1ull << (W % 64)) - 1);
      cnt[is_col][i] = W;
    }
  }
};

// The final verification's results, read back in one copy: every root of the square and
// the encoding-check flags by (direction, axis).
struct Verify {
  const uint8_t* got;  // [2][W][90]
  const int32_t* flags;
  const uint8_t *row_roots, *col_roots;
  uint32_t W;
  bool root_ok(int is_col, int32_t i) const {
    const uint8_t* exp = (is_col ? col_roots : row_roots) + (size_t)i * kNode;
    return std::memcmp(got + (size_t)is_col * W * kNode + (size_t)i * kNode, exp, kNode) == 0;
  }
  bool enc_ok(int is_col, int32_t i) const { return flags[(size_t)is_col * W + i] == 0; }
  // rsmt2d's order of checks: the first that fails (index into order, -1 if none) and
  // its status
  long first_failure(const std::vector<Check>& order, cel_status* code) const {
    for (size_t t = 0; t < order.size(); t++) {
      const Check& c = order[t];
      bool ok = true;
      *code = CEL_EBYZANTINE;
      switch (c.kind) {
        case Check::SANITY:
          if (!root_ok(c.is_col, c.idx)) {
            *code = CEL_EBADROOT;
            ok = false;
          } else {
            ok = enc_ok(c.is_col, c.idx);
          }
          break;
        case Check::SOLVE: ok = enc_ok(c.is_col, c.idx) && root_ok(c.is_col, c.idx); break;
        case Check::ORTH: ok = root_ok(c.is_col, c.idx) && enc_ok(c.is_col, c.idx); break;
      }
      if (!ok) return (long)t;
    }
    return -1;
  }
};

// hm := the presence mask before solve `upto` of `solves` (each solve completes its axis)
static void rollback(std::vector<uint8_t>& hm, uint32_t W, const std::vector<Solve>& solves, size_t upto) {
  for (size_t t = 0; t < upto; t++) {
    const uint32_t i = (uint32_t)solves[t].idx;
    if (solves[t].is_col)
      for (uint32_t j = 0; j < W; j++) hm[(size_t)j * W + i] = 1;
    else
      std::memset(hm.data() + (size_t)i * W, 1, W);
  }
}

// Report a failing axis: status, axis, index, and for CEL_EBYZANTINE rsmt2d's
// ErrByzantineData.Shares: the axis's cells from the square (complete axes never change;
// cells of a solved axis present before its solve kept their bytes), with the axis's mask
// from hm (masked: hm is rolled back to the mask before the failing solve) or all present.
static cel_status fail_axis(cel_ctx* ctx, const RepairBufs& b, const std::vector<uint8_t>& hm, const RepairOut& out,
                            cel_status code, int is_col, int32_t idx, bool masked) {
  const uint32_t W = b.W;
  if (out.bad_axis) *out.bad_axis = is_col;
  if (out.bad_index) *out.bad_index = idx;
  if (code == CEL_EBYZANTINE && (out.byz_shares || out.byz_present)) {
    std::vector<uint8_t> axis((size_t)W * kShare);
    const uint8_t* src = b.eds + (is_col ? (size_t)idx * kShare : (size_t)idx * W * kShare);
    const hipError_t ce = is_col ? hipMemcpy2D(axis.data(), kShare, src, (size_t)W * kShare, kShare, W,
                                                hipMemcpyDeviceToHost)
                                 : hipMemcpy(axis.data(), src, axis.size(), hipMemcpyDeviceToHost);
    if (ce != hipSuccess) return hip_fail(ctx, ce, "byzantine shares");
    for (uint32_t j = 0; j < W; j++) {
      const uint8_t p = masked ? hm[is_col ? (size_t)j * W + (uint32_t)idx : (size_t)idx * W + j] : 1;
      if (out.byz_present) out.byz_present[j] = p;
      if (out.byz_shares) {
        if (p) std::memcpy(out.byz_shares + (size_t)j * kShare, axis.data() + (size_t)j * kShare, kShare);
        else std::memset(out.byz_shares + (size_t)j * kShare, 0, kShare);
      }
    }
  }
  const char* dir = is_col ? "col" : "row";
  return fail(ctx, code, code == CEL_EBADROOT
                             ? std::string("bad root input: ") + dir + " " + std::to_string(idx)
                             : std::string("byzantine ") + (is_col ? "column" : "row") + " " + std::to_string(idx));
}

// Commit every root of the square on the main stream beside the side stream's last checks,
// join the streams and read roots and flags back (one page-locked copy).
static cel_status verify_square(cel_ctx* ctx, RepairBufs& b, uint32_t k, int last_col, const Issued& last,
                                int pending_col, const std::vector<int32_t>& pending, Verify* v) {
  const uint32_t W = 2 * k;
  const size_t roots_b = (size_t)W * kNode;
  hipError_t e;
  cel_status st;
  if ((st = fuzz(ctx, b.main)) != CEL_OK) return st;
  // the last pass's checks go to the side stream ahead of the commit's dozen launches, so
  // they run beside its leaf hashing instead of trailing its tree levels
  if ((st = solve_check(ctx, b, k, last_col, last)) != CEL_OK ||
      (st = check_pass(ctx, b, k, pending_col, pending, false)) != CEL_OK)
    return st;
  if ((e = launch_commit(b.eds, k, 1, b.roots, b.roots + roots_b, nullptr, nullptr, b.work, false, b.main)) !=
      hipSuccess)
    return hip_fail(ctx, e, "roots");
  if ((e = hipEventRecord(b.ev_done, b.side)) != hipSuccess || (e = hipStreamWaitEvent(b.main, b.ev_done, 0)) != hipSuccess)
    return hip_fail(ctx, e, "join");
  if ((e = hipMemcpyAsync(b.hres, b.roots, b.res_bytes, hipMemcpyDeviceToHost, b.main)) != hipSuccess)
    return hip_fail(ctx, e, "D2H");
  if ((e = hipStreamSynchronize(b.main)) != hipSuccess) return hip_fail(ctx, e, "sync");
  v->got = b.hres;
  v->flags = reinterpret_cast<const int32_t*>(b.hres + (b.res_bytes - 2 * (size_t)W * 4));
  v->W = W;
  return CEL_OK;
}

// rsmt2d's own solve order, for a square the pass-parallel schedule found byzantine.
//
// solveCrossword sweeps `for i { solveCrosswordRow(i); solveCrosswordCol(i) }`, and on
// inconsistent data which axis fails first, and with which Shares, depends on that order.
// The host replays the sweeps over the mask alone (every solve completes its axis): the
// solve sequence, the orthogonal axes each solve completes, and each solve's level, one
// more than the highest level among the solves that filled a cell it reads. Solves of one
// level touch no cell another of them fills, so a level runs as one row and one column
// launch; level by level the device sees every axis exactly as rsmt2d's sequence does.
// hm0: the mask the repair started from; cells present in it still hold their bytes
// (every decoder stores erased cells only).
// rsmt2d's sweeps over the mask alone (every solve completes its axis): the solve
// sequence, each solve's level and the check order (SOLVE, then the ORTH axes it
// completes, ascending); cnt = known cells per axis at the end.
struct SweepPlan {
  std::vector<Solve> solves;
  std::vector<int32_t> level;
  std::vector<Check> order;
  std::vector<uint32_t> cnt[2];
  int32_t nlevels = 0;
  bool solved = false;
};

static SweepPlan plan_sweeps(const std::vector<uint8_t>& hm, uint32_t k) {
  const uint32_t W = 2 * k;
  const size_t cells = (size_t)W * W;
  SweepPlan p;
  std::vector<uint8_t> m(hm);
  p.cnt[0].assign(W, 0);
  p.cnt[1].assign(W, 0);
  auto& cnt = p.cnt;
  size_t total = 0;
  for (uint32_t i = 0; i < W; i++)
    for (uint32_t j = 0; j < W; j++)
      if (m[(size_t)i * W + j]) {
        cnt[0][i]++;
        cnt[1][j]++;
        total++;
      }
  std::vector<int32_t> lvl_of(cells, 0);
  p.solved = total == cells;
  while (!p.solved) {
    bool progress = false;
    for (uint32_t i = 0; i < W; i++)
      for (int d = 0; d < 2; d++) {
        if (cnt[d][i] == W || cnt[d][i] < k) continue;
        const size_t base_c = d ? i : (size_t)i * W, step = d ? W : 1;
        int32_t L = 0;
        for (uint32_t j = 0; j < W; j++) {
          const size_t c = base_c + j * step;
          if (m[c] && lvl_of[c] > L) L = lvl_of[c];
        }
        L++;
        const int32_t si = (int32_t)p.solves.size();
        p.order.push_back({Check::SOLVE, d, (int32_t)i, si});
        for (uint32_t j = 0; j < W; j++) {
          const size_t c = base_c + j * step;
          if (m[c]) continue;
          if (cnt[!d][j] == W - 1) p.order.push_back({Check::ORTH, !d, (int32_t)j, si});
          m[c] = 1;
          lvl_of[c] = L;
          cnt[!d][j]++;
          total++;
        }
        cnt[d][i] = W;
        p.solves.push_back({d, (int32_t)i});
        p.level.push_back(L);
        if (L > p.nlevels) p.nlevels = L;
        progress = true;
      }
    if (total == cells) p.solved = true;
    if (!progress) break;
  }
  return p;
}

static cel_status repair_exact(cel_ctx* ctx, RepairBufs& b, std::vector<uint8_t>& hm, uint32_t k,
                               const uint8_t* row_roots, const uint8_t* col_roots, const RepairOut& out) {
  const Range range("repair.exact");
  const uint32_t W = 2 * k;
  const size_t cells = (size_t)W * W;
  const SweepPlan plan = plan_sweeps(hm, k);
  const std::vector<Solve>& solves = plan.solves;
  const std::vector<int32_t>& level = plan.level;
  const std::vector<Check>& order = plan.order;
  const size_t S = solves.size();
  // order[first[t] .. first[t + 1]) = solve t's checks (SOLVE, then its ORTH axes)
  std::vector<size_t> first(S + 1, order.size());
  for (size_t o = 0; o < order.size(); o++)
    if (order[o].kind == Check::SOLVE) first[(size_t)order[o].solve] = o;
  const bool in_square = rs_decode_axis_supported(W, kShare);
  // roots of the checked axes: 96-byte records after the axes-roots workspace (b.work holds
  // the whole-square commit's workspace, which is larger)
  const size_t ws_axes = (axes_roots_workspace_size(k, W) + 255) & ~(size_t)255;
  uint32_t* d_rec = reinterpret_cast<uint32_t*>(b.work + ws_axes);
  std::vector<uint8_t> h_rec((size_t)2 * W * kNodeWords * 4);
  std::vector<int32_t> h_flags((size_t)2 * W);
  hipError_t e;
  cel_status st;
  // both streams are idle (verify_square synchronised the joined streams); the square keeps
  // the bytes of every cell known at the start (decoders store erased cells only)
  std::memcpy(b.hmask, hm.data(), cells);
  if ((e = hipMemcpyAsync(b.mask, b.hmask, cells, hipMemcpyHostToDevice, b.main)) != hipSuccess ||
      (e = hipMemsetAsync(b.flags, 0, 2 * (size_t)W * 4, b.main)) != hipSuccess)
    return hip_fail(ctx, e, "H2D");
  // The sequence runs in prefixes of CH solves. A prefix's solves depend only on earlier
  // solves, so each prefix runs level by level after the previous one; then its checks
  // (encoding and root of every axis it solves or completes) come back, and the first
  // failure in sweep order ends the replay there: rsmt2d returns at its first failing check.
  const size_t CH = std::max<size_t>(16, W / 4);
  for (size_t s0 = 0; s0 < S; s0 += CH) {
    const size_t s1 = std::min(S, s0 + CH);
    std::vector<int32_t> lists;
    struct Group {
      uint32_t off, n;
      int is_col;  // -1: mixed (register decoder, direction in bit 30)
    };
    std::vector<Group> groups;
    {
      int32_t lo = INT32_MAX, hi = 0;
      for (size_t t = s0; t < s1; t++) {
        lo = std::min(lo, level[t]);
        hi = std::max(hi, level[t]);
      }
      std::vector<std::vector<int32_t>> by[2];
      by[0].resize((size_t)(hi - lo + 1));
      by[1].resize((size_t)(hi - lo + 1));
      for (size_t t = s0; t < s1; t++) by[solves[t].is_col][(size_t)(level[t] - lo)].push_back(solves[t].idx);
      for (size_t L = 0; L < by[0].size(); L++) {
        if (in_square) {
          const uint32_t off = (uint32_t)lists.size();
          for (int d = 0; d < 2; d++)
            for (int32_t i : by[d][L]) lists.push_back(d ? (int32_t)((uint32_t)i | (1u << 30)) : i);
          if ((uint32_t)lists.size() > off) groups.push_back({off, (uint32_t)lists.size() - off, -1});
          continue;
        }
        for (int d = 0; d < 2; d++)
          if (!by[d][L].empty()) {
            groups.push_back({(uint32_t)lists.size(), (uint32_t)by[d][L].size(), d});
            lists.insert(lists.end(), by[d][L].begin(), by[d][L].end());
          }
      }
    }
    // the axes this prefix's checks look at, by direction (each axis is checked once)
    std::vector<int32_t> chk[2];
    for (size_t o = first[s0]; o < first[s1]; o++) chk[order[o].is_col].push_back(order[o].idx);
    const uint32_t off_chk0 = (uint32_t)lists.size();
    lists.insert(lists.end(), chk[0].begin(), chk[0].end());
    const uint32_t off_chk1 = (uint32_t)lists.size();
    lists.insert(lists.end(), chk[1].begin(), chk[1].end());
    std::memcpy(b.hidx, lists.data(), lists.size() * 4);
    if ((e = hipMemcpyAsync(b.idx, b.hidx, lists.size() * 4, hipMemcpyHostToDevice, b.main)) != hipSuccess)
      return hip_fail(ctx, e, "H2D");
    for (const Group& g : groups) {
      const int32_t* idx = b.idx + g.off;
      if ((st = fuzz(ctx, b.main)) != CEL_OK) return st;
      if (in_square) {
        e = launch_rs_decode_in_square(b.eds, b.mask, W, idx, g.is_col, g.n, ctx->tables.mul8, b.main);
      } else if ((e = launch_gather_axes(b.eds, b.mask, W, idx, g.is_col, g.n, b.dense[0], b.dmask, b.main)) ==
                     hipSuccess &&
                 (e = launch_rs_decode(b.dense[0], b.dmask, g.n, k, kShare, ctx->tables, nullptr, b.main)) ==
                     hipSuccess) {
        e = launch_scatter_axes(b.eds, b.mask, W, idx, g.is_col, g.n, b.dense[0], b.main);
      }
      if (e != hipSuccess) return hip_fail(ctx, e, "solve");
    }
    // encoding check and root of every checked axis, one direction at a time through dchk
    for (int d = 0; d < 2; d++) {
      const uint32_t na = (uint32_t)chk[d].size();
      if (!na) continue;
      const int32_t* idx = b.idx + (d ? off_chk1 : off_chk0);
      uint32_t* rec = d_rec + (size_t)d * W * kNodeWords;
      if ((e = launch_gather_axes(b.eds, b.mask, W, idx, d, na, b.dchk, b.dmask_chk, b.main)) != hipSuccess)
        return hip_fail(ctx, e, "gather");
      if ((st = encode_check(ctx, b, k, d, na, b.dchk, idx, b.main)) != CEL_OK) return st;
      if ((e = launch_axes_roots(b.dchk, k, idx, na, rec, b.work, b.main)) != hipSuccess)
        return hip_fail(ctx, e, "roots");
    }
    if ((e = hipMemcpyAsync(h_flags.data(), b.flags, h_flags.size() * 4, hipMemcpyDeviceToHost, b.main)) !=
            hipSuccess ||
        (e = hipMemcpyAsync(h_rec.data(), d_rec, h_rec.size(), hipMemcpyDeviceToHost, b.main)) != hipSuccess ||
        (e = hipStreamSynchronize(b.main)) != hipSuccess)
      return hip_fail(ctx, e, "D2H");
    // replay the prefix's checks in sweep order
    size_t pos[2] = {0, 0};
    for (size_t o = first[s0]; o < first[s1]; o++) {
      const Check& c = order[o];
      const uint8_t* got = h_rec.data() + ((size_t)c.is_col * W + pos[c.is_col]++) * kNodeWords * 4;
      const uint8_t* exp = (c.is_col ? col_roots : row_roots) + (size_t)c.idx * kNode;
      const bool root_ok = std::memcmp(got, exp, kNode) == 0;
      const bool enc_ok = h_flags[(size_t)c.is_col * W + (size_t)c.idx] == 0;
      if (!root_ok || !enc_ok) {
        rollback(hm, W, solves, (size_t)c.solve);
        return fail_axis(ctx, b, hm, out, CEL_EBYZANTINE, c.is_col, c.idx, c.kind == Check::SOLVE);
      }
    }
  }
  // not reached for a square the pass schedule found byzantine (the outcome does not depend
  // on the order when every check passes), kept for completeness
  if (!plan.solved) {
    rollback(hm, W, solves, S);
    return fail(ctx, CEL_EUNREPAIRABLE, "failed to solve data square");
  }
  std::fill(hm.begin(), hm.end(), (uint8_t)1);
  return CEL_OK;
}

// rsmt2d Repair over the EDS resident at b.eds. hm = host presence mask (updated: all
// ones on success, the mask before the failing solve on a byzantine / bad-root error,
// the mask after the last solve when stuck). No pass waits for the device. Root checks
// are deferred: an axis, once complete, never changes, so one commit pass over the final
// square gives every root rsmt2d checks on the way, and the checks are replayed in
// rsmt2d's order, reporting the first failure.
//
// The solves run in passes (every solvable row, then every solvable column, ...), which
// decodes whole directions at once. When every check passes, the outcome equals that of
// rsmt2d's sweep order (row i, then column i): all cells of the final square then agree
// with valid codewords whose roots match, so any order decodes the same bytes and passes
// the same checks, and the set of axes that can be solved is the same closure. Only a
// failing solve or orthogonal check depends on the order; that square is replayed in
// rsmt2d's order by repair_exact.
static cel_status repair_core(cel_ctx* ctx, RepairBufs& b, std::vector<uint8_t>& hm, uint32_t k,
                              const uint8_t* row_roots, const uint8_t* col_roots, const RepairOut& out) {
  const uint32_t W = 2 * k;
  const size_t cells = (size_t)W * W;
  hipStream_t s = b.main;
  hipError_t e = hipSuccess;
  cel_status st;
  // an early return leaves no side-stream work running on the ctx's scratch buffers
  struct SideDrain {
    hipStream_t side;
    ~SideDrain() { (void)hipStreamSynchronize(side); }
  } drain{b.side};
  // The first row pass goes to the device before the host builds its bookkeeping (the
  // mask bitsets, the sanity lists), which then runs beside the decode; its axis list
  // rides in the mask's upload.
  std::vector<int32_t> list, orth, first;
  for (uint32_t i = 0; i < W; i++) {  // hm bytes are 0 / 1: a word's popcount is its count
    const uint8_t* r = hm.data() + (size_t)i * W;
    uint32_t c = 0;
    uint32_t j = 0;
    for (; j + 8 <= W; j += 8) {
      uint64_t x;
      std::memcpy(&x, r + j, 8);
      c += (uint32_t)__builtin_popcountll(x);
    }
    for (; j < W; j++) c += r[j];
    if (c >= k && c < W) first.push_back((int32_t)i);
  }
  const size_t cells_a = (cells + 255) & ~(size_t)255;
  std::memcpy(b.hmask, hm.data(), cells);
  if (!first.empty()) std::memcpy(b.hmask + cells_a, first.data(), first.size() * 4);
  // the flags are the side stream's (its checks), zeroed there after the mask is up
  if ((e = hipMemcpyAsync(b.mask, b.hmask, cells_a + first.size() * 4, hipMemcpyHostToDevice, s)) != hipSuccess ||
      (e = hipEventRecord(b.ev_main, s)) != hipSuccess || (e = hipStreamWaitEvent(b.side, b.ev_main, 0)) != hipSuccess ||
      (e = hipMemsetAsync(b.flags, 0, 2 * (size_t)W * 4, b.side)) != hipSuccess)
    return hip_fail(ctx, e, "H2D");
  // Each pass's encoding check (side stream) is enqueued after the next pass's decode, so
  // the host's enqueue of it is off the solve chain (the checked axes are final from their
  // pass on; the dense path's buffer dense[d] is reused two passes later, after the check
  // has recorded ev_side[d]).
  Issued prev;
  int prev_col = 0;
  if ((st = solve_issue(ctx, b, k, 0, first, &prev, b.list0)) != CEL_OK) return st;
  bool first_issued = !first.empty();
  std::unique_ptr<Range> plan_range(new Range("repair.plan"));
  MaskBits mb(hm, W);
  std::vector<Check> order;
  std::vector<Solve> solves;
  // preRepairSanityCheck: for i: row i, column i
  {
    std::vector<int32_t> comp[2];
    for (uint32_t i = 0; i < W; i++)
      for (int is_col = 0; is_col < 2; is_col++)
        if (mb.cnt[is_col][i] == W) {
          order.push_back({Check::SANITY, is_col, (int32_t)i, -1});
          comp[is_col].push_back((int32_t)i);
        }
    for (int is_col = 0; is_col < 2; is_col++)
      if ((st = check_pass(ctx, b, k, is_col, comp[is_col], true)) != CEL_OK) return st;
  }
  // The orthogonal checks of a pass are issued after the next pass's decode (or the final
  // commit), so the host's enqueue of them is not on the solve chain; the side stream runs
  // them right after that pass's own encoding checks.
  std::vector<int32_t> pending;
  int pending_col = 0;
  plan_range.reset();
  // passes: all solvable rows, then all solvable columns, until solved or stuck
  bool solved = false;
  std::vector<std::vector<int32_t>> by_solve;
  for (;;) {
    bool progress = false;
    for (int is_col = 0; is_col < 2; is_col++) {
      list.clear();
      orth.clear();
      for (uint32_t i = 0; i < W; i++) {
        const uint32_t c = mb.cnt[is_col][i];
        if (c >= k && c < W) list.push_back((int32_t)i);
      }
      if (list.empty()) continue;
      if (first_issued) {  // the first row pass (the same list, issued above)
        first_issued = false;
      } else {
        Issued s1;
        if ((st = solve_issue(ctx, b, k, is_col, list, &s1)) != CEL_OK ||
            (st = solve_check(ctx, b, k, prev_col, prev)) != CEL_OK ||
            (st = check_pass(ctx, b, k, pending_col, pending, false)) != CEL_OK)
          return st;
        prev = s1;
        prev_col = is_col;
        pending.clear();
      }
      // sequential view of the pass: solve i fills its missing cells, completing the
      // orthogonal axes whose last missing cell it held
      const Range fill_range("repair.fill");
      mb.fill_pass(is_col, list, by_solve);
      for (size_t t = 0; t < list.size(); t++) {
        const int32_t si = (int32_t)solves.size();
        order.push_back({Check::SOLVE, is_col, list[t], si});
        for (int32_t j : by_solve[t]) {
          order.push_back({Check::ORTH, !is_col, j, si});
          orth.push_back(j);
        }
        solves.push_back({is_col, list[t]});
      }
      std::sort(orth.begin(), orth.end());
      // pending is empty here: the previous pass's orthogonal checks were issued (and
      // cleared) right after this pass's solve above, or this is the first pass
      pending.swap(orth);
      pending_col = !is_col;
      progress = true;
    }
    if (mb.total == cells) {
      solved = true;
      break;
    }
    if (!progress) break;
  }
  Verify v{nullptr, nullptr, row_roots, col_roots, W};
  if ((st = verify_square(ctx, b, k, prev_col, prev, pending_col, pending, &v)) != CEL_OK) return st;
  cel_status code;
  const long f = v.first_failure(order, &code);
  if (f >= 0) {
    const Check& c = order[(size_t)f];
    if (c.kind == Check::SANITY) return fail_axis(ctx, b, hm, out, code, c.is_col, c.idx, false);
    return repair_exact(ctx, b, hm, k, row_roots, col_roots, out);
  }
  if (!solved) {
    rollback(hm, W, solves, solves.size());
    return fail(ctx, CEL_EUNREPAIRABLE, "failed to solve data square");
  }
  std::fill(hm.begin(), hm.end(), (uint8_t)1);
  return CEL_OK;
}

static cel_status repair_bufs(cel_ctx* ctx, uint32_t k, bool own_eds, RepairBufs* b) {
  const uint32_t W = 2 * k;
  const size_t cells = (size_t)W * W, eds_b = cells * kShare;
  const size_t cells_a = (cells + 255) & ~(size_t)255;
  hipError_t e = hipSuccess;
  b->W = W;
  if (own_eds) b->eds = static_cast<uint8_t*>(scratch(ctx, S_EDS, eds_b, &e));
  b->dense[0] = static_cast<uint8_t*>(scratch(ctx, S_IN, 3 * eds_b, &e));
  b->tmp = static_cast<uint8_t*>(scratch(ctx, S_AUX, eds_b / 2 + (size_t)kIdxSlots * W * 4 + 256, &e));
  const size_t list_a = ((size_t)W * 4 + 255) & ~(size_t)255;
  b->mask = static_cast<uint8_t*>(scratch(ctx, S_MASK, 3 * cells_a + list_a, &e));
  b->work = static_cast<uint8_t*>(scratch(ctx, S_WORK, nmt_workspace_size(k, 1), &e));
  const size_t roots_a = (2 * (size_t)W * kNode + 255) & ~(size_t)255;
  b->res_bytes = roots_a + 2 * (size_t)W * 4;
  b->roots = static_cast<uint8_t*>(scratch(ctx, S_ROOTS, b->res_bytes, &e));
  if (!b->eds || !b->dense[0] || !b->tmp || !b->mask || !b->work || !b->roots)
    return fail(ctx, CEL_ENOMEM, "device allocation failed");
  b->dense[1] = b->dense[0] + eds_b;
  b->dchk = b->dense[1] + eds_b;
  b->list0 = reinterpret_cast<int32_t*>(b->mask + cells_a);
  b->dmask = b->mask + cells_a + list_a;
  b->dmask_chk = b->dmask + cells_a;
  b->flags = reinterpret_cast<int32_t*>(b->roots + roots_a);
  b->idx = reinterpret_cast<int32_t*>(b->tmp + eds_b / 2);
  const size_t cells_h = (cells + 255) & ~(size_t)255;
  // axis lists, mask + first list, results
  const size_t hb = (size_t)kIdxSlots * W * 4 + cells_h + list_a + b->res_bytes;
  if (!host_stage(ctx, hb)) return fail(ctx, CEL_ENOMEM, "page-locked allocation failed");
  b->hidx = static_cast<int32_t*>(ctx->hstage);
  b->hmask = static_cast<uint8_t*>(ctx->hstage) + (size_t)kIdxSlots * W * 4;
  b->hres = b->hmask + cells_h + list_a;
  b->slot = 0;
  b->solves = 0;
  // the side stream and the events are the batch pipeline's (the ctx lock is held)
  b->main = ctx->stream;
  b->side = ctx->sub[0];
  b->ev_main = ctx->ev_rs[0];
  b->ev_side[0] = ctx->ev_rs[1];
  b->ev_side[1] = ctx->ev_rs[2];
  b->ev_done = ctx->ev_rs[3];
  // no stale record of an earlier call may gate this one: both streams start from here
  if ((e = hipEventRecord(b->ev_side[0], b->side)) != hipSuccess || (e = hipEventRecord(b->ev_side[1], b->side)) != hipSuccess)
    return hip_fail(ctx, e, "event");
  return CEL_OK;
}

}  // namespace


cel_status cel_repair(cel_ctx* ctx, uint8_t* eds, uint8_t* present, uint32_t k, uint32_t share_size,
                      const uint8_t* row_roots, const uint8_t* col_roots, int32_t* bad_axis, int32_t* bad_index,
                      uint8_t* byz_shares, uint8_t* byz_present) {
  if (!ctx) return CEL_EINVAL;
  std::lock_guard<std::mutex> lock(ctx->mu);
  if (!eds || !present || !row_roots || !col_roots) return fail(ctx, CEL_EINVAL, "nil argument");
  cel_status st = validate_square(ctx, k, share_size);
  if (st) return st;
  if (bad_axis) *bad_axis = -1;
  if (bad_index) *bad_index = -1;
  DeviceGuard g(ctx->device);
  const uint32_t W = 2 * k;
  const size_t cells = (size_t)W * W, eds_b = cells * kShare;
  RepairBufs b{};
  if ((st = repair_bufs(ctx, k, true, &b)) != CEL_OK) return st;
  hipStream_t s = ctx->stream;
  hipError_t e;
  std::vector<uint8_t> hm(cells);
  for (size_t i = 0; i < cells; i++) hm[i] = present[i] != 0;
  if ((e = hipMemcpyAsync(b.eds, eds, eds_b, hipMemcpyHostToDevice, s)) != hipSuccess) return hip_fail(ctx, e, "H2D");
  st = repair_core(ctx, b, hm, k, row_roots, col_roots, RepairOut{bad_axis, bad_index, byz_shares, byz_present});
  if (st != CEL_OK && st != CEL_EBYZANTINE && st != CEL_EBADROOT && st != CEL_EUNREPAIRABLE) return st;
  // the (partially) repaired square goes back either way, with the mask it is valid under
  if ((e = hipMemcpyAsync(eds, b.eds, eds_b, hipMemcpyDeviceToHost, s)) != hipSuccess) return hip_fail(ctx, e, "D2H");
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return hip_fail(ctx, e, "sync");
  std::memcpy(present, hm.data(), cells);
  return st;
}

cel_status cel_debug_repair_plan(const uint8_t* present, uint32_t k, int32_t* solve_axis, int32_t* solve_index,
                                 int32_t* solve_level, uint32_t* nsolves, int32_t* solved) {
  if (!present || !solve_axis || !solve_index || !solve_level || !nsolves || !solved || !k || (k & (k - 1)) ||
      k > 512)
    return CEL_EINVAL;
  const size_t cells = (size_t)4 * k * k;
  std::vector<uint8_t> hm(cells);
  for (size_t i = 0; i < cells; i++) hm[i] = present[i] != 0;
  const SweepPlan p = plan_sweeps(hm, k);
  for (size_t t = 0; t < p.solves.size(); t++) {
    solve_axis[t] = p.solves[t].is_col;
    solve_index[t] = p.solves[t].idx;
    solve_level[t] = p.level[t];
  }
  *nsolves = (uint32_t)p.solves.size();
  *solved = p.solved ? 1 : 0;
  return CEL_OK;
}

cel_status cel_debug_schedule_fuzz(cel_ctx* ctx, uint64_t seed, uint32_t max_us) {
  if (!ctx) return CEL_EINVAL;
  std::lock_guard<std::mutex> lock(ctx->mu);
  if (max_us > 100000) return fail(ctx, CEL_EINVAL, "max_us above 100 ms");
  ctx->fuzz_state = seed;
  ctx->fuzz_max_us = max_us;
  return CEL_OK;
}

cel_status cel_dev_repair(cel_ctx* ctx, void* d_eds, uint8_t* present, uint32_t k, const uint8_t* row_roots,
                          const uint8_t* col_roots, int32_t* bad_axis, int32_t* bad_index, uint8_t* byz_shares,
                          uint8_t* byz_present) {
  if (!ctx) return CEL_EINVAL;
  std::lock_guard<std::mutex> lock(ctx->mu);
  if (!d_eds || !present || !row_roots || !col_roots) return fail(ctx, CEL_EINVAL, "nil argument");
  cel_status st = validate_square(ctx, k, kShare);
  if (st) return st;
  if (bad_axis) *bad_axis = -1;
  if (bad_index) *bad_index = -1;
  DeviceGuard g(ctx->device);
  const size_t cells = (size_t)4 * k * k;
  RepairBufs b{};
  b.eds = static_cast<uint8_t*>(d_eds);
  if ((st = repair_bufs(ctx, k, false, &b)) != CEL_OK) return st;
  std::vector<uint8_t> hm(cells);
  for (size_t i = 0; i < cells; i++) hm[i] = present[i] != 0;
  st = repair_core(ctx, b, hm, k, row_roots, col_roots, RepairOut{bad_axis, bad_index, byz_shares, byz_present});
  if (st == CEL_OK || st == CEL_EBYZANTINE || st == CEL_EBADROOT || st == CEL_EUNREPAIRABLE)
    std::memcpy(present, hm.data(), cells);
  return st;
}

}  // extern "C"
