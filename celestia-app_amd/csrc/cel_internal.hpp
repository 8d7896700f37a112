// Internal declarations shared by the HIP kernels and the C-ABI host layer.
#pragma once
#include <hip/hip_runtime.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <cstddef>
#include <cstdint>
#include <mutex>
#include <string>

#include "../../include/celestia_eds.h"

namespace cel {

constexpr uint32_t kShare = CEL_SHARE_SIZE;
constexpr uint32_t kNs = CEL_NAMESPACE_SIZE;
constexpr uint32_t kNode = CEL_NMT_NODE_SIZE;
constexpr uint32_t kNodeWords = 24;  // 90-byte node padded to 96 B (24 dwords) on the device
constexpr uint32_t kMaxGf8Width = 128;   // k <= 128 -> 2k <= 256 shards -> GF(2^8)
constexpr uint32_t kMaxGf16Width = 2048; // LDS holds 2048 shards x 64 B per workgroup

// One RS encode launch: `axes` independent axes of n data shards each, for `nsq`
// squares. Shard i of axis a of square s lives at
//   in + s*in_sq + a*in_axis + i*in_shard        (len bytes)
// and its parity shard i goes to out + s*out_sq + a*out_axis + i*out_shard.
struct RsGeom {
  const uint8_t* in;
  uint8_t* out;
  uint64_t in_sq, in_axis, in_shard;
  uint64_t out_sq, out_axis, out_shard;
  // Optional copy of the data shards (the row pass writes Q0 into the EDS while it
  // has them in registers): dcopy + s*dc_sq + a*dc_axis + i*dc_shard. nullptr = none.
  uint8_t* dcopy;
  uint64_t dc_sq, dc_axis, dc_shard;
  // Blocked shard placement (row-sharded mode: the row pass writes straight into the
  // all-to-all send layout). When blk_log != 0, output / dcopy shard j goes to
  //   ((j >> blk_log) * *_blk) + (j & ((1 << blk_log) - 1)) * *_shard
  // instead of j * *_shard. Only the GF(2^16) register kernel supports it.
  uint32_t blk_log;
  uint64_t out_blk, dc_blk;
  uint32_t n;     // data shards per axis (power of two)
  uint32_t len;   // bytes per shard (multiple of 64)
  uint32_t axes;  // axes per square
  uint32_t nsq;   // squares
  // Check mode (GF(2^16) register kernel, n = 256/512, nsq == 1): nothing is stored; the
  // computed parity is compared with the bytes at `out` and a mismatch in axis a sets
  // chk_flags[chk_idx ? chk_idx[a] : a]. nullptr = encode.
  int32_t* chk_flags;
  const int32_t* chk_idx;
  // Check mode only: axis a of the launch is axis chk_axes[a] of the square (in/out bases
  // in + chk_axes[a]*in_axis, out + chk_axes[a]*out_axis), so the check reads the square in
  // place. nullptr = axis a.
  const int32_t* chk_axes;
};

struct DeviceTables {
  uint32_t* tw8 = nullptr;     // [255][8] GF(2^8) twiddle product tables, indexed by skew index
  uint16_t* exp16 = nullptr;   // [65536]
  uint16_t* log16 = nullptr;   // [65536]
  uint32_t* mul8 = nullptr;    // [256][8] GF(2^8) product tables indexed by log value (decoder)
  uint32_t* tw16 = nullptr;    // [4095][8] GF(2^16) bit-plane twiddles: products c*b_i in tower coordinates
  uint16_t* tower16 = nullptr; // [256 + 256 + 16] Cantor -> tower coordinates (lo, hi byte), b_i (decoder)
};

// Block size 2^J of the GF(2^16) decoder's products by twiddles below 2^r (Cantor
// representation): such a twiddle lies in GF(2^(2^J)), the smallest Cantor subfield holding
// span(beta_0 .. beta_{r-1}).
constexpr uint32_t decode16_level(uint32_t r) { return r <= 1 ? 0 : r <= 2 ? 1 : r <= 4 ? 2 : r <= 8 ? 3 : 4; }

// roctx range over a phase's launches (rocprofv3 --marker-trace shows them on the host
// timeline; the launches themselves are asynchronous, so a range brackets their enqueue).
struct Range {
  explicit Range(const char* name) { roctxRangePushA(name); }
  ~Range() { roctxRangePop(); }
  Range(const Range&) = delete;
  Range& operator=(const Range&) = delete;
};

// XCD-aware workgroup order. Workgroups are dealt round-robin over the 8 XCDs
// (MI355X_MICROARCH.md, "Workgroup dispatch"), so workgroup b shares an L2 with b + 8.
// Map them so that each XCD works through one contiguous range of logical ids: the
// column passes then stream adjacent column blocks through each XCD's L2 channels instead
// of one fixed residue of column offsets per XCD. A bijection of [0, nb) for any nb;
// for speed only (nothing relies on where a workgroup runs).
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t nb) {
  const uint32_t q = nb >> 3, r = nb & 7u, x = b & 7u;
  return x * q + (x < r ? x : r) + (b >> 3);
}

hipError_t upload_tables(DeviceTables* t);
void free_tables(DeviceTables* t);

// Kernel launchers (rs_kernels.hip / nmt_kernels.hip). All asynchronous on `s`.
hipError_t launch_rs_encode(const RsGeom& g, const DeviceTables& t, hipStream_t s);
hipError_t launch_rs_encode_bitslice(const RsGeom& g, hipStream_t s);  // GF(2^8), n <= 16
hipError_t launch_rs_encode_axis(const RsGeom& g, hipStream_t s);       // GF(2^8), 32 <= n <= 128
// Two launches' worth of GF(2^8) axes (same n, len, axes count and squares, no data copy) in
// one launch with their tiles interleaved per square (rs_axis.hip, k_rs_axis_gf8_pair).
hipError_t launch_rs_encode_axis_pair(const RsGeom& g1, const RsGeom& g2, hipStream_t s);
// Encoding check of listed axes in place in a resident EDS (flags[axis] |= 1 on mismatch),
// GF(2^8), k = 32, 64, 128.
hipError_t launch_rs_check_axes(const uint8_t* eds, uint32_t k, const int32_t* idx, int is_col, uint32_t naxes,
                                int32_t* flags, hipStream_t s);
hipError_t launch_rs_encode_gf16x(const RsGeom& g, hipStream_t s);     // GF(2^16), n = 256 / 512
// Full 2D extension of nsq squares: Q0 rows -> Q1, then all 2k columns -> Q2|Q3.
// ods == nullptr means Q0 is already in place inside eds.
hipError_t launch_extend(const uint8_t* ods, uint8_t* eds, uint32_t k, uint32_t nsq,
                         const DeviceTables& t, hipStream_t s);
// The two passes apart, for one square's latency path: Q0 rows [row0, row1) -> Q1 (Q0
// read in place in the EDS, or from a contiguous k x k ODS `ods` and then also written into
// Q0), and all 2k columns -> Q2|Q3 of nsq squares.
hipError_t launch_extend_rows(uint8_t* eds, uint32_t k, uint32_t row0, uint32_t row1, const DeviceTables& t,
                              hipStream_t s, const uint8_t* ods = nullptr);
hipError_t launch_extend_cols(uint8_t* eds, uint32_t k, uint32_t nsq, const DeviceTables& t, hipStream_t s);

// NMT + DAH over resident EDSs. work: scratch of nmt_workspace_size(k, nsq) bytes.
size_t nmt_workspace_size(uint32_t k, uint32_t nsq);
hipError_t launch_commit(const uint8_t* eds, uint32_t k, uint32_t nsq, uint8_t* row_roots,
                         uint8_t* col_roots, uint8_t* dah, int32_t* status, void* work,
                         bool order_check, hipStream_t s);
// The same commit in two steps: the leaves of EDS rows [row0, row1) of every square
// (init_bad: reset the push-order flags first; it must precede every leaf launch of the
// commit in stream order), then, after every leaf, the tree levels, roots and DAH.
hipError_t launch_commit_leaves(const uint8_t* eds, uint32_t k, uint32_t nsq, void* work, bool order_check,
                                uint32_t row0, uint32_t row1, bool init_bad, hipStream_t s);
// host_out (nsq == 1, optional): page-locked host memory that receives out_bytes (a multiple of
// 16) starting at row_roots from the DAH launch itself; row_roots, col_roots, dah and status
// must then be one contiguous block in that order.
hipError_t launch_commit_trees(uint32_t k, uint32_t nsq, uint8_t* row_roots, uint8_t* col_roots, uint8_t* dah,
                               int32_t* status, void* work, hipStream_t s, uint8_t* host_out = nullptr,
                               uint32_t out_bytes = 0);
// One erasured axis root (cells contiguous) or plain NMT root over leaves.
hipError_t launch_axis_root(const uint8_t* cells, uint32_t k, uint32_t axis, uint8_t* root,
                            void* work, hipStream_t s);
size_t axis_root_workspace_size(uint32_t k);
hipError_t launch_nmt_root(const uint8_t* leaves, uint32_t n, uint32_t leaf_len, uint8_t* root,
                           void* work, hipStream_t s);
size_t nmt_root_workspace_size(uint32_t n);
// RFC-6962 root over n items of item_len bytes (DataAvailabilityHeader.Hash).
hipError_t launch_merkle_root(const uint8_t* items, uint32_t n, uint32_t item_len, uint8_t* out,
                              void* work, hipStream_t s);
size_t merkle_workspace_size(uint32_t n);
// merkle.HashFromByteSlices over n slices of any length (data + off[i] .. off[i + 1]),
// all device pointers; work: slices_workspace_size(n) bytes.
hipError_t launch_hash_slices(const uint8_t* data, const uint64_t* off, uint32_t n, uint8_t* out, void* work,
                              hipStream_t s);
size_t slices_workspace_size(uint32_t n);

// Row-sharded mode (one column slab of one square per rank).
size_t slab_workspace_size(uint32_t k, uint32_t w);
// The slab commit in two steps: leaves of slab rows [row0, row1) (the rows < k half first,
// init_bad resetting the push-order flag), then, after every leaf, the trees and status.
hipError_t launch_slab_leaves(const uint8_t* slab, uint32_t k, uint32_t c0, uint32_t w, uint32_t row0, uint32_t row1,
                              void* work, bool order_check, bool init_bad, hipStream_t s);
hipError_t launch_slab_trees(uint32_t k, uint32_t w, uint32_t* col_rec, uint32_t* row_sub, int32_t* status,
                             void* work, hipStream_t s);
// A rank's two device steps (api_shard.cpp): the row pass into the all-to-all send layout
// [nranks][k/nranks][w][512], and the column pass + slab commit over [2k][w][512].
hipError_t shard_rows_enqueue(const DeviceTables& t, const uint8_t* ods_rows, uint32_t k, uint32_t nranks,
                              uint8_t* send, hipStream_t s);
hipError_t shard_cols_enqueue(const DeviceTables& t, uint8_t* slab, uint32_t k, uint32_t nranks, uint32_t rank,
                              uint32_t* col_rec, uint32_t* row_sub, int32_t* status, void* work, bool order_check,
                              hipStream_t s);
size_t shard_finish_workspace_size(uint32_t k, uint32_t nranks);
// gathered: [nranks][2k + w + 1] records, rank order (row subtrees, column roots, status).
hipError_t launch_shard_finish(const uint32_t* gathered, uint32_t k, uint32_t nranks, uint8_t* row_roots,
                               uint8_t* col_roots, uint8_t* dah, int32_t* status, void* work, bool order_check,
                               hipStream_t s);

// Same-run probes (probe_kernels.hip): SHA-256 chained in registers (out: blocks*256 words,
// clk: 2 counters per wave), and a streaming copy of `bytes` (a multiple of 16).
hipError_t launch_probe_sha(uint32_t* out, unsigned long long* clk, uint32_t blocks, int n, hipStream_t s);
// mode 0: copy `bytes` from src to dst (one lane per 16-byte element; blocks unused); 1: read
// src only; 2 / 3: write dst only, 16 / 4 bytes per lane (grid-strided over `blocks` workgroups)
hipError_t launch_probe_copy(const void* src, void* dst, uint64_t bytes, uint32_t blocks, int mode, bool nt,
                             hipStream_t s);
// GF(2^8) encode transform alone (rs_axis.hip), k = 32/64/128: ntiles tiles reading the same
// k x 256 B of src; dst (k x 256 B) written only when store != 0.
hipError_t launch_probe_rs_transform(uint32_t k, const uint32_t* src, uint32_t* dst, uint32_t ntiles, uint32_t store,
                                     hipStream_t s);
// GF(2^16) register kernel alone (rs_gf16x.hip), k = 256/512: ntiles 64-byte-block tiles, all
// loads from the 512 bytes at src, nothing stored.
hipError_t launch_probe_rs_transform_gf16(uint32_t k, const uint8_t* src, uint8_t* dst, uint32_t ntiles,
                                          hipStream_t s);

// Repair helpers (repair_kernels.hip, nmt_kernels.hip).
hipError_t launch_gather_axes(const uint8_t* eds, const uint8_t* mask, uint32_t W, const int32_t* idx, int is_col,
                              uint32_t naxes, uint8_t* dense, uint8_t* dmask, hipStream_t s);
hipError_t launch_scatter_axes(uint8_t* eds, uint8_t* mask, uint32_t W, const int32_t* idx, int is_col,
                               uint32_t naxes, const uint8_t* dense, hipStream_t s);
hipError_t launch_cmp(const uint8_t* x, uint64_t xstride, const uint8_t* y, uint64_t ystride, uint64_t bytes,
                      uint32_t naxes, int32_t* flags, hipStream_t s, const int32_t* idx = nullptr);
size_t axes_roots_workspace_size(uint32_t k, uint32_t naxes);
// A single-wave kernel that idles `us` microseconds on s (schedule fuzzing only).
hipError_t launch_delay(uint32_t us, hipStream_t s);
hipError_t launch_axes_roots(const uint8_t* cells, uint32_t k, const int32_t* axis_idx, uint32_t naxes,
                             uint32_t* roots, void* work, hipStream_t s);

// Exported trees (proofs): all NMT levels of gathered axes (level-major, 96-byte records,
// axes_trees_nodes(k, naxes) records) and all RFC-6962 levels over n = 2^m 90-byte items
// (2n - 1 nodes of 8 big-endian words; work: merkle_workspace_size(n) bytes).
size_t axes_trees_nodes(uint32_t k, uint32_t naxes);
hipError_t launch_axes_trees(const uint8_t* cells, uint32_t k, const int32_t* axis_idx, uint32_t naxes,
                             uint32_t* nodes, hipStream_t s);
hipError_t launch_rfc_tree(const uint8_t* items90, uint32_t n, uint32_t* levels, void* work, hipStream_t s);

hipError_t launch_gather_nodes(const uint32_t* nodes, const int32_t* rec, uint32_t n, uint8_t* out, hipStream_t s);
// Blob share commitment (inclusion.cpp): trees of the gathered rows, subtree roots at
// (rows[i], depths[i], positions[i]) of the rows' ODS halves, RFC-6962 root -> d_out[32].
hipError_t launch_commitment(const uint8_t* d_cells, uint32_t k, uint32_t r0, uint32_t nrows, const uint32_t* rows,
                             const uint32_t* depths, const uint32_t* positions, uint32_t npaths, int32_t* d_idx,
                             uint32_t* d_nodes, uint8_t* d_items, void* d_merkle_work, uint8_t* d_out,
                             hipStream_t s);

// Erasure decode of `naxes` axes of 2n shards each, gathered into a dense
// [naxes][2n][len] buffer with a [naxes][2n] present mask. In place.
// GF(2^16) erasure decode over n = 512, 1024 or 2048 points (rs_decode_gf16.hip).
bool rs_decode_gf16_supported(uint32_t n);
// GF(2^16) encode of 1024 or 2048 data shards in bit planes (codec API).
hipError_t launch_rs_encode_gf16p(const RsGeom& g, const DeviceTables& t, hipStream_t s);
hipError_t launch_rs_decode_gf16(uint8_t* shards, const uint8_t* present, uint32_t naxes, uint32_t n, uint32_t len,
                                 const DeviceTables& t, hipStream_t s);
hipError_t launch_rs_decode(uint8_t* shards, const uint8_t* present, uint32_t naxes, uint32_t n,
                            uint32_t len, const DeviceTables& t, void* work, hipStream_t s);
size_t decode_workspace_size(uint32_t naxes, uint32_t n);
// GF(2^8) register-resident decode (rs_decode_axis.hip): n = 32..256 points, len % 64 == 0.
bool rs_decode_axis_supported(uint32_t n, uint32_t len);
hipError_t launch_rs_decode_axis(uint8_t* shards, const uint8_t* present, uint32_t naxes, uint32_t n, uint32_t len,
                                 const uint32_t* mul8, hipStream_t s);
// The repair's solve of naxes axes (rows if is_col == 0, columns if 1, indices idx; with
// is_col < 0 every entry carries its direction in bit 30) of a W x W square of 512-byte
// cells in place: erased cells decoded straight into the square, the axes marked present
// in mask (W = 32 .. 256, the register decoder's range).
hipError_t launch_rs_decode_in_square(uint8_t* eds, uint8_t* mask, uint32_t W, const int32_t* idx, int is_col,
                                      uint32_t naxes, const uint32_t* mul8, hipStream_t s);

}  // namespace cel

// The opaque context of the C ABI.
struct cel_ctx {
  static constexpr int kPipe = 4;     // internal streams of the chunked batch pipeline
  static constexpr int kChunks = 16;  // max chunks per batch call
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t sub[kPipe] = {nullptr, nullptr, nullptr, nullptr};
  hipEvent_t ev_start = nullptr;
  // CEL_FLAG_CALLER_STREAM batches: the previous one's extension-done event (recorded
  // once ext_pending); the next such batch starts after it (api.cpp)
  hipEvent_t ev_ext = nullptr;
  bool ext_pending = false;
  hipEvent_t ev_done[kChunks] = {};
  hipEvent_t ev_rs[kChunks] = {};
  // EDS downloads of the host pipeline, one per pipeline stream (beside the hashing)
  hipStream_t dl[kPipe] = {nullptr, nullptr, nullptr, nullptr};
  hipEvent_t ev_dl[kPipe] = {};
  std::mutex mu;
  cel::DeviceTables tables;
  std::string last_error;
  // Grow-only device scratch (reused across calls on this ctx).
  void* scratch[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  size_t scratch_size[6] = {0, 0, 0, 0, 0, 0};
  // Grow-only page-locked host staging (the repair's axis lists).
  void* hstage = nullptr;
  size_t hstage_size = 0;
  // Schedule fuzzing of the repair's two streams (cel_debug_schedule_fuzz; tests only):
  // before each enqueue point, an idle kernel of 0..fuzz_max_us microseconds.
  uint64_t fuzz_state = 0;
  uint32_t fuzz_max_us = 0;
  // cel_extend_sharded's plan (buffers, streams, RCCL communicators), kept while the device
  // list, k and flags stay the same (api_multi.cpp)
  cel_shard_plan* shard_cache = nullptr;
  // cel_extend_batch_multi's host worker thread for this ctx (api_multi.cpp), made on first use
  void* worker = nullptr;
};

namespace cel {
void destroy_ctx_worker(cel_ctx* c);  // api_multi.cpp: joins the ctx's worker, if any
}
