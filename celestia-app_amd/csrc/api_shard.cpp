// C ABI of the row-sharded single square (include/celestia_eds.h): a rank's
// row pass into the all-to-all send layout, its column slab, and the finish over the
// gathered records; collectives are the caller's (RCCL). Split from api.cpp.
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

namespace cel {

// Step 1 of a rank (shared by cel_dev_shard_rows and the in-library plan, api_multi.cpp):
// row-encode the rank's k/nranks ODS rows into the all-to-all send layout.
hipError_t shard_rows_enqueue(const DeviceTables& t, const uint8_t* ods_rows, uint32_t k, uint32_t nranks,
                              uint8_t* send, hipStream_t s) {
  const uint32_t rows = k / nranks, w = 2 * k / nranks;
  const uint64_t blk = (uint64_t)rows * w * kShare;  // one destination rank's block
  uint32_t wlog = 0;
  while ((1u << wlog) < w) wlog++;
  RsGeom gm{};
  gm.in = ods_rows;
  gm.in_sq = (uint64_t)rows * k * kShare;
  gm.in_axis = (uint64_t)k * kShare;
  gm.in_shard = kShare;
  // Q0 cell (i, j) -> block j / w, row i, slot j % w; Q1 cell (i, k + j) likewise
  gm.dcopy = send;
  gm.dc_sq = gm.in_sq;
  gm.dc_axis = (uint64_t)w * kShare;
  gm.dc_shard = kShare;
  gm.dc_blk = blk;
  gm.out = send + (uint64_t)(k / w) * blk + (uint64_t)(k % w) * kShare;
  gm.out_sq = gm.in_sq;
  gm.out_axis = (uint64_t)w * kShare;
  gm.out_shard = kShare;
  gm.out_blk = blk;
  gm.blk_log = wlog;
  gm.n = k;
  gm.len = kShare;
  gm.axes = rows;
  gm.nsq = 1;
  return launch_rs_encode(gm, t, s);
}

// Step 2 of a rank: column-encode its slab in place, hash the slab's leaves once, build its
// column-root and row-subtree records.
hipError_t shard_cols_enqueue(const DeviceTables& t, uint8_t* slab, uint32_t k, uint32_t nranks, uint32_t rank,
                              uint32_t* col_rec, uint32_t* row_sub, int32_t* status, void* work, bool order_check,
                              hipStream_t s) {
  const uint32_t w = 2 * k / nranks;
  RsGeom gm{};
  gm.in = slab;
  gm.in_sq = (uint64_t)2 * k * w * kShare;
  gm.in_axis = kShare;
  gm.in_shard = (uint64_t)w * kShare;
  gm.out = slab + (uint64_t)k * w * kShare;
  gm.out_sq = gm.in_sq;
  gm.out_axis = kShare;
  gm.out_shard = (uint64_t)w * kShare;
  gm.n = k;
  gm.len = kShare;
  gm.axes = w;
  gm.nsq = 1;
  // Column pass, then the slab's leaves and trees. Hashing the top half's leaves on a
  // second stream beside the column pass measured no faster (profiles/r3_rank_latency.txt).
  hipError_t e = launch_rs_encode(gm, t, s);
  if (e == hipSuccess) e = launch_slab_leaves(slab, k, rank * w, w, 0, 2 * k, work, order_check, true, s);
  if (e == hipSuccess) e = launch_slab_trees(k, w, col_rec, row_sub, status, work, s);
  return e;
}

}  // namespace cel

using namespace cel;
using namespace cel::abi;

extern "C" {

// ------------------------------------------------------------ row-sharded mode

static cel_status validate_shard(cel_ctx* ctx, uint32_t k, uint32_t nranks) {
  if (k != 256 && k != 512)
    return fail(ctx, CEL_EINVAL, "row-sharded mode supports k = 256 or 512 (GF(2^16)): got " + std::to_string(k));
  if (!is_pow2(nranks) || nranks > k)
    return fail(ctx, CEL_EINVAL, "nranks must be a power of two <= k: got " + std::to_string(nranks));
  return CEL_OK;
}

size_t cel_dev_shard_workspace_size(uint32_t k, uint32_t nranks) {
  if (!nranks) return 0;
  const size_t a = slab_workspace_size(k, 2 * k / nranks), b = shard_finish_workspace_size(k, nranks);
  return a > b ? a : b;
}

cel_status cel_dev_shard_rows(cel_ctx* ctx, const void* d_ods_rows, uint32_t k, uint32_t nranks, void* d_send,
                              void* stream) {
  if (!ctx || !d_ods_rows || !d_send) return CEL_EINVAL;
  std::lock_guard<std::mutex> lock(ctx->mu);
  cel_status st = validate_shard(ctx, k, nranks);
  if (st) return st;
  DeviceGuard g(ctx->device);
  hipError_t e = shard_rows_enqueue(ctx->tables, static_cast<const uint8_t*>(d_ods_rows), k, nranks,
                                    static_cast<uint8_t*>(d_send), pick_stream(ctx, stream));
  return e == hipSuccess ? CEL_OK : hip_fail(ctx, e, "shard rows");
}

cel_status cel_dev_shard_cols(cel_ctx* ctx, void* d_slab, uint32_t k, uint32_t nranks, uint32_t rank,
                              void* d_col_rec, void* d_row_sub, int32_t* d_status, void* d_work, void* stream,
                              uint32_t flags) {
  if (!ctx || !d_slab || !d_col_rec || !d_row_sub || !d_status || !d_work) return CEL_EINVAL;
  std::lock_guard<std::mutex> lock(ctx->mu);
  cel_status st = validate_shard(ctx, k, nranks);
  if (st) return st;
  if (rank >= nranks) return fail(ctx, CEL_EINVAL, "rank out of range");
  DeviceGuard g(ctx->device);
  hipError_t e = shard_cols_enqueue(ctx->tables, static_cast<uint8_t*>(d_slab), k, nranks, rank,
                                    static_cast<uint32_t*>(d_col_rec), static_cast<uint32_t*>(d_row_sub), d_status,
                                    d_work, (flags & CEL_FLAG_ORDER_CHECK) != 0, pick_stream(ctx, stream));
  return e == hipSuccess ? CEL_OK : hip_fail(ctx, e, "shard cols");
}

cel_status cel_dev_shard_finish(cel_ctx* ctx, const void* d_gathered, uint32_t k, uint32_t nranks, void* d_row_roots,
                                void* d_col_roots, void* d_dah, int32_t* d_status, void* d_work, void* stream,
                                uint32_t flags) {
  if (!ctx || !d_gathered || !d_row_roots || !d_col_roots || !d_dah || !d_status || !d_work) return CEL_EINVAL;
  std::lock_guard<std::mutex> lock(ctx->mu);
  cel_status st = validate_shard(ctx, k, nranks);
  if (st) return st;
  DeviceGuard g(ctx->device);
  hipError_t e = launch_shard_finish(static_cast<const uint32_t*>(d_gathered), k, nranks,
                                     static_cast<uint8_t*>(d_row_roots), static_cast<uint8_t*>(d_col_roots),
                                     static_cast<uint8_t*>(d_dah), d_status, d_work,
                                     (flags & CEL_FLAG_ORDER_CHECK) != 0, pick_stream(ctx, stream));
  return e == hipSuccess ? CEL_OK : hip_fail(ctx, e, "shard finish");
}

}  // extern "C"
