// C ABI of the trees (include/celestia_eds.h): one axis's NMT root, NMT roots over any
// leaves, the DAH hash, and every node of axis / DAH trees for the proofs.
// Split from api.cpp.
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

// -------------------------------------------------------------------- trees

cel_status cel_axis_root(cel_ctx* ctx, const uint8_t* cells, uint32_t k, uint32_t axis_index, uint32_t share_size,
                         uint8_t* root_out, uint32_t flags) {
  if (!ctx) return CEL_EINVAL;
  std::lock_guard<std::mutex> lock(ctx->mu);
  if (!cells || !root_out || !k) return fail(ctx, CEL_EINVAL, "nil argument");
  if (share_size != kShare) return fail(ctx, CEL_ECHUNK, "share size must be 512 on the device path");
  if (axis_index >= 2 * k)  // nmt_wrapper.go:94-96 (no uint32 wrap at 0xFFFFFFFF)
    return fail(ctx, CEL_EPUSHPAST, "pushed past predetermined square size: boundary at " + std::to_string(2 * k) +
                                        " index at " + std::to_string(axis_index) + " 0");
  if (flags & CEL_FLAG_ORDER_CHECK) {
    // honest nmt push order over the Q0 part of the axis (the rest carries the max namespace)
    if (axis_index < k)
      for (uint32_t i = 1; i < k; i++)
        if (std::memcmp(cells + (size_t)i * kShare, cells + (size_t)(i - 1) * kShare, kNs) < 0)
          return fail(ctx, CEL_EORDER, "invalid push order: namespace of leaf " + std::to_string(i) +
                                           " is smaller than the previous one");
  }
  DeviceGuard g(ctx->device);
  hipError_t e = hipSuccess;
  const size_t b = (size_t)2 * k * kShare;
  uint8_t* d_c = static_cast<uint8_t*>(scratch(ctx, S_IN, b, &e));
  void* d_w = scratch(ctx, S_WORK, axis_root_workspace_size(k), &e);
  uint8_t* d_r = static_cast<uint8_t*>(scratch(ctx, S_ROOTS, 256, &e));
  if (!d_c || !d_w || !d_r) return fail(ctx, CEL_ENOMEM, "device allocation failed");
  hipStream_t s = ctx->stream;
  if ((e = hipMemcpyAsync(d_c, cells, b, hipMemcpyHostToDevice, s)) != hipSuccess) return hip_fail(ctx, e, "H2D");
  if ((e = launch_axis_root(d_c, k, axis_index, d_r, d_w, s)) != hipSuccess) return hip_fail(ctx, e, "axis root");
  if ((e = hipMemcpyAsync(root_out, d_r, kNode, hipMemcpyDeviceToHost, s)) != hipSuccess) return hip_fail(ctx, e, "D2H");
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return hip_fail(ctx, e, "sync");
  return CEL_OK;
}

cel_status cel_nmt_root(cel_ctx* ctx, const uint8_t* leaves, uint32_t n, uint32_t leaf_len, uint8_t* root_out,
                        uint32_t flags) {
  if (!ctx) return CEL_EINVAL;
  std::lock_guard<std::mutex> lock(ctx->mu);
  if ((!leaves && n) || !root_out) return fail(ctx, CEL_EINVAL, "nil argument");
  if (n && leaf_len < kNs) return fail(ctx, CEL_ESHORT, "data is too short to contain namespace ID");
  if ((flags & CEL_FLAG_ORDER_CHECK) && n > 1)
    for (uint32_t i = 1; i < n; i++)
      if (std::memcmp(leaves + (size_t)i * leaf_len, leaves + (size_t)(i - 1) * leaf_len, kNs) < 0)
        return fail(ctx, CEL_EORDER, "invalid push order: namespace of leaf " + std::to_string(i) +
                                         " is smaller than the previous one");
  DeviceGuard g(ctx->device);
  hipError_t e = hipSuccess;
  const size_t b = (size_t)n * leaf_len;
  uint8_t* d_l = static_cast<uint8_t*>(scratch(ctx, S_IN, b, &e));
  void* d_w = scratch(ctx, S_WORK, nmt_root_workspace_size(n), &e);
  uint8_t* d_r = static_cast<uint8_t*>(scratch(ctx, S_ROOTS, 256, &e));
  if (!d_l || !d_w || !d_r) return fail(ctx, CEL_ENOMEM, "device allocation failed");
  hipStream_t s = ctx->stream;
  if (b && (e = hipMemcpyAsync(d_l, leaves, b, hipMemcpyHostToDevice, s)) != hipSuccess) return hip_fail(ctx, e, "H2D");
  if ((e = launch_nmt_root(d_l, n, leaf_len, d_r, d_w, s)) != hipSuccess) return hip_fail(ctx, e, "nmt root");
  if ((e = hipMemcpyAsync(root_out, d_r, kNode, hipMemcpyDeviceToHost, s)) != hipSuccess) return hip_fail(ctx, e, "D2H");
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return hip_fail(ctx, e, "sync");
  return CEL_OK;
}

cel_status cel_dah_hash(cel_ctx* ctx, const uint8_t* row_roots, const uint8_t* col_roots, uint32_t w, uint8_t* out) {
  if (!ctx) return CEL_EINVAL;
  std::lock_guard<std::mutex> lock(ctx->mu);
  if (!out || (w && (!row_roots || !col_roots))) return fail(ctx, CEL_EINVAL, "nil argument");
  if (2 * (size_t)w > 2048) return fail(ctx, CEL_ETOOBIG, "too many roots for the device DAH kernel");
  DeviceGuard g(ctx->device);
  hipError_t e = hipSuccess;
  const size_t b = (size_t)2 * w * kNode;
  uint8_t* d_items = static_cast<uint8_t*>(scratch(ctx, S_IN, b, &e));
  void* d_w = scratch(ctx, S_WORK, merkle_workspace_size(2 * w), &e);
  uint8_t* d_o = static_cast<uint8_t*>(scratch(ctx, S_ROOTS, 256, &e));
  if (!d_items || !d_w || !d_o) return fail(ctx, CEL_ENOMEM, "device allocation failed");
  hipStream_t s = ctx->stream;
  if (w) {
    if ((e = hipMemcpyAsync(d_items, row_roots, (size_t)w * kNode, hipMemcpyHostToDevice, s)) != hipSuccess ||
        (e = hipMemcpyAsync(d_items + (size_t)w * kNode, col_roots, (size_t)w * kNode, hipMemcpyHostToDevice, s)) !=
            hipSuccess)
      return hip_fail(ctx, e, "H2D");
  }
  if ((e = launch_merkle_root(d_items, 2 * w, kNode, d_o, d_w, s)) != hipSuccess) return hip_fail(ctx, e, "merkle");
  if ((e = hipMemcpyAsync(out, d_o, 32, hipMemcpyDeviceToHost, s)) != hipSuccess) return hip_fail(ctx, e, "D2H");
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return hip_fail(ctx, e, "sync");
  return CEL_OK;
}

cel_status cel_merkle_hash_slices(cel_ctx* ctx, const uint8_t* data, const uint64_t* offsets, uint32_t n,
                                  uint8_t* out) {
  if (!ctx) return CEL_EINVAL;
  std::lock_guard<std::mutex> lock(ctx->mu);
  if (!out || !offsets || (n && !data && offsets[n] > offsets[0])) return fail(ctx, CEL_EINVAL, "nil argument");
  for (uint32_t i = 0; i < n; i++)
    if (offsets[i + 1] < offsets[i]) return fail(ctx, CEL_EINVAL, "slice offsets must be non-decreasing");
  if (n > (1u << 20)) return fail(ctx, CEL_ETOOBIG, "too many slices for the device merkle kernel");
  const uint64_t bytes = n ? offsets[n] - offsets[0] : 0;
  DeviceGuard g(ctx->device);
  hipError_t e = hipSuccess;
  const size_t ob = ((size_t)(n + 1) * 8 + 255) / 256 * 256;
  uint8_t* d_in = static_cast<uint8_t*>(scratch(ctx, S_IN, ob + (bytes ? bytes : 1), &e));
  void* d_w = scratch(ctx, S_WORK, slices_workspace_size(n), &e);
  uint8_t* d_o = static_cast<uint8_t*>(scratch(ctx, S_ROOTS, 256, &e));
  if (!d_in || !d_w || !d_o) return fail(ctx, CEL_ENOMEM, "device allocation failed");
  std::vector<uint64_t> off(n + 1);
  for (uint32_t i = 0; i <= n; i++) off[i] = offsets[i] - offsets[0];
  hipStream_t s = ctx->stream;
  if ((e = hipMemcpyAsync(d_in, off.data(), (size_t)(n + 1) * 8, hipMemcpyHostToDevice, s)) != hipSuccess ||
      (bytes && (e = hipMemcpyAsync(d_in + ob, data + offsets[0], bytes, hipMemcpyHostToDevice, s)) != hipSuccess))
    return hip_fail(ctx, e, "H2D");
  if ((e = launch_hash_slices(d_in + ob, reinterpret_cast<const uint64_t*>(d_in), n, d_o, d_w, s)) != hipSuccess)
    return hip_fail(ctx, e, "merkle");
  if ((e = hipMemcpyAsync(out, d_o, 32, hipMemcpyDeviceToHost, s)) != hipSuccess) return hip_fail(ctx, e, "D2H");
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return hip_fail(ctx, e, "sync");
  return CEL_OK;
}

// ------------------------------------------------------------- exported trees
//
// Inner nodes for proofs: pkg/proof/proof.go:151-201 rebuilds
// each row's NMT on the CPU to call ProveRange; here the device hashes the trees and
// hands every node back, and the host proof builders (proof.cpp) only pick nodes.

// Every node of the NMTs of `idx.size()` axes whose cells sit densely in `cells` (axis a
// = cells [a * 2k, (a + 1) * 2k)), per axis level-major into nodes_out. ctx->mu held.
static cel_status dense_axes_trees(cel_ctx* ctx, const std::vector<uint8_t>& cells, const std::vector<int32_t>& idx,
                                   uint32_t k, uint8_t* nodes_out) {
  const uint32_t W = 2 * k, count = (uint32_t)idx.size();
  DeviceGuard g(ctx->device);
  hipError_t e = hipSuccess;
  const size_t nodes = axes_trees_nodes(k, count);
  uint8_t* d_c = static_cast<uint8_t*>(scratch(ctx, S_IN, cells.size(), &e));
  uint32_t* d_n = static_cast<uint32_t*>(scratch(ctx, S_WORK, nodes * kNodeWords * 4, &e));
  int32_t* d_idx = static_cast<int32_t*>(scratch(ctx, S_AUX, (size_t)count * 4, &e));
  if (!d_c || !d_n || !d_idx) return fail(ctx, CEL_ENOMEM, "device allocation failed");
  hipStream_t s = ctx->stream;
  if ((e = hipMemcpyAsync(d_c, cells.data(), cells.size(), hipMemcpyHostToDevice, s)) != hipSuccess ||
      (e = hipMemcpyAsync(d_idx, idx.data(), (size_t)count * 4, hipMemcpyHostToDevice, s)) != hipSuccess)
    return hip_fail(ctx, e, "H2D");
  if ((e = launch_axes_trees(d_c, k, d_idx, count, d_n, s)) != hipSuccess) return hip_fail(ctx, e, "axis trees");
  std::vector<uint32_t> recs(nodes * kNodeWords);
  if ((e = hipMemcpyAsync(recs.data(), d_n, recs.size() * 4, hipMemcpyDeviceToHost, s)) != hipSuccess)
    return hip_fail(ctx, e, "D2H");
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return hip_fail(ctx, e, "sync");
  // level-major across axes on the device -> per axis, level-major, 90-byte nodes
  size_t level_off = 0;
  uint32_t in_axis_off = 0;
  for (uint32_t n = W; n >= 1; n /= 2) {
    for (uint32_t a = 0; a < count; a++)
      for (uint32_t j = 0; j < n; j++)
        std::memcpy(nodes_out + ((size_t)a * (2 * W - 1) + in_axis_off + j) * kNode,
                    &recs[(level_off + (size_t)a * n + j) * kNodeWords], kNode);
    level_off += (size_t)count * n;
    in_axis_off += n;
    if (n == 1) break;
  }
  return CEL_OK;
}

cel_status cel_axis_trees(cel_ctx* ctx, const uint8_t* eds, uint32_t k, uint32_t share_size, uint32_t axis,
                          uint32_t first, uint32_t count, uint8_t* nodes_out) {
  if (!ctx) return CEL_EINVAL;
  std::lock_guard<std::mutex> lock(ctx->mu);
  if (!eds || !nodes_out || !count) return fail(ctx, CEL_EINVAL, "nil argument");
  cel_status st = validate_square(ctx, k, share_size);
  if (st) return st;
  const uint32_t W = 2 * k;
  if (axis > 1 || first >= W || count > W - first) return fail(ctx, CEL_EINVAL, "axis range outside the square");
  // gather the axes densely on the host: rows are contiguous, columns strided
  std::vector<uint8_t> cells((size_t)count * W * kShare);
  std::vector<int32_t> idx(count);
  for (uint32_t a = 0; a < count; a++) {
    idx[a] = (int32_t)(first + a);
    for (uint32_t j = 0; j < W; j++) {
      const size_t cell = axis == 0 ? (size_t)(first + a) * W + j : (size_t)j * W + first + a;
      std::memcpy(&cells[((size_t)a * W + j) * kShare], eds + cell * kShare, kShare);
    }
  }
  return dense_axes_trees(ctx, cells, idx, k, nodes_out);
}

cel_status cel_axis_tree(cel_ctx* ctx, const uint8_t* cells, uint32_t k, uint32_t axis_index, uint32_t share_size,
                         uint8_t* nodes_out) {
  if (!ctx) return CEL_EINVAL;
  std::lock_guard<std::mutex> lock(ctx->mu);
  if (!cells || !nodes_out) return fail(ctx, CEL_EINVAL, "nil argument");
  cel_status st = validate_square(ctx, k, share_size);
  if (st) return st;
  if (axis_index >= 2 * k)  // nmt_wrapper.go:94-96 (no uint32 wrap at 0xFFFFFFFF)
    return fail(ctx, CEL_EPUSHPAST, "pushed past predetermined square size: boundary at " + std::to_string(2 * k) +
                                        " index at " + std::to_string(axis_index) + " 0");
  std::vector<uint8_t> dense(cells, cells + (size_t)2 * k * kShare);
  return dense_axes_trees(ctx, dense, std::vector<int32_t>{(int32_t)axis_index}, k, nodes_out);
}

cel_status cel_dah_tree(cel_ctx* ctx, const uint8_t* row_roots, const uint8_t* col_roots, uint32_t w,
                        uint8_t* nodes_out) {
  if (!ctx) return CEL_EINVAL;
  std::lock_guard<std::mutex> lock(ctx->mu);
  if (!row_roots || !col_roots || !nodes_out || !w) return fail(ctx, CEL_EINVAL, "nil argument");
  const uint32_t n = 2 * w;
  if (n & (n - 1)) return fail(ctx, CEL_ENOTPOW2, "DAH tree export needs a power-of-two root count");
  DeviceGuard g(ctx->device);
  hipError_t e = hipSuccess;
  uint8_t* d_items = static_cast<uint8_t*>(scratch(ctx, S_IN, (size_t)n * kNode, &e));
  void* d_w = scratch(ctx, S_WORK, merkle_workspace_size(n), &e);
  uint32_t* d_l = static_cast<uint32_t*>(scratch(ctx, S_ROOTS, (size_t)(2 * n - 1) * 32, &e));
  if (!d_items || !d_w || !d_l) return fail(ctx, CEL_ENOMEM, "device allocation failed");
  hipStream_t s = ctx->stream;
  if ((e = hipMemcpyAsync(d_items, row_roots, (size_t)w * kNode, hipMemcpyHostToDevice, s)) != hipSuccess ||
      (e = hipMemcpyAsync(d_items + (size_t)w * kNode, col_roots, (size_t)w * kNode, hipMemcpyHostToDevice, s)) !=
          hipSuccess)
    return hip_fail(ctx, e, "H2D");
  if ((e = launch_rfc_tree(d_items, n, d_l, d_w, s)) != hipSuccess) return hip_fail(ctx, e, "rfc tree");
  std::vector<uint32_t> words((size_t)(2 * n - 1) * 8);
  if ((e = hipMemcpyAsync(words.data(), d_l, words.size() * 4, hipMemcpyDeviceToHost, s)) != hipSuccess)
    return hip_fail(ctx, e, "D2H");
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return hip_fail(ctx, e, "sync");
  for (size_t i = 0; i < words.size(); i++) {  // big-endian words -> digest bytes
    nodes_out[4 * i] = (uint8_t)(words[i] >> 24);
    nodes_out[4 * i + 1] = (uint8_t)(words[i] >> 16);
    nodes_out[4 * i + 2] = (uint8_t)(words[i] >> 8);
    nodes_out[4 * i + 3] = (uint8_t)words[i];
  }
  return CEL_OK;
}

cel_status cel_get_commitment(cel_ctx* ctx, const uint8_t* eds, uint32_t k, uint32_t share_size, uint32_t start,
                              uint32_t blob_share_len, uint32_t subtree_root_threshold, uint8_t* commitment) {
  if (!ctx) return CEL_EINVAL;
  std::lock_guard<std::mutex> lock(ctx->mu);
  if (!eds || !commitment || !blob_share_len || !subtree_root_threshold) return fail(ctx, CEL_EINVAL, "nil argument");
  cel_status st = validate_square(ctx, k, share_size);
  if (st) return st;
  if ((uint64_t)start + blob_share_len > (uint64_t)k * k)  // get_commit.go:14-16
    return fail(ctx, CEL_ETOOBIG, "cannot get commitment for blob that doesn't fit in square");
  uint32_t n = 0;
  if ((st = cel_commitment_paths(k, start, blob_share_len, subtree_root_threshold, nullptr, nullptr, nullptr, 0, &n)))
    return fail(ctx, st, "commitment paths");
  std::vector<uint32_t> rows(n), depths(n), pos(n);
  cel_commitment_paths(k, start, blob_share_len, subtree_root_threshold, rows.data(), depths.data(), pos.data(), n,
                       &n);
  if (n > 2048) return fail(ctx, CEL_ETOOBIG, "too many subtree roots for the device merkle kernel");
  const uint32_t r0 = rows.front(), nrows = rows.back() - r0 + 1, W = 2 * k;
  DeviceGuard g(ctx->device);
  hipError_t e = hipSuccess;
  const size_t cells_b = (size_t)nrows * W * kShare;
  uint8_t* d_c = static_cast<uint8_t*>(scratch(ctx, S_IN, cells_b, &e));
  uint32_t* d_n = static_cast<uint32_t*>(scratch(ctx, S_WORK, axes_trees_nodes(k, nrows) * kNodeWords * 4, &e));
  int32_t* d_idx = static_cast<int32_t*>(scratch(ctx, S_AUX, (size_t)(nrows + n) * 4, &e));
  uint8_t* d_items = static_cast<uint8_t*>(scratch(ctx, S_ROOTS, (size_t)n * kNode + 64, &e));
  void* d_mw = scratch(ctx, S_MASK, merkle_workspace_size(n), &e);
  if (!d_c || !d_n || !d_idx || !d_items || !d_mw) return fail(ctx, CEL_ENOMEM, "device allocation failed");
  uint8_t* d_out = d_items + (size_t)n * kNode + (64 - ((size_t)n * kNode) % 32) % 32;
  hipStream_t s = ctx->stream;
  if ((e = hipMemcpyAsync(d_c, eds + (size_t)r0 * W * kShare, cells_b, hipMemcpyHostToDevice, s)) != hipSuccess)
    return hip_fail(ctx, e, "H2D");
  if ((e = launch_commitment(d_c, k, r0, nrows, rows.data(), depths.data(), pos.data(), n, d_idx, d_n, d_items, d_mw,
                             d_out, s)) != hipSuccess)
    return hip_fail(ctx, e, "commitment");
  if ((e = hipMemcpyAsync(commitment, d_out, 32, hipMemcpyDeviceToHost, s)) != hipSuccess) return hip_fail(ctx, e, "D2H");
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return hip_fail(ctx, e, "sync");
  return CEL_OK;
}

}  // extern "C"
