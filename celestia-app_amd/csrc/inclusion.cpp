// Blob share commitments from the EDS, device half (the paths
// are computed on the host, inclusion_paths.cpp).
//
//   cel_get_commitment   <- pkg/inclusion/get_commit.go:12-30 GetCommitment over the
//                           EDSSubTreeRootCacher of nmt_caching.go:96-124
//
// The reference caches, per row tree, every (parent -> children) pair seen by an nmt
// NodeVisitor while rsmt2d computes the roots, then walks from the row root. Here the
// device hashes the row trees (launch_axes_trees, every node kept) and a walk is an
// index: the subtree root at depth d, position p of a row's ODS half is node
// (level log2(2k) - 1 - d, index p) of that row's tree. The commitment is the RFC-6962
// root of the selected subtree roots (launch_merkle_root, on the device).
#include <hip/hip_runtime.h>

#include <vector>

#include "cel_internal.hpp"

namespace cel {

static uint32_t ilog2(uint32_t n) {
  uint32_t l = 0;
  while ((1u << l) < n) l++;
  return l;
}

// Device half of cel_get_commitment (api.cpp): trees of rows [r0, r1], node selection,
// RFC-6962 root. cells: the gathered rows [r1 - r0 + 1][2k][512] on the device.
hipError_t launch_commitment(const uint8_t* d_cells, uint32_t k, uint32_t r0, uint32_t nrows, const uint32_t* rows,
                             const uint32_t* depths, const uint32_t* positions, uint32_t npaths, int32_t* d_idx,
                             uint32_t* d_nodes, uint8_t* d_items, void* d_merkle_work, uint8_t* d_out,
                             hipStream_t s) {
  // host tables: the gathered rows' indices, then the record of every selected node
  // (level-major across rows: level L holds nrows * (2k >> L) records)
  const uint32_t W = 2 * k, depth_full = ilog2(W);
  std::vector<int32_t> tab(nrows + npaths);
  for (uint32_t i = 0; i < nrows; i++) tab[i] = (int32_t)(r0 + i);
  for (uint32_t p = 0; p < npaths; p++) {
    const uint32_t level = depth_full - 1 - depths[p];  // -1: the walk starts with WalkLeft (ODS half)
    size_t off = 0;
    for (uint32_t l = 0; l < level; l++) off += (size_t)nrows * (W >> l);
    tab[nrows + p] = (int32_t)(off + (size_t)(rows[p] - r0) * (W >> level) + positions[p]);
  }
  // synchronous upload: the table is pageable host memory local to this call
  hipError_t e = hipMemcpyAsync(d_idx, tab.data(), tab.size() * 4, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return e;
  if ((e = launch_axes_trees(d_cells, k, d_idx, nrows, d_nodes, s)) != hipSuccess) return e;
  if ((e = launch_gather_nodes(d_nodes, d_idx + nrows, npaths, d_items, s)) != hipSuccess) return e;
  return launch_merkle_root(d_items, npaths, kNode, d_out, d_merkle_work, s);
}

}  // namespace cel
