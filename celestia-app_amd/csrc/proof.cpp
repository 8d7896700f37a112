// Proof builders over exported trees. Host code: the device
// hashed every node (cel_axis_trees, cel_dah_tree); building a proof only selects nodes.
//
//   cel_nmt_prove_range  <- nmt v0.22.0 NamespacedMerkleTree.ProveRange / buildRangeProof
//                           [dep], as called by pkg/proof/proof.go:190 (tree.ProveRange)
//   cel_merkle_aunts     <- go-square merkle.ProofsFromByteSlices [dep] aunts, as used by
//                           pkg/proof/proof.go:98-111 for the row-root-to-data-root proofs
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/celestia_eds.h"

namespace {

constexpr uint32_t kNode = CEL_NMT_NODE_SIZE;

bool pow2(uint32_t n) { return n && !(n & (n - 1)); }

// Node (level, index) of a perfect tree stored level-major from the leaves up:
// level 0 = nleaves nodes, level 1 = nleaves/2, ...
size_t node_offset(uint32_t nleaves, uint32_t level, uint32_t index) {
  size_t off = 0;
  for (uint32_t l = 0; l < level; l++) off += nleaves >> l;
  return off + index;
}

// buildRangeProof: left-to-right, the roots of the maximal subtrees of [0, n) that do
// not overlap [ps, pe) (a leaf counts as a subtree of size 1).
void collect(uint32_t nleaves, uint32_t start, uint32_t end, uint32_t ps, uint32_t pe, std::vector<size_t>& out) {
  if (end <= ps || start >= pe) {
    uint32_t level = 0;
    while ((1u << level) < end - start) level++;
    out.push_back(node_offset(nleaves, level, start >> level));
    return;
  }
  if (end - start == 1) return;  // a leaf inside the range
  const uint32_t half = (end - start) / 2;
  collect(nleaves, start, start + half, ps, pe, out);
  collect(nleaves, start + half, end, ps, pe, out);
}

}  // namespace

extern "C" {

cel_status cel_nmt_prove_range(const uint8_t* tree_nodes, uint32_t nleaves, uint32_t start, uint32_t end,
                               uint8_t* nodes_out, uint32_t* nnodes) {
  if (!tree_nodes || !nnodes || !pow2(nleaves) || start >= end || end > nleaves) return CEL_EINVAL;
  std::vector<size_t> sel;
  collect(nleaves, 0, nleaves, start, end, sel);
  *nnodes = (uint32_t)sel.size();
  if (nodes_out)
    for (size_t i = 0; i < sel.size(); i++) std::memcpy(nodes_out + i * kNode, tree_nodes + sel[i] * kNode, kNode);
  return CEL_OK;
}

cel_status cel_merkle_aunts(const uint8_t* tree, uint32_t n, uint32_t index, uint8_t* aunts_out, uint32_t* naunts) {
  if (!tree || !naunts || !pow2(n) || index >= n) return CEL_EINVAL;
  // perfect tree (n = 2^m): the aunt at height h is the sibling of the ancestor of
  // `index` at height h; Aunts are listed from the leaf's sibling up (merkle
  // computeHashFromAunts consumes the last one at the root).
  uint32_t h = 0;
  for (uint32_t w = n, i = index; w > 1; w /= 2, i /= 2, h++)
    if (aunts_out) std::memcpy(aunts_out + (size_t)h * 32, tree + node_offset(n, h, i ^ 1u) * 32, 32);
  *naunts = h;
  return CEL_OK;
}

}  // extern "C"
