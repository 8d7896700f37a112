// Blob share commitment paths, host-only:
//
//   cel_commitment_paths          <- pkg/inclusion/paths.go:16-47 calculateCommitmentPaths
//                                    (+ go-square v1.1.0 inclusion.NextShareIndex / SubTreeWidth)
//   cel_subtree_root_coordinates  <- pkg/inclusion/paths.go:95-173
//
// The device half of cel_get_commitment (the row trees and the RFC-6962 root of the
// selected subtree roots) is in inclusion.cpp.
#include <cmath>
#include <cstdint>
#include <vector>

#include "../../include/celestia_eds.h"

namespace cel {
namespace incl {
namespace {

uint32_t pow2ceil(uint64_t n) {
  uint32_t r = 1;
  while (r < n) r <<= 1;
  return r;
}
uint32_t log2u(uint32_t n) {
  uint32_t l = 0;
  while ((1u << l) < n) l++;
  return l;
}
// go-square inclusion.SubTreeWidth: min(RoundUpPow2(ceil(n / threshold)), BlobMinSquareSize(n))
uint32_t subtree_width(uint32_t shares, uint32_t threshold) {
  const uint32_t s = pow2ceil((shares + threshold - 1) / threshold);
  const uint32_t m = pow2ceil((uint64_t)std::ceil(std::sqrt((double)shares)));
  return s < m ? s : m;
}

struct Coord {
  uint32_t depth, position;
};

// calculateSubTreeRootCoordinates: the leaves [start, end) of a tree of depth max_depth
// covered left to right by the largest aligned subtrees whose depth is >= min_depth
// (at most 2^(max_depth - min_depth) leaves each).
void cover(uint32_t max_depth, uint32_t min_depth, uint32_t start, uint32_t end, std::vector<Coord>& out) {
  const uint32_t cap_log = max_depth - min_depth;
  for (uint32_t c = start; c < end;) {
    uint32_t j = 0;
    while (j < cap_log && c % (2u << j) == 0 && c + (2u << j) <= end) j++;
    out.push_back(Coord{max_depth - j, c >> j});
    c += 1u << j;
  }
}

struct Path {
  uint32_t row, depth, position;  // ODS-half coordinates (the walk skips the leading WalkLeft)
};

std::vector<Path> commitment_paths(uint32_t square, uint32_t start, uint32_t len, uint32_t threshold) {
  const uint32_t w = subtree_width(len, threshold);
  start = (start + w - 1) / w * w;  // inclusion.NextShareIndex
  const uint32_t r0 = start / square, r1 = (start + len - 1) / square;
  const uint32_t max_depth = log2u(square), min_depth = max_depth - log2u(w);
  std::vector<Path> out;
  for (uint32_t r = r0; r <= r1; r++) {
    const uint32_t s = r == r0 ? start % square : 0;
    const uint32_t e = r == r1 ? start + len - r1 * square : square;
    std::vector<Coord> cs;
    cover(max_depth, min_depth, s, e, cs);
    for (const Coord& c : cs) out.push_back(Path{r, c.depth, c.position});
  }
  return out;
}

bool pow2(uint32_t n) { return n && !(n & (n - 1)); }

}  // namespace
}  // namespace incl
}  // namespace cel

extern "C" {

cel_status cel_commitment_paths(uint32_t square_size, uint32_t start, uint32_t blob_share_len,
                                uint32_t subtree_root_threshold, uint32_t* rows, uint32_t* depths,
                                uint32_t* positions, uint32_t cap, uint32_t* n_out) {
  using namespace cel::incl;
  if (!n_out || !pow2(square_size) || !blob_share_len || !subtree_root_threshold) return CEL_EINVAL;
  if ((uint64_t)start + blob_share_len > (uint64_t)square_size * square_size) return CEL_ETOOBIG;
  const std::vector<Path> ps = commitment_paths(square_size, start, blob_share_len, subtree_root_threshold);
  *n_out = (uint32_t)ps.size();
  if (rows && depths && positions)
    for (size_t i = 0; i < ps.size() && i < cap; i++) {
      rows[i] = ps[i].row;
      depths[i] = ps[i].depth;
      positions[i] = ps[i].position;
    }
  return CEL_OK;
}

cel_status cel_subtree_root_coordinates(uint32_t max_depth, uint32_t min_depth, uint32_t start, uint32_t end,
                                        uint32_t* depths, uint32_t* positions, uint32_t cap, uint32_t* n_out) {
  using namespace cel::incl;
  if (!n_out || min_depth > max_depth || max_depth > 31 || start >= end || end > (1u << max_depth)) return CEL_EINVAL;
  std::vector<Coord> cs;
  cover(max_depth, min_depth, start, end, cs);
  *n_out = (uint32_t)cs.size();
  if (depths && positions)
    for (size_t i = 0; i < cs.size() && i < cap; i++) {
      depths[i] = cs[i].depth;
      positions[i] = cs[i].position;
    }
  return CEL_OK;
}

}  // extern "C"
