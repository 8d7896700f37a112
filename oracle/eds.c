/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * NMT, erasured-NMT wrapper, RFC-6962 DAH, 2D extension and crossword repair.
 *
 *  - NMT hasher: nmt v0.22.0 (go.mod:12) [dep]; formulas follow the text copy in
 *    test/util/malicious/hasher.go:186-310 (HashLeaf :196-223, HashNode :271-299,
 *    computeNsRange :302-310) with the honest push-order check restored.
 *  - Wrapper: pkg/wrapper/nmt_wrapper.go:93-114 (Push: Q0 cells keep their own
 *    namespace, every other cell gets the parity namespace 0xFF*29),
 *    :138-140 (isQuadrantZero), :55-63 (NamespaceIDSize 29, IgnoreMaxNamespace).
 *  - DAH: pkg/da/data_availability_header.go:92-108 -> go-square/merkle
 *    HashFromByteSlices (RFC-6962; specs/src/specs/data_structures.md:173-211).
 *  - Extension order: rsmt2d v0.14.0 erasureExtendSquare [dep] as described in
 *    specs/src/specs/data_structures.md:295-305 (Q0->Q1 rows, Q0->Q2 cols, Q2->Q3 rows).
 *  - Repair: rsmt2d ExtendedDataSquare.Repair [dep] crossword loop.
 */
#include <stdlib.h>
#include <string.h>
#include "oracle.h"
#include "oracle_internal.h"

static const uint8_t kParityNs[ORC_NS] = {
    0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF,
    0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF};

/* ------------------------------------------------------------------- NMT */

/* HashLeaf: ns || ns || SHA256(0x00 || ns || data) where ndata = ns || data. */
static void nmt_leaf(const uint8_t* ns, const uint8_t* data, size_t len, uint8_t out[ORC_NODE]) {
  static const uint8_t zero = 0x00;
  uint8_t d[32];
  sha256_3(&zero, 1, ns, ORC_NS, data, len, d);
  memcpy(out, ns, ORC_NS);
  memcpy(out + ORC_NS, ns, ORC_NS);
  memcpy(out + 2 * ORC_NS, d, 32);
}

/* HashNode with IgnoreMaxNamespace: min = L.min; max = (R.min == MAX) ? L.max : R.max. */
static void nmt_node(const uint8_t* l, const uint8_t* r, uint8_t out[ORC_NODE]) {
  static const uint8_t one = 0x01;
  uint8_t d[32];
  sha256_3(&one, 1, l, ORC_NODE, r, ORC_NODE, d);
  uint8_t res[ORC_NODE];
  memcpy(res, l, ORC_NS);
  if (memcmp(r, kParityNs, ORC_NS) == 0) memcpy(res + ORC_NS, l + ORC_NS, ORC_NS);
  else memcpy(res + ORC_NS, r + ORC_NS, ORC_NS);
  memcpy(res + 2 * ORC_NS, d, 32);
  memcpy(out, res, ORC_NODE);
}

/* Root of a tree over n leaf nodes (n may be any size; nmt splits at the largest
 * power of two < n, like RFC-6962). Empty tree: 0*58 || SHA256(""). */
static void nmt_reduce(uint8_t* nodes, uint32_t n, uint8_t out[ORC_NODE]) {
  if (n == 0) {
    memset(out, 0, 2 * ORC_NS);
    sha256_3(NULL, 0, NULL, 0, NULL, 0, out + 2 * ORC_NS);
    return;
  }
  if (n == 1) { memcpy(out, nodes, ORC_NODE); return; }
  uint32_t k = 1;
  while (k * 2 < n) k *= 2;
  uint8_t l[ORC_NODE], r[ORC_NODE];
  nmt_reduce(nodes, k, l);
  nmt_reduce(nodes + (size_t)k * ORC_NODE, n - k, r);
  nmt_node(l, r, out);
}

int orc_nmt_root(const uint8_t* leaves, uint32_t n, size_t len, uint8_t out[ORC_NODE],
                 int check_order) {
  uint8_t* nodes = (uint8_t*)malloc((size_t)(n ? n : 1) * ORC_NODE);
  for (uint32_t i = 0; i < n; i++) {
    const uint8_t* lf = leaves + (size_t)i * len;
    if (len < ORC_NS) { free(nodes); return ORC_EINVAL; }
    if (check_order && i > 0 && memcmp(lf, leaves + (size_t)(i - 1) * len, ORC_NS) < 0) {
      free(nodes);
      return ORC_EORDER;
    }
    nmt_leaf(lf, lf + ORC_NS, len - ORC_NS, nodes + (size_t)i * ORC_NODE);
  }
  nmt_reduce(nodes, n, out);
  free(nodes);
  return ORC_OK;
}

/* Erasured NMT over the 2k cells of axis `axis` (wrapper.Push semantics). */
int orc_axis_root(const uint8_t* cells, size_t cell_stride, uint32_t k, uint32_t axis,
                  size_t share, uint8_t out[ORC_NODE], int check_order) {
  uint32_t w = 2 * k;
  uint8_t* nodes = (uint8_t*)malloc((size_t)w * ORC_NODE);
  const uint8_t* prev_ns = NULL;
  for (uint32_t i = 0; i < w; i++) {
    const uint8_t* c = cells + (size_t)i * cell_stride;
    const uint8_t* ns = (i < k && axis < k) ? c : kParityNs;
    if (check_order && prev_ns && memcmp(ns, prev_ns, ORC_NS) < 0) {
      free(nodes);
      return ORC_EORDER;
    }
    prev_ns = ns;
    nmt_leaf(ns, c, share, nodes + (size_t)i * ORC_NODE);
  }
  nmt_reduce(nodes, w, out);
  free(nodes);
  return ORC_OK;
}

/* ------------------------------------------------------------ RFC-6962 */

static void merkle_rec(const uint8_t* items, uint32_t n, size_t il, uint8_t out[32]) {
  static const uint8_t zero = 0x00, one = 0x01;
  if (n == 0) { sha256_3(NULL, 0, NULL, 0, NULL, 0, out); return; }
  if (n == 1) { sha256_3(&zero, 1, items, il, NULL, 0, out); return; }
  uint32_t k = 1;
  while (k * 2 < n) k *= 2;
  uint8_t lr[64];
  merkle_rec(items, k, il, lr);
  merkle_rec(items + (size_t)k * il, n - k, il, lr + 32);
  sha256_3(&one, 1, lr, 64, NULL, 0, out);
}

void orc_merkle_root(const uint8_t* items, uint32_t n, size_t item_len, uint8_t out[32]) {
  merkle_rec(items, n, item_len, out);
}

void orc_dah_hash(const uint8_t* row_roots, const uint8_t* col_roots, uint32_t w, uint8_t out[32]) {
  uint8_t* all = (uint8_t*)malloc((size_t)((2 * w) ? (2 * w) : 1) * ORC_NODE);
  memcpy(all, row_roots, (size_t)w * ORC_NODE);
  memcpy(all + (size_t)w * ORC_NODE, col_roots, (size_t)w * ORC_NODE);
  merkle_rec(all, 2 * w, ORC_NODE, out);
  free(all);
}

/* ----------------------------------------------------------- extension */

static int encode_axis(uint32_t k, size_t share, const uint8_t* src, size_t sstride, uint8_t* dst,
                       size_t dstride) {
  uint8_t* d = (uint8_t*)malloc((size_t)k * share);
  uint8_t* p = (uint8_t*)malloc((size_t)k * share);
  for (uint32_t i = 0; i < k; i++) memcpy(d + (size_t)i * share, src + (size_t)i * sstride, share);
  int rc = orc_rs_encode(k, share, d, p);
  if (rc == ORC_OK)
    for (uint32_t i = 0; i < k; i++) memcpy(dst + (size_t)i * dstride, p + (size_t)i * share, share);
  free(d);
  free(p);
  return rc;
}

int orc_extend(const uint8_t* ods, uint32_t k, size_t share, uint8_t* eds) {
  orc_init();
  if (!k || (k & (k - 1))) return ORC_ENOTPOW2;
  if (share % 64) return ORC_ECHUNK;
  uint32_t w = 2 * k;
  size_t row = (size_t)w * share;
  for (uint32_t r = 0; r < k; r++) memcpy(eds + r * row, ods + (size_t)r * k * share, (size_t)k * share);
  int rc = ORC_OK;
  /* Q0 -> Q1 (rows) and Q0 -> Q2 (columns) */
#pragma omp parallel for schedule(dynamic, 1) reduction(| : rc)
  for (int i = 0; i < (int)(2 * k); i++) {
    if (i < (int)k)
      rc |= encode_axis(k, share, eds + (size_t)i * row, share, eds + (size_t)i * row + (size_t)k * share,
                        share);
    else {
      uint32_t c = (uint32_t)i - k;
      rc |= encode_axis(k, share, eds + (size_t)c * share, row, eds + (size_t)k * row + (size_t)c * share,
                        row);
    }
  }
  /* Q2 -> Q3 (rows) */
#pragma omp parallel for schedule(dynamic, 1) reduction(| : rc)
  for (int r = (int)k; r < (int)w; r++)
    rc |= encode_axis(k, share, eds + (size_t)r * row, share, eds + (size_t)r * row + (size_t)k * share,
                      share);
  return rc;
}

int orc_roots(const uint8_t* eds, uint32_t k, size_t share, uint8_t* row_roots, uint8_t* col_roots,
              int check_order, int32_t* bad_axis) {
  orc_init();
  uint32_t w = 2 * k;
  size_t row = (size_t)w * share;
  int first_bad = -1;
#pragma omp parallel for schedule(dynamic, 1)
  for (int i = 0; i < (int)(2 * w); i++) {
    int rc;
    if (i < (int)w)
      rc = orc_axis_root(eds + (size_t)i * row, share, k, (uint32_t)i, share,
                         row_roots + (size_t)i * ORC_NODE, check_order);
    else
      rc = orc_axis_root(eds + (size_t)(i - w) * share, row, k, (uint32_t)(i - w), share,
                         col_roots + (size_t)(i - w) * ORC_NODE, check_order);
    if (rc != ORC_OK) {
#pragma omp critical(orc_bad)
      if (first_bad < 0 || i < first_bad) first_bad = i;
    }
  }
  if (first_bad >= 0) {
    if (bad_axis) *bad_axis = first_bad;
    return ORC_EORDER;
  }
  return ORC_OK;
}

int orc_extend_and_commit(const uint8_t* ods, uint32_t k, size_t share, uint8_t* eds,
                          uint8_t* row_roots, uint8_t* col_roots, uint8_t dah[32]) {
  uint8_t* e = eds ? eds : (uint8_t*)malloc((size_t)4 * k * k * share);
  int rc = orc_extend(ods, k, share, e);
  if (rc == ORC_OK) rc = orc_roots(e, k, share, row_roots, col_roots, 1, NULL);
  if (rc == ORC_OK) orc_dah_hash(row_roots, col_roots, 2 * k, dah);
  if (!eds) free(e);
  return rc;
}

/* -------------------------------------------------------------- repair */

/* Decode one axis (2k cells gathered from the EDS) if it is incomplete but has >= k
 * cells. Returns 1 if solved, 0 if nothing to do / not enough, <0 on byzantine. */
static int repair_axis(uint8_t* eds, uint8_t* present, uint32_t k, size_t share, int is_col,
                       uint32_t idx, const uint8_t* root) {
  uint32_t w = 2 * k;
  size_t row = (size_t)w * share;
  size_t base = is_col ? (size_t)idx * share : (size_t)idx * row;
  size_t stride = is_col ? row : share;
  size_t pbase = is_col ? idx : (size_t)idx * w;
  size_t pstride = is_col ? w : 1;
  uint32_t have = 0;
  for (uint32_t i = 0; i < w; i++) have += present[pbase + i * pstride] ? 1 : 0;
  if (have == w || have < k) return 0;
  uint8_t* cells = (uint8_t*)malloc((size_t)w * share);
  uint8_t* pm = (uint8_t*)malloc(w);
  for (uint32_t i = 0; i < w; i++) {
    pm[i] = present[pbase + i * pstride];
    if (pm[i]) memcpy(cells + (size_t)i * share, eds + base + i * stride, share);
    else memset(cells + (size_t)i * share, 0, share);
  }
  int rc = orc_rs_decode(k, share, cells, pm);
  if (rc != ORC_OK) { free(cells); free(pm); return -1; }
  /* Re-encode check: parity recomputed from the data half must match every known cell. */
  uint8_t* par = (uint8_t*)malloc((size_t)k * share);
  orc_rs_encode(k, share, cells, par);
  int bad = memcmp(par, cells + (size_t)k * share, (size_t)k * share) != 0;
  free(par);
  /* Root check against the committed root. */
  if (!bad) {
    uint8_t r[ORC_NODE];
    orc_axis_root(cells, share, k, idx, share, r, 0);
    bad = memcmp(r, root, ORC_NODE) != 0;
  }
  if (bad) { free(cells); free(pm); return -1; }
  for (uint32_t i = 0; i < w; i++)
    if (!pm[i]) {
      memcpy(eds + base + i * stride, cells + (size_t)i * share, share);
      present[pbase + i * pstride] = 1;
    }
  free(cells);
  free(pm);
  return 1;
}

int orc_repair(uint8_t* eds, uint8_t* present, uint32_t k, size_t share, const uint8_t* row_roots,
               const uint8_t* col_roots, int32_t* bad_axis, int32_t* bad_index) {
  orc_init();
  uint32_t w = 2 * k;
  size_t row = (size_t)w * share;
  /* rsmt2d prerepairSanityCheck: axes complete before the repair must match their
   * roots (rows, then columns, in index order). */
  for (int is_col = 0; is_col < 2; is_col++)
    for (uint32_t i = 0; i < w; i++) {
      uint32_t have = 0;
      for (uint32_t j = 0; j < w; j++) have += present[is_col ? (size_t)j * w + i : (size_t)i * w + j] ? 1 : 0;
      if (have != w) continue;
      uint8_t r[ORC_NODE];
      if (is_col) orc_axis_root(eds + (size_t)i * share, row, k, i, share, r, 0);
      else orc_axis_root(eds + (size_t)i * row, share, k, i, share, r, 0);
      if (memcmp(r, (is_col ? col_roots : row_roots) + (size_t)i * ORC_NODE, ORC_NODE) != 0) {
        if (bad_axis) *bad_axis = is_col;
        if (bad_index) *bad_index = (int32_t)i;
        return ORC_EBYZANTINE;
      }
    }
  /* crossword: all rows, then all columns, until solved or stuck */
  for (;;) {
    int progress = 0;
    for (int is_col = 0; is_col < 2; is_col++)
      for (uint32_t i = 0; i < w; i++) {
        int rc = repair_axis(eds, present, k, share, is_col, i,
                             (is_col ? col_roots : row_roots) + (size_t)i * ORC_NODE);
        if (rc < 0) {
          if (bad_axis) *bad_axis = is_col;
          if (bad_index) *bad_index = (int32_t)i;
          return ORC_EBYZANTINE;
        }
        progress |= rc;
      }
    uint64_t have = 0;
    for (size_t i = 0; i < (size_t)w * w; i++) have += present[i] ? 1 : 0;
    if (have == (uint64_t)w * w) break;
    if (!progress) return ORC_EUNREPAIRABLE;
  }
  /* Final consistency: every axis root must match. */
  for (int is_col = 0; is_col < 2; is_col++)
    for (uint32_t i = 0; i < w; i++) {
      uint8_t r[ORC_NODE];
      if (is_col) orc_axis_root(eds + (size_t)i * share, row, k, i, share, r, 0);
      else orc_axis_root(eds + (size_t)i * row, share, k, i, share, r, 0);
      if (memcmp(r, (is_col ? col_roots : row_roots) + (size_t)i * ORC_NODE, ORC_NODE) != 0) {
        if (bad_axis) *bad_axis = is_col;
        if (bad_index) *bad_index = (int32_t)i;
        return ORC_EBYZANTINE;
      }
    }
  return ORC_OK;
}
