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
#ifdef _OPENMP
#include <omp.h>
#endif
#include "oracle.h"
#include "oracle_internal.h"

static const uint8_t kParityNs[ORC_NS] = {
    0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF,
    0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF};

/* ------------------------------------------------------------------- NMT */

/* HashLeaf: ns || ns || SHA256(0x00 || ns || data) where ndata = ns || data. The
 * message (542 B for a share) is laid out once with its padding and hashed in one
 * block-function call (9 blocks), like Go crypto/sha256's block loop over a Write. */
static void nmt_leaf(const uint8_t* ns, const uint8_t* data, size_t len, uint8_t out[ORC_NODE]) {
  uint8_t d[32];
  if (len <= 512) {
    uint8_t msg[640];
    msg[0] = 0x00;
    memcpy(msg + 1, ns, ORC_NS);
    memcpy(msg + 1 + ORC_NS, data, len);
    sha256_blocks(msg, sha256_pad(msg, 1 + ORC_NS + len), d);
  } else {
    static const uint8_t zero = 0x00;
    sha256_3(&zero, 1, ns, ORC_NS, data, len, d);
  }
  memcpy(out, ns, ORC_NS);
  memcpy(out + ORC_NS, ns, ORC_NS);
  memcpy(out + 2 * ORC_NS, d, 32);
}

/* HashNode with IgnoreMaxNamespace: min = L.min; max = (R.min == MAX) ? L.max : R.max.
 * 0x01 || L || R = 181 B: three padded blocks, one block-function call. */
static void nmt_node(const uint8_t* l, const uint8_t* r, uint8_t out[ORC_NODE]) {
  uint8_t d[32];
  uint8_t msg[192];
  msg[0] = 0x01;
  memcpy(msg + 1, l, ORC_NODE);
  memcpy(msg + 1 + ORC_NODE, r, ORC_NODE);
  sha256_blocks(msg, sha256_pad(msg, 1 + 2 * ORC_NODE), d);
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
  const size_t nroots = w ? (size_t)2 * w : 1;
  uint8_t* all = (uint8_t*)malloc(nroots * ORC_NODE);
  memcpy(all, row_roots, (size_t)w * ORC_NODE);
  memcpy(all + (size_t)w * ORC_NODE, col_roots, (size_t)w * ORC_NODE);
  merkle_rec(all, 2 * w, ORC_NODE, out);
  free(all);
}

/* ----------------------------------------------------------- extension */

static int encode_axis(uint32_t k, size_t share, const uint8_t* src, size_t sstride, uint8_t* dst,
                       size_t dstride) {
  if (k == 0 || share == 0) return ORC_EINVAL;
  uint8_t* d = (uint8_t*)malloc((size_t)k * share);
  memcpy(d, src, share);
  uint8_t* p = (uint8_t*)malloc((size_t)k * share);
  for (uint32_t i = 1; i < k; i++) memcpy(d + (size_t)i * share, src + (size_t)i * sstride, share);
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
/*
 * rsmt2d v0.14.0 ExtendedDataSquare.Repair [dep] (extendeddatacrossword.go), restated:
 *  1. preRepairSanityCheck: every axis complete before the repair must match its root
 *     (else ORC_EBADROOT: rsmt2d's plain "bad root input" error, not ErrByzantineData)
 *     and its parity half must equal Encode(data half) (else ORC_EBYZANTINE, shares =
 *     the whole axis). rsmt2d runs these checks in goroutines; this restatement fixes
 *     the order: for i in 0..W-1: row i (root, encoding), then column i.
 *  2. solveCrossword: sweeps `for i in 0..W-1 { solveCrosswordRow(i); solveCrosswordCol(i) }`
 *     (row i, then column i, each solve seeing the square as every earlier solve left it),
 *     until solved or a sweep makes no progress (ORC_EUNREPAIRABLE).
 *     Every incomplete axis with >= k known cells is decoded; its
 *     parity half must equal Encode(data half) and its root must match (else
 *     ORC_EBYZANTINE, shares = the axis before the solve, missing cells absent); then
 *     every orthogonal axis the solve completes (in index order) must match its root
 *     and its encoding (else ORC_EBYZANTINE, shares = that complete axis).
 *  On ORC_EBYZANTINE / ORC_EBADROOT the presence mask is left as it was before the
 *  failing solve ("the most-repaired square prior to the byzantine axis"); cells
 *  outside it are undefined. byz_shares (W*share) / byz_present (W) may be NULL.
 */

typedef struct {
  uint8_t* eds;
  uint8_t* present;
  uint32_t k, w;
  size_t share, row;
  const uint8_t *row_roots, *col_roots;
  int32_t *bad_axis, *bad_index;
  uint8_t *byz_shares, *byz_present;
} rep_t;

static uint8_t* cell(const rep_t* R, int is_col, uint32_t idx, uint32_t j) {
  return is_col ? R->eds + (size_t)j * R->row + (size_t)idx * R->share
                : R->eds + (size_t)idx * R->row + (size_t)j * R->share;
}
static uint8_t* pres(const rep_t* R, int is_col, uint32_t idx, uint32_t j) {
  return is_col ? R->present + (size_t)j * R->w + idx : R->present + (size_t)idx * R->w + j;
}
static uint32_t count_axis(const rep_t* R, int is_col, uint32_t idx) {
  uint32_t c = 0;
  for (uint32_t j = 0; j < R->w; j++) c += *pres(R, is_col, idx, j) ? 1 : 0;
  return c;
}

/* cells: W contiguous shares of one axis. 1 = root matches. */
static int root_ok(const rep_t* R, int is_col, uint32_t idx, const uint8_t* cells) {
  uint8_t r[ORC_NODE];
  orc_axis_root(cells, R->share, R->k, idx, R->share, r, 0);
  return memcmp(r, (is_col ? R->col_roots : R->row_roots) + (size_t)idx * ORC_NODE, ORC_NODE) == 0;
}
/* 1 = parity half equals Encode(data half). */
static int encoding_ok(const rep_t* R, const uint8_t* cells) {
  size_t half = (size_t)R->k * R->share;
  uint8_t* par = (uint8_t*)malloc(half);
  orc_rs_encode(R->k, R->share, cells, par);
  int ok = memcmp(par, cells + half, half) == 0;
  free(par);
  return ok;
}
static void gather(const rep_t* R, int is_col, uint32_t idx, uint8_t* cells, uint8_t* pm) {
  for (uint32_t j = 0; j < R->w; j++) {
    pm[j] = *pres(R, is_col, idx, j) ? 1 : 0;
    if (pm[j]) memcpy(cells + (size_t)j * R->share, cell(R, is_col, idx, j), R->share);
    else memset(cells + (size_t)j * R->share, 0, R->share);
  }
}
static int byzantine(const rep_t* R, int is_col, uint32_t idx, const uint8_t* cells, const uint8_t* pm) {
  if (R->bad_axis) *R->bad_axis = is_col;
  if (R->bad_index) *R->bad_index = (int32_t)idx;
  if (R->byz_shares)
    for (uint32_t j = 0; j < R->w; j++) {
      if (pm[j]) memcpy(R->byz_shares + (size_t)j * R->share, cells + (size_t)j * R->share, R->share);
      else memset(R->byz_shares + (size_t)j * R->share, 0, R->share);
    }
  if (R->byz_present) memcpy(R->byz_present, pm, R->w);
  return ORC_EBYZANTINE;
}

static int sanity_axis(const rep_t* R, int is_col, uint32_t idx, uint8_t* cells, uint8_t* pm) {
  if (count_axis(R, is_col, idx) != R->w) return ORC_OK;
  gather(R, is_col, idx, cells, pm);
  if (!root_ok(R, is_col, idx, cells)) {
    if (R->bad_axis) *R->bad_axis = is_col;
    if (R->bad_index) *R->bad_index = (int32_t)idx;
    return ORC_EBADROOT;
  }
  if (!encoding_ok(R, cells)) return byzantine(R, is_col, idx, cells, pm);
  return ORC_OK;
}

/* Solve one axis (>= k known, incomplete). 1 = solved, <0 = status. */
static int solve_axis(const rep_t* R, int is_col, uint32_t idx, uint8_t* cells, uint8_t* pm, uint8_t* ocells,
                      uint8_t* opm) {
  gather(R, is_col, idx, cells, pm);
  uint8_t* dec = (uint8_t*)malloc((size_t)R->w * R->share);
  memcpy(dec, cells, (size_t)R->w * R->share);
  int rc = orc_rs_decode(R->k, R->share, dec, pm);
  if (rc != ORC_OK || !encoding_ok(R, dec) || !root_ok(R, is_col, idx, dec)) {
    free(dec);
    return -byzantine(R, is_col, idx, cells, pm);
  }
  /* orthogonal axes this solve completes */
  for (uint32_t j = 0; j < R->w; j++) {
    if (pm[j]) continue;
    int o_col = !is_col;
    if (count_axis(R, o_col, j) != R->w - 1) continue;
    gather(R, o_col, j, ocells, opm);
    memcpy(ocells + (size_t)idx * R->share, dec + (size_t)j * R->share, R->share);
    opm[idx] = 1;
    if (!root_ok(R, o_col, j, ocells) || !encoding_ok(R, ocells)) {
      free(dec);
      return -byzantine(R, o_col, j, ocells, opm);
    }
  }
  for (uint32_t j = 0; j < R->w; j++)
    if (!pm[j]) {
      memcpy(cell(R, is_col, idx, j), dec + (size_t)j * R->share, R->share);
      *pres(R, is_col, idx, j) = 1;
    }
  free(dec);
  return 1;
}

/* order 0: rsmt2d's sweep (row i, column i); order 1: every row, then every column, per
 * sweep (the order of the round-1/2 restatement, kept only so a test can show that a case
 * tells the two apart). */
int orc_repair_order(uint8_t* eds, uint8_t* present, uint32_t k, size_t share, const uint8_t* row_roots,
                     const uint8_t* col_roots, int32_t* bad_axis, int32_t* bad_index, uint8_t* byz_shares,
                     uint8_t* byz_present, int order) {
  orc_init();
  rep_t R = {eds, present, k, 2 * k, share, (size_t)2 * k * share, row_roots, col_roots,
             bad_axis, bad_index, byz_shares, byz_present};
  const uint32_t w = R.w;
  if (bad_axis) *bad_axis = -1;
  if (bad_index) *bad_index = -1;
  uint8_t* cells = (uint8_t*)malloc((size_t)w * share);
  uint8_t* ocells = (uint8_t*)malloc((size_t)w * share);
  uint8_t* pm = (uint8_t*)malloc(w);
  uint8_t* opm = (uint8_t*)malloc(w);
  int rc = ORC_OK;
  for (uint32_t i = 0; i < w && rc == ORC_OK; i++) {
    rc = sanity_axis(&R, 0, i, cells, pm);
    if (rc == ORC_OK) rc = sanity_axis(&R, 1, i, cells, pm);
  }
  while (rc == ORC_OK) {
    int progress = 0;
    for (uint32_t t = 0; t < 2 * w && rc == ORC_OK; t++) {
      const int is_col = order ? (t >= w) : (int)(t & 1);
      const uint32_t i = order ? t % w : t >> 1;
      uint32_t c = count_axis(&R, is_col, i);
      if (c == w || c < k) continue;
      int s = solve_axis(&R, is_col, i, cells, pm, ocells, opm);
      if (s < 0) { rc = -s; break; }
      progress = 1;
    }
    if (rc != ORC_OK) break;
    uint64_t have = 0;
    for (size_t i = 0; i < (size_t)w * w; i++) have += present[i] ? 1 : 0;
    if (have == (uint64_t)w * w) break;
    if (!progress) rc = ORC_EUNREPAIRABLE;
  }
  free(cells);
  free(ocells);
  free(pm);
  free(opm);
  return rc;
}

int orc_repair(uint8_t* eds, uint8_t* present, uint32_t k, size_t share, const uint8_t* row_roots,
               const uint8_t* col_roots, int32_t* bad_axis, int32_t* bad_index, uint8_t* byz_shares,
               uint8_t* byz_present) {
  return orc_repair_order(eds, present, k, share, row_roots, col_roots, bad_axis, bad_index, byz_shares,
                          byz_present, 0);
}

/* ------------------------------------------------------- CPU baseline (bench) */
/*
 * Throughput form of the reference's CPU path on a multi-core host: independent squares
 * (or repairs) on independent threads, each single-threaded inside with buffers reused
 * across its squares, the way a node extends one block per goroutine set. Not a checker.
 */
/* Per-thread scratch that outlives a call (OpenMP keeps its threads across parallel
 * regions): a fresh 32 MiB EDS per call would be page-faulted in again every time. */
static __thread uint8_t* tl_buf;
static __thread size_t tl_cap;

static uint8_t* thread_scratch(size_t bytes) {
  if (bytes > tl_cap) {
    free(tl_buf);
    tl_buf = (uint8_t*)malloc(bytes);
    tl_cap = tl_buf ? bytes : 0;
  }
  return tl_buf;
}

/* End of a call: a thread keeps its scratch only up to a k=128 square's size, so a k=512
 * repair's ~0.5 GiB per thread is not held by the process after the call. */
#define ORC_SCRATCH_KEEP ((size_t)64 << 20)
static void thread_scratch_trim(void) {
  if (tl_cap > ORC_SCRATCH_KEEP) {
    free(tl_buf);
    tl_buf = NULL;
    tl_cap = 0;
  }
}

int orc_extend_commit_many(const uint8_t* ods, uint32_t n, uint32_t k, size_t share, uint8_t* dah_out) {
  orc_init();
  const size_t ods_b = (size_t)k * k * share, eds_b = 4 * ods_b, roots_b = (size_t)2 * k * ORC_NODE;
  int rc = ORC_OK;
#ifdef _OPENMP
  const int levels = omp_get_max_active_levels();
  omp_set_max_active_levels(1);
#endif
#pragma omp parallel reduction(| : rc)
  {
    uint8_t* eds = thread_scratch(eds_b + 2 * roots_b);
    uint8_t* rr = eds ? eds + eds_b : NULL;
    uint8_t* cr = rr ? rr + roots_b : NULL;
#pragma omp for schedule(dynamic, 1)
    for (int64_t i = 0; i < (int64_t)n; i++) {
      int r = eds ? orc_extend(ods + (size_t)i * ods_b, k, share, eds) : ORC_ENOMEM;
      if (r == ORC_OK) r = orc_roots(eds, k, share, rr, cr, 1, NULL);
      if (r == ORC_OK) orc_dah_hash(rr, cr, 2 * k, dah_out + (size_t)i * 32);
      rc |= r;
    }
    thread_scratch_trim();
  }
#ifdef _OPENMP
  omp_set_max_active_levels(levels);
#endif
  return rc;
}

int orc_repair_many(const uint8_t* eds, const uint8_t* present, uint32_t k, size_t share, const uint8_t* row_roots,
                    const uint8_t* col_roots, uint32_t n, int32_t* status_out) {
  orc_init();
  const size_t cells = (size_t)4 * k * k, eds_b = cells * share;
#pragma omp parallel
  {
    uint8_t* e = thread_scratch(eds_b + cells);
    uint8_t* p = e ? e + eds_b : NULL;
#pragma omp for schedule(dynamic, 1)
    for (int64_t i = 0; i < (int64_t)n; i++) {
      if (!e) {
        status_out[i] = ORC_ENOMEM;
        continue;
      }
      memcpy(e, eds, eds_b);
      memcpy(p, present, cells);
      status_out[i] = orc_repair(e, p, k, share, row_roots, col_roots, NULL, NULL, NULL, NULL);
    }
    thread_scratch_trim();
  }
  return ORC_OK;
}
