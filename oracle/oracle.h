/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C CPU restatement of the reference's EDS / NMT / DAH hot path.
 * It is the checker for the HIP product path (tests/, __graft_entry__.smoke())
 * and the CPU baseline leg of bench.py. Product code (celestia-app_amd/) never
 * links, loads or calls anything in this directory.
 *
 * What it restates (see each .c for file:line citations):
 *   - klauspost/reedsolomon v1.12.1 Leopard GF(2^8) / GF(2^16) encode
 *     (rsmt2d v0.14.0 LeoRSCodec; reached from pkg/appconsts/global_consts.go:92)
 *   - a simple O(k^3) erasure decoder of the same code (the decoded codeword is
 *     unique for an MDS code, so any correct decoder is bit-exact)
 *   - SHA-256 (FIPS 180-4; Go crypto/sha256 via pkg/appconsts/global_consts.go:86)
 *   - nmt v0.22.0 hasher (text copy: test/util/malicious/hasher.go:186-310) with
 *     the wrapper semantics of pkg/wrapper/nmt_wrapper.go:93-140
 *   - go-square/merkle RFC-6962 HashFromByteSlices (pkg/da/data_availability_header.go:92-108)
 *   - rsmt2d ComputeExtendedDataSquare order (Q0->Q1 rows, Q0->Q2 cols, Q2->Q3 rows)
 *   - rsmt2d Repair crossword loop
 *
 * Parity pinning: GF(2^8) + NMT + DAH are pinned by the reference's DAH known
 * answers (pkg/da/data_availability_header_test.go:15-68) and by mainnet block 408
 * (x/blob/test/testdata/block_response.json data_hash). GF(2^16) (k >= 256) is
 * "parity unpinned": the reference holds no test with more than 256 shards.
 */
#ifndef CEL_ORACLE_H
#define CEL_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_OK 0
#define ORC_EINVAL 1
#define ORC_ENOTPOW2 2
#define ORC_ECHUNK 3
#define ORC_EORDER 5
#define ORC_ETOOFEW 6
#define ORC_EBYZANTINE 7
#define ORC_EUNREPAIRABLE 8
#define ORC_ENOMEM 10  /* host allocation failed (CPU baseline scratch) */
#define ORC_EBADROOT 13 /* rsmt2d preRepairSanityCheck "bad root input" (not ErrByzantineData) */

#define ORC_NS 29
#define ORC_NODE 90

void orc_init(void);
/* 0 = scalar everywhere, 1 = SIMD (AVX2 nibble mulAdd, SHA-NI) where the CPU has it. */
void orc_set_simd(int on);
int orc_simd_available(void);
void orc_set_threads(int n);
int orc_get_threads(void);

/* GF table access (debug values of SURVEY Appendix A). field = 8 or 16. */
int orc_gf_exp(int field, int i);
int orc_gf_log(int field, int i);
int orc_gf_skew(int field, int i);
int orc_gf_mul(int field, int a, int b); /* field multiplication in Leopard representation */

/* SHA-256 of one message. */
void orc_sha256(const uint8_t* msg, size_t len, uint8_t out[32]);

/* Leopard encode of n data shards -> n parity shards (n power of two, 1..32768).
 * GF(2^8) when 2n <= 256 else GF(2^16). data: n*len contiguous, parity: n*len. */
int orc_rs_encode(uint32_t n, size_t len, const uint8_t* data, uint8_t* parity);

/* Erasure decode of one axis of 2n shards (n data + n parity), in place.
 * present[i] != 0 marks shard i as known. Fills every missing shard. */
int orc_rs_decode(uint32_t n, size_t len, uint8_t* shards, const uint8_t* present);

/* ODS (k*k*share row-major) -> EDS (2k*2k*share row-major) in rsmt2d's order. */
int orc_extend(const uint8_t* ods, uint32_t k, size_t share, uint8_t* eds);

/* Row and column NMT roots (2k*90 B each) of an EDS. check_order != 0 enforces
 * the honest nmt push order. Returns ORC_EORDER (and the axis) on violation. */
int orc_roots(const uint8_t* eds, uint32_t k, size_t share, uint8_t* row_roots,
              uint8_t* col_roots, int check_order, int32_t* bad_axis);

/* NMT root over n leaves (each leaf = namespaced data of len bytes, ns = first 29 B). */
int orc_nmt_root(const uint8_t* leaves, uint32_t n, size_t len, uint8_t out[ORC_NODE],
                 int check_order);
/* Erasured (wrapper) root for one axis: cells = 2k shares of `share` bytes. */
int orc_axis_root(const uint8_t* cells, size_t cell_stride, uint32_t k, uint32_t axis,
                  size_t share, uint8_t out[ORC_NODE], int check_order);

/* RFC-6962 root over n items of item_len bytes. */
void orc_merkle_root(const uint8_t* items, uint32_t n, size_t item_len, uint8_t out[32]);
/* DAH hash = merkle(rowRoots || colRoots), w = 2k roots each. */
void orc_dah_hash(const uint8_t* row_roots, const uint8_t* col_roots, uint32_t w, uint8_t out[32]);

/* Full path: ODS -> EDS, roots, DAH. eds may be NULL. */
int orc_extend_and_commit(const uint8_t* ods, uint32_t k, size_t share, uint8_t* eds,
                          uint8_t* row_roots, uint8_t* col_roots, uint8_t dah[32]);

/* rsmt2d v0.14.0 Repair (eds.c has the full restatement): eds (2k*2k*share) with present
 * mask (2k*2k). On success every cell is filled and present[] set to all ones. On
 * EBYZANTINE / EBADROOT, bad_axis (0 row, 1 col) and bad_index are set; on EBYZANTINE
 * byz_shares (2k*share, nullable) / byz_present (2k, nullable) get the byzantine axis's
 * shares (rsmt2d ErrByzantineData.Shares; absent cells zero with byz_present 0), and
 * present[] is the mask before the failing solve. */
int orc_repair(uint8_t* eds, uint8_t* present, uint32_t k, size_t share,
               const uint8_t* row_roots, const uint8_t* col_roots, int32_t* bad_axis,
               int32_t* bad_index, uint8_t* byz_shares, uint8_t* byz_present);
/* Same, with the sweep order as a parameter: 0 = rsmt2d's (row i, then column i), 1 = all
 * rows, then all columns (test use only: shows that a case distinguishes the orders). */
int orc_repair_order(uint8_t* eds, uint8_t* present, uint32_t k, size_t share,
                     const uint8_t* row_roots, const uint8_t* col_roots, int32_t* bad_axis,
                     int32_t* bad_index, uint8_t* byz_shares, uint8_t* byz_present, int order);

/* CPU baseline (bench.py only): n independent squares (ods: n*k*k*share) extended,
 * committed and hashed on parallel threads, single-threaded each -> dah_out (n*32); and
 * n independent repairs of copies of one damaged square (status_out: n codes). */
int orc_extend_commit_many(const uint8_t* ods, uint32_t n, uint32_t k, size_t share, uint8_t* dah_out);
int orc_repair_many(const uint8_t* eds, const uint8_t* present, uint32_t k, size_t share,
                    const uint8_t* row_roots, const uint8_t* col_roots, uint32_t n, int32_t* status_out);

#ifdef __cplusplus
}
#endif
#endif
