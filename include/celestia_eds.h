/*
 * celestia_eds.h — C ABI of the MI355X-native extended-data-square hot path.
 *
 * This library replaces, behind an unchanged Go surface, the hot path of
 * celestia-app's pkg/da (reference /root/reference):
 *
 *   da.ExtendShares                 pkg/da/data_availability_header.go:65-75
 *   da.NewDataAvailabilityHeader    pkg/da/data_availability_header.go:44-63
 *   DataAvailabilityHeader.Hash     pkg/da/data_availability_header.go:92-108
 *   rsmt2d.Codec (LeoRSCodec)       pkg/appconsts/global_consts.go:92 (DefaultCodec)
 *   rsmt2d.Tree via wrapper         pkg/wrapper/nmt_wrapper.go:14-17,83,93-124
 *   rsmt2d ExtendedDataSquare.Repair (rsmt2d v0.14.0 [dep]; used by celestia-node)
 *
 * Every entry point returns cel_status (0 = OK) and never aborts. Buffers are
 * borrowed for the duration of the call only (cgo forbids retaining Go pointers);
 * outputs go to caller-allocated memory. A cel_ctx binds one HIP device and one
 * stream; calls on one ctx are serialised internally, so a ctx may be shared by
 * goroutines; use one ctx per device for concurrency.
 *
 * Layouts (all row-major, share = 512 B = appconsts.ShareSize):
 *   ODS   k*k shares                         (the [][]byte of da.ExtendShares, flattened)
 *   EDS   2k*2k shares                       (rsmt2d flattened square: Q0 Q1 / Q2 Q3)
 *   roots 2k entries of 90 B                 (minNs(29) || maxNs(29) || sha256(32))
 *   dah   32 B                               (RFC-6962 root of rowRoots || colRoots)
 */
#ifndef CELESTIA_EDS_H
#define CELESTIA_EDS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int32_t cel_status;

/* Status codes; each maps 1:1 onto a Go error of the reference surface. */
#define CEL_OK 0
#define CEL_EINVAL 1         /* bad argument (nil pointer, zero size)                          */
#define CEL_ENOTPOW2 2       /* "number of shares is not a power of 2: got %d" (data_availability_header.go:68) */
#define CEL_ECHUNK 3         /* chunk size not a positive multiple of 64 (rsmt2d ValidateChunkSize) */
#define CEL_ETOOBIG 4        /* square / codeword wider than the device path supports: the Go shim
                                answers these calls with the reference path instead */
#define CEL_EORDER 5         /* nmt: leaves pushed out of namespace order (nmt_wrapper_test.go:106-111) */
#define CEL_ETOOFEW 6        /* decode: fewer than k of 2k shards present                      */
#define CEL_EBYZANTINE 7     /* rsmt2d ErrByzantineData: axis fails re-encoding or root check  */
#define CEL_EUNREPAIRABLE 8  /* rsmt2d ErrUnrepairableDataSquare                               */
#define CEL_EDEVICE 9        /* HIP runtime / kernel failure                                   */
#define CEL_ENOMEM 10        /* device allocation failed                                       */
#define CEL_ESHORT 11        /* "data is too short to contain namespace ID" (nmt_wrapper.go:98) */
#define CEL_EPUSHPAST 12     /* "pushed past predetermined square size" (nmt_wrapper.go:95)     */
#define CEL_EBADROOT 13      /* rsmt2d preRepairSanityCheck "bad root input": a complete axis does
                                not match its root (a plain error, not ErrByzantineData)       */
#define CEL_ENODATA 14       /* codec: zero-length shards (klauspost reedsolomon ErrShardNoData,
                                "no shard data", which LeoRSCodec.Encode / Decode pass through) */

/* Flags for the square entry points. */
#define CEL_FLAG_ORDER_CHECK 0x1u   /* enforce the honest nmt push order (default in the Go path) */
#define CEL_FLAG_PARITY_ONLY 0x2u   /* host entry points: eds_out receives the parity cells only
                                       (Q1, Q2, Q3); its Q0 cells are not written, the caller
                                       holds the ODS already (the Go shim points Q0's cells of the
                                       imported square at the input shares): 3/4 of the PCIe bytes */
#define CEL_FLAG_CALLER_STREAM 0x4u /* cel_dev_extend_batch: the whole batch as one chunk on the
                                       caller's stream, no internal streams (a caller keeping
                                       several batches in flight on its own streams). Such
                                       batches on one ctx are chained: each starts its extension
                                       after the previous CALLER_STREAM batch's extension on that
                                       ctx has finished (an event wait, whatever stream either
                                       ran on), so its extension runs beside the previous batch's
                                       hashing. Independent pipelines that must not be ordered
                                       use one ctx each. */

#define CEL_SHARE_SIZE 512u
#define CEL_NAMESPACE_SIZE 29u
#define CEL_NMT_NODE_SIZE 90u
#define CEL_HASH_SIZE 32u

typedef struct cel_ctx cel_ctx;

/* ---------------------------------------------------------------- context */
cel_status cel_ctx_create(int device, cel_ctx** out);
void cel_ctx_destroy(cel_ctx* ctx);
const char* cel_strerror(cel_status st);
/* Go-style message of the last failing call on ctx (e.g. the exact
 * "number of shares is not a power of 2: got 5" string). */
const char* cel_last_error(const cel_ctx* ctx);
/* Name of the device (for reports). */
cel_status cel_device_name(cel_ctx* ctx, char* buf, size_t len);

/* ------------------------------------------------------- square (host I/O) */
/* da.ExtendShares + da.NewDataAvailabilityHeader in one device pass.
 * shares: n_shares * share_size bytes (n_shares must be a power of two and a
 * perfect square, i.e. k*k; replaces data_availability_header.go:65-75,44-63).
 * eds_out may be NULL (PrepareProposal/ProcessProposal discard the EDS:
 * app/prepare_proposal.go:81-83). row_roots/col_roots: 2k*90 B each; dah: 32 B. */
cel_status cel_extend_shares(cel_ctx* ctx, const uint8_t* shares, uint32_t n_shares,
                             uint32_t share_size, uint8_t* eds_out, uint8_t* row_roots,
                             uint8_t* col_roots, uint8_t* dah, uint32_t flags);

/* Batch replay: n independent k*k squares laid out back to back (config 4).
 * eds_out (nullable): n * 4k^2 * share; roots: n * 2k * 90 each; dah: n * 32.
 * status_out (nullable): per-square status (CEL_EORDER for a bad square). */
cel_status cel_extend_batch(cel_ctx* ctx, const uint8_t* ods, uint32_t n, uint32_t k,
                            uint32_t share_size, uint8_t* eds_out, uint8_t* row_roots,
                            uint8_t* col_roots, uint8_t* dah, int32_t* status_out,
                            uint32_t flags);

/* Page-locked host memory for the buffers of the host entry points (the ODS, the EDS
 * output): with it every PCIe copy of cel_extend_batch is an asynchronous DMA that
 * overlaps the other chunks' kernels. Any host memory works; pageable memory is
 * staged by the runtime. cel_host_alloc returns NULL on failure. */
void* cel_host_alloc(size_t bytes);
void cel_host_free(void* p);

/* -------------------------------------------------- square (device resident)
 * Same as cel_extend_batch with every pointer in device memory of ctx's device.
 * stream: a hipStream_t (NULL = ctx's own stream). Asynchronous: returns after
 * enqueueing. d_status: n int32 (0 or CEL_EORDER). Required d_eds: n*4k^2*share
 * (the EDS is always materialised on the device). d_work: scratch of
 * cel_dev_workspace_size(k, n) bytes. */
size_t cel_dev_workspace_size(uint32_t k, uint32_t n);
cel_status cel_dev_extend_batch(cel_ctx* ctx, const void* d_ods, uint32_t n, uint32_t k,
                                void* d_eds, void* d_row_roots, void* d_col_roots, void* d_dah,
                                int32_t* d_status, void* d_work, void* stream, uint32_t flags);
/* Input layout of the device path: d_ods == NULL means every ODS already sits in
 * quadrant Q0 of its EDS buffer (row pitch 2k shares, the flattened rsmt2d square)
 * and is extended in place. cel_dev_place_ods puts n
 * row-major ODSs (host or device memory, as da.ExtendShares receives them flattened,
 * data_availability_header.go:65-75) there with strided copies on `stream`.
 * cel_extend_batch uses this path; a separate d_ods buffer makes the row pass also
 * copy Q0 into the EDS. */
cel_status cel_dev_place_ods(cel_ctx* ctx, const void* ods, uint32_t n, uint32_t k, void* d_eds,
                             void* stream);
/* Phase entry points of the same pipeline (for profiling and the row-sharded
 * multi-GPU mode): RS extension only, and NMT roots + DAH over a resident EDS. */
cel_status cel_dev_extend_only(cel_ctx* ctx, const void* d_ods, uint32_t n, uint32_t k,
                               void* d_eds, void* stream);
cel_status cel_dev_commit_only(cel_ctx* ctx, const void* d_eds, uint32_t n, uint32_t k,
                               void* d_row_roots, void* d_col_roots, void* d_dah,
                               int32_t* d_status, void* d_work, void* stream, uint32_t flags);

/* ------------------------------------------- row-sharded square (multi-GPU)
 * One square extended by nranks processes, one per GPU (config 3).
 * Replaces, for a square too large for one device's share of the work, the same
 * da.ExtendShares + NewDataAvailabilityHeader pair (data_availability_header.go:65-75,
 * :44-63). Rank r owns ODS rows [r*k/nranks, (r+1)*k/nranks) and, after the column
 * transpose, EDS columns [r*w, (r+1)*w) with w = 2k/nranks. The two collectives (one
 * all-to-all of cells, one all-gather of node records) belong to the caller (RCCL
 * through torch.distributed); these calls are the per-rank device steps.
 * Supported for k in {256, 512} (Leopard GF(2^16)), nranks a power of two <= k.
 * Node records are 96 bytes: the 90-byte NMT node and 6 zero bytes. */
#define CEL_NODE_RECORD 96u
size_t cel_dev_shard_workspace_size(uint32_t k, uint32_t nranks);
/* Step 1: row-encode this rank's k/nranks ODS rows (d_ods_rows: [k/nranks][k][512])
 * straight into the all-to-all send buffer d_send: [nranks][k/nranks][w][512]
 * (block h = the cells of columns [h*w, (h+1)*w), Q0 and Q1 alike). */
cel_status cel_dev_shard_rows(cel_ctx* ctx, const void* d_ods_rows, uint32_t k, uint32_t nranks, void* d_send,
                              void* stream);
/* Step 2 (after the all-to-all into the top half of d_slab): d_slab is [2k][w][512]
 * with rows [0, k) received in rank order. Column-encodes the slab in place (rows
 * [k, 2k)), hashes its 2k*w leaves once, and writes the w column-root records
 * (d_col_rec: [w][96]) and the 2k row-subtree records over this slab's columns
 * (d_row_sub: [2k][96]). *d_status = 0 or CEL_EORDER (within-slab push order).
 * Step 3 all-gathers one record block per rank, [2k + w + 1][96]: the row subtrees,
 * then the column roots, then a record whose first 4 bytes are the status; pointing
 * d_row_sub, d_col_rec and d_status into that block makes it the send buffer. */
cel_status cel_dev_shard_cols(cel_ctx* ctx, void* d_slab, uint32_t k, uint32_t nranks, uint32_t rank,
                              void* d_col_rec, void* d_row_sub, int32_t* d_status, void* d_work, void* stream,
                              uint32_t flags);
/* Step 3 (after all-gathering every rank's record block, rank order):
 * d_gathered [nranks][2k + w + 1][96] -> d_row_roots, d_col_roots (2k x 90 B each) and
 * d_dah (32 B). *d_status = the max over ranks of the step-2 status, or CEL_EORDER if
 * the push order breaks across slab boundaries. */
cel_status cel_dev_shard_finish(cel_ctx* ctx, const void* d_gathered, uint32_t k, uint32_t nranks, void* d_row_roots,
                                void* d_col_roots, void* d_dah, int32_t* d_status, void* d_work, void* stream,
                                uint32_t flags);

/* --------------------------------------- multi-GPU inside the library (configs 3, 4)
 * One process, one host thread, several devices: ctxs[0..ngpu) as cel_ctx_create made them.
 * The collectives run inside the library over RCCL: one communicator rank per device
 * (ncclCommInitAll), every rank's sends / receives / all-gathers issued inside
 * ncclGroupStart / ncclGroupEnd. librccl.so.1 is loaded (dlopen) by the first plan over
 * distinct devices; the single-device entry points never need it. RCCL refuses two ranks on
 * one device, so a plan whose ctxs repeat a device moves the same blocks with device copies
 * instead (transport "copy": the same schedule, e.g. N ranks rehearsed on one GPU). Distinct
 * devices without RCCL (CEL_FLAG_SHARD_PEERCOPY, or RCCL not loadable / ncclCommInitAll
 * failing at plan creation) move them with hipMemcpyPeerAsync, peer access enabled (transport
 * "peer", "peer-fallback" when RCCL failed; cel_shard_plan_note keeps RCCL's message).
 *
 * cel_extend_sharded: da.ExtendShares + da.NewDataAvailabilityHeader
 * (data_availability_header.go:65-75, :44-63) for ONE square row-sharded over ngpu devices
 * (config 3): rank r row-encodes ODS rows [r k/N, (r+1) k/N) straight into
 * the all-to-all layout, grouped ncclSend / ncclRecv transpose the column blocks (k/N x 2k/N
 * cells per peer), each rank column-encodes and commits its [2k][2k/N] slab, one ncclAllGather
 * of 96-byte record blocks, rank 0 combines the row subtrees and hashes the DAH. Same
 * arguments and outputs as cel_extend_shares (ods: k*k*512 host bytes; eds_out nullable, with
 * CEL_FLAG_PARITY_ONLY its Q0 cells are not written). k = 256 or 512 (Leopard GF(2^16)), ngpu a
 * power of two <= k. The plan (buffers, streams, communicators) is kept in ctxs[0] for the
 * next call with the same device list, k and flags; ctxs[0]'s lock serialises such calls. */
cel_status cel_extend_sharded(cel_ctx* const* ctxs, uint32_t ngpu, const uint8_t* ods, uint32_t k,
                              uint32_t share_size, uint8_t* eds_out, uint8_t* row_roots, uint8_t* col_roots,
                              uint8_t* dah, uint32_t flags);
/* The same square as an explicit plan, for callers that keep ODSs resident or several squares
 * in flight (each plan has its own streams and communicators):
 *   create   per-rank buffers, streams, tables and the communicators (the expensive part);
 *   upload   ods (k*k*512 bytes, host or device memory) -> each rank's row block;
 *   run      one square, asynchronous on the ranks' streams;
 *   wait     sync, then (each nullable) the EDS (from every rank's column slab), the roots and
 *            the DAH (rank 0); returns the square's status (CEL_EORDER) or a device error.
 * flags: CEL_FLAG_ORDER_CHECK, CEL_FLAG_PARITY_ONLY (wait's eds_out), CEL_FLAG_SHARD_EXCHANGE,
 * CEL_FLAG_SHARD_PEERCOPY. */
typedef struct cel_shard_plan cel_shard_plan;
#define CEL_FLAG_SHARD_EXCHANGE 0x8u /* the exchange through RCCL wherever it is asked for: ngpu = 1
                                        gets a one-rank RCCL communicator, a separate send buffer, the
                                        all-to-all through it (self send / receive) and the record
                                        all-gather too, instead of the row pass writing the slab in
                                        place and no collective (tests the N > 1 exchange on one GPU);
                                        ctxs repeating a device try RCCL too (which refuses them) and
                                        fall back to device copies ("copy-fallback") */
#define CEL_FLAG_SHARD_PEERCOPY 0x10u /* never RCCL: distinct devices exchange with hipMemcpyPeerAsync
                                         (transport "peer"), repeated devices with device copies */
cel_status cel_shard_plan_create(cel_ctx* const* ctxs, uint32_t ngpu, uint32_t k, uint32_t flags,
                                 cel_shard_plan** out);
void cel_shard_plan_destroy(cel_shard_plan* plan);
const char* cel_shard_plan_transport(const cel_shard_plan* plan); /* "rccl", "copy" (ctxs repeat a
                                                                      device), "peer" (distinct
                                                                      devices, peer copies), "local"
                                                                      (one rank, no collective);
                                                                      "copy-fallback" /
                                                                      "peer-fallback" when RCCL
                                                                      could not start */
const char* cel_shard_plan_note(const cel_shard_plan* plan); /* why RCCL was not used ("" if it was,
                                                               or was not asked for) */
const char* cel_shard_plan_last_error(const cel_shard_plan* plan);
cel_status cel_shard_plan_upload(cel_shard_plan* plan, const uint8_t* ods);
cel_status cel_shard_plan_run(cel_shard_plan* plan);
cel_status cel_shard_plan_wait(cel_shard_plan* plan, uint8_t* eds_out, uint8_t* row_roots, uint8_t* col_roots,
                               uint8_t* dah);
/* The plan's all-to-all alone, `reps` times back to back after one warm-up exchange: the
 * slowest rank's microseconds per exchange (a report's figure next to SURVEY.md §8e's
 * one-link estimate; CEL_EINVAL for a one-rank plan in place, which has no exchange). */
cel_status cel_shard_plan_time_exchange(cel_shard_plan* plan, uint32_t reps, double* us_per_exchange);
/* Config 4 over several devices: cel_extend_batch's arguments, the n squares split into ngpu
 * contiguous ranges (sizes differ by at most one) each extended by cel_extend_batch on ctxs[i]
 * from its own host thread, so every device's PCIe copies and kernels run side by side
 * (page-locked buffers from cel_host_alloc keep the copies asynchronous). ctxs may repeat a
 * device. Returns the first failing range's status (its message in ctxs[0]). */
cel_status cel_extend_batch_multi(cel_ctx* const* ctxs, uint32_t ngpu, const uint8_t* ods, uint32_t n, uint32_t k,
                                  uint32_t share_size, uint8_t* eds_out, uint8_t* row_roots, uint8_t* col_roots,
                                  uint8_t* dah, int32_t* status_out, uint32_t flags);

/* ------------------------------------------------------- same-run probes
 * The ceilings a report prices the hot path against, measured on ctx's device in the same
 * process (bench.py's line): cel_probe_sha256 runs the NMT kernels' SHA-256 compression
 * chained in registers on every lane with no memory traffic (G compressions/s, best of 5
 * launches) and reports the sustained shader clock over that launch (MHz, nullable: shader
 * clock ticks per constant-rate tick of every wave); cel_probe_hbm_copy streams a copy over
 * `bytes` of HBM (half read, half written; one 16-byte element per lane) and reports read +
 * write GB/s (best of 5); cel_probe_hbm_stream adds the read-only and write-only rates over
 * the same half (each nullable: HBM writes stream slower than reads, which prices a
 * write-heavy kernel such as the extension, 3 bytes written per byte read);
 * cel_probe_rs_transform runs the encode tile (GF(2^8): k = 32, 64 or 128; GF(2^16): k = 256
 * or 512) with its HBM traffic taken away and reports the microseconds one square's
 * extension (3k axis encodes) spends in the transform alone, whole chip (best of 5). */
cel_status cel_probe_sha256(cel_ctx* ctx, double* g_compressions_per_s, double* shader_mhz);
cel_status cel_probe_hbm_copy(cel_ctx* ctx, uint64_t bytes, double* gbps);
cel_status cel_probe_hbm_stream(cel_ctx* ctx, uint64_t bytes, double* copy_gbps, double* read_gbps,
                                double* write_gbps);
cel_status cel_probe_rs_transform(cel_ctx* ctx, uint32_t k, double* us_per_square);

/* ------------------------------------------------------ rsmt2d.Codec surface
 * Leopard RS (klauspost/reedsolomon v1.12.1 New(n, n, WithLeopardGF(true))):
 * GF(2^8) when 2n <= 256, GF(2^16) otherwise. len must be a positive multiple
 * of 64. data: n*len contiguous -> parity: n*len. */
cel_status cel_codec_encode(cel_ctx* ctx, const uint8_t* data, uint32_t n, uint32_t len,
                            uint8_t* parity);
/* shards: 2n*len (n data then n parity), present: 2n flags (nil shard = 0).
 * Fills every missing shard in place (rsmt2d Codec.Decode). */
cel_status cel_codec_decode(cel_ctx* ctx, uint8_t* shards, const uint8_t* present, uint32_t n,
                            uint32_t len);
/* Device-resident batch of rsmt2d Codec.Decode calls (one per axis), as the repair's
 * crossword passes issue them: d_shards [naxes][2n][len] (data then parity, filled in
 * place), d_present [naxes][2n] (0 = missing; every axis needs >= n present). n <= 1024,
 * len a positive multiple of 64. Asynchronous on stream (NULL = ctx's stream). */
cel_status cel_dev_decode(cel_ctx* ctx, void* d_shards, const void* d_present, uint32_t naxes, uint32_t n,
                          uint32_t len, void* stream);
uint64_t cel_codec_max_chunks(void);             /* 32768 * 32768 */
const char* cel_codec_name(void);                /* "Leopard" */
cel_status cel_codec_validate_chunk_size(uint32_t len);

/* ---------------------------------------------------- rsmt2d.Tree surface
 * Root of one erasured NMT axis: the 2k cells of row/column `axis_index` of a
 * square of original width k (wrapper.Push x 2k then Root,
 * pkg/wrapper/nmt_wrapper.go:93-124). cells: 2k*share contiguous. */
cel_status cel_axis_root(cel_ctx* ctx, const uint8_t* cells, uint32_t k, uint32_t axis_index,
                         uint32_t share_size, uint8_t* root_out, uint32_t flags);
/* Plain NMT root over n namespaced leaves of leaf_len bytes (ns = first 29 B). */
cel_status cel_nmt_root(cel_ctx* ctx, const uint8_t* leaves, uint32_t n, uint32_t leaf_len,
                        uint8_t* root_out, uint32_t flags);
/* DataAvailabilityHeader.Hash: RFC-6962 root over rowRoots || colRoots (w each). */
cel_status cel_dah_hash(cel_ctx* ctx, const uint8_t* row_roots, const uint8_t* col_roots,
                        uint32_t w, uint8_t* out);
/* merkle.HashFromByteSlices (RFC-6962; tendermint crypto/merkle, the hash
 * DataAvailabilityHeader.Hash applies to rowRoots || colRoots,
 * data_availability_header.go:92-108) over n byte slices of any length: slice i is
 * data[offsets[i] .. offsets[i+1]) (offsets: n + 1 entries, non-decreasing). For DAHs
 * whose roots are not all 90-byte NMT roots (FromProto accepts any length). n = 0 gives
 * SHA-256 of the empty string. */
cel_status cel_merkle_hash_slices(cel_ctx* ctx, const uint8_t* data, const uint64_t* offsets, uint32_t n,
                                  uint8_t* out);

/* ------------------------------------------------------------------ repair
 * rsmt2d ExtendedDataSquare.Repair(rowRoots, colRoots) (rsmt2d v0.14.0
 * extendeddatacrossword.go [dep]; oracle/eds.c restates it): eds is 2k*2k*share with
 * present[2k*2k] marking known cells.
 *   CEL_OK            every cell filled, present[] all ones.
 *   CEL_EBADROOT      an axis complete before the repair does not match its root
 *                     (preRepairSanityCheck "bad root input", a plain error).
 *   CEL_EBYZANTINE    rsmt2d *ErrByzantineData{Axis, Index, Shares}: *bad_axis (0 = row,
 *                     1 = col), *bad_index, and (both nullable) byz_shares (2k*share) /
 *                     byz_present (2k) = that axis's shares as rsmt2d reports them
 *                     (absent cells zero with byz_present 0). Raised by a complete axis
 *                     whose parity differs from Encode(data) (sanity check), a decoded axis
 *                     failing its re-encoding or root check, or an orthogonal axis the
 *                     decode completed failing its root or encoding.
 *   CEL_EUNREPAIRABLE ErrUnrepairableDataSquare: no progress possible.
 * On CEL_EBYZANTINE / CEL_EBADROOT present[] is the mask before the failing solve (the
 * "most-repaired square prior to the byzantine axis"); on CEL_EUNREPAIRABLE the mask of
 * the most-repaired square. Cells outside present[] are undefined. Checks are reported
 * in rsmt2d's order: sanity row i then column i; then solveCrossword's sweeps, row i then
 * column i for i = 0..2k-1, each solve followed by the orthogonal axes it completes.
 * rsmt2d runs its sanity checks in goroutines, so which failing complete axis it reports
 * first is not fixed there. */
cel_status cel_repair(cel_ctx* ctx, uint8_t* eds, uint8_t* present, uint32_t k,
                      uint32_t share_size, const uint8_t* row_roots, const uint8_t* col_roots,
                      int32_t* bad_axis, int32_t* bad_index, uint8_t* byz_shares,
                      uint8_t* byz_present);
/* Same repair over an EDS resident on ctx's device (d_eds: 2k*2k*512 bytes, filled in
 * place); present, the roots and the byzantine outputs stay host memory (the crossword
 * control loop runs on the host over the presence mask). Synchronous. */
cel_status cel_dev_repair(cel_ctx* ctx, void* d_eds, uint8_t* present, uint32_t k,
                          const uint8_t* row_roots, const uint8_t* col_roots, int32_t* bad_axis,
                          int32_t* bad_index, uint8_t* byz_shares, uint8_t* byz_present);
/* Tests only: from the next repair on ctx, an idle kernel of a pseudo-random 0..max_us
 * microseconds (seeded by seed) goes in front of every operation the repair enqueues on
 * either of its two streams, so the streams interleave differently; max_us = 0 turns it
 * off. Outcomes must not change: it checks that the schedule's cross-stream dependencies
 * are complete. */
cel_status cel_debug_schedule_fuzz(cel_ctx* ctx, uint64_t seed, uint32_t max_us);
/* Tests only, host-only (no device): the plan of the byzantine replay in rsmt2d's sweep
 * order for a presence mask (2k*2k): for each solve in sequence its axis (0 row, 1 col),
 * index and level (solves of one level run together on the device; a solve's level is
 * one more than that of every earlier solve that filled a cell it reads). The outputs
 * hold up to 4k entries (each axis is solved at most once); *solved = 1 if the sweeps
 * complete the square. */
cel_status cel_debug_repair_plan(const uint8_t* present, uint32_t k, int32_t* solve_axis, int32_t* solve_index,
                                 int32_t* solve_level, uint32_t* nsolves, int32_t* solved);

/* ------------------------------------------------------- exported trees, proofs
 * pkg/proof (proof.go:78-202, row_proof.go, share_proof.go) and the subtree-root
 * cacher (pkg/inclusion/nmt_caching.go:96-124) need inner nodes, which the reference
 * gets by rebuilding row trees on the CPU. Here the device hashes the trees and
 * returns every node; proof building only selects nodes (host, no device).
 *
 * cel_axis_trees: all nodes of the NMTs of EDS axes [first, first + count) (axis 0 =
 * rows, row i = cells (i, 0..2k-1); 1 = columns), eds = 2k*2k*share host bytes.
 * nodes_out: count * (4k - 1) nodes of 90 B; per axis level-major from the 2k leaves
 * up to the root (leaf j at [j], level-1 node j at [2k + j], ..., root last). */
cel_status cel_axis_trees(cel_ctx* ctx, const uint8_t* eds, uint32_t k, uint32_t share_size,
                          uint32_t axis, uint32_t first, uint32_t count, uint8_t* nodes_out);
/* cel_axis_tree: all 4k - 1 nodes of the NMT of one axis from its 2k cells (contiguous
 * shares, the wrapper's pushed data), axis_index deciding the Q0 namespace rule as in
 * nmt_wrapper.go:100-107; same layout as one axis of cel_axis_trees. For
 * ErasuredNamespacedMerkleTree.ProveRange (nmt_wrapper.go:127-130) on a full axis. */
cel_status cel_axis_tree(cel_ctx* ctx, const uint8_t* cells, uint32_t k, uint32_t axis_index,
                         uint32_t share_size, uint8_t* nodes_out);
/* RFC-6962 tree over rowRoots || colRoots (w each, 2w a power of two), every level:
 * nodes_out (4w - 1) * 32 B, level 0 = the 2w leaf hashes, ..., the root last (equal to
 * cel_dah_hash). */
cel_status cel_dah_tree(cel_ctx* ctx, const uint8_t* row_roots, const uint8_t* col_roots,
                        uint32_t w, uint8_t* nodes_out);
/* nmt ProveRange(start, end) on one tree of cel_axis_trees (nleaves = 2k): the proof
 * nodes (90 B each, nmt order: maximal subtrees outside [start, end), left to right)
 * to nodes_out (nullable: count only) and their count to *nnodes. */
cel_status cel_nmt_prove_range(const uint8_t* tree_nodes, uint32_t nleaves, uint32_t start,
                               uint32_t end, uint8_t* nodes_out, uint32_t* nnodes);
/* merkle.ProofsFromByteSlices Aunts of item `index` (n items, a power of two) from a
 * cel_dah_tree table: leaf sibling first, 32 B each, count to *naunts. */
cel_status cel_merkle_aunts(const uint8_t* tree, uint32_t n, uint32_t index, uint8_t* aunts_out,
                            uint32_t* naunts);

/* Blob share commitments from an EDS (pkg/inclusion).
 * cel_commitment_paths: calculateCommitmentPaths (paths.go:16-47) for a blob of
 * blob_share_len shares placed at the first aligned index >= start of a square of
 * width square_size: per subtree root, its row and its (depth, position) inside the
 * row's ODS half (the reference walk is WalkLeft then the depth bits of position,
 * most significant first). n_out = count; arrays (nullable) hold up to cap entries.
 * cel_get_commitment: GetCommitment (get_commit.go:12-30) over device-built row
 * trees: the RFC-6962 root of those subtree roots (eds = 2k*2k*share host bytes). */
cel_status cel_commitment_paths(uint32_t square_size, uint32_t start, uint32_t blob_share_len,
                                uint32_t subtree_root_threshold, uint32_t* rows, uint32_t* depths,
                                uint32_t* positions, uint32_t cap, uint32_t* n_out);
/* calculateSubTreeRootCoordinates (paths.go:95-173): leaves [start, end) of a tree of
 * depth max_depth covered left to right by the largest aligned subtrees of depth >=
 * min_depth, as (depth, position) pairs. */
cel_status cel_subtree_root_coordinates(uint32_t max_depth, uint32_t min_depth, uint32_t start,
                                        uint32_t end, uint32_t* depths, uint32_t* positions,
                                        uint32_t cap, uint32_t* n_out);
cel_status cel_get_commitment(cel_ctx* ctx, const uint8_t* eds, uint32_t k, uint32_t share_size,
                              uint32_t start, uint32_t blob_share_len,
                              uint32_t subtree_root_threshold, uint8_t* commitment);

/* ---------------------------------------------------- data-square construction
 * go-square v1.1.0 (host code, no device needed):
 *   greedy = 0: square.Construct (app/extend_block.go:16-25, app/process_proposal.go:121-130):
 *               normal txs must precede blob txs; a tx that does not fit is an error
 *               (CEL_ETOOBIG "not enough space to append tx at index i",
 *               CEL_EINVAL "normal transaction at index i can not be appended after blob tx");
 *   greedy = 1: square.Build (app/prepare_proposal.go:48-61): txs that do not fit are
 *               skipped (the square orders kept normal txs before kept blob txs).
 * included (nullable, ntx bytes): 0 = tx not in the square, 1 = normal tx kept,
 * 2 = blob tx kept.
 * txs: the ntx transactions concatenated, tx_lens[ntx] their lengths.
 * max_square_size / subtree_root_threshold: appconsts SquareSizeUpperBound (128) and
 * SubtreeRootThreshold (64) (pkg/appconsts/v1,v2/app_consts.go).
 * Writes k*k shares (the ODS handed to cel_extend_shares) to shares_out (capacity
 * cap_shares shares; shares_out == NULL only reports *k_out). */
cel_status cel_square_construct(const uint8_t* txs, const uint32_t* tx_lens, uint32_t ntx,
                                uint32_t max_square_size, uint32_t subtree_root_threshold,
                                uint32_t greedy, uint8_t* shares_out, uint32_t cap_shares,
                                uint32_t* k_out, uint8_t* included);
/* go-square Builder.FindTxShareRange after Construct (pkg/proof/proof.go:21-48,
 * NewTxInclusionProof): the ODS shares [*start, *end) holding tx `tx_index` (a normal tx,
 * or the index wrapper of a blob tx, which lives in the PayForBlob namespace). */
cel_status cel_square_tx_range(const uint8_t* txs, const uint32_t* tx_lens, uint32_t ntx,
                               uint32_t max_square_size, uint32_t subtree_root_threshold,
                               uint32_t tx_index, uint32_t* start, uint32_t* end);
/* Message of the last cel_square_construct / cel_square_tx_range failure on this thread. */
const char* cel_square_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* CELESTIA_EDS_H */
