// C ABI of the MI355X EDS hot path (include/celestia_eds.h).
//
// Host-side mirror of the reference surface, in C++ because the reference host
// (Go) is compiled code and no Go toolchain is available here:
//   cel_extend_shares  <- da.ExtendShares + da.NewDataAvailabilityHeader
//                         (pkg/da/data_availability_header.go:65-75, :44-63)
//   cel_codec_*        <- rsmt2d.LeoRSCodec (pkg/appconsts/global_consts.go:92)
//   cel_axis_root      <- wrapper.ErasuredNamespacedMerkleTree Push/Root (pkg/wrapper/nmt_wrapper.go:93-124)
//   cel_dah_hash       <- DataAvailabilityHeader.Hash (data_availability_header.go:92-108)
//                         (these two and the exported trees: api_trees.cpp)
//   cel_dev_shard_*    <- the row-sharded square of config 3 (api_shard.cpp)
//   cel_repair         <- rsmt2d ExtendedDataSquare.Repair [dep] (api_repair.cpp)
// Every computation runs in the HIP kernels; this layer validates arguments with
// the reference's error semantics, stages host buffers and orders the launches.
// There is no CPU fallback: without a usable device every call fails with
// CEL_EDEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cmath>
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

cel_status cel_ctx_create(int device, cel_ctx** out) {
  if (!out) return CEL_EINVAL;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return CEL_EDEVICE;
  if (device < 0 || device >= n) return CEL_EINVAL;
  cel_ctx* ctx = new cel_ctx();
  ctx->device = device;
  DeviceGuard g(device);
  hipError_t e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
  for (int i = 0; i < cel_ctx::kPipe && e == hipSuccess; i++) e = hipStreamCreateWithFlags(&ctx->sub[i], hipStreamNonBlocking);
  for (int i = 0; i < cel_ctx::kChunks && e == hipSuccess; i++) {
    e = hipEventCreateWithFlags(&ctx->ev_done[i], hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->ev_rs[i], hipEventDisableTiming);
  }
  if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->ev_start, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->ev_ext, hipEventDisableTiming);
  for (int i = 0; i < cel_ctx::kPipe && e == hipSuccess; i++) {
    e = hipEventCreateWithFlags(&ctx->ev_dl[i], hipEventDisableTiming);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->dl[i], hipStreamNonBlocking);
  }
  if (e == hipSuccess) e = upload_tables(&ctx->tables);
  if (e != hipSuccess) {
    cel_ctx_destroy(ctx);
    return CEL_EDEVICE;
  }
  *out = ctx;
  return CEL_OK;
}

void cel_ctx_destroy(cel_ctx* ctx) {
  if (!ctx) return;
  destroy_ctx_worker(ctx);
  cel_shard_plan_destroy(ctx->shard_cache);
  {
    DeviceGuard g(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    for (int i = 0; i < 6; i++)
      if (ctx->scratch[i]) (void)hipFree(ctx->scratch[i]);
    if (ctx->hstage) (void)hipHostFree(ctx->hstage);
    free_tables(&ctx->tables);
    for (int i = 0; i < cel_ctx::kPipe; i++)
      if (ctx->sub[i]) (void)hipStreamDestroy(ctx->sub[i]);
    for (int i = 0; i < cel_ctx::kChunks; i++) {
      if (ctx->ev_done[i]) (void)hipEventDestroy(ctx->ev_done[i]);
      if (ctx->ev_rs[i]) (void)hipEventDestroy(ctx->ev_rs[i]);
    }
    if (ctx->ev_start) (void)hipEventDestroy(ctx->ev_start);
    if (ctx->ev_ext) (void)hipEventDestroy(ctx->ev_ext);
    for (int i = 0; i < cel_ctx::kPipe; i++) {
      if (ctx->dl[i]) {
        (void)hipStreamSynchronize(ctx->dl[i]);
        (void)hipStreamDestroy(ctx->dl[i]);
      }
      if (ctx->ev_dl[i]) (void)hipEventDestroy(ctx->ev_dl[i]);
    }
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  }
  delete ctx;
}

const char* cel_strerror(cel_status st) {
  switch (st) {
    case CEL_OK: return "ok";
    case CEL_EINVAL: return "invalid argument";
    case CEL_ENOTPOW2: return "number of shares is not a power of 2";
    case CEL_ECHUNK: return "chunk size must be a positive multiple of 64";
    case CEL_ETOOBIG: return "square too large for the device path";
    case CEL_EORDER: return "invalid push order: namespaces must be non-decreasing";
    case CEL_ETOOFEW: return "too few shards given";
    case CEL_EBYZANTINE: return "byzantine data: axis failed re-encoding or root verification";
    case CEL_EUNREPAIRABLE: return "failed to solve data square";
    case CEL_EDEVICE: return "HIP device error";
    case CEL_ENOMEM: return "device out of memory";
    case CEL_ESHORT: return "data is too short to contain namespace ID";
    case CEL_EPUSHPAST: return "pushed past predetermined square size";
    case CEL_EBADROOT: return "bad root input";
    case CEL_ENODATA: return "no shard data";
    default: return "unknown status";
  }
}

const char* cel_last_error(const cel_ctx* ctx) { return ctx ? ctx->last_error.c_str() : ""; }

cel_status cel_device_name(cel_ctx* ctx, char* buf, size_t len) {
  if (!ctx || !buf || !len) return CEL_EINVAL;
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, ctx->device) != hipSuccess) return CEL_EDEVICE;
  // the marketing name can be empty on a box (a driver without the product table): then
  // the PCI device id stands in for it
  if (p.name[0])
    std::snprintf(buf, len, "%s (%s, %d CUs)", p.name, p.gcnArchName, p.multiProcessorCount);
  else
    std::snprintf(buf, len, "AMD GPU %04x:%02x:%02x (%s, %d CUs)", p.pciDomainID, p.pciBusID, p.pciDeviceID,
                  p.gcnArchName, p.multiProcessorCount);
  return CEL_OK;
}

// ------------------------------------------------------------------ squares

// Chunking of a batch over the internal streams: chunk c runs RS extension then NMT +
// DAH on stream sub[c % kPipe]; the chunks start together, so one chunk's latency-bound
// tree top + DAH runs beside the other's work. Two chunks (profiles/r1g_pipe_chunks_ab.txt);
// chaining the extensions so each runs beside the previous chunk's hashing buys nothing,
// the step is the sum of the two VALU-bound phases (profiles/r2_pipe_overlap_ab.txt).
// Equal halves: uneven splits (5/8 .. 7/8 of the batch in the first chunk, so the small
// chunk's tree top would run under the large chunk's bulk) measured slower at both k=64
// B=128 and k=128 B=256 (profiles/r4_pipe_split_ab.txt).
constexpr uint32_t kPipeChunks = 2;

struct PipePlan {
  uint32_t nchunks;
  uint32_t first[kPipeChunks], cnt[kPipeChunks];
  size_t work_off[kPipeChunks], work_bytes;  // NMT workspace of each chunk
};

static PipePlan pipe_plan(uint32_t k, uint32_t n) {
  PipePlan p{};
  uint32_t c0 = n < 2 ? n : (n + 1) / 2;
  if (c0 >= n) c0 = n;
  if (c0 == 0) c0 = n;
  p.nchunks = c0 < n ? 2 : 1;
  p.first[0] = 0;
  p.cnt[0] = c0;
  p.first[1] = c0;
  p.cnt[1] = n - c0;
  size_t off = 0;
  for (uint32_t c = 0; c < p.nchunks; c++) {
    p.work_off[c] = off;
    off += (nmt_workspace_size(k, p.cnt[c]) + 255) & ~(size_t)255;
  }
  p.work_bytes = off;
  return p;
}

// Chunks of the host-buffer pipeline: the upload of chunk c + 1, the compute of chunk c
// and the copy-back of chunk c - 1 overlap (profiles/r1c_host_io.txt).
constexpr uint32_t kHostChunks = 4;

void* cel_host_alloc(size_t bytes) {
  void* p = nullptr;
  return hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault) == hipSuccess ? p : nullptr;
}

void cel_host_free(void* p) {
  if (p) (void)hipHostFree(p);
}

size_t cel_dev_workspace_size(uint32_t k, uint32_t n) {
  const size_t a = nmt_workspace_size(k, n), b = pipe_plan(k, n).work_bytes;
  return a > b ? a : b;
}


// n row-major k x k ODSs (host or device memory) -> Q0 of n row-major 2k x 2k EDSs.
static hipError_t place_ods(const void* src, uint32_t n, uint32_t k, void* d_eds, hipStream_t s) {
  const size_t w = (size_t)k * kShare, sq_ods = (size_t)k * w, sq_eds = 4 * sq_ods;
  for (uint32_t i = 0; i < n; i++) {
    const hipError_t e = hipMemcpy2DAsync(static_cast<uint8_t*>(d_eds) + i * sq_eds, 2 * w,
                                          static_cast<const uint8_t*>(src) + i * sq_ods, w, w, k, hipMemcpyDefault, s);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

cel_status cel_dev_place_ods(cel_ctx* ctx, const void* ods, uint32_t n, uint32_t k, void* d_eds, void* stream) {
  if (!ctx || !ods || !d_eds || !n) return CEL_EINVAL;
  std::lock_guard<std::mutex> lock(ctx->mu);
  cel_status st = validate_square(ctx, k, kShare);
  if (st) return st;
  DeviceGuard g(ctx->device);
  const hipError_t e = place_ods(ods, n, k, d_eds, pick_stream(ctx, stream));
  return e == hipSuccess ? CEL_OK : hip_fail(ctx, e, "place ods");
}

cel_status cel_dev_extend_only(cel_ctx* ctx, const void* d_ods, uint32_t n, uint32_t k, void* d_eds, void* stream) {
  if (!ctx || !d_eds || !n) return CEL_EINVAL;
  std::lock_guard<std::mutex> lock(ctx->mu);
  cel_status st = validate_square(ctx, k, kShare);
  if (st) return st;
  DeviceGuard g(ctx->device);
  const hipError_t e = launch_extend(static_cast<const uint8_t*>(d_ods), static_cast<uint8_t*>(d_eds), k, n,
                                     ctx->tables, pick_stream(ctx, stream));
  return e == hipSuccess ? CEL_OK : hip_fail(ctx, e, "extend");
}

cel_status cel_dev_commit_only(cel_ctx* ctx, const void* d_eds, uint32_t n, uint32_t k, void* d_row_roots,
                               void* d_col_roots, void* d_dah, int32_t* d_status, void* d_work, void* stream,
                               uint32_t flags) {
  if (!ctx || !d_eds || !n || !d_row_roots || !d_col_roots || !d_dah || !d_work) return CEL_EINVAL;
  std::lock_guard<std::mutex> lock(ctx->mu);
  cel_status st = validate_square(ctx, k, kShare);
  if (st) return st;
  DeviceGuard g(ctx->device);
  hipError_t e = launch_commit(static_cast<const uint8_t*>(d_eds), k, n, static_cast<uint8_t*>(d_row_roots),
                               static_cast<uint8_t*>(d_col_roots), static_cast<uint8_t*>(d_dah), d_status, d_work,
                               (flags & CEL_FLAG_ORDER_CHECK) != 0, pick_stream(ctx, stream));
  return e == hipSuccess ? CEL_OK : hip_fail(ctx, e, "commit");
}

cel_status cel_dev_extend_batch(cel_ctx* ctx, const void* d_ods, uint32_t n, uint32_t k, void* d_eds,
                                void* d_row_roots, void* d_col_roots, void* d_dah, int32_t* d_status, void* d_work,
                                void* stream, uint32_t flags) {
  if (!ctx || !d_eds || !n || !d_row_roots || !d_col_roots || !d_dah || !d_work) return CEL_EINVAL;
  std::lock_guard<std::mutex> lock(ctx->mu);
  cel_status st = validate_square(ctx, k, kShare);
  if (st) return st;
  DeviceGuard g(ctx->device);
  const PipePlan plan = pipe_plan(k, n);
  const uint64_t ods_sq = (uint64_t)k * k * kShare, eds_sq = 4 * ods_sq, roots_sq = (uint64_t)2 * k * kNode;
  hipStream_t us = pick_stream(ctx, stream);
  if (flags & CEL_FLAG_CALLER_STREAM) {
    // One chunk on the caller's stream, for a caller with several batches in flight on
    // its own streams; no internal stream is touched, so the batches do not meet on
    // shared hardware queues. Each such batch starts when the previous one's extension
    // is done: its (HBM-bound) extension runs beside the previous batch's leaf hashing,
    // its hashing beside the previous batch's latency-bound tree top and DAH
    // (profiles/r4_inflight_ab.txt).
    hipError_t e = ctx->ext_pending ? hipStreamWaitEvent(us, ctx->ev_ext, 0) : hipSuccess;
    if (e == hipSuccess)
      e = launch_extend(static_cast<const uint8_t*>(d_ods), static_cast<uint8_t*>(d_eds), k, n, ctx->tables, us);
    if (e == hipSuccess) e = hipEventRecord(ctx->ev_ext, us);
    if (e == hipSuccess)
      e = launch_commit(static_cast<const uint8_t*>(d_eds), k, n, static_cast<uint8_t*>(d_row_roots),
                        static_cast<uint8_t*>(d_col_roots), static_cast<uint8_t*>(d_dah), d_status, d_work,
                        (flags & CEL_FLAG_ORDER_CHECK) != 0, us);
    if (e != hipSuccess) return hip_fail(ctx, e, "extend batch");
    ctx->ext_pending = true;
    return CEL_OK;
  }
  hipError_t e = hipEventRecord(ctx->ev_start, us);
  for (uint32_t c = 0; c < plan.nchunks && e == hipSuccess; c++) {
    const uint32_t first = plan.first[c], cnt = plan.cnt[c];
    hipStream_t s = ctx->sub[c % cel_ctx::kPipe];
    if ((e = hipStreamWaitEvent(s, ctx->ev_start, 0)) != hipSuccess) break;
    const uint8_t* ods = d_ods ? static_cast<const uint8_t*>(d_ods) + first * ods_sq : nullptr;
    uint8_t* eds = static_cast<uint8_t*>(d_eds) + first * eds_sq;
    if ((e = launch_extend(ods, eds, k, cnt, ctx->tables, s)) != hipSuccess) break;
    e = launch_commit(eds, k, cnt, static_cast<uint8_t*>(d_row_roots) + first * roots_sq,
                      static_cast<uint8_t*>(d_col_roots) + first * roots_sq, static_cast<uint8_t*>(d_dah) + first * 32,
                      d_status ? d_status + first : nullptr, static_cast<uint8_t*>(d_work) + plan.work_off[c],
                      (flags & CEL_FLAG_ORDER_CHECK) != 0, s);
    if (e != hipSuccess) break;
    if ((e = hipEventRecord(ctx->ev_done[c], s)) != hipSuccess) break;
    e = hipStreamWaitEvent(us, ctx->ev_done[c], 0);
  }
  return e == hipSuccess ? CEL_OK : hip_fail(ctx, e, "extend batch");
}

static cel_status order_status(cel_ctx* ctx, int32_t st) {
  if (st == CEL_EORDER) return fail(ctx, CEL_EORDER, "invalid push order: leaf namespaces must be non-decreasing");
  return st;
}

// Device address of host memory the GPU can read directly (page-locked: cel_host_alloc,
// hipHostMalloc / hipHostRegister), or nullptr for pageable memory.
static const uint8_t* mapped_host(const uint8_t* p) {
  hipPointerAttribute_t at;
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();  // clear the sticky "invalid value" of a pageable pointer
    return nullptr;
  }
  if (at.type != hipMemoryTypeHost || !at.devicePointer || !at.hostPointer) return nullptr;
  return static_cast<const uint8_t*>(at.devicePointer) + (p - static_cast<const uint8_t*>(at.hostPointer));
}

// One square from host buffers, latency first: PrepareProposal and ProcessProposal extend
// one block at a time and keep only the header (app/prepare_proposal.go:61-92,
// app/process_proposal.go:138-156). Everything on one stream, so nothing waits on another
// queue (round 5: row chunks uploaded on a copy stream with the row passes waiting on
// their events serialized behind the whole upload, profiles/r5_header_host_timeline.txt):
//   - page-locked ODS: the row pass reads it straight from host memory over PCIe and
//     writes Q0 and Q1 (the upload and the row transform are one launch);
//     pageable ODS: one contiguous copy to the device first, then the row pass;
//   - the column pass, every leaf, the tree levels and the DAH;
//   - the DAH launch writes every result (roots, DAH, status) into page-locked staging
//     itself (round 4: four copies into pageable memory, each a staging kernel and a host
//     wait; round 5 first: one copy after the DAH launch).
// The EDS download, if asked for, runs on a download stream after the column pass.
static cel_status extend_one(cel_ctx* ctx, const uint8_t* ods, uint32_t k, uint8_t* eds_out, uint8_t* row_roots,
                             uint8_t* col_roots, uint8_t* dah, int32_t* status_out, uint32_t flags) {
  const size_t ods_b = (size_t)k * k * kShare, eds_b = 4 * ods_b, roots_b = (size_t)2 * k * kNode;
  const size_t out_b = (2 * roots_b + 32 + 4 + 15) & ~(size_t)15;
  hipError_t e = hipSuccess;
  // The GF(2^8) row pass reads a page-locked ODS straight over PCIe (256-byte segments per
  // shard: the upload and the row transform are one launch). The GF(2^16) row kernel reads
  // 64-byte segments, which cross PCIe at ~39 GB/s, so at k = 256 / 512, and for pageable
  // memory, DMA copies put the ODS into Q0 and the rows are extended in place (k=512 header
  // 4.82 -> 3.43 ms, k=256 1.24 -> 1.03 ms, profiles/r5_header_gf16_dma_ab.txt).
  const uint8_t* src = k <= kMaxGf8Width ? mapped_host(ods) : nullptr;
  uint8_t* d_eds = static_cast<uint8_t*>(scratch(ctx, S_EDS, eds_b, &e));
  uint8_t* d_work = static_cast<uint8_t*>(scratch(ctx, S_WORK, nmt_workspace_size(k, 1), &e));
  uint8_t* d_out = static_cast<uint8_t*>(scratch(ctx, S_ROOTS, out_b, &e));
  uint8_t* h_out = static_cast<uint8_t*>(host_stage(ctx, out_b));
  if (!d_eds || !d_work || !d_out || !h_out) return fail(ctx, CEL_ENOMEM, "allocation failed");
  uint8_t* h_dev = const_cast<uint8_t*>(mapped_host(h_out));
  if (!h_dev) return fail(ctx, CEL_EDEVICE, "page-locked staging is not mapped for the device");
  int32_t* d_st = reinterpret_cast<int32_t*>(d_out + 2 * roots_b + 32);
  hipStream_t s = ctx->stream, d = ctx->dl[0];
  auto enqueue = [&]() -> hipError_t {
    hipError_t r;
    const bool order = (flags & CEL_FLAG_ORDER_CHECK) != 0;
    const size_t rowb = (size_t)2 * k * kShare, odsrow = (size_t)k * kShare;
    uint32_t leaf0 = 0;  // EDS rows whose leaves are hashed already
    // Page-locked output: EDS rows [r0, r1) < k go back as soon as the row pass wrote them,
    // beside the later uploads, the column pass and the hashing (k=512 parity only 9.94 ->
    // 8.20 ms, full EDS 12.3 -> 10.6-11.0 ms; k <= 256 -2 %: profiles/r5_eds_early_dl_ab.txt).
    // A copy into pageable memory blocks this thread, so it stays after every launch.
    const bool early = eds_out && mapped_host(eds_out);
    auto dl_top = [&](uint32_t r0, uint32_t r1, int ev) -> hipError_t {
      hipError_t q;
      if ((q = hipEventRecord(ctx->ev_rs[ev], s)) != hipSuccess || (q = hipStreamWaitEvent(d, ctx->ev_rs[ev], 0)))
        return q;
      const size_t half = (size_t)k * kShare;
      return (flags & CEL_FLAG_PARITY_ONLY)
                 ? hipMemcpy2DAsync(eds_out + r0 * rowb + half, rowb, d_eds + r0 * rowb + half, rowb, half, r1 - r0,
                                    hipMemcpyDeviceToHost, d)
                 : hipMemcpyAsync(eds_out + r0 * rowb, d_eds + r0 * rowb, (r1 - r0) * rowb, hipMemcpyDeviceToHost, d);
    };
    if (k == 512 && mapped_host(ods)) {
      // One k=512 block from page-locked memory: 128 MiB crosses PCIe in 4 row chunks on a
      // copy stream, and each chunk's rows are extended and their leaves hashed on the
      // compute stream while the next one crosses (3.58 -> 3.43 ms; at k = 256 the chunks
      // cost more than they hide: profiles/r5_header_gf16_dma_ab.txt). The push-order check
      // of a chunk's first row reads the row above, which the previous chunk brought.
      constexpr uint32_t kUp = 4;
      const uint32_t rows = k / kUp;
      hipStream_t cp = ctx->dl[1];
      if ((r = hipEventRecord(ctx->ev_start, s)) != hipSuccess || (r = hipStreamWaitEvent(cp, ctx->ev_start, 0)))
        return r;
      for (uint32_t c = 0; c < kUp; c++) {
        const uint32_t r0 = c * rows;
        if ((r = hipMemcpy2DAsync(d_eds + r0 * rowb, rowb, ods + r0 * odsrow, odsrow, odsrow, rows,
                                  hipMemcpyHostToDevice, cp)) != hipSuccess ||
            (r = hipEventRecord(ctx->ev_done[c], cp)) != hipSuccess ||
            (r = hipStreamWaitEvent(s, ctx->ev_done[c], 0)) != hipSuccess ||
            (r = launch_extend_rows(d_eds, k, r0, r0 + rows, ctx->tables, s)) != hipSuccess ||
            (early && (r = dl_top(r0, r0 + rows, 1 + (int)c)) != hipSuccess) ||
            (r = launch_commit_leaves(d_eds, k, 1, d_work, order, r0, r0 + rows, c == 0, s)) != hipSuccess)
          return r;
      }
      leaf0 = k;
    } else {
      if (!src && (r = hipMemcpy2DAsync(d_eds, rowb, ods, odsrow, odsrow, k, hipMemcpyHostToDevice, s)) != hipSuccess)
        return r;
      if ((r = launch_extend_rows(d_eds, k, 0, k, ctx->tables, s, src)) != hipSuccess) return r;
      if (early && (r = dl_top(0, k, 1)) != hipSuccess) return r;
    }
    if ((r = launch_extend_cols(d_eds, k, 1, ctx->tables, s)) != hipSuccess) return r;
    if (eds_out &&
        ((r = hipEventRecord(ctx->ev_rs[0], s)) != hipSuccess || (r = hipStreamWaitEvent(d, ctx->ev_rs[0], 0))))
      return r;
    // the DAH launch writes every result into the page-locked staging itself
    if ((r = launch_commit_leaves(d_eds, k, 1, d_work, order, leaf0, 2 * k, leaf0 == 0, s)) != hipSuccess ||
        (r = launch_commit_trees(k, 1, d_out, d_out + roots_b, d_out + 2 * roots_b, d_st, d_work, s, h_dev,
                                 (uint32_t)out_b)) != hipSuccess)
      return r;
    if (eds_out) {
      // after every kernel is enqueued: a copy into pageable memory blocks the calling thread
      const size_t half = (size_t)k * kShare;
      r = early ? hipSuccess
          : (flags & CEL_FLAG_PARITY_ONLY)
              ? hipMemcpy2DAsync(eds_out + half, rowb, d_eds + half, rowb, half, k, hipMemcpyDeviceToHost, d)
              : hipMemcpyAsync(eds_out, d_eds, k * rowb, hipMemcpyDeviceToHost, d);
      if (r == hipSuccess)
        r = hipMemcpyAsync(eds_out + k * rowb, d_eds + k * rowb, k * rowb, hipMemcpyDeviceToHost, d);
      if (r == hipSuccess) r = hipEventRecord(ctx->ev_dl[0], d);
      if (r == hipSuccess) r = hipStreamWaitEvent(s, ctx->ev_dl[0], 0);
    }
    return r;
  };
  if ((e = enqueue()) != hipSuccess) return hip_fail(ctx, e, "extend square");
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return hip_fail(ctx, e, "sync");
  std::memcpy(row_roots, h_out, roots_b);
  std::memcpy(col_roots, h_out + roots_b, roots_b);
  std::memcpy(dah, h_out + 2 * roots_b, 32);
  int32_t stv = 0;
  std::memcpy(&stv, h_out + 2 * roots_b + 32, 4);
  if (status_out) *status_out = stv;
  return order_status(ctx, stv);
}

cel_status cel_extend_batch(cel_ctx* ctx, const uint8_t* ods, uint32_t n, uint32_t k, uint32_t share_size,
                            uint8_t* eds_out, uint8_t* row_roots, uint8_t* col_roots, uint8_t* dah,
                            int32_t* status_out, uint32_t flags) {
  if (!ctx) return CEL_EINVAL;
  std::lock_guard<std::mutex> lock(ctx->mu);
  if (!ods || !row_roots || !col_roots || !dah || !n) return fail(ctx, CEL_EINVAL, "nil argument");
  cel_status st = validate_square(ctx, k, share_size);
  if (st) return st;
  DeviceGuard g(ctx->device);
  if (n == 1 && k >= 32) return extend_one(ctx, ods, k, eds_out, row_roots, col_roots, dah, status_out, flags);
  const size_t ods_b = (size_t)n * k * k * kShare, eds_b = 4 * ods_b;
  const size_t roots_b = (size_t)n * 2 * k * kNode;
  hipError_t e = hipSuccess;
  // Chunked host pipeline: chunk c goes through upload (ODS into Q0) -> extension ->
  // commit -> download on internal stream c % kPipe, so the PCIe copies of one chunk
  // overlap the kernels and copies of the others (the copies dominate: 40 MiB of
  // PCIe traffic per k=128 square against ~50 us of kernels). Host buffers from
  // cel_host_alloc (pinned) make every copy asynchronous.
  const uint32_t nc = std::min<uint32_t>(n, kHostChunks);
  const uint32_t chunk = (n + nc - 1) / nc;
  const uint32_t nchunks = (n + chunk - 1) / chunk;
  const uint32_t nstreams = std::min<uint32_t>(nchunks, cel_ctx::kPipe);
  const size_t ws = nmt_workspace_size(k, chunk);
  uint8_t* d_eds = static_cast<uint8_t*>(scratch(ctx, S_EDS, eds_b, &e));
  if (!d_eds) return fail(ctx, CEL_ENOMEM, "device allocation failed");
  uint8_t* d_work = static_cast<uint8_t*>(scratch(ctx, S_WORK, nstreams * ws, &e));
  if (!d_work) return fail(ctx, CEL_ENOMEM, "device allocation failed");
  const size_t out_b = 2 * roots_b + (size_t)n * 32 + (size_t)n * 4;
  uint8_t* d_out = static_cast<uint8_t*>(scratch(ctx, S_ROOTS, out_b, &e));
  if (!d_out) return fail(ctx, CEL_ENOMEM, "device allocation failed");
  uint8_t* h_out = static_cast<uint8_t*>(host_stage(ctx, out_b));
  if (!h_out) return fail(ctx, CEL_ENOMEM, "page-locked allocation failed");
  uint8_t* d_rr = d_out;
  uint8_t* d_cr = d_out + roots_b;
  uint8_t* d_dah = d_out + 2 * roots_b;
  int32_t* d_st = reinterpret_cast<int32_t*>(d_out + 2 * roots_b + (size_t)n * 32);
  std::vector<int32_t> stv(n);
  hipStream_t s = ctx->stream;
  const uint64_t ods_sq = (uint64_t)k * k * kShare, eds_sq = 4 * ods_sq, roots_sq = (uint64_t)2 * k * kNode;
  if ((e = hipEventRecord(ctx->ev_start, s)) != hipSuccess) return hip_fail(ctx, e, "event");
  for (uint32_t c = 0; c < nchunks; c++) {
    const uint32_t first = c * chunk, cnt = (first + chunk <= n) ? chunk : n - first;
    hipStream_t cs = ctx->sub[c % cel_ctx::kPipe];
    uint8_t* eds_c = d_eds + first * eds_sq;
    if ((e = hipStreamWaitEvent(cs, ctx->ev_start, 0)) != hipSuccess ||
        (e = place_ods(ods + first * ods_sq, cnt, k, eds_c, cs)) != hipSuccess ||
        (e = launch_extend(nullptr, eds_c, k, cnt, ctx->tables, cs)) != hipSuccess ||
        (e = hipEventRecord(ctx->ev_rs[c % cel_ctx::kChunks], cs)) != hipSuccess ||
        (e = launch_commit(eds_c, k, cnt, d_rr + first * roots_sq, d_cr + first * roots_sq, d_dah + first * 32,
                           d_st + first, d_work + (c % cel_ctx::kPipe) * ws, (flags & CEL_FLAG_ORDER_CHECK) != 0,
                           cs)) != hipSuccess)
      return hip_fail(ctx, e, "extend batch");
  }
  // Downloads after every chunk is enqueued: a copy into pageable memory blocks the
  // calling thread, and the later chunks' kernels run meanwhile. A chunk's EDS goes back
  // on the download stream as soon as its extension is done, beside its own hashing.
  for (uint32_t c = 0; c < nchunks; c++) {
    const uint32_t first = c * chunk, cnt = (first + chunk <= n) ? chunk : n - first;
    hipStream_t cs = ctx->sub[c % cel_ctx::kPipe];
    uint8_t* eds_c = d_eds + first * eds_sq;
    // one download stream, chunks in order: one DMA stream at the link's rate (four
    // concurrent ones measured 1.75K -> 1.0K squares/s on the parity-only copies)
    hipStream_t ds = ctx->dl[0];
    if (eds_out && (e = hipStreamWaitEvent(ds, ctx->ev_rs[c % cel_ctx::kChunks], 0)) != hipSuccess)
      return hip_fail(ctx, e, "event");
    if (eds_out && (flags & CEL_FLAG_PARITY_ONLY)) {
      // Q1 (the right half of rows 0..k-1, one strided copy) then Q2|Q3 (contiguous)
      const size_t half = (size_t)k * kShare;
      for (uint32_t i = 0; i < cnt && e == hipSuccess; i++) {
        uint8_t* h = eds_out + (first + i) * eds_sq;
        const uint8_t* d = eds_c + i * eds_sq;
        if ((e = hipMemcpy2DAsync(h + half, 2 * half, d + half, 2 * half, half, k, hipMemcpyDeviceToHost, ds)) ==
            hipSuccess)
          e = hipMemcpyAsync(h + eds_sq / 2, d + eds_sq / 2, eds_sq / 2, hipMemcpyDeviceToHost, ds);
      }
      if (e != hipSuccess) return hip_fail(ctx, e, "D2H");
    } else if (eds_out && (e = hipMemcpyAsync(eds_out + first * eds_sq, eds_c, cnt * eds_sq, hipMemcpyDeviceToHost,
                                              ds)) != hipSuccess) {
      return hip_fail(ctx, e, "D2H");
    }
    if ((e = hipEventRecord(ctx->ev_done[c % cel_ctx::kChunks], cs)) != hipSuccess ||
        (e = hipStreamWaitEvent(s, ctx->ev_done[c % cel_ctx::kChunks], 0)) != hipSuccess)
      return hip_fail(ctx, e, "event");
  }
  if (eds_out && ((e = hipEventRecord(ctx->ev_dl[0], ctx->dl[0])) != hipSuccess ||
                  (e = hipStreamWaitEvent(s, ctx->ev_dl[0], 0)) != hipSuccess))
    return hip_fail(ctx, e, "event");
  // every result in one copy into page-locked staging (one D2H into pageable memory costs
  // a staging kernel and a host wait each: four of them per chunk were ~25 us apiece)
  if ((e = hipMemcpyAsync(h_out, d_out, out_b, hipMemcpyDeviceToHost, s)) != hipSuccess) return hip_fail(ctx, e, "D2H");
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return hip_fail(ctx, e, "sync");
  std::memcpy(row_roots, h_out, roots_b);
  std::memcpy(col_roots, h_out + roots_b, roots_b);
  std::memcpy(dah, h_out + 2 * roots_b, (size_t)n * 32);
  std::memcpy(stv.data(), h_out + 2 * roots_b + (size_t)n * 32, (size_t)n * 4);
  cel_status worst = CEL_OK;
  for (uint32_t i = 0; i < n; i++) {
    if (status_out) status_out[i] = stv[i];
    if (stv[i] != CEL_OK && worst == CEL_OK) worst = stv[i];
  }
  return order_status(ctx, worst);
}

cel_status cel_extend_shares(cel_ctx* ctx, const uint8_t* shares, uint32_t n_shares, uint32_t share_size,
                             uint8_t* eds_out, uint8_t* row_roots, uint8_t* col_roots, uint8_t* dah, uint32_t flags) {
  if (!ctx) return CEL_EINVAL;
  // data_availability_header.go:67-69
  if (!is_pow2(n_shares))
    return fail(ctx, CEL_ENOTPOW2, "number of shares is not a power of 2: got " + std::to_string(n_shares));
  const uint32_t k = square_size(n_shares);
  if ((uint64_t)k * k != n_shares)
    // rsmt2d.ComputeExtendedDataSquare rejects a share count that is not a perfect square
    return fail(ctx, CEL_EINVAL, "number of chunks must be a square number: got " + std::to_string(n_shares));
  return cel_extend_batch(ctx, shares, 1, k, share_size, eds_out, row_roots, col_roots, dah, nullptr, flags);
}

// -------------------------------------------------------------------- codec

uint64_t cel_codec_max_chunks(void) { return 32768ull * 32768ull; }
const char* cel_codec_name(void) { return "Leopard"; }
// rsmt2d LeoRSCodec.ValidateChunkSize: chunkSize % 64 == 0 (zero passes).
cel_status cel_codec_validate_chunk_size(uint32_t len) { return (len % 64) != 0 ? CEL_ECHUNK : CEL_OK; }

cel_status cel_codec_encode(cel_ctx* ctx, const uint8_t* data, uint32_t n, uint32_t len, uint8_t* parity) {
  if (!ctx) return CEL_EINVAL;
  std::lock_guard<std::mutex> lock(ctx->mu);
  if (!data || !parity || !n) return fail(ctx, CEL_EINVAL, "nil argument");
  if (cel_codec_validate_chunk_size(len)) return fail(ctx, CEL_ECHUNK, "shard size must be a multiple of 64");
  if (!is_pow2(n)) return fail(ctx, CEL_ENOTPOW2, "number of data shards is not a power of 2");
  if (n > kMaxGf16Width) return fail(ctx, CEL_ETOOBIG, "too many shards for the device path");
  if (len == 0) return fail(ctx, CEL_ENODATA, "no shard data");  // klauspost ErrShardNoData
  DeviceGuard g(ctx->device);
  hipError_t e = hipSuccess;
  const size_t b = (size_t)n * len;
  uint8_t* d_in = static_cast<uint8_t*>(scratch(ctx, S_IN, b, &e));
  uint8_t* d_out = static_cast<uint8_t*>(scratch(ctx, S_EDS, b, &e));
  if (!d_in || !d_out) return fail(ctx, CEL_ENOMEM, "device allocation failed");
  hipStream_t s = ctx->stream;
  if ((e = hipMemcpyAsync(d_in, data, b, hipMemcpyHostToDevice, s)) != hipSuccess) return hip_fail(ctx, e, "H2D");
  RsGeom gm{};
  gm.in = d_in;
  gm.out = d_out;
  gm.in_sq = gm.out_sq = b;
  gm.in_axis = gm.out_axis = b;
  gm.in_shard = gm.out_shard = len;
  gm.n = n;
  gm.len = len;
  gm.axes = 1;
  gm.nsq = 1;
  if ((e = launch_rs_encode(gm, ctx->tables, s)) != hipSuccess) return hip_fail(ctx, e, "encode");
  if ((e = hipMemcpyAsync(parity, d_out, b, hipMemcpyDeviceToHost, s)) != hipSuccess) return hip_fail(ctx, e, "D2H");
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return hip_fail(ctx, e, "sync");
  return CEL_OK;
}

cel_status cel_codec_decode(cel_ctx* ctx, uint8_t* shards, const uint8_t* present, uint32_t n, uint32_t len) {
  if (!ctx) return CEL_EINVAL;
  std::lock_guard<std::mutex> lock(ctx->mu);
  if (!shards || !present || !n) return fail(ctx, CEL_EINVAL, "nil argument");
  if (cel_codec_validate_chunk_size(len)) return fail(ctx, CEL_ECHUNK, "shard size must be a multiple of 64");
  if (!is_pow2(n)) return fail(ctx, CEL_ENOTPOW2, "number of data shards is not a power of 2");
  if (n > 1024) return fail(ctx, CEL_ETOOBIG, "too many shards for the device decoder");
  uint32_t have = 0;
  for (uint32_t i = 0; i < 2 * n; i++) have += present[i] ? 1 : 0;
  if (len == 0) return fail(ctx, CEL_ENODATA, "no shard data");  // klauspost ErrShardNoData
  if (have == 2 * n) return CEL_OK;
  if (have < n) return fail(ctx, CEL_ETOOFEW, "too few shards given");
  DeviceGuard g(ctx->device);
  hipError_t e = hipSuccess;
  const size_t b = (size_t)2 * n * len;
  uint8_t* d_sh = static_cast<uint8_t*>(scratch(ctx, S_IN, b, &e));
  uint8_t* d_pr = static_cast<uint8_t*>(scratch(ctx, S_MASK, 2 * n, &e));
  if (!d_sh || !d_pr) return fail(ctx, CEL_ENOMEM, "device allocation failed");
  hipStream_t s = ctx->stream;
  if ((e = hipMemcpyAsync(d_sh, shards, b, hipMemcpyHostToDevice, s)) != hipSuccess ||
      (e = hipMemcpyAsync(d_pr, present, 2 * n, hipMemcpyHostToDevice, s)) != hipSuccess)
    return hip_fail(ctx, e, "H2D");
  if ((e = launch_rs_decode(d_sh, d_pr, 1, n, len, ctx->tables, nullptr, s)) != hipSuccess)
    return hip_fail(ctx, e, "decode");
  if ((e = hipMemcpyAsync(shards, d_sh, b, hipMemcpyDeviceToHost, s)) != hipSuccess) return hip_fail(ctx, e, "D2H");
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return hip_fail(ctx, e, "sync");
  return CEL_OK;
}

cel_status cel_dev_decode(cel_ctx* ctx, void* d_shards, const void* d_present, uint32_t naxes, uint32_t n,
                          uint32_t len, void* stream) {
  if (!ctx) return CEL_EINVAL;
  std::lock_guard<std::mutex> lock(ctx->mu);
  if (!d_shards || !d_present || !naxes || !n) return fail(ctx, CEL_EINVAL, "nil argument");
  if (len == 0 || cel_codec_validate_chunk_size(len)) return fail(ctx, CEL_ECHUNK, "shard size must be a multiple of 64");
  if (!is_pow2(n)) return fail(ctx, CEL_ENOTPOW2, "number of data shards is not a power of 2");
  if (n > 1024) return fail(ctx, CEL_ETOOBIG, "too many shards for the device decoder");
  DeviceGuard g(ctx->device);
  const hipError_t e = launch_rs_decode(static_cast<uint8_t*>(d_shards), static_cast<const uint8_t*>(d_present), naxes,
                                        n, len, ctx->tables, nullptr, pick_stream(ctx, stream));
  return e == hipSuccess ? CEL_OK : hip_fail(ctx, e, "decode");
}

}  // extern "C"
