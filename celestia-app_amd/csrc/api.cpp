// C ABI of the MI355X EDS hot path (include/celestia_eds.h).
//
// Host-side mirror of the reference surface, in C++ because the reference host
// (Go) is compiled code and no Go toolchain is available here:
//   cel_extend_shares  <- da.ExtendShares + da.NewDataAvailabilityHeader
//                         (pkg/da/data_availability_header.go:65-75, :44-63)
//   cel_codec_*        <- rsmt2d.LeoRSCodec (pkg/appconsts/global_consts.go:92)
//   cel_axis_root      <- wrapper.ErasuredNamespacedMerkleTree Push/Root (pkg/wrapper/nmt_wrapper.go:93-124)
//   cel_dah_hash       <- DataAvailabilityHeader.Hash (data_availability_header.go:92-108)
//   cel_repair         <- rsmt2d ExtendedDataSquare.Repair [dep]
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

#include "cel_internal.hpp"

using namespace cel;

namespace {

enum ScratchSlot { S_IN = 0, S_EDS = 1, S_WORK = 2, S_ROOTS = 3, S_AUX = 4, S_MASK = 5 };

cel_status fail(cel_ctx* ctx, cel_status st, const std::string& msg) {
  if (ctx) ctx->last_error = msg;
  return st;
}

cel_status hip_fail(cel_ctx* ctx, hipError_t e, const char* what) {
  return fail(ctx, CEL_EDEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

void* scratch(cel_ctx* ctx, int slot, size_t bytes, hipError_t* err) {
  if (bytes == 0) bytes = 256;
  if (ctx->scratch_size[slot] >= bytes) return ctx->scratch[slot];
  if (ctx->scratch[slot]) (void)hipFree(ctx->scratch[slot]);
  ctx->scratch[slot] = nullptr;
  ctx->scratch_size[slot] = 0;
  void* p = nullptr;
  *err = hipMalloc(&p, bytes);
  if (*err != hipSuccess) return nullptr;
  ctx->scratch[slot] = p;
  ctx->scratch_size[slot] = bytes;
  return p;
}

bool is_pow2(uint64_t n) { return n && !(n & (n - 1)); }

// da.SquareSize: RoundUpPowerOfTwo(ceil(sqrt(len))) (data_availability_header.go:205-215)
uint32_t square_size(uint32_t n) {
  const uint32_t s = (uint32_t)std::ceil(std::sqrt((double)n));
  uint32_t r = 1;
  while (r < s) r <<= 1;
  return r;
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

hipStream_t pick_stream(cel_ctx* ctx, void* stream) {
  return stream ? static_cast<hipStream_t>(stream) : ctx->stream;
}

}  // namespace

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

static cel_status validate_square(cel_ctx* ctx, uint32_t k, uint32_t share_size) {
  if (share_size != kShare)
    return fail(ctx, CEL_ECHUNK, "share size must be appconsts.ShareSize (512) on the device path");
  if (!is_pow2(k)) return fail(ctx, CEL_ENOTPOW2, "square width is not a power of 2: got " + std::to_string(k));
  if (k > 512) return fail(ctx, CEL_ETOOBIG, "square width " + std::to_string(k) + " exceeds the device path (512)");
  return CEL_OK;
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

cel_status cel_extend_batch(cel_ctx* ctx, const uint8_t* ods, uint32_t n, uint32_t k, uint32_t share_size,
                            uint8_t* eds_out, uint8_t* row_roots, uint8_t* col_roots, uint8_t* dah,
                            int32_t* status_out, uint32_t flags) {
  if (!ctx) return CEL_EINVAL;
  std::lock_guard<std::mutex> lock(ctx->mu);
  if (!ods || !row_roots || !col_roots || !dah || !n) return fail(ctx, CEL_EINVAL, "nil argument");
  cel_status st = validate_square(ctx, k, share_size);
  if (st) return st;
  DeviceGuard g(ctx->device);
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
  uint8_t* d_out = static_cast<uint8_t*>(scratch(ctx, S_ROOTS, 2 * roots_b + (size_t)n * 32 + (size_t)n * 4, &e));
  if (!d_out) return fail(ctx, CEL_ENOMEM, "device allocation failed");
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
    hipStream_t ds = ctx->dl[c % cel_ctx::kPipe];
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
    if ((e = hipMemcpyAsync(row_roots + first * roots_sq, d_rr + first * roots_sq, cnt * roots_sq,
                            hipMemcpyDeviceToHost, cs)) != hipSuccess ||
        (e = hipMemcpyAsync(col_roots + first * roots_sq, d_cr + first * roots_sq, cnt * roots_sq,
                            hipMemcpyDeviceToHost, cs)) != hipSuccess ||
        (e = hipMemcpyAsync(dah + first * 32, d_dah + first * 32, (size_t)cnt * 32, hipMemcpyDeviceToHost, cs)) !=
            hipSuccess ||
        (e = hipMemcpyAsync(stv.data() + first, d_st + first, (size_t)cnt * 4, hipMemcpyDeviceToHost, cs)) !=
            hipSuccess)
      return hip_fail(ctx, e, "D2H");
    if ((e = hipEventRecord(ctx->ev_done[c % cel_ctx::kChunks], cs)) != hipSuccess ||
        (e = hipStreamWaitEvent(s, ctx->ev_done[c % cel_ctx::kChunks], 0)) != hipSuccess)
      return hip_fail(ctx, e, "event");
  }
  for (uint32_t i = 0; eds_out && i < nstreams; i++)
    if ((e = hipEventRecord(ctx->ev_dl[i], ctx->dl[i])) != hipSuccess ||
        (e = hipStreamWaitEvent(s, ctx->ev_dl[i], 0)) != hipSuccess)
      return hip_fail(ctx, e, "event");
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return hip_fail(ctx, e, "sync");
  cel_status worst = CEL_OK;
  for (uint32_t i = 0; i < n; i++) {
    if (status_out) status_out[i] = stv[i];
    if (stv[i] != CEL_OK && worst == CEL_OK) worst = stv[i];
  }
  if (worst == CEL_EORDER) return fail(ctx, CEL_EORDER, "invalid push order: leaf namespaces must be non-decreasing");
  return worst;
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
  const uint32_t rows = k / nranks, w = 2 * k / nranks;
  const uint64_t blk = (uint64_t)rows * w * kShare;  // one destination rank's block
  uint8_t* send = static_cast<uint8_t*>(d_send);
  uint32_t wlog = 0;
  while ((1u << wlog) < w) wlog++;
  RsGeom gm{};
  gm.in = static_cast<const uint8_t*>(d_ods_rows);
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
  hipError_t e = launch_rs_encode(gm, ctx->tables, pick_stream(ctx, stream));
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
  const uint32_t w = 2 * k / nranks;
  uint8_t* slab = static_cast<uint8_t*>(d_slab);
  hipStream_t s = pick_stream(ctx, stream);
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
  const bool order = (flags & CEL_FLAG_ORDER_CHECK) != 0;
  hipError_t e;
  if ((e = launch_rs_encode(gm, ctx->tables, s)) != hipSuccess) return hip_fail(ctx, e, "shard cols");
  if ((e = launch_slab_leaves(slab, k, rank * w, w, 0, 2 * k, d_work, order, true, s)) != hipSuccess ||
      (e = launch_slab_trees(k, w, static_cast<uint32_t*>(d_col_rec), static_cast<uint32_t*>(d_row_sub), d_status,
                             d_work, s)) != hipSuccess)
    return hip_fail(ctx, e, "shard commit");
  return CEL_OK;
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

// -------------------------------------------------------------------- trees

cel_status cel_axis_root(cel_ctx* ctx, const uint8_t* cells, uint32_t k, uint32_t axis_index, uint32_t share_size,
                         uint8_t* root_out, uint32_t flags) {
  if (!ctx) return CEL_EINVAL;
  std::lock_guard<std::mutex> lock(ctx->mu);
  if (!cells || !root_out || !k) return fail(ctx, CEL_EINVAL, "nil argument");
  if (share_size != kShare) return fail(ctx, CEL_ECHUNK, "share size must be 512 on the device path");
  if (axis_index + 1 > 2 * k)  // nmt_wrapper.go:94-96
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
  if (axis_index + 1 > 2 * k)  // nmt_wrapper.go:94-96
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

// ------------------------------------------------------------------- repair

// rsmt2d v0.14.0 ExtendedDataSquare.Repair [dep] (extendeddatacrossword.go), with the
// oracle's restatement (oracle/eds.c) as the checker. The crossword control loop runs on
// the host over the presence mask; decoding, re-encoding, byte comparisons and root
// computation run on the device over the EDS kept resident.
namespace {

// Axis lists of the passes of one repair: each pass gets its own slot of a page-locked
// host buffer and of the device index buffer, so its upload is asynchronous and no pass
// waits for the previous one's kernels (a pageable upload into one shared buffer
// serialised the host against the stream). Slots wrap with one stream sync.
constexpr uint32_t kIdxSlots = 64;

struct RepairBufs {
  uint32_t W;
  uint8_t* eds;
  uint8_t* mask;
  int32_t* list0;     // the first pass's axis list, right after the mask (one upload for both)
  uint8_t* dense[2];  // gathered axes of the solve passes, alternating (main stream)
  uint8_t* dmask;
  uint8_t* dchk;      // gathered axes of the check passes (side stream)
  uint8_t* dmask_chk;
  uint8_t* tmp;       // re-encoded parity halves (side stream)
  uint8_t* work;      // NMT workspace of the final verification
  uint8_t* roots;     // [2][W][90] row then column roots of the final verification, then flags
  uint8_t* hres;      // page-locked copy of roots + flags (one D2H at the end)
  size_t res_bytes;
  int32_t* idx;       // [kIdxSlots][W] device axis lists
  int32_t* hidx;      // [kIdxSlots][W] page-locked staging of the same
  uint8_t* hmask;     // [W][W] page-locked staging of the presence mask
  uint32_t slot;      // next free slot
  uint32_t solves;    // solve passes so far (which dense buffer is next)
  int32_t* flags;     // [2][W] encoding-check flags by (direction, axis), right after the roots
  // Two streams: the solve chain (gather -> decode -> scatter) runs on `main`; every
  // re-encode check (of the solved axes, the sanity and the orthogonal checks) runs on
  // `side`, off the chain's critical path: its outcome is only read at the end.
  hipStream_t main, side;
  hipEvent_t ev_main;     // the square after the main stream's latest pass
  hipEvent_t ev_side[2];  // the side stream is done with dense[i]
  hipEvent_t ev_done;     // the side stream's last check
};

// `list` into the next axis-list slot, uploaded on stream s. Every slot in flight: drain
// both streams (the side stream's compares read the lists too), then reuse.
static cel_status upload_list(cel_ctx* ctx, RepairBufs& b, const std::vector<int32_t>& list, hipStream_t s,
                              int32_t** d_list) {
  hipError_t e;
  if (b.slot == kIdxSlots) {
    if ((e = hipStreamSynchronize(b.main)) != hipSuccess || (e = hipStreamSynchronize(b.side)) != hipSuccess)
      return hip_fail(ctx, e, "sync");
    b.slot = 0;
  }
  int32_t* hidx = b.hidx + (size_t)b.slot * b.W;
  *d_list = b.idx + (size_t)b.slot * b.W;
  b.slot++;
  std::memcpy(hidx, list.data(), list.size() * 4);
  if ((e = hipMemcpyAsync(*d_list, hidx, list.size() * 4, hipMemcpyHostToDevice, s)) != hipSuccess)
    return hip_fail(ctx, e, "H2D");
  return CEL_OK;
}

// Randomised idle time in front of an enqueue point (cel_debug_schedule_fuzz; off = 0).
static cel_status fuzz(cel_ctx* ctx, hipStream_t s) {
  if (!ctx->fuzz_max_us) return CEL_OK;
  uint64_t x = (ctx->fuzz_state += 0x9E3779B97F4A7C15ull);  // splitmix64
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  x ^= x >> 31;
  const hipError_t e = launch_delay((uint32_t)(x % (ctx->fuzz_max_us + 1ull)), s);
  return e == hipSuccess ? CEL_OK : hip_fail(ctx, e, "delay");
}

// Re-encode check of na gathered axes at `dense` on stream s: the data half of each axis
// is encoded again and compared with its parity half; mismatches set flags[is_col*W + axis].
// k = 256, 512: one launch of the GF(2^16) register kernel in check mode; else encode into
// b.tmp and k_cmp.
static cel_status encode_check(cel_ctx* ctx, RepairBufs& b, uint32_t k, int is_col, uint32_t na, const uint8_t* dense,
                               const int32_t* idx, hipStream_t s) {
  const uint32_t W = 2 * k;
  RsGeom g{};
  g.in = dense;
  g.in_sq = (uint64_t)na * W * kShare;
  g.in_axis = (uint64_t)W * kShare;
  g.in_shard = kShare;
  g.out = b.tmp;
  g.out_sq = (uint64_t)na * k * kShare;
  g.out_axis = (uint64_t)k * kShare;
  g.out_shard = kShare;
  g.n = k;
  g.len = kShare;
  g.axes = na;
  g.nsq = 1;
  hipError_t e;
  if (k == 256 || k == 512) {  // GF(2^16): the register kernel compares with the parity half as it goes
    g.out = const_cast<uint8_t*>(dense) + (uint64_t)k * kShare;
    g.out_sq = g.in_sq;
    g.out_axis = g.in_axis;
    g.chk_flags = b.flags + (size_t)is_col * W;
    g.chk_idx = idx;
    if ((e = launch_rs_encode(g, ctx->tables, s)) != hipSuccess) return hip_fail(ctx, e, "encoding check");
    return CEL_OK;
  }
  if ((e = launch_rs_encode(g, ctx->tables, s)) != hipSuccess) return hip_fail(ctx, e, "re-encode");
  if ((e = launch_cmp(b.tmp, (uint64_t)k * kShare, dense + (uint64_t)k * kShare, (uint64_t)W * kShare,
                      (uint64_t)k * kShare, na, b.flags + (size_t)is_col * W, s, idx)) != hipSuccess)
    return hip_fail(ctx, e, "compare");
  return CEL_OK;
}

// Encoding check of na complete axes of the square (list idx on the device) on stream s:
// one in-place launch for k = 32..128 (k_rs_check_axes) and k = 256/512 (k_rs_gf16x in
// check mode), else gather into dchk and encode_check.
static cel_status check_in_square(cel_ctx* ctx, RepairBufs& b, uint32_t k, int is_col, uint32_t na,
                                  const int32_t* idx, hipStream_t s) {
  const uint32_t W = 2 * k;
  hipError_t e;
  if (k >= 32 && k <= kMaxGf8Width) {
    if ((e = launch_rs_check_axes(b.eds, k, idx, is_col, na, b.flags + (size_t)is_col * W, s)) != hipSuccess)
      return hip_fail(ctx, e, "encoding check");
    return CEL_OK;
  }
  if (k == 256 || k == 512) {  // the GF(2^16) register kernel in check mode, in place
    const uint64_t row = (uint64_t)W * kShare;
    RsGeom g{};
    g.in = b.eds;
    g.out = b.eds + (is_col ? (uint64_t)k * row : (uint64_t)k * kShare);
    g.in_axis = g.out_axis = is_col ? kShare : row;
    g.in_shard = g.out_shard = is_col ? row : kShare;
    g.in_sq = g.out_sq = row * W;
    g.n = k;
    g.len = kShare;
    g.axes = na;
    g.nsq = 1;
    g.chk_flags = b.flags + (size_t)is_col * W;
    g.chk_idx = idx;
    g.chk_axes = idx;
    if ((e = launch_rs_encode(g, ctx->tables, s)) != hipSuccess) return hip_fail(ctx, e, "encoding check");
    return CEL_OK;
  }
  if ((e = launch_gather_axes(b.eds, b.mask, W, idx, is_col, na, b.dchk, b.dmask_chk, s)) != hipSuccess)
    return hip_fail(ctx, e, "gather");
  return encode_check(ctx, b, k, is_col, na, b.dchk, idx, s);
}

// rsmt2d solveCrossword's decode of `list` (incomplete axes of one direction), in two
// halves so the host can put other side-stream work between them:
//   solve_issue  the decode on the main stream (in place in the square, or gather ->
//                decode -> scatter), then ev_main;
//   solve_check  the encoding check of the solved axes on the side stream, after ev_main.
// Nothing is synchronised: every flag is read back once at the end of the repair.
struct Issued {
  uint32_t na = 0;
  uint32_t d = 0;
  int32_t* idx = nullptr;
};

static cel_status solve_issue(cel_ctx* ctx, RepairBufs& b, uint32_t k, int is_col, const std::vector<int32_t>& list,
                              Issued* out, int32_t* uploaded = nullptr) {
  const Range range("repair.solve");
  const uint32_t W = 2 * k, na = (uint32_t)list.size();
  out->na = na;
  if (!na) return CEL_OK;
  const uint32_t d = out->d = b.solves++ & 1u;
  cel_status st;
  if (uploaded) out->idx = uploaded;  // `list` is already on the device there
  else if ((st = upload_list(ctx, b, list, b.main, &out->idx)) != CEL_OK) return st;
  if ((st = fuzz(ctx, b.main)) != CEL_OK) return st;
  const int32_t* idx = out->idx;
  hipError_t e;
  if (rs_decode_axis_supported(W, kShare)) {
    // register decoder in place: erased cells straight into the square (no gather /
    // scatter on the chain)
    if ((e = launch_rs_decode_in_square(b.eds, b.mask, W, idx, is_col, na, ctx->tables.mul8, b.main)) != hipSuccess ||
        (e = hipEventRecord(b.ev_main, b.main)) != hipSuccess)
      return hip_fail(ctx, e, "solve");
    return CEL_OK;
  }
  uint8_t* dense = b.dense[d];
  if ((e = hipStreamWaitEvent(b.main, b.ev_side[d], 0)) != hipSuccess ||  // the side stream is done with dense[d]
      (e = launch_gather_axes(b.eds, b.mask, W, idx, is_col, na, dense, b.dmask, b.main)) != hipSuccess ||
      (e = launch_rs_decode(dense, b.dmask, na, k, kShare, ctx->tables, nullptr, b.main)) != hipSuccess ||
      (e = launch_scatter_axes(b.eds, b.mask, W, idx, is_col, na, dense, b.main)) != hipSuccess ||
      (e = hipEventRecord(b.ev_main, b.main)) != hipSuccess)
    return hip_fail(ctx, e, "solve");
  return CEL_OK;
}

// The side half of a solve_issue, enqueued after it with ev_main that solve's record or a
// later one of the main stream (the axes it checks are final from their pass on). Dense
// path: it must be enqueued before the solve after next, which reuses dense[s.d] once
// this check has recorded ev_side[s.d].
static cel_status solve_check(cel_ctx* ctx, RepairBufs& b, uint32_t k, int is_col, const Issued& s) {
  if (!s.na) return CEL_OK;
  const uint32_t W = 2 * k;
  hipError_t e;
  if ((e = hipStreamWaitEvent(b.side, b.ev_main, 0)) != hipSuccess) return hip_fail(ctx, e, "event");
  cel_status st;
  if ((st = fuzz(ctx, b.side)) != CEL_OK) return st;
  if (rs_decode_axis_supported(W, kShare))  // the completed axes are checked in the square
    return check_in_square(ctx, b, k, is_col, s.na, s.idx, b.side);
  if ((st = encode_check(ctx, b, k, is_col, s.na, b.dense[s.d], s.idx, b.side)) != CEL_OK) return st;
  if ((e = hipEventRecord(b.ev_side[s.d], b.side)) != hipSuccess) return hip_fail(ctx, e, "event");
  return CEL_OK;
}

// Encoding check of complete axes (preRepairSanityCheck, and the orthogonal axes a solve
// completed) on the side stream. wait_main: after the main stream's latest work; without
// it the caller guarantees the axes are final in the side stream's order already (the
// orthogonal axes of a pass whose solve_check the side stream has passed).
static cel_status check_pass(cel_ctx* ctx, RepairBufs& b, uint32_t k, int is_col, const std::vector<int32_t>& list,
                             bool wait_main) {
  const Range range("repair.check");
  const uint32_t na = (uint32_t)list.size();
  if (!na) return CEL_OK;
  hipError_t e;
  if (wait_main &&
      ((e = hipEventRecord(b.ev_main, b.main)) != hipSuccess || (e = hipStreamWaitEvent(b.side, b.ev_main, 0)) != hipSuccess))
    return hip_fail(ctx, e, "event");
  int32_t* idx;
  cel_status st;
  if ((st = upload_list(ctx, b, list, b.side, &idx)) != CEL_OK || (st = fuzz(ctx, b.side)) != CEL_OK) return st;
  return check_in_square(ctx, b, k, is_col, na, idx, b.side);
}

// One check of the replay, in rsmt2d's order (oracle/eds.c orc_repair):
//   SANITY  an axis complete before the repair: root (else "bad root input"), encoding
//   SOLVE   an axis decoded by solve `solve`: encoding, root
//   ORTH    an axis that solve `solve` completed: root, encoding
struct Check {
  enum Kind { SANITY, SOLVE, ORTH } kind;
  int is_col;
  int32_t idx;
  int32_t solve;  // index into the solve log (-1 for SANITY)
};
struct Solve {
  int is_col;
  int32_t idx;
};

struct RepairOut {
  int32_t* bad_axis;
  int32_t* bad_index;
  uint8_t* byz_shares;   // nullable, W * 512
  uint8_t* byz_present;  // nullable, W
};

// a[i] bit j <-> a[j] bit i
static void transpose64(uint64_t* a) {
  uint64_t m = 0x00000000FFFFFFFFull;
  for (int j = 32; j != 0; j >>= 1, m ^= (m << j)) {
    for (int k = 0; k < 64; k = ((k | j) + 1) & ~j) {
      const uint64_t t = ((a[k] >> j) ^ a[k | j]) & m;
      a[k | j] ^= t;
      a[k] ^= t << j;
    }
  }
}

// The presence mask as bitsets by row and by column (bit j of axis i = cell j of it) with
// per-axis counts, so a solve's bookkeeping visits only the cells it fills.
struct MaskBits {
  uint32_t W, nw;
  std::vector<uint64_t> bits[2];  // [is_col][axis * nw + word]
  std::vector<uint32_t> cnt[2];
  uint64_t total = 0;
  MaskBits(const std::vector<uint8_t>& hm, uint32_t w) : W(w), nw((w + 63) / 64) {
    const uint32_t P = nw * 64;  // padded to whole 64x64 tiles for the transpose
    std::vector<uint64_t> rows((size_t)P * nw, 0), cols((size_t)P * nw, 0);
    for (uint32_t i = 0; i < W; i++) {
      const uint8_t* r = hm.data() + (size_t)i * W;
      for (uint32_t j = 0; j < W; j += 8) {
        uint64_t x = 0;
        const uint32_t n = W - j < 8 ? W - j : 8;
        std::memcpy(&x, r + j, n);  // bytes 0 / 1
        rows[(size_t)i * nw + j / 64] |= ((x * 0x0102040810204080ull) >> 56) << (j % 64);
      }
    }
    // cols = rows transposed, tile by tile
    uint64_t t[64];
    for (uint32_t bi = 0; bi < nw; bi++)
      for (uint32_t bj = 0; bj < nw; bj++) {
        for (int r = 0; r < 64; r++) t[r] = rows[(size_t)(bi * 64 + r) * nw + bj];
        transpose64(t);
        for (int r = 0; r < 64; r++) cols[(size_t)(bj * 64 + r) * nw + bi] = t[r];
      }
    rows.resize((size_t)W * nw);
    cols.resize((size_t)W * nw);
    bits[0] = std::move(rows);
    bits[1] = std::move(cols);
    for (int d = 0; d < 2; d++) {
      cnt[d].assign(W, 0);
      for (uint32_t i = 0; i < W; i++) {
        uint32_t c = 0;
        for (uint32_t q = 0; q < nw; q++) c += (uint32_t)__builtin_popcountll(bits[d][(size_t)i * nw + q]);
        cnt[d][i] = c;
      }
    }
    for (uint32_t i = 0; i < W; i++) total += cnt[0][i];
  }
  // A pass: every axis of `list` (direction is_col, ascending) gets all its cells.
  // orth[t] = the orthogonal axes that solve list[t] completes, ascending: those whose
  // missing cells all lie in listed axes, the last of them in list[t] (rsmt2d fills the
  // axes one by one in list order). Word operations over the bitsets, O(W^2 / 64).
  void fill_pass(int is_col, const std::vector<int32_t>& list, std::vector<std::vector<int32_t>>& orth) {
    std::vector<uint64_t> S(nw, 0);
    std::vector<int32_t> pos(W, -1);
    for (size_t t = 0; t < list.size(); t++) {
      S[(uint32_t)list[t] / 64] |= 1ull << ((uint32_t)list[t] % 64);
      pos[list[t]] = (int32_t)t;
    }
    orth.assign(list.size(), {});
    for (uint32_t j = 0; j < W; j++) {
      if (cnt[!is_col][j] == W) continue;
      uint64_t* a = bits[!is_col].data() + (size_t)j * nw;
      bool inside = true;
      int32_t last = -1;
      uint32_t c = 0;
      for (uint32_t q = 0; q < nw; q++) {
        const uint64_t valid = (q + 1) * 64 <= W ? ~0ull : ((1ull << (W % 64)) - 1);
        const uint64_t miss = ~a[q] & valid;
        if (miss & ~S[q]) inside = false;
        if (miss) last = (int32_t)(q * 64 + 63 - __builtin_clzll(miss));
        a[q] |= S[q];
        c += (uint32_t)__builtin_popcountll(a[q] & valid);
      }
      total += c - cnt[!is_col][j];
      cnt[!is_col][j] = c;
      if (inside && last >= 0) orth[pos[last]].push_back((int32_t)j);
    }
    for (int32_t i : list) {
      uint64_t* a = bits[is_col].data() + (size_t)i * nw;
      for (uint32_t q = 0; q < nw; q++) a[q] = (q + 1) * 64 <= W ? ~0ull : ((1ull << (W % 64)) - 1);
      cnt[is_col][i] = W;
    }
  }
};

// The final verification's results, read back in one copy: every root of the square and
// the encoding-check flags by (direction, axis).
struct Verify {
  const uint8_t* got;  // [2][W][90]
  const int32_t* flags;
  const uint8_t *row_roots, *col_roots;
  uint32_t W;
  bool root_ok(int is_col, int32_t i) const {
    const uint8_t* exp = (is_col ? col_roots : row_roots) + (size_t)i * kNode;
    return std::memcmp(got + (size_t)is_col * W * kNode + (size_t)i * kNode, exp, kNode) == 0;
  }
  bool enc_ok(int is_col, int32_t i) const { return flags[(size_t)is_col * W + i] == 0; }
  // rsmt2d's order of checks: the first that fails (index into order, -1 if none) and
  // its status
  long first_failure(const std::vector<Check>& order, cel_status* code) const {
    for (size_t t = 0; t < order.size(); t++) {
      const Check& c = order[t];
      bool ok = true;
      *code = CEL_EBYZANTINE;
      switch (c.kind) {
        case Check::SANITY:
          if (!root_ok(c.is_col, c.idx)) {
            *code = CEL_EBADROOT;
            ok = false;
          } else {
            ok = enc_ok(c.is_col, c.idx);
          }
          break;
        case Check::SOLVE: ok = enc_ok(c.is_col, c.idx) && root_ok(c.is_col, c.idx); break;
        case Check::ORTH: ok = root_ok(c.is_col, c.idx) && enc_ok(c.is_col, c.idx); break;
      }
      if (!ok) return (long)t;
    }
    return -1;
  }
};

// hm := the presence mask before solve `upto` of `solves` (each solve completes its axis)
static void rollback(std::vector<uint8_t>& hm, uint32_t W, const std::vector<Solve>& solves, size_t upto) {
  for (size_t t = 0; t < upto; t++) {
    const uint32_t i = (uint32_t)solves[t].idx;
    if (solves[t].is_col)
      for (uint32_t j = 0; j < W; j++) hm[(size_t)j * W + i] = 1;
    else
      std::memset(hm.data() + (size_t)i * W, 1, W);
  }
}

// Report a failing axis: status, axis, index, and for CEL_EBYZANTINE rsmt2d's
// ErrByzantineData.Shares: the axis's cells from the square (complete axes never change;
// cells of a solved axis present before its solve kept their bytes), with the axis's mask
// from hm (masked: hm is rolled back to the mask before the failing solve) or all present.
static cel_status fail_axis(cel_ctx* ctx, const RepairBufs& b, const std::vector<uint8_t>& hm, const RepairOut& out,
                            cel_status code, int is_col, int32_t idx, bool masked) {
  const uint32_t W = b.W;
  if (out.bad_axis) *out.bad_axis = is_col;
  if (out.bad_index) *out.bad_index = idx;
  if (code == CEL_EBYZANTINE && (out.byz_shares || out.byz_present)) {
    std::vector<uint8_t> axis((size_t)W * kShare);
    const uint8_t* src = b.eds + (is_col ? (size_t)idx * kShare : (size_t)idx * W * kShare);
    const hipError_t ce = is_col ? hipMemcpy2D(axis.data(), kShare, src, (size_t)W * kShare, kShare, W,
                                                hipMemcpyDeviceToHost)
                                 : hipMemcpy(axis.data(), src, axis.size(), hipMemcpyDeviceToHost);
    if (ce != hipSuccess) return hip_fail(ctx, ce, "byzantine shares");
    for (uint32_t j = 0; j < W; j++) {
      const uint8_t p = masked ? hm[is_col ? (size_t)j * W + (uint32_t)idx : (size_t)idx * W + j] : 1;
      if (out.byz_present) out.byz_present[j] = p;
      if (out.byz_shares) {
        if (p) std::memcpy(out.byz_shares + (size_t)j * kShare, axis.data() + (size_t)j * kShare, kShare);
        else std::memset(out.byz_shares + (size_t)j * kShare, 0, kShare);
      }
    }
  }
  const char* dir = is_col ? "col" : "row";
  return fail(ctx, code, code == CEL_EBADROOT
                             ? std::string("bad root input: ") + dir + " " + std::to_string(idx)
                             : std::string("byzantine ") + (is_col ? "column" : "row") + " " + std::to_string(idx));
}

// Commit every root of the square on the main stream beside the side stream's last checks,
// join the streams and read roots and flags back (one page-locked copy).
static cel_status verify_square(cel_ctx* ctx, RepairBufs& b, uint32_t k, int last_col, const Issued& last,
                                int pending_col, const std::vector<int32_t>& pending, Verify* v) {
  const uint32_t W = 2 * k;
  const size_t roots_b = (size_t)W * kNode;
  hipError_t e;
  cel_status st;
  if ((st = fuzz(ctx, b.main)) != CEL_OK) return st;
  // the last pass's checks go to the side stream ahead of the commit's dozen launches, so
  // they run beside its leaf hashing instead of trailing its tree levels
  if ((st = solve_check(ctx, b, k, last_col, last)) != CEL_OK ||
      (st = check_pass(ctx, b, k, pending_col, pending, false)) != CEL_OK)
    return st;
  if ((e = launch_commit(b.eds, k, 1, b.roots, b.roots + roots_b, nullptr, nullptr, b.work, false, b.main)) !=
      hipSuccess)
    return hip_fail(ctx, e, "roots");
  if ((e = hipEventRecord(b.ev_done, b.side)) != hipSuccess || (e = hipStreamWaitEvent(b.main, b.ev_done, 0)) != hipSuccess)
    return hip_fail(ctx, e, "join");
  if ((e = hipMemcpyAsync(b.hres, b.roots, b.res_bytes, hipMemcpyDeviceToHost, b.main)) != hipSuccess)
    return hip_fail(ctx, e, "D2H");
  if ((e = hipStreamSynchronize(b.main)) != hipSuccess) return hip_fail(ctx, e, "sync");
  v->got = b.hres;
  v->flags = reinterpret_cast<const int32_t*>(b.hres + (b.res_bytes - 2 * (size_t)W * 4));
  v->W = W;
  return CEL_OK;
}

// rsmt2d's own solve order, for a square the pass-parallel schedule found byzantine.
//
// solveCrossword sweeps `for i { solveCrosswordRow(i); solveCrosswordCol(i) }`, and on
// inconsistent data which axis fails first, and with which Shares, depends on that order.
// The host replays the sweeps over the mask alone (every solve completes its axis): the
// solve sequence, the orthogonal axes each solve completes, and each solve's level, one
// more than the highest level among the solves that filled a cell it reads. Solves of one
// level touch no cell another of them fills, so a level runs as one row and one column
// launch; level by level the device sees every axis exactly as rsmt2d's sequence does.
// hm0: the mask the repair started from; cells present in it still hold their bytes
// (every decoder stores erased cells only).
// rsmt2d's sweeps over the mask alone (every solve completes its axis): the solve
// sequence, each solve's level and the check order (SOLVE, then the ORTH axes it
// completes, ascending); cnt = known cells per axis at the end.
struct SweepPlan {
  std::vector<Solve> solves;
  std::vector<int32_t> level;
  std::vector<Check> order;
  std::vector<uint32_t> cnt[2];
  int32_t nlevels = 0;
  bool solved = false;
};

static SweepPlan plan_sweeps(const std::vector<uint8_t>& hm, uint32_t k) {
  const uint32_t W = 2 * k;
  const size_t cells = (size_t)W * W;
  SweepPlan p;
  std::vector<uint8_t> m(hm);
  p.cnt[0].assign(W, 0);
  p.cnt[1].assign(W, 0);
  auto& cnt = p.cnt;
  size_t total = 0;
  for (uint32_t i = 0; i < W; i++)
    for (uint32_t j = 0; j < W; j++)
      if (m[(size_t)i * W + j]) {
        cnt[0][i]++;
        cnt[1][j]++;
        total++;
      }
  std::vector<int32_t> lvl_of(cells, 0);
  p.solved = total == cells;
  while (!p.solved) {
    bool progress = false;
    for (uint32_t i = 0; i < W; i++)
      for (int d = 0; d < 2; d++) {
        if (cnt[d][i] == W || cnt[d][i] < k) continue;
        const size_t base_c = d ? i : (size_t)i * W, step = d ? W : 1;
        int32_t L = 0;
        for (uint32_t j = 0; j < W; j++) {
          const size_t c = base_c + j * step;
          if (m[c] && lvl_of[c] > L) L = lvl_of[c];
        }
        L++;
        const int32_t si = (int32_t)p.solves.size();
        p.order.push_back({Check::SOLVE, d, (int32_t)i, si});
        for (uint32_t j = 0; j < W; j++) {
          const size_t c = base_c + j * step;
          if (m[c]) continue;
          if (cnt[!d][j] == W - 1) p.order.push_back({Check::ORTH, !d, (int32_t)j, si});
          m[c] = 1;
          lvl_of[c] = L;
          cnt[!d][j]++;
          total++;
        }
        cnt[d][i] = W;
        p.solves.push_back({d, (int32_t)i});
        p.level.push_back(L);
        if (L > p.nlevels) p.nlevels = L;
        progress = true;
      }
    if (total == cells) p.solved = true;
    if (!progress) break;
  }
  return p;
}

static cel_status repair_exact(cel_ctx* ctx, RepairBufs& b, std::vector<uint8_t>& hm, uint32_t k,
                               const uint8_t* row_roots, const uint8_t* col_roots, const RepairOut& out) {
  const Range range("repair.exact");
  const uint32_t W = 2 * k;
  const size_t cells = (size_t)W * W;
  const SweepPlan plan = plan_sweeps(hm, k);
  const std::vector<Solve>& solves = plan.solves;
  const std::vector<int32_t>& level = plan.level;
  const std::vector<Check>& order = plan.order;
  const size_t S = solves.size();
  // order[first[t] .. first[t + 1]) = solve t's checks (SOLVE, then its ORTH axes)
  std::vector<size_t> first(S + 1, order.size());
  for (size_t o = 0; o < order.size(); o++)
    if (order[o].kind == Check::SOLVE) first[(size_t)order[o].solve] = o;
  const bool in_square = rs_decode_axis_supported(W, kShare);
  // roots of the checked axes: 96-byte records after the axes-roots workspace (b.work holds
  // the whole-square commit's workspace, which is larger)
  const size_t ws_axes = (axes_roots_workspace_size(k, W) + 255) & ~(size_t)255;
  uint32_t* d_rec = reinterpret_cast<uint32_t*>(b.work + ws_axes);
  std::vector<uint8_t> h_rec((size_t)2 * W * kNodeWords * 4);
  std::vector<int32_t> h_flags((size_t)2 * W);
  hipError_t e;
  cel_status st;
  // both streams are idle (verify_square synchronised the joined streams); the square keeps
  // the bytes of every cell known at the start (decoders store erased cells only)
  std::memcpy(b.hmask, hm.data(), cells);
  if ((e = hipMemcpyAsync(b.mask, b.hmask, cells, hipMemcpyHostToDevice, b.main)) != hipSuccess ||
      (e = hipMemsetAsync(b.flags, 0, 2 * (size_t)W * 4, b.main)) != hipSuccess)
    return hip_fail(ctx, e, "H2D");
  // The sequence runs in prefixes of CH solves. A prefix's solves depend only on earlier
  // solves, so each prefix runs level by level after the previous one; then its checks
  // (encoding and root of every axis it solves or completes) come back, and the first
  // failure in sweep order ends the replay there: rsmt2d returns at its first failing check.
  const size_t CH = std::max<size_t>(16, W / 4);
  for (size_t s0 = 0; s0 < S; s0 += CH) {
    const size_t s1 = std::min(S, s0 + CH);
    std::vector<int32_t> lists;
    struct Group {
      uint32_t off, n;
      int is_col;  // -1: mixed (register decoder, direction in bit 30)
    };
    std::vector<Group> groups;
    {
      int32_t lo = INT32_MAX, hi = 0;
      for (size_t t = s0; t < s1; t++) {
        lo = std::min(lo, level[t]);
        hi = std::max(hi, level[t]);
      }
      std::vector<std::vector<int32_t>> by[2];
      by[0].resize((size_t)(hi - lo + 1));
      by[1].resize((size_t)(hi - lo + 1));
      for (size_t t = s0; t < s1; t++) by[solves[t].is_col][(size_t)(level[t] - lo)].push_back(solves[t].idx);
      for (size_t L = 0; L < by[0].size(); L++) {
        if (in_square) {
          const uint32_t off = (uint32_t)lists.size();
          for (int d = 0; d < 2; d++)
            for (int32_t i : by[d][L]) lists.push_back(d ? (int32_t)((uint32_t)i | (1u << 30)) : i);
          if ((uint32_t)lists.size() > off) groups.push_back({off, (uint32_t)lists.size() - off, -1});
          continue;
        }
        for (int d = 0; d < 2; d++)
          if (!by[d][L].empty()) {
            groups.push_back({(uint32_t)lists.size(), (uint32_t)by[d][L].size(), d});
            lists.insert(lists.end(), by[d][L].begin(), by[d][L].end());
          }
      }
    }
    // the axes this prefix's checks look at, by direction (each axis is checked once)
    std::vector<int32_t> chk[2];
    for (size_t o = first[s0]; o < first[s1]; o++) chk[order[o].is_col].push_back(order[o].idx);
    const uint32_t off_chk0 = (uint32_t)lists.size();
    lists.insert(lists.end(), chk[0].begin(), chk[0].end());
    const uint32_t off_chk1 = (uint32_t)lists.size();
    lists.insert(lists.end(), chk[1].begin(), chk[1].end());
    std::memcpy(b.hidx, lists.data(), lists.size() * 4);
    if ((e = hipMemcpyAsync(b.idx, b.hidx, lists.size() * 4, hipMemcpyHostToDevice, b.main)) != hipSuccess)
      return hip_fail(ctx, e, "H2D");
    for (const Group& g : groups) {
      const int32_t* idx = b.idx + g.off;
      if ((st = fuzz(ctx, b.main)) != CEL_OK) return st;
      if (in_square) {
        e = launch_rs_decode_in_square(b.eds, b.mask, W, idx, g.is_col, g.n, ctx->tables.mul8, b.main);
      } else if ((e = launch_gather_axes(b.eds, b.mask, W, idx, g.is_col, g.n, b.dense[0], b.dmask, b.main)) ==
                     hipSuccess &&
                 (e = launch_rs_decode(b.dense[0], b.dmask, g.n, k, kShare, ctx->tables, nullptr, b.main)) ==
                     hipSuccess) {
        e = launch_scatter_axes(b.eds, b.mask, W, idx, g.is_col, g.n, b.dense[0], b.main);
      }
      if (e != hipSuccess) return hip_fail(ctx, e, "solve");
    }
    // encoding check and root of every checked axis, one direction at a time through dchk
    for (int d = 0; d < 2; d++) {
      const uint32_t na = (uint32_t)chk[d].size();
      if (!na) continue;
      const int32_t* idx = b.idx + (d ? off_chk1 : off_chk0);
      uint32_t* rec = d_rec + (size_t)d * W * kNodeWords;
      if ((e = launch_gather_axes(b.eds, b.mask, W, idx, d, na, b.dchk, b.dmask_chk, b.main)) != hipSuccess)
        return hip_fail(ctx, e, "gather");
      if ((st = encode_check(ctx, b, k, d, na, b.dchk, idx, b.main)) != CEL_OK) return st;
      if ((e = launch_axes_roots(b.dchk, k, idx, na, rec, b.work, b.main)) != hipSuccess)
        return hip_fail(ctx, e, "roots");
    }
    if ((e = hipMemcpyAsync(h_flags.data(), b.flags, h_flags.size() * 4, hipMemcpyDeviceToHost, b.main)) !=
            hipSuccess ||
        (e = hipMemcpyAsync(h_rec.data(), d_rec, h_rec.size(), hipMemcpyDeviceToHost, b.main)) != hipSuccess ||
        (e = hipStreamSynchronize(b.main)) != hipSuccess)
      return hip_fail(ctx, e, "D2H");
    // replay the prefix's checks in sweep order
    size_t pos[2] = {0, 0};
    for (size_t o = first[s0]; o < first[s1]; o++) {
      const Check& c = order[o];
      const uint8_t* got = h_rec.data() + ((size_t)c.is_col * W + pos[c.is_col]++) * kNodeWords * 4;
      const uint8_t* exp = (c.is_col ? col_roots : row_roots) + (size_t)c.idx * kNode;
      const bool root_ok = std::memcmp(got, exp, kNode) == 0;
      const bool enc_ok = h_flags[(size_t)c.is_col * W + (size_t)c.idx] == 0;
      if (!root_ok || !enc_ok) {
        rollback(hm, W, solves, (size_t)c.solve);
        return fail_axis(ctx, b, hm, out, CEL_EBYZANTINE, c.is_col, c.idx, c.kind == Check::SOLVE);
      }
    }
  }
  // not reached for a square the pass schedule found byzantine (the outcome does not depend
  // on the order when every check passes), kept for completeness
  if (!plan.solved) {
    rollback(hm, W, solves, S);
    return fail(ctx, CEL_EUNREPAIRABLE, "failed to solve data square");
  }
  std::fill(hm.begin(), hm.end(), (uint8_t)1);
  return CEL_OK;
}

// rsmt2d Repair over the EDS resident at b.eds. hm = host presence mask (updated: all
// ones on success, the mask before the failing solve on a byzantine / bad-root error,
// the mask after the last solve when stuck). No pass waits for the device. Root checks
// are deferred: an axis, once complete, never changes, so one commit pass over the final
// square gives every root rsmt2d checks on the way, and the checks are replayed in
// rsmt2d's order, reporting the first failure.
//
// The solves run in passes (every solvable row, then every solvable column, ...), which
// decodes whole directions at once. When every check passes, the outcome equals that of
// rsmt2d's sweep order (row i, then column i): all cells of the final square then agree
// with valid codewords whose roots match, so any order decodes the same bytes and passes
// the same checks, and the set of axes that can be solved is the same closure. Only a
// failing solve or orthogonal check depends on the order; that square is replayed in
// rsmt2d's order by repair_exact.
static cel_status repair_core(cel_ctx* ctx, RepairBufs& b, std::vector<uint8_t>& hm, uint32_t k,
                              const uint8_t* row_roots, const uint8_t* col_roots, const RepairOut& out) {
  const uint32_t W = 2 * k;
  const size_t cells = (size_t)W * W;
  hipStream_t s = b.main;
  hipError_t e = hipSuccess;
  cel_status st;
  // an early return leaves no side-stream work running on the ctx's scratch buffers
  struct SideDrain {
    hipStream_t side;
    ~SideDrain() { (void)hipStreamSynchronize(side); }
  } drain{b.side};
  // The first row pass goes to the device before the host builds its bookkeeping (the
  // mask bitsets, the sanity lists), which then runs beside the decode; its axis list
  // rides in the mask's upload.
  std::vector<int32_t> list, orth, first;
  for (uint32_t i = 0; i < W; i++) {  // hm bytes are 0 / 1: a word's popcount is its count
    const uint8_t* r = hm.data() + (size_t)i * W;
    uint32_t c = 0;
    uint32_t j = 0;
    for (; j + 8 <= W; j += 8) {
      uint64_t x;
      std::memcpy(&x, r + j, 8);
      c += (uint32_t)__builtin_popcountll(x);
    }
    for (; j < W; j++) c += r[j];
    if (c >= k && c < W) first.push_back((int32_t)i);
  }
  const size_t cells_a = (cells + 255) & ~(size_t)255;
  std::memcpy(b.hmask, hm.data(), cells);
  if (!first.empty()) std::memcpy(b.hmask + cells_a, first.data(), first.size() * 4);
  // the flags are the side stream's (its checks), zeroed there after the mask is up
  if ((e = hipMemcpyAsync(b.mask, b.hmask, cells_a + first.size() * 4, hipMemcpyHostToDevice, s)) != hipSuccess ||
      (e = hipEventRecord(b.ev_main, s)) != hipSuccess || (e = hipStreamWaitEvent(b.side, b.ev_main, 0)) != hipSuccess ||
      (e = hipMemsetAsync(b.flags, 0, 2 * (size_t)W * 4, b.side)) != hipSuccess)
    return hip_fail(ctx, e, "H2D");
  // Each pass's encoding check (side stream) is enqueued after the next pass's decode, so
  // the host's enqueue of it is off the solve chain (the checked axes are final from their
  // pass on; the dense path's buffer dense[d] is reused two passes later, after the check
  // has recorded ev_side[d]).
  Issued prev;
  int prev_col = 0;
  if ((st = solve_issue(ctx, b, k, 0, first, &prev, b.list0)) != CEL_OK) return st;
  bool first_issued = !first.empty();
  std::unique_ptr<Range> plan_range(new Range("repair.plan"));
  MaskBits mb(hm, W);
  std::vector<Check> order;
  std::vector<Solve> solves;
  // preRepairSanityCheck: for i: row i, column i
  {
    std::vector<int32_t> comp[2];
    for (uint32_t i = 0; i < W; i++)
      for (int is_col = 0; is_col < 2; is_col++)
        if (mb.cnt[is_col][i] == W) {
          order.push_back({Check::SANITY, is_col, (int32_t)i, -1});
          comp[is_col].push_back((int32_t)i);
        }
    for (int is_col = 0; is_col < 2; is_col++)
      if ((st = check_pass(ctx, b, k, is_col, comp[is_col], true)) != CEL_OK) return st;
  }
  // The orthogonal checks of a pass are issued after the next pass's decode (or the final
  // commit), so the host's enqueue of them is not on the solve chain; the side stream runs
  // them right after that pass's own encoding checks.
  std::vector<int32_t> pending;
  int pending_col = 0;
  plan_range.reset();
  // passes: all solvable rows, then all solvable columns, until solved or stuck
  bool solved = false;
  std::vector<std::vector<int32_t>> by_solve;
  for (;;) {
    bool progress = false;
    for (int is_col = 0; is_col < 2; is_col++) {
      list.clear();
      orth.clear();
      for (uint32_t i = 0; i < W; i++) {
        const uint32_t c = mb.cnt[is_col][i];
        if (c >= k && c < W) list.push_back((int32_t)i);
      }
      if (list.empty()) continue;
      if (first_issued) {  // the first row pass (the same list, issued above)
        first_issued = false;
      } else {
        Issued s1;
        if ((st = solve_issue(ctx, b, k, is_col, list, &s1)) != CEL_OK ||
            (st = solve_check(ctx, b, k, prev_col, prev)) != CEL_OK ||
            (st = check_pass(ctx, b, k, pending_col, pending, false)) != CEL_OK)
          return st;
        prev = s1;
        prev_col = is_col;
        pending.clear();
      }
      // sequential view of the pass: solve i fills its missing cells, completing the
      // orthogonal axes whose last missing cell it held
      const Range fill_range("repair.fill");
      mb.fill_pass(is_col, list, by_solve);
      for (size_t t = 0; t < list.size(); t++) {
        const int32_t si = (int32_t)solves.size();
        order.push_back({Check::SOLVE, is_col, list[t], si});
        for (int32_t j : by_solve[t]) {
          order.push_back({Check::ORTH, !is_col, j, si});
          orth.push_back(j);
        }
        solves.push_back({is_col, list[t]});
      }
      std::sort(orth.begin(), orth.end());
      // pending is empty here: the previous pass's orthogonal checks were issued (and
      // cleared) right after this pass's solve above, or this is the first pass
      pending.swap(orth);
      pending_col = !is_col;
      progress = true;
    }
    if (mb.total == cells) {
      solved = true;
      break;
    }
    if (!progress) break;
  }
  Verify v{nullptr, nullptr, row_roots, col_roots, W};
  if ((st = verify_square(ctx, b, k, prev_col, prev, pending_col, pending, &v)) != CEL_OK) return st;
  cel_status code;
  const long f = v.first_failure(order, &code);
  if (f >= 0) {
    const Check& c = order[(size_t)f];
    if (c.kind == Check::SANITY) return fail_axis(ctx, b, hm, out, code, c.is_col, c.idx, false);
    return repair_exact(ctx, b, hm, k, row_roots, col_roots, out);
  }
  if (!solved) {
    rollback(hm, W, solves, solves.size());
    return fail(ctx, CEL_EUNREPAIRABLE, "failed to solve data square");
  }
  std::fill(hm.begin(), hm.end(), (uint8_t)1);
  return CEL_OK;
}

static cel_status repair_bufs(cel_ctx* ctx, uint32_t k, bool own_eds, RepairBufs* b) {
  const uint32_t W = 2 * k;
  const size_t cells = (size_t)W * W, eds_b = cells * kShare;
  const size_t cells_a = (cells + 255) & ~(size_t)255;
  hipError_t e = hipSuccess;
  b->W = W;
  if (own_eds) b->eds = static_cast<uint8_t*>(scratch(ctx, S_EDS, eds_b, &e));
  b->dense[0] = static_cast<uint8_t*>(scratch(ctx, S_IN, 3 * eds_b, &e));
  b->tmp = static_cast<uint8_t*>(scratch(ctx, S_AUX, eds_b / 2 + (size_t)kIdxSlots * W * 4 + 256, &e));
  const size_t list_a = ((size_t)W * 4 + 255) & ~(size_t)255;
  b->mask = static_cast<uint8_t*>(scratch(ctx, S_MASK, 3 * cells_a + list_a, &e));
  b->work = static_cast<uint8_t*>(scratch(ctx, S_WORK, nmt_workspace_size(k, 1), &e));
  const size_t roots_a = (2 * (size_t)W * kNode + 255) & ~(size_t)255;
  b->res_bytes = roots_a + 2 * (size_t)W * 4;
  b->roots = static_cast<uint8_t*>(scratch(ctx, S_ROOTS, b->res_bytes, &e));
  if (!b->eds || !b->dense[0] || !b->tmp || !b->mask || !b->work || !b->roots)
    return fail(ctx, CEL_ENOMEM, "device allocation failed");
  b->dense[1] = b->dense[0] + eds_b;
  b->dchk = b->dense[1] + eds_b;
  b->list0 = reinterpret_cast<int32_t*>(b->mask + cells_a);
  b->dmask = b->mask + cells_a + list_a;
  b->dmask_chk = b->dmask + cells_a;
  b->flags = reinterpret_cast<int32_t*>(b->roots + roots_a);
  b->idx = reinterpret_cast<int32_t*>(b->tmp + eds_b / 2);
  const size_t cells_h = (cells + 255) & ~(size_t)255;
  // axis lists, mask + first list, results
  const size_t hb = (size_t)kIdxSlots * W * 4 + cells_h + list_a + b->res_bytes;
  if (ctx->hstage_size < hb) {
    if (ctx->hstage) (void)hipHostFree(ctx->hstage);
    ctx->hstage = nullptr;
    ctx->hstage_size = 0;
    if (hipHostMalloc(&ctx->hstage, hb, hipHostMallocDefault) != hipSuccess)
      return fail(ctx, CEL_ENOMEM, "page-locked allocation failed");
    ctx->hstage_size = hb;
  }
  b->hidx = static_cast<int32_t*>(ctx->hstage);
  b->hmask = static_cast<uint8_t*>(ctx->hstage) + (size_t)kIdxSlots * W * 4;
  b->hres = b->hmask + cells_h + list_a;
  b->slot = 0;
  b->solves = 0;
  // the side stream and the events are the batch pipeline's (the ctx lock is held)
  b->main = ctx->stream;
  b->side = ctx->sub[0];
  b->ev_main = ctx->ev_rs[0];
  b->ev_side[0] = ctx->ev_rs[1];
  b->ev_side[1] = ctx->ev_rs[2];
  b->ev_done = ctx->ev_rs[3];
  // no stale record of an earlier call may gate this one: both streams start from here
  if ((e = hipEventRecord(b->ev_side[0], b->side)) != hipSuccess || (e = hipEventRecord(b->ev_side[1], b->side)) != hipSuccess)
    return hip_fail(ctx, e, "event");
  return CEL_OK;
}

}  // namespace


cel_status cel_repair(cel_ctx* ctx, uint8_t* eds, uint8_t* present, uint32_t k, uint32_t share_size,
                      const uint8_t* row_roots, const uint8_t* col_roots, int32_t* bad_axis, int32_t* bad_index,
                      uint8_t* byz_shares, uint8_t* byz_present) {
  if (!ctx) return CEL_EINVAL;
  std::lock_guard<std::mutex> lock(ctx->mu);
  if (!eds || !present || !row_roots || !col_roots) return fail(ctx, CEL_EINVAL, "nil argument");
  cel_status st = validate_square(ctx, k, share_size);
  if (st) return st;
  if (bad_axis) *bad_axis = -1;
  if (bad_index) *bad_index = -1;
  DeviceGuard g(ctx->device);
  const uint32_t W = 2 * k;
  const size_t cells = (size_t)W * W, eds_b = cells * kShare;
  RepairBufs b{};
  if ((st = repair_bufs(ctx, k, true, &b)) != CEL_OK) return st;
  hipStream_t s = ctx->stream;
  hipError_t e;
  std::vector<uint8_t> hm(cells);
  for (size_t i = 0; i < cells; i++) hm[i] = present[i] != 0;
  if ((e = hipMemcpyAsync(b.eds, eds, eds_b, hipMemcpyHostToDevice, s)) != hipSuccess) return hip_fail(ctx, e, "H2D");
  st = repair_core(ctx, b, hm, k, row_roots, col_roots, RepairOut{bad_axis, bad_index, byz_shares, byz_present});
  if (st != CEL_OK && st != CEL_EBYZANTINE && st != CEL_EBADROOT && st != CEL_EUNREPAIRABLE) return st;
  // the (partially) repaired square goes back either way, with the mask it is valid under
  if ((e = hipMemcpyAsync(eds, b.eds, eds_b, hipMemcpyDeviceToHost, s)) != hipSuccess) return hip_fail(ctx, e, "D2H");
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return hip_fail(ctx, e, "sync");
  std::memcpy(present, hm.data(), cells);
  return st;
}

cel_status cel_debug_repair_plan(const uint8_t* present, uint32_t k, int32_t* solve_axis, int32_t* solve_index,
                                 int32_t* solve_level, uint32_t* nsolves, int32_t* solved) {
  if (!present || !solve_axis || !solve_index || !solve_level || !nsolves || !solved || !k || (k & (k - 1)) ||
      k > 512)
    return CEL_EINVAL;
  const size_t cells = (size_t)4 * k * k;
  std::vector<uint8_t> hm(cells);
  for (size_t i = 0; i < cells; i++) hm[i] = present[i] != 0;
  const SweepPlan p = plan_sweeps(hm, k);
  for (size_t t = 0; t < p.solves.size(); t++) {
    solve_axis[t] = p.solves[t].is_col;
    solve_index[t] = p.solves[t].idx;
    solve_level[t] = p.level[t];
  }
  *nsolves = (uint32_t)p.solves.size();
  *solved = p.solved ? 1 : 0;
  return CEL_OK;
}

cel_status cel_debug_schedule_fuzz(cel_ctx* ctx, uint64_t seed, uint32_t max_us) {
  if (!ctx) return CEL_EINVAL;
  std::lock_guard<std::mutex> lock(ctx->mu);
  if (max_us > 100000) return fail(ctx, CEL_EINVAL, "max_us above 100 ms");
  ctx->fuzz_state = seed;
  ctx->fuzz_max_us = max_us;
  return CEL_OK;
}

cel_status cel_dev_repair(cel_ctx* ctx, void* d_eds, uint8_t* present, uint32_t k, const uint8_t* row_roots,
                          const uint8_t* col_roots, int32_t* bad_axis, int32_t* bad_index, uint8_t* byz_shares,
                          uint8_t* byz_present) {
  if (!ctx) return CEL_EINVAL;
  std::lock_guard<std::mutex> lock(ctx->mu);
  if (!d_eds || !present || !row_roots || !col_roots) return fail(ctx, CEL_EINVAL, "nil argument");
  cel_status st = validate_square(ctx, k, kShare);
  if (st) return st;
  if (bad_axis) *bad_axis = -1;
  if (bad_index) *bad_index = -1;
  DeviceGuard g(ctx->device);
  const size_t cells = (size_t)4 * k * k;
  RepairBufs b{};
  b.eds = static_cast<uint8_t*>(d_eds);
  if ((st = repair_bufs(ctx, k, false, &b)) != CEL_OK) return st;
  std::vector<uint8_t> hm(cells);
  for (size_t i = 0; i < cells; i++) hm[i] = present[i] != 0;
  st = repair_core(ctx, b, hm, k, row_roots, col_roots, RepairOut{bad_axis, bad_index, byz_shares, byz_present});
  if (st == CEL_OK || st == CEL_EBYZANTINE || st == CEL_EBADROOT || st == CEL_EUNREPAIRABLE)
    std::memcpy(present, hm.data(), cells);
  return st;
}

}  // extern "C"
