// Multi-GPU inside the library (include/celestia_eds.h, "multi-GPU" section): one process,
// one host thread, several devices.
//
//   cel_shard_plan_*, cel_extend_sharded   config 3: one square row-sharded over ngpu devices
//                                           with the all-to-all transpose and the
//                                          record all-gather issued here over RCCL
//   cel_extend_batch_multi                 config 4: independent squares split over ngpu ctxs,
//                                          one host thread per ctx (cel_extend_batch each)
//
// Both replace, for a block too large for one device's share of the work, the same
// da.ExtendShares + da.NewDataAvailabilityHeader pair (pkg/da/data_availability_header.go:65-75,
// :44-63), so a Go node reaches configs 3 and 4 through cgo without torchrun.
//
// RCCL is loaded with dlopen on the first plan (librccl.so.1: the copy a process already has,
// e.g. PyTorch's, or ROCm's), so the single-device entry points never pull it in. One
// communicator rank per device (ncclCommInitAll) and every rank's work issued from this
// thread inside ncclGroupStart / ncclGroupEnd, NCCL's single-process multi-device pattern.
// RCCL refuses two ranks on one device ("Duplicate GPU detected", profiles/r3_rccl_probe.txt);
// a plan whose ctxs repeat a device therefore moves the same blocks with device copies
// (transport "copy") in the same schedule, which is how the plan's N > 1 schedule is tested
// on a one-GPU box. Distinct devices use RCCL, or hipMemcpyPeerAsync with peer access
// enabled (transport "peer") when CEL_FLAG_SHARD_PEERCOPY asks for it or when RCCL cannot
// start (not loadable, ncclCommInitAll failing): the plan then reports "peer-fallback" and
// keeps RCCL's message in cel_shard_plan_note, so a node's first multi-GPU run cannot come
// back empty-handed. One rank needs no collective (transport "local": the all-to-all is the
// identity, the row pass writes the slab in place, and the gather is the rank's own record
// block) unless CEL_FLAG_SHARD_EXCHANGE asks for the exchange through a one-rank RCCL
// communicator. The selection is shard_transport.hpp's (unit-tested on the host).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "api_common.hpp"
#include "cel_internal.hpp"
#include "shard_transport.hpp"

using namespace cel;
using namespace cel::abi;

namespace {

// The RCCL entry points the plan uses, resolved from librccl.so.1.
struct Rccl {
  decltype(&ncclCommInitAll) CommInitAll = nullptr;
  decltype(&ncclCommDestroy) CommDestroy = nullptr;
  decltype(&ncclGroupStart) GroupStart = nullptr;
  decltype(&ncclGroupEnd) GroupEnd = nullptr;
  decltype(&ncclSend) Send = nullptr;
  decltype(&ncclRecv) Recv = nullptr;
  decltype(&ncclAllGather) AllGather = nullptr;
  decltype(&ncclGetErrorString) GetErrorString = nullptr;
  decltype(&ncclGetVersion) GetVersion = nullptr;
  std::string error;
};

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      const char* e = dlerror();
      r.error = std::string("RCCL is not loadable: ") + (e ? e : "librccl.so.1");
      return;
    }
    bool ok = true;
    auto sym = [&](auto& fn, const char* name) {
      fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
      ok = ok && fn != nullptr;
    };
    sym(r.CommInitAll, "ncclCommInitAll");
    sym(r.CommDestroy, "ncclCommDestroy");
    sym(r.GroupStart, "ncclGroupStart");
    sym(r.GroupEnd, "ncclGroupEnd");
    sym(r.Send, "ncclSend");
    sym(r.Recv, "ncclRecv");
    sym(r.AllGather, "ncclAllGather");
    sym(r.GetErrorString, "ncclGetErrorString");
    sym(r.GetVersion, "ncclGetVersion");
    if (!ok) r.error = "librccl.so.1 lacks an NCCL entry point the plan needs";
  });
  return r;
}

}  // namespace

// One row-sharded square over ngpu devices: per-rank buffers, streams and communicators.
struct cel_shard_plan {
  using Transport = ShardTransport;
  static constexpr Transport kRccl = Transport::kRccl, kCopy = Transport::kCopy, kLocal = Transport::kLocal,
                             kPeer = Transport::kPeer;
  struct Rank {
    int device = 0;
    hipStream_t s = nullptr;
    DeviceTables tables;
    uint8_t* ods_rows = nullptr;  // [k/N][k][512]
    uint8_t* send = nullptr;      // [N][k/N][w][512] (the slab's top half when aliased)
    uint8_t* slab = nullptr;      // [2k][w][512]
    uint8_t* pack = nullptr;      // [2k + w + 1][96]: row subtrees, column roots, status record
    uint8_t* gathered = nullptr;  // [N][2k + w + 1][96] (the record block itself when local)
    uint8_t* work = nullptr;
    // rank 0: the finish's outputs, contiguous so one copy brings them back
    uint8_t* out = nullptr;  // row roots [2k][90] | col roots [2k][90] | dah [32] | status int32
    hipEvent_t ev_rows = nullptr, ev_exch = nullptr, ev_cols = nullptr;
  };
  uint32_t ngpu = 0, k = 0, w = 0, flags = 0;
  bool alias = false, ran = false;
  Transport transport = kRccl;
  bool fallback = false;  // RCCL could not start: copies instead (note says why)
  std::string note;
  std::vector<Rank> r;
  std::vector<ncclComm_t> comms;
  hipEvent_t ev_fin = nullptr;  // on rank 0's stream: the gather copies and the finish
  void* host_out = nullptr;     // page-locked copy of rank 0's `out`
  std::string last_error;
  std::mutex mu;

  size_t pack_bytes() const { return (size_t)(2 * k + w + 1) * CEL_NODE_RECORD; }
  size_t out_bytes() const { return (size_t)4 * k * kNode + 32 + 4; }
  uint64_t block_bytes() const { return (uint64_t)(k / ngpu) * w * kShare; }  // one all-to-all block
};

namespace {

cel_status plan_fail(cel_shard_plan* p, cel_status st, const std::string& msg) {
  p->last_error = msg;
  return st;
}

cel_status plan_hip(cel_shard_plan* p, hipError_t e, const char* what) {
  return plan_fail(p, CEL_EDEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

cel_status plan_nccl(cel_shard_plan* p, ncclResult_t e, const char* what) {
  return plan_fail(p, CEL_EDEVICE, std::string(what) + ": " + rccl().GetErrorString(e));
}

void plan_free(cel_shard_plan* p) {
  for (auto& rk : p->r) {
    DeviceGuard g(rk.device);
    if (rk.s) (void)hipStreamSynchronize(rk.s);
  }
  for (ncclComm_t c : p->comms)
    if (c) (void)rccl().CommDestroy(c);
  for (size_t i = 0; i < p->r.size(); i++) {
    auto& rk = p->r[i];
    DeviceGuard g(rk.device);
    for (uint8_t* b : {rk.ods_rows, rk.slab, rk.pack, rk.work, rk.out})
      if (b) (void)hipFree(b);
    if (rk.gathered && rk.gathered != rk.pack) (void)hipFree(rk.gathered);
    if (rk.send && !p->alias) (void)hipFree(rk.send);
    free_tables(&rk.tables);
    for (hipEvent_t ev : {rk.ev_rows, rk.ev_exch, rk.ev_cols})
      if (ev) (void)hipEventDestroy(ev);
    if (i == 0 && p->ev_fin) (void)hipEventDestroy(p->ev_fin);
    if (rk.s) (void)hipStreamDestroy(rk.s);
  }
  if (p->host_out) (void)hipHostFree(p->host_out);
}

// A ctx's host worker for cel_extend_batch_multi: one thread running posted jobs in order.
// Members before the thread, so the thread starts on constructed state.
struct CtxWorker {
  std::mutex m;
  std::condition_variable cv;
  std::deque<std::function<void()>> q;
  bool stop = false;
  std::thread th;
  CtxWorker() : th([this] { loop(); }) {}
  ~CtxWorker() {
    {
      std::lock_guard<std::mutex> l(m);
      stop = true;
    }
    cv.notify_one();
    th.join();
  }
  void post(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> l(m);
      q.push_back(std::move(f));
    }
    cv.notify_one();
  }
  void loop() {
    for (;;) {
      std::function<void()> f;
      {
        std::unique_lock<std::mutex> l(m);
        cv.wait(l, [&] { return stop || !q.empty(); });
        if (q.empty()) return;  // stop, queue drained
        f = std::move(q.front());
        q.pop_front();
      }
      f();
    }
  }
};

std::mutex g_worker_mu;  // creation of the ctxs' workers

CtxWorker* ctx_worker(cel_ctx* c) {
  std::lock_guard<std::mutex> l(g_worker_mu);
  if (!c->worker) c->worker = new CtxWorker();
  return static_cast<CtxWorker*>(c->worker);
}

// Device copy of `bytes` from (src_dev, src) to (dst_dev, dst) on stream s (of dst_dev).
hipError_t dcopy(void* dst, int dst_dev, const void* src, int src_dev, size_t bytes, hipStream_t s) {
  if (dst_dev == src_dev) return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s);
  return hipMemcpyPeerAsync(dst, dst_dev, src, src_dev, bytes, s);
}

}  // namespace

namespace cel {
void destroy_ctx_worker(cel_ctx* c) {
  std::lock_guard<std::mutex> l(g_worker_mu);
  delete static_cast<CtxWorker*>(c->worker);  // joins after the queued jobs
  c->worker = nullptr;
}
}  // namespace cel

extern "C" {

cel_status cel_shard_plan_create(cel_ctx* const* ctxs, uint32_t ngpu, uint32_t k, uint32_t flags,
                                 cel_shard_plan** out) {
  if (!out) return CEL_EINVAL;
  *out = nullptr;
  if (!ctxs || !ngpu) return CEL_EINVAL;
  for (uint32_t i = 0; i < ngpu; i++)
    if (!ctxs[i]) return CEL_EINVAL;
  cel_ctx* c0 = ctxs[0];
  if (k != 256 && k != 512)
    return fail(c0, CEL_EINVAL, "row-sharded mode supports k = 256 or 512 (GF(2^16)): got " + std::to_string(k));
  if (!is_pow2(ngpu) || ngpu > k)
    return fail(c0, CEL_EINVAL, "ngpu must be a power of two <= k: got " + std::to_string(ngpu));
  auto* p = new cel_shard_plan();
  p->ngpu = ngpu;
  p->k = k;
  p->w = 2 * k / ngpu;
  p->flags = flags;
  p->r.resize(ngpu);
  std::vector<int> devs(ngpu);
  for (uint32_t i = 0; i < ngpu; i++) devs[i] = p->r[i].device = ctxs[i]->device;
  const ShardChoice choice = shard_choose(devs.data(), ngpu, (flags & CEL_FLAG_SHARD_EXCHANGE) != 0,
                                          (flags & CEL_FLAG_SHARD_PEERCOPY) != 0);
  p->alias = choice.alias;  // one rank, no collective
  p->transport = choice.want;
  auto bail = [&](cel_status st, const std::string& msg) {
    c0->last_error = msg;
    plan_free(p);
    delete p;
    return st;
  };
  const size_t ods_b = (size_t)(k / ngpu) * k * kShare, slab_b = (size_t)2 * k * p->w * kShare;
  const size_t work_b = cel_dev_shard_workspace_size(k, ngpu);
  for (uint32_t i = 0; i < ngpu; i++) {
    auto& rk = p->r[i];
    DeviceGuard g(rk.device);
    hipError_t e = hipStreamCreateWithFlags(&rk.s, hipStreamNonBlocking);
    if (e == hipSuccess) e = upload_tables(&rk.tables);
    if (e == hipSuccess) e = hipMalloc(&rk.ods_rows, ods_b);
    if (e == hipSuccess) e = hipMalloc(&rk.slab, slab_b);
    if (e == hipSuccess) e = hipMalloc(&rk.pack, p->pack_bytes());
    if (e == hipSuccess) {
      if (p->alias)
        rk.gathered = rk.pack;
      else
        e = hipMalloc(&rk.gathered, (size_t)ngpu * p->pack_bytes());
    }
    if (e == hipSuccess) e = hipMalloc(&rk.work, work_b);
    if (e == hipSuccess) e = hipMemset(rk.pack, 0, p->pack_bytes());
    if (e == hipSuccess && i == 0) e = hipMalloc(&rk.out, p->out_bytes());
    if (e == hipSuccess) {
      if (p->alias)
        rk.send = rk.slab;  // one rank: the all-to-all is the identity, the row pass writes the slab
      else
        e = hipMalloc(&rk.send, (size_t)ngpu * p->block_bytes());
    }
    for (hipEvent_t* ev : {&rk.ev_rows, &rk.ev_exch, &rk.ev_cols})
      if (e == hipSuccess) e = hipEventCreateWithFlags(ev, hipEventDisableTiming);
    if (e == hipSuccess && i == 0) e = hipEventCreateWithFlags(&p->ev_fin, hipEventDisableTiming);
    if (e != hipSuccess)
      return bail(e == hipErrorOutOfMemory ? CEL_ENOMEM : CEL_EDEVICE,
                  std::string("shard plan: device ") + std::to_string(rk.device) + ": " + hipGetErrorString(e));
  }
  if (hipHostMalloc(&p->host_out, p->out_bytes(), hipHostMallocDefault) != hipSuccess)
    return bail(CEL_ENOMEM, "shard plan: page-locked host buffer");
  if (p->transport == cel_shard_plan::kRccl) {
    const Rccl& nc = rccl();
    bool ok = nc.error.empty();
    if (!ok) {
      p->note = nc.error;
    } else {
      p->comms.assign(ngpu, nullptr);
      const ncclResult_t r = nc.CommInitAll(p->comms.data(), (int)ngpu, devs.data());
      ok = r == ncclSuccess;
      if (!ok) {
        p->comms.clear();
        p->note = std::string("ncclCommInitAll: ") + nc.GetErrorString(r);
      }
    }
    p->transport = shard_settle(choice, ok);
    p->fallback = !ok;
  }
  if (p->transport == cel_shard_plan::kPeer) {
    // direct reads of the peers' buffers where the link allows it; hipMemcpyPeerAsync works
    // either way (staged by the runtime when it does not)
    for (uint32_t i = 0; i < ngpu; i++)
      for (uint32_t j = 0; j < ngpu; j++) {
        int can = 0;
        if (i == j || hipDeviceCanAccessPeer(&can, devs[i], devs[j]) != hipSuccess || !can) continue;
        DeviceGuard g(devs[i]);
        const hipError_t e = hipDeviceEnablePeerAccess(devs[j], 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
          return bail(CEL_EDEVICE, std::string("shard plan: peer access ") + std::to_string(devs[i]) + " -> " +
                                       std::to_string(devs[j]) + ": " + hipGetErrorString(e));
        (void)hipGetLastError();
      }
  }
  *out = p;
  return CEL_OK;
}

void cel_shard_plan_destroy(cel_shard_plan* plan) {
  if (!plan) return;
  plan_free(plan);
  delete plan;
}

const char* cel_shard_plan_transport(const cel_shard_plan* plan) {
  return plan ? shard_transport_name(plan->transport, plan->fallback) : "";
}

const char* cel_shard_plan_note(const cel_shard_plan* plan) { return plan ? plan->note.c_str() : ""; }

const char* cel_shard_plan_last_error(const cel_shard_plan* plan) { return plan ? plan->last_error.c_str() : ""; }

cel_status cel_shard_plan_upload(cel_shard_plan* p, const uint8_t* ods) {
  if (!p || !ods) return CEL_EINVAL;
  std::lock_guard<std::mutex> lock(p->mu);
  const size_t rows_b = (size_t)(p->k / p->ngpu) * p->k * kShare;
  for (uint32_t i = 0; i < p->ngpu; i++) {
    auto& rk = p->r[i];
    DeviceGuard g(rk.device);
    // the next upload must not overwrite rows a queued run still reads: stream order
    const hipError_t e = hipMemcpyAsync(rk.ods_rows, ods + i * rows_b, rows_b, hipMemcpyDefault, rk.s);
    if (e != hipSuccess) return plan_hip(p, e, "shard plan upload");
  }
  return CEL_OK;
}

// The all-to-all of one run on the ranks' streams: rank h receives block h of every rank r
// into its slab rows [r k/N, (r+1) k/N). Copy / peer transports wait for every rank's row pass
// (ev_rows) and record ev_exch; RCCL orders it on the streams itself.
static cel_status exchange(cel_shard_plan* p) {
  const uint32_t N = p->ngpu;
  const uint64_t blk = p->block_bytes();
  hipError_t e = hipSuccess;
  if (p->transport == cel_shard_plan::kCopy || p->transport == cel_shard_plan::kPeer) {
    for (uint32_t h = 0; h < N && e == hipSuccess; h++) {
      auto& dst = p->r[h];
      DeviceGuard g(dst.device);
      for (uint32_t r = 0; r < N && e == hipSuccess; r++) e = hipStreamWaitEvent(dst.s, p->r[r].ev_rows, 0);
      for (uint32_t r = 0; r < N && e == hipSuccess; r++)
        e = dcopy(dst.slab + r * blk, dst.device, p->r[r].send + h * blk, p->r[r].device, blk, dst.s);
      if (e == hipSuccess) e = hipEventRecord(dst.ev_exch, dst.s);
    }
    return e == hipSuccess ? CEL_OK : plan_hip(p, e, "shard exchange");
  }
  const Rccl& nc = rccl();
  ncclResult_t rc = nc.GroupStart();
  for (uint32_t r = 0; r < N && rc == ncclSuccess; r++) {
    auto& rk = p->r[r];
    for (uint32_t h = 0; h < N && rc == ncclSuccess; h++) {
      rc = nc.Send(rk.send + h * blk, blk, ncclUint8, (int)h, p->comms[r], rk.s);
      if (rc == ncclSuccess) rc = nc.Recv(rk.slab + h * blk, blk, ncclUint8, (int)h, p->comms[r], rk.s);
    }
  }
  const ncclResult_t rc2 = nc.GroupEnd();
  if (rc != ncclSuccess || rc2 != ncclSuccess) return plan_nccl(p, rc != ncclSuccess ? rc : rc2, "all-to-all");
  return CEL_OK;
}

// One square through the plan, asynchronous on the ranks' streams:
//   rows (each rank) -> all-to-all of the column blocks -> cols + slab commit (each rank)
//   -> all-gather of the record blocks -> finish (rank 0: row-root combine + DAH).
cel_status cel_shard_plan_run(cel_shard_plan* p) {
  if (!p) return CEL_EINVAL;
  std::lock_guard<std::mutex> lock(p->mu);
  const uint32_t N = p->ngpu, k = p->k;
  const bool order = (p->flags & CEL_FLAG_ORDER_CHECK) != 0;
  const size_t pb = p->pack_bytes();
  const bool copy = p->transport == cel_shard_plan::kCopy || p->transport == cel_shard_plan::kPeer;
  hipError_t e = hipSuccess;
  // 1. rows. With copy transport, a rank's send buffer and record block are read by other
  //    ranks' streams: wait for the previous run's exchange and gather first.
  for (uint32_t i = 0; i < N; i++) {
    auto& rk = p->r[i];
    DeviceGuard g(rk.device);
    if (copy && p->ran) {
      for (uint32_t h = 0; h < N && e == hipSuccess; h++) e = hipStreamWaitEvent(rk.s, p->r[h].ev_exch, 0);
      if (e == hipSuccess) e = hipStreamWaitEvent(rk.s, p->ev_fin, 0);
    }
    if (e == hipSuccess) e = shard_rows_enqueue(rk.tables, rk.ods_rows, k, N, rk.send, rk.s);
    if (e == hipSuccess && copy) e = hipEventRecord(rk.ev_rows, rk.s);
    if (e != hipSuccess) return plan_hip(p, e, "shard rows");
  }
  // 2. all-to-all: rank h receives block h of every rank r into slab rows [r k/N, (r+1) k/N)
  if (!p->alias) {
    const cel_status xs = exchange(p);
    if (xs) return xs;
  }
  // 3. cols + slab commit: the record block is [row subtrees 2k | column roots w | status]
  for (uint32_t i = 0; i < N; i++) {
    auto& rk = p->r[i];
    DeviceGuard g(rk.device);
    uint32_t* pack = reinterpret_cast<uint32_t*>(rk.pack);
    e = shard_cols_enqueue(rk.tables, rk.slab, k, N, i, pack + (size_t)2 * k * kNodeWords, pack,
                           reinterpret_cast<int32_t*>(pack + (size_t)(2 * k + p->w) * kNodeWords), rk.work, order,
                           rk.s);
    if (e == hipSuccess && copy) e = hipEventRecord(rk.ev_cols, rk.s);
    if (e != hipSuccess) return plan_hip(p, e, "shard cols");
  }
  // 4. gather every rank's record block (rank order)
  auto& r0 = p->r[0];
  if (p->transport == cel_shard_plan::kLocal) {
    // one rank: its record block is the gathered block (finish reads it in place)
  } else if (copy) {
    DeviceGuard g(r0.device);
    for (uint32_t r = 0; r < N && e == hipSuccess; r++) e = hipStreamWaitEvent(r0.s, p->r[r].ev_cols, 0);
    for (uint32_t r = 0; r < N && e == hipSuccess; r++)
      e = dcopy(r0.gathered + r * pb, r0.device, p->r[r].pack, p->r[r].device, pb, r0.s);
    if (e != hipSuccess) return plan_hip(p, e, "shard gather");
  } else {
    const Rccl& nc = rccl();
    ncclResult_t rc = nc.GroupStart();
    for (uint32_t r = 0; r < N && rc == ncclSuccess; r++)
      rc = nc.AllGather(p->r[r].pack, p->r[r].gathered, pb, ncclUint8, p->comms[r], p->r[r].s);
    const ncclResult_t rc2 = nc.GroupEnd();
    if (rc != ncclSuccess || rc2 != ncclSuccess) return plan_nccl(p, rc != ncclSuccess ? rc : rc2, "all-gather");
  }
  // 5. finish on rank 0
  {
    DeviceGuard g(r0.device);
    uint8_t* o = r0.out;
    e = launch_shard_finish(reinterpret_cast<const uint32_t*>(r0.gathered), k, N, o, o + 2 * k * kNode,
                            o + 4 * k * kNode, reinterpret_cast<int32_t*>(o + 4 * k * kNode + 32), r0.work, order,
                            r0.s);
    if (e == hipSuccess) e = hipEventRecord(p->ev_fin, r0.s);
    if (e != hipSuccess) return plan_hip(p, e, "shard finish");
  }
  p->ran = true;
  return CEL_OK;
}

// Waits for the queued runs and copies the last square's results out (every output
// nullable): roots and the DAH from rank 0, the EDS from each rank's column slab (columns
// [r w, (r+1) w) of every row; with CEL_FLAG_PARITY_ONLY in the plan's flags, Q0 cells are
// not written). Returns the square's push-order status (CEL_EORDER) or a device error.
cel_status cel_shard_plan_wait(cel_shard_plan* p, uint8_t* eds_out, uint8_t* row_roots, uint8_t* col_roots,
                               uint8_t* dah) {
  if (!p) return CEL_EINVAL;
  std::lock_guard<std::mutex> lock(p->mu);
  if (!p->ran) return plan_fail(p, CEL_EINVAL, "shard plan: nothing has run");
  const uint32_t k = p->k, W = 2 * k, w = p->w;
  hipError_t e = hipSuccess;
  if (eds_out) {
    const size_t rowb = (size_t)W * kShare;
    for (uint32_t i = 0; i < p->ngpu && e == hipSuccess; i++) {
      auto& rk = p->r[i];
      DeviceGuard g(rk.device);
      const uint32_t c0 = i * w, c1 = c0 + w;
      // top half: columns [max(c0, k), c1) unless Q0 is skipped; bottom half: all w columns
      const uint32_t t0 = (p->flags & CEL_FLAG_PARITY_ONLY) ? std::max(c0, k) : c0;
      if (t0 < c1)
        e = hipMemcpy2DAsync(eds_out + (size_t)t0 * kShare, rowb, rk.slab + (size_t)(t0 - c0) * kShare,
                             (size_t)w * kShare, (size_t)(c1 - t0) * kShare, k, hipMemcpyDeviceToHost, rk.s);
      if (e == hipSuccess)
        e = hipMemcpy2DAsync(eds_out + (size_t)k * rowb + (size_t)c0 * kShare, rowb,
                             rk.slab + (size_t)k * w * kShare, (size_t)w * kShare, (size_t)w * kShare, k,
                             hipMemcpyDeviceToHost, rk.s);
    }
    if (e != hipSuccess) return plan_hip(p, e, "shard plan download");
  }
  auto& r0 = p->r[0];
  {
    DeviceGuard g(r0.device);
    e = hipMemcpyAsync(p->host_out, r0.out, p->out_bytes(), hipMemcpyDeviceToHost, r0.s);
    if (e != hipSuccess) return plan_hip(p, e, "shard plan download");
  }
  for (auto& rk : p->r) {
    DeviceGuard g(rk.device);
    if ((e = hipStreamSynchronize(rk.s)) != hipSuccess) return plan_hip(p, e, "shard plan sync");
  }
  const uint8_t* h = static_cast<const uint8_t*>(p->host_out);
  if (row_roots) std::memcpy(row_roots, h, (size_t)W * kNode);
  if (col_roots) std::memcpy(col_roots, h + (size_t)W * kNode, (size_t)W * kNode);
  if (dah) std::memcpy(dah, h + (size_t)2 * W * kNode, 32);
  int32_t st = 0;
  std::memcpy(&st, h + (size_t)2 * W * kNode + 32, 4);
  if (st == CEL_EORDER) return plan_fail(p, CEL_EORDER, "invalid push order: leaf namespaces must be non-decreasing");
  return st ? plan_fail(p, st, "shard plan: device status " + std::to_string(st)) : CEL_OK;
}

// The all-to-all alone (bench.py's rowshard512_lib): one exchange to warm up, then `reps`
// back to back on every rank's stream, bracketed by timing events per rank after the queued
// runs drain; the longest rank's average. The send buffers and slabs hold whatever the last
// run left (the bytes moved are the same).
cel_status cel_shard_plan_time_exchange(cel_shard_plan* p, uint32_t reps, double* us_per_exchange) {
  if (!p || !us_per_exchange || !reps) return CEL_EINVAL;
  std::lock_guard<std::mutex> lock(p->mu);
  if (p->alias) return plan_fail(p, CEL_EINVAL, "shard plan: one rank in place, no exchange to time");
  const uint32_t N = p->ngpu;
  std::vector<hipEvent_t> a(N, nullptr), b(N, nullptr);
  hipError_t e = hipSuccess;
  cel_status st = CEL_OK;
  for (uint32_t i = 0; i < N && e == hipSuccess; i++) {
    DeviceGuard g(p->r[i].device);
    e = hipStreamSynchronize(p->r[i].s);
    if (e == hipSuccess) e = hipEventCreate(&a[i]);
    if (e == hipSuccess) e = hipEventCreate(&b[i]);
    if (e == hipSuccess) e = hipEventRecord(p->r[i].ev_rows, p->r[i].s);  // the copies' wait: satisfied
  }
  for (uint32_t it = 0; it <= reps && e == hipSuccess && !st; it++) {
    if (it == 1)
      for (uint32_t i = 0; i < N && e == hipSuccess; i++) {
        DeviceGuard g(p->r[i].device);
        e = hipEventRecord(a[i], p->r[i].s);
      }
    if (e == hipSuccess) st = exchange(p);
  }
  double worst = 0;
  for (uint32_t i = 0; i < N && e == hipSuccess && !st; i++) {
    DeviceGuard g(p->r[i].device);
    e = hipEventRecord(b[i], p->r[i].s);
    if (e == hipSuccess) e = hipEventSynchronize(b[i]);
    float ms = 0;
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, a[i], b[i]);
    worst = std::max(worst, (double)ms);
  }
  for (uint32_t i = 0; i < N; i++) {
    DeviceGuard g(p->r[i].device);
    if (a[i]) (void)hipEventDestroy(a[i]);
    if (b[i]) (void)hipEventDestroy(b[i]);
  }
  if (st) return st;
  if (e != hipSuccess) return plan_hip(p, e, "shard exchange timing");
  *us_per_exchange = worst * 1e3 / reps;
  return CEL_OK;
}

// da.ExtendShares + NewDataAvailabilityHeader for one square over ngpu devices. The plan
// (buffers, streams, communicators: ncclCommInitAll is the expensive part) is kept in
// ctxs[0] and reused while the device list, k and flags stay the same.
cel_status cel_extend_sharded(cel_ctx* const* ctxs, uint32_t ngpu, const uint8_t* ods, uint32_t k,
                              uint32_t share_size, uint8_t* eds_out, uint8_t* row_roots, uint8_t* col_roots,
                              uint8_t* dah, uint32_t flags) {
  if (!ctxs || !ngpu || !ctxs[0]) return CEL_EINVAL;
  cel_ctx* c0 = ctxs[0];
  std::lock_guard<std::mutex> lock(c0->mu);
  if (!ods || !row_roots || !col_roots || !dah) return fail(c0, CEL_EINVAL, "nil argument");
  if (share_size != kShare)
    return fail(c0, CEL_ECHUNK, "share size must be appconsts.ShareSize (512) on the device path");
  cel_shard_plan* p = c0->shard_cache;
  bool same = p && p->ngpu == ngpu && p->k == k && p->flags == flags;
  for (uint32_t i = 0; same && i < ngpu; i++) same = ctxs[i] && p->r[i].device == ctxs[i]->device;
  if (!same) {
    cel_shard_plan_destroy(p);
    c0->shard_cache = nullptr;
    cel_status st = cel_shard_plan_create(ctxs, ngpu, k, flags, &p);
    if (st) return st;  // message already in ctxs[0]
    c0->shard_cache = p;
  }
  cel_status st = cel_shard_plan_upload(p, ods);
  if (!st) st = cel_shard_plan_run(p);
  if (!st) st = cel_shard_plan_wait(p, eds_out, row_roots, col_roots, dah);
  if (st) c0->last_error = p->last_error;
  return st;
}

// Config 4 over several devices: squares [first_i, first_i + n_i) go to ctxs[i] (an equal
// split, the remainder to the first ctxs), each through cel_extend_batch on that ctx's host
// worker thread (ctxs[0]'s part on the caller's), so the ctxs' PCIe copies and kernels run
// side by side. The workers live as long as their ctx: a call posts its parts and waits on
// a per-call latch, no thread is started per call.
cel_status cel_extend_batch_multi(cel_ctx* const* ctxs, uint32_t ngpu, const uint8_t* ods, uint32_t n, uint32_t k,
                                  uint32_t share_size, uint8_t* eds_out, uint8_t* row_roots, uint8_t* col_roots,
                                  uint8_t* dah, int32_t* status_out, uint32_t flags) {
  if (!ctxs || !ngpu) return CEL_EINVAL;
  for (uint32_t i = 0; i < ngpu; i++)
    if (!ctxs[i]) return CEL_EINVAL;
  if (!ods || !row_roots || !col_roots || !dah || !n) return fail(ctxs[0], CEL_EINVAL, "nil argument");
  const uint64_t ods_sq = (uint64_t)k * k * share_size, eds_sq = 4 * ods_sq, roots_sq = (uint64_t)2 * k * kNode;
  std::vector<cel_status> st(ngpu, CEL_OK);
  std::vector<uint32_t> first(ngpu), cnt(ngpu);
  for (uint32_t i = 0, f = 0; i < ngpu; i++) {
    cnt[i] = n / ngpu + (i < n % ngpu ? 1 : 0);
    first[i] = f;
    f += cnt[i];
  }
  auto part = [&](uint32_t i) {
    const uint64_t f = first[i];
    st[i] = cel_extend_batch(ctxs[i], ods + f * ods_sq, cnt[i], k, share_size, eds_out ? eds_out + f * eds_sq : nullptr,
                             row_roots + f * roots_sq, col_roots + f * roots_sq, dah + f * 32,
                             status_out ? status_out + f : nullptr, flags);
  };
  std::mutex m;
  std::condition_variable cv;
  uint32_t pending = 0;
  for (uint32_t i = 1; i < ngpu; i++) {
    if (!cnt[i]) continue;
    {
      std::lock_guard<std::mutex> l(m);
      pending++;
    }
    ctx_worker(ctxs[i])->post([&, i] {
      part(i);
      std::lock_guard<std::mutex> l(m);
      if (--pending == 0) cv.notify_one();
    });
  }
  if (cnt[0]) part(0);
  {
    std::unique_lock<std::mutex> l(m);
    cv.wait(l, [&] { return pending == 0; });
  }
  // the first failing part's status; its message to ctxs[0] (order failures are per square),
  // read and written under each ctx's lock
  for (uint32_t i = 0; i < ngpu; i++)
    if (st[i] != CEL_OK) {
      if (ctxs[i] != ctxs[0]) {
        std::string msg;
        {
          std::lock_guard<std::mutex> l(ctxs[i]->mu);
          msg = ctxs[i]->last_error;
        }
        std::lock_guard<std::mutex> l(ctxs[0]->mu);
        ctxs[0]->last_error = msg;
      }
      return st[i];
    }
  return CEL_OK;
}

}  // extern "C"
