// C ABI of the same-run probes (include/celestia_eds.h, cel_probe_*): the ceilings a report
// prices the hot path against, measured on the ctx's device in the same process as the
// measurement itself, so a line from another box or clock carries its own denominators.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>
#include <vector>

#include "api_common.hpp"
#include "cel_internal.hpp"

using namespace cel;
using namespace cel::abi;

namespace {

// Best of `reps` timed launches of fn on s (one untimed warm-up launch first), in seconds.
template <class F>
hipError_t best_time(F fn, int reps, hipStream_t s, double* secs) {
  hipEvent_t a = nullptr, b = nullptr;
  hipError_t e = hipEventCreate(&a);
  if (e == hipSuccess) e = hipEventCreate(&b);
  if (e == hipSuccess) e = fn();
  double best = 1e30;
  for (int i = 0; i < reps && e == hipSuccess; i++) {
    if ((e = hipEventRecord(a, s)) != hipSuccess || (e = fn()) != hipSuccess || (e = hipEventRecord(b, s)) != hipSuccess ||
        (e = hipEventSynchronize(b)) != hipSuccess)
      break;
    float ms = 0;
    if ((e = hipEventElapsedTime(&ms, a, b)) != hipSuccess) break;
    best = std::min(best, (double)ms * 1e-3);
  }
  if (a) (void)hipEventDestroy(a);
  if (b) (void)hipEventDestroy(b);
  *secs = best;
  return e;
}

}  // namespace

extern "C" {

cel_status cel_probe_sha256(cel_ctx* ctx, double* g_compressions_per_s, double* shader_mhz) {
  if (!ctx || !g_compressions_per_s) return CEL_EINVAL;
  std::lock_guard<std::mutex> lock(ctx->mu);
  DeviceGuard g(ctx->device);
  int cus = 0, wall_khz = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess ||
      hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, ctx->device) != hipSuccess)
    return fail(ctx, CEL_EDEVICE, "device attributes");
  const uint32_t blocks = (uint32_t)cus * 16;  // 16 workgroups of 256 per CU (sha_rate.hip sweep)
  const int n = 64;                            // compressions per lane
  const uint32_t waves = blocks * 4;
  hipError_t e = hipSuccess;
  uint8_t* buf = static_cast<uint8_t*>(scratch(ctx, S_AUX, (size_t)blocks * 256 * 4 + (size_t)waves * 16, &e));
  if (!buf) return fail(ctx, CEL_ENOMEM, "device allocation failed");
  uint32_t* out = reinterpret_cast<uint32_t*>(buf);
  auto* clk = reinterpret_cast<unsigned long long*>(buf + (size_t)blocks * 256 * 4);
  hipStream_t s = ctx->stream;
  double secs = 0;
  e = best_time([&] { return launch_probe_sha(out, clk, blocks, n, s); }, 5, s, &secs);
  if (e != hipSuccess) return hip_fail(ctx, e, "sha probe");
  *g_compressions_per_s = (double)blocks * 256 * n / secs / 1e9;
  if (shader_mhz) {
    // the last launch's waves: shader-clock ticks per constant-rate tick
    std::vector<unsigned long long> h((size_t)waves * 2);
    if ((e = hipMemcpy(h.data(), clk, h.size() * 8, hipMemcpyDeviceToHost)) != hipSuccess)
      return hip_fail(ctx, e, "sha probe clock");
    double ticks = 0, real = 0;
    for (uint32_t i = 0; i < waves; i++) {
      ticks += (double)h[2 * i];
      real += (double)h[2 * i + 1];
    }
    *shader_mhz = real > 0 ? ticks / real * (wall_khz / 1e3) : 0.0;
  }
  return CEL_OK;
}

cel_status cel_probe_hbm_copy(cel_ctx* ctx, uint64_t bytes, double* gbps) {
  return cel_probe_hbm_stream(ctx, bytes, gbps, nullptr, nullptr);
}

cel_status cel_probe_hbm_stream(cel_ctx* ctx, uint64_t bytes, double* copy_gbps, double* read_gbps,
                                double* write_gbps) {
  if (!ctx || !copy_gbps || bytes < 2 * 4096) return CEL_EINVAL;
  std::lock_guard<std::mutex> lock(ctx->mu);
  DeviceGuard g(ctx->device);
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess)
    return fail(ctx, CEL_EDEVICE, "device attributes");
  const uint64_t half = (bytes / 2) & ~(uint64_t)4095;  // copy: read half, write half
  void *src = nullptr, *dst = nullptr;
  hipError_t e = hipMalloc(&src, half);
  if (e == hipSuccess) e = hipMalloc(&dst, half);
  if (e == hipSuccess) e = hipMemsetAsync(src, 0x5A, half, ctx->stream);
  // copy: the faster of {non-temporal, default policy}
  double secs = 1e30;
  for (int v = 0; v < 2 && e == hipSuccess; v++) {
    double t = 0;
    e = best_time([&] { return launch_probe_copy(src, dst, half, 0, 0, v == 0, ctx->stream); }, 5, ctx->stream, &t);
    secs = std::min(secs, t);
  }
  // read-only and write-only streams over the same half: the fastest of 4 / 8 / 16 workgroups
  // per CU (writes: also of 16 or 4 bytes per lane)
  double rsecs = 1e30, wsecs = 1e30;
  for (int v = 0; v < 9 && e == hipSuccess && (read_gbps || write_gbps); v++) {
    const int mode = v < 3 ? 1 : v < 6 ? 2 : 3;
    if ((mode == 1 && !read_gbps) || (mode != 1 && !write_gbps)) continue;
    const uint32_t blocks = (uint32_t)cus * (4u << (v % 3));
    double t = 0;
    e = best_time([&] { return launch_probe_copy(src, dst, half, blocks, mode, true, ctx->stream); }, 5, ctx->stream,
                  &t);
    (mode == 1 ? rsecs : wsecs) = std::min(mode == 1 ? rsecs : wsecs, t);
  }
  if (src) (void)hipFree(src);
  if (dst) (void)hipFree(dst);
  if (e != hipSuccess) return e == hipErrorOutOfMemory ? fail(ctx, CEL_ENOMEM, "device allocation failed")
                                                       : hip_fail(ctx, e, "hbm probe");
  *copy_gbps = 2.0 * (double)half / secs / 1e9;
  if (read_gbps) *read_gbps = (double)half / rsecs / 1e9;
  if (write_gbps) *write_gbps = (double)half / wsecs / 1e9;
  return CEL_OK;
}

cel_status cel_probe_rs_transform(cel_ctx* ctx, uint32_t k, double* us_per_square) {
  const bool gf16 = k == 256 || k == 512;
  if (!ctx || !us_per_square || (k != 32 && k != 64 && k != 128 && !gf16)) return CEL_EINVAL;
  std::lock_guard<std::mutex> lock(ctx->mu);
  DeviceGuard g(ctx->device);
  // one square's extension = 3k axis encodes (Q0 rows, then all 2k columns); a GF(2^8) tile
  // is one 256-byte slice of an axis, a GF(2^16) tile one 64-byte Leopard block. Time about
  // 196,608 tiles (~770 waves per CU).
  const uint32_t per_sq = 3 * k * (kShare / (gf16 ? 64 : 256));
  const uint32_t nsq = std::max(1u, (196608u + per_sq - 1) / per_sq), ntiles = per_sq * nsq;
  const size_t region = gf16 ? (size_t)kShare : (size_t)k * 256;  // what every tile reads
  hipError_t e = hipSuccess;
  uint8_t* buf = static_cast<uint8_t*>(scratch(ctx, S_AUX, 2 * region, &e));
  if (!buf) return fail(ctx, CEL_ENOMEM, "device allocation failed");
  hipStream_t s = ctx->stream;
  if ((e = hipMemsetAsync(buf, 0x3C, region, s)) != hipSuccess) return hip_fail(ctx, e, "rs probe");
  double secs = 0;
  e = best_time(
      [&] {
        return gf16 ? launch_probe_rs_transform_gf16(k, buf, buf + region, ntiles, s)
                    : launch_probe_rs_transform(k, reinterpret_cast<const uint32_t*>(buf),
                                                reinterpret_cast<uint32_t*>(buf + region), ntiles, 0, s);
      },
      5, s, &secs);
  if (e != hipSuccess) return hip_fail(ctx, e, "rs probe");
  *us_per_square = secs / nsq * 1e6;
  return CEL_OK;
}

}  // extern "C"
