// Shared helpers of the C-ABI host layer (api.cpp, api_repair.cpp): error reporting with
// the reference's messages, grow-only device scratch per ctx, device selection.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <string>

#include "cel_internal.hpp"

namespace cel {
namespace abi {

enum ScratchSlot { S_IN = 0, S_EDS = 1, S_WORK = 2, S_ROOTS = 3, S_AUX = 4, S_MASK = 5 };

inline cel_status fail(cel_ctx* ctx, cel_status st, const std::string& msg) {
  if (ctx) ctx->last_error = msg;
  return st;
}

inline cel_status hip_fail(cel_ctx* ctx, hipError_t e, const char* what) {
  return fail(ctx, CEL_EDEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

inline void* scratch(cel_ctx* ctx, int slot, size_t bytes, hipError_t* err) {
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

// Grow-only page-locked host staging of a ctx (calls on a ctx hold its lock, so one buffer
// serves them all): device results come back in one asynchronous copy into it, then a host
// memcpy to the caller's (often pageable) buffers. nullptr if the allocation fails.
inline void* host_stage(cel_ctx* ctx, size_t bytes) {
  if (ctx->hstage_size >= bytes) return ctx->hstage;
  if (ctx->hstage) (void)hipHostFree(ctx->hstage);
  ctx->hstage = nullptr;
  ctx->hstage_size = 0;
  // coherent: kernels may store results into it directly (the one-square DAH launch)
  if (hipHostMalloc(&ctx->hstage, bytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return nullptr;
  ctx->hstage_size = bytes;
  return ctx->hstage;
}

inline bool is_pow2(uint64_t n) { return n && !(n & (n - 1)); }

// da.SquareSize: RoundUpPowerOfTwo(ceil(sqrt(len))) (data_availability_header.go:205-215)
inline uint32_t square_size(uint32_t n) {
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

inline hipStream_t pick_stream(cel_ctx* ctx, void* stream) {
  return stream ? static_cast<hipStream_t>(stream) : ctx->stream;
}


inline cel_status validate_square(cel_ctx* ctx, uint32_t k, uint32_t share_size) {
  if (share_size != kShare)
    return fail(ctx, CEL_ECHUNK, "share size must be appconsts.ShareSize (512) on the device path");
  if (!is_pow2(k)) return fail(ctx, CEL_ENOTPOW2, "square width is not a power of 2: got " + std::to_string(k));
  if (k > 512) return fail(ctx, CEL_ETOOBIG, "square width " + std::to_string(k) + " exceeds the device path (512)");
  return CEL_OK;
}

}  // namespace abi
}  // namespace cel
