// Device helpers for rsmt2d-style Repair (ExtendedDataSquare.Repair, rsmt2d v0.14.0
// [dep]; not called inside celestia-app itself but used by celestia-node):
// gather axes out of a resident EDS, batch axis roots, byte comparison, scatter back.
#include <hip/hip_runtime.h>

#include "cel_internal.hpp"
#include "sha256_device.hpp"

namespace cel {

// dense[a][i] <- cell i of axis a (row axes: eds row idx[a]; column axes: eds column idx[a]).
__global__ __launch_bounds__(256) void k_gather_axes(const uint8_t* __restrict__ eds, const uint8_t* __restrict__ mask,
                                                     uint32_t W, const int32_t* __restrict__ idx, int is_col,
                                                     uint32_t naxes, uint8_t* __restrict__ dense,
                                                     uint8_t* __restrict__ dmask) {
  const uint64_t t = (uint64_t)blockIdx.x * 256u + threadIdx.x;  // one uint4 per thread
  const uint64_t per_axis = (uint64_t)W * (kShare / 16);
  if (t >= per_axis * naxes) return;
  const uint32_t a = (uint32_t)(t / per_axis);
  const uint32_t rem = (uint32_t)(t % per_axis);
  const uint32_t i = rem / (kShare / 16), q = rem % (kShare / 16);
  const uint32_t ax = (uint32_t)idx[a];
  const uint64_t cell = is_col ? (uint64_t)i * W + ax : (uint64_t)ax * W + i;
  reinterpret_cast<uint4*>(dense)[t] = reinterpret_cast<const uint4*>(eds + cell * kShare)[q];
  if (q == 0) dmask[(uint64_t)a * W + i] = mask[cell];
}

__global__ __launch_bounds__(256) void k_scatter_axes(uint8_t* __restrict__ eds, uint8_t* __restrict__ mask, uint32_t W,
                                                      const int32_t* __restrict__ idx, int is_col, uint32_t naxes,
                                                      const uint8_t* __restrict__ dense) {
  const uint64_t t = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  const uint64_t per_axis = (uint64_t)W * (kShare / 16);
  if (t >= per_axis * naxes) return;
  const uint32_t a = (uint32_t)(t / per_axis);
  const uint32_t rem = (uint32_t)(t % per_axis);
  const uint32_t i = rem / (kShare / 16), q = rem % (kShare / 16);
  const uint32_t ax = (uint32_t)idx[a];
  const uint64_t cell = is_col ? (uint64_t)i * W + ax : (uint64_t)ax * W + i;
  reinterpret_cast<uint4*>(eds + cell * kShare)[q] = reinterpret_cast<const uint4*>(dense)[t];
  if (q == 0) mask[cell] = 1;
}

// flags[a] |= 1 if the n bytes of a[axis] and b[axis] differ (uint4 granularity).
__global__ __launch_bounds__(256) void k_cmp(const uint8_t* __restrict__ x, uint64_t xstride,
                                             const uint8_t* __restrict__ y, uint64_t ystride, uint64_t bytes,
                                             uint32_t naxes, int32_t* __restrict__ flags,
                                             const int32_t* __restrict__ idx) {
  const uint64_t t = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  const uint64_t per = bytes / 16;
  if (t >= per * naxes) return;
  const uint32_t a = (uint32_t)(t / per);
  const uint64_t q = t % per;
  const uint4 u = reinterpret_cast<const uint4*>(x + a * xstride)[q];
  const uint4 v = reinterpret_cast<const uint4*>(y + a * ystride)[q];
  if (u.x != v.x || u.y != v.y || u.z != v.z || u.w != v.w) atomicOr(flags + (idx ? idx[a] : (int32_t)a), 1);
}

// Schedule fuzzing (cel_debug_schedule_fuzz): one wave that idles for `ticks` of the
// 100 MHz constant clock, so a stream's next operation starts later. The loop reads only
// the clock, so it always ends.
__global__ __launch_bounds__(64) void k_delay(uint64_t ticks) {
  const uint64_t t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

hipError_t launch_delay(uint32_t us, hipStream_t s) {
  hipLaunchKernelGGL(k_delay, dim3(1), dim3(64), 0, s, (uint64_t)us * 100u);
  return hipGetLastError();
}

hipError_t launch_gather_axes(const uint8_t* eds, const uint8_t* mask, uint32_t W, const int32_t* idx, int is_col,
                              uint32_t naxes, uint8_t* dense, uint8_t* dmask, hipStream_t s) {
  const uint64_t total = (uint64_t)naxes * W * (kShare / 16);
  hipLaunchKernelGGL(k_gather_axes, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, eds, mask, W, idx, is_col,
                     naxes, dense, dmask);
  return hipGetLastError();
}

hipError_t launch_scatter_axes(uint8_t* eds, uint8_t* mask, uint32_t W, const int32_t* idx, int is_col,
                               uint32_t naxes, const uint8_t* dense, hipStream_t s) {
  const uint64_t total = (uint64_t)naxes * W * (kShare / 16);
  hipLaunchKernelGGL(k_scatter_axes, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, eds, mask, W, idx,
                     is_col, naxes, dense);
  return hipGetLastError();
}

hipError_t launch_cmp(const uint8_t* x, uint64_t xstride, const uint8_t* y, uint64_t ystride, uint64_t bytes,
                      uint32_t naxes, int32_t* flags, hipStream_t s, const int32_t* idx) {
  const uint64_t total = (bytes / 16) * naxes;
  hipLaunchKernelGGL(k_cmp, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, x, xstride, y, ystride, bytes,
                     naxes, flags, idx);
  return hipGetLastError();
}

}  // namespace cel
