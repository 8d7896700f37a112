// Memory-side probe of an XCD-resident two-pass RS extension at k = 64 (VERDICT r4 ask 5),
// against the shipped two-pass flow's memory shape; no transform in either (an xor stands in
// for it), so this prices the data flow alone.
//
// k = 64: Q0 + Q1 of one square = 4 MiB, one XCD's L2. The shipped flow runs the row pass of
// the whole batch, then the column pass, so the column pass re-reads [Q0|Q1] from HBM
// (1.5x the algorithmic bytes). Here a persistent grid keeps one ticket queue per XCD
// (logical XCD = blockIdx % 8, the observed round-robin dispatch; placement decides speed
// only): queue x deals square x, x + 8, ... as 128 row tiles (64 rows x 2 slices of 256 B)
// then 256 column tiles (128 columns x 2 slices). A column tile waits until its square's 128
// row tiles have counted in, so its [Q0|Q1] re-read comes from the XCD's L2 (or the Infinity
// Cache) right after the row pass wrote / read it. Tickets are taken in order by running
// waves and row tiles wait on nothing, so the grid always drains; polls are bounded anyway.
// Hand-off: plain stores, s_waitcnt, agent-scope atomic add; the consumer polls with
// agent-scope atomic loads, then reads with default-policy (or nt) loads. That is correct only
// while producer and consumer share an L2 (same XCD): an upper bound for the data flow, not a
// shippable form (DESIGN.md §4.1.1 has the placement-independent hand-offs and their cost).
// Build: hipcc --offload-arch=gfx950 -O3 -o xcd_two_pass xcd_two_pass.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

constexpr uint32_t K = 64, W = 2 * K;
constexpr uint64_t ROW = (uint64_t)W * 512, SQ = (uint64_t)W * ROW;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}

// one wave's tile: a dword per lane of 64 shards in, 64 shards out (shard i at base + i * in_shard,
// its output at base + (K + i) * in_shard). NT: non-temporal accesses (the shipped policy).
template <bool NT>
__device__ __forceinline__ void tile(uint8_t* base, uint32_t in_shard, uint32_t lane) {
  const uint32_t* src = reinterpret_cast<const uint32_t*>(base + lane * 4u);
  uint32_t* dst = reinterpret_cast<uint32_t*>(base + (uint64_t)K * in_shard + lane * 4u);
  const uint32_t step = in_shard / 4u;
  uint32_t w[K];
#pragma unroll
  for (int i = 0; i < (int)K; i++) w[i] = NT ? __builtin_nontemporal_load(src + i * step) : src[i * step];
#pragma unroll
  for (int i = 0; i < (int)K; i++) {
    if (NT)
      __builtin_nontemporal_store(w[i] ^ (uint32_t)i, dst + i * step);
    else
      dst[i * step] = w[i] ^ (uint32_t)i;
  }
}

// shipped shape: one wave per (square, axis, slice), rows launch then columns launch, nt
__global__ __launch_bounds__(256, 3) void k_rows(uint8_t* eds, uint32_t nsq) {
  const uint32_t t = blockIdx.x * 4u + (threadIdx.x >> 6);
  if (t >= nsq * K * 2) return;
  const uint32_t sl = t & 1, rw = (t >> 1) % K, z = (t >> 1) / K;
  tile<true>(eds + z * SQ + rw * ROW + sl * 256u, 512u, threadIdx.x & 63);
}
__global__ __launch_bounds__(256, 3) void k_cols(uint8_t* eds, uint32_t nsq) {
  const uint32_t t = blockIdx.x * 4u + (threadIdx.x >> 6);
  if (t >= nsq * W * 2) return;
  const uint32_t sl = t & 1, c = (t >> 1) % W, z = (t >> 1) / W;
  tile<true>(eds + z * SQ + c * 512u + sl * 256u, (uint32_t)ROW, threadIdx.x & 63);
}

// XCD queues. tick[x]: queue x's next ticket; done[z]: row tiles of square z counted in;
// late: polls that ran out of budget (the result would be wrong; the timing is still read).
template <bool NTR>
__global__ __launch_bounds__(256, 2) void k_xcd(uint8_t* eds, uint32_t nsq, uint32_t* tick, uint32_t* done,
                                                uint32_t* late) {
  const uint32_t x = blockIdx.x & 7u, lane = threadIdx.x & 63;
  const uint32_t per = nsq / 8, total = per * (K * 2 + W * 2);
  // the ticket loop has its one exit at the loop test (a `for (;;)` with a break was the
  // round-2 hang: a second loop header that re-entered the body with the ticket zeroed)
  auto next = [&]() {
    uint32_t v = 0;
    if (lane == 0) v = __hip_atomic_fetch_add(tick + x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return __builtin_amdgcn_readfirstlane(v);
  };
  for (uint32_t t = next(); t < total; t = next()) {
    const uint32_t j = t / (K * 2 + W * 2), u = t % (K * 2 + W * 2), z = x + 8 * j;
    uint8_t* sq = eds + z * SQ;
    if (u < K * 2) {
      const uint32_t sl = u & 1, rw = u >> 1;
      tile<NTR>(sq + rw * ROW + sl * 256u, 512u, lane);
      __builtin_amdgcn_s_waitcnt(0);  // the stores have left the wave before the count
      if (lane == 0) __hip_atomic_fetch_add(done + z, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      const uint32_t v = u - K * 2, sl = v & 1, c = v >> 1;
      uint32_t polls = 0;  // every lane polls the same word: wave-uniform control flow
      while (__hip_atomic_load(done + z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < K * 2 && ++polls < (1u << 16))
        __builtin_amdgcn_s_sleep(2);
      if (polls >= (1u << 16) && lane == 0) __hip_atomic_fetch_add(late, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      tile<NTR>(sq + c * 512u + sl * 256u, (uint32_t)ROW, lane);
    }
  }
}

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IONBF, 0);
  const uint32_t nsq = argc > 1 ? (uint32_t)atoi(argv[1]) : 256;  // squares (multiple of 8)
  const char* only = argc > 2 ? argv[2] : nullptr;
  uint8_t* eds;
  uint32_t *tick, *done, *late;
  CK(hipMalloc(&eds, SQ * nsq));
  CK(hipMemset(eds, 1, SQ * nsq));
  CK(hipMalloc(&tick, 8 * 4));
  CK(hipMalloc(&done, nsq * 4));
  CK(hipMalloc(&late, 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const double alg = 2048.0 * K * K * nsq;
  auto run = [&](const char* name, auto launch) {
    if (only && !strstr(name, only)) return;
    float best = 1e30f;
    uint32_t lt = 0;
    for (int r = 0; r < 4; r++) {
      CK(hipMemset(tick, 0, 32));
      CK(hipMemset(done, 0, nsq * 4));
      CK(hipMemset(late, 0, 4));
      CK(hipEventRecord(a));
      launch();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      if (r && ms < best) best = ms;
      uint32_t l;
      CK(hipMemcpy(&l, late, 4, hipMemcpyDeviceToHost));
      lt += l;
    }
    printf("k=64 nsq=%u %-34s %8.1f us  %5.2f us/square  %5.2f TB/s algorithmic (frac %.3f)  late polls %u\n", nsq,
           name, best * 1e3, best * 1e3 / nsq, alg / (best * 1e-3) / 1e12, alg / (best * 1e-3) / 8e12, lt);
  };
  if (only && strstr(only, "debug")) {  // one launch, then the counters
    CK(hipMemset(tick, 0, 32));
    CK(hipMemset(done, 0, nsq * 4));
    CK(hipMemset(late, 0, 4));
    hipLaunchKernelGGL(k_xcd<false>, dim3(256), dim3(256), 0, 0, eds, nsq, tick, done, late);
    CK(hipDeviceSynchronize());
    uint32_t ht[8], hd[64], hl;
    CK(hipMemcpy(ht, tick, 32, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hd, done, 4 * (nsq < 64 ? nsq : 64), hipMemcpyDeviceToHost));
    CK(hipMemcpy(&hl, late, 4, hipMemcpyDeviceToHost));
    printf("tick:");
    for (int i = 0; i < 8; i++) printf(" %u", ht[i]);
    printf("\ndone:");
    for (uint32_t i = 0; i < (nsq < 64 ? nsq : 64); i++) printf(" %u", hd[i]);
    printf("\nlate %u\n", hl);
    return 0;
  }
  run("two-pass rows + cols (nt)", [&] {
    hipLaunchKernelGGL(k_rows, dim3((nsq * K * 2 + 3) / 4), dim3(256), 0, 0, eds, nsq);
    hipLaunchKernelGGL(k_cols, dim3((nsq * W * 2 + 3) / 4), dim3(256), 0, 0, eds, nsq);
  });
  for (uint32_t wg : {256u, 512u}) {
    char n[64];
    snprintf(n, sizeof n, "xcd queues default, %u WG", wg);
    run(n, [&] { hipLaunchKernelGGL(k_xcd<false>, dim3(wg), dim3(256), 0, 0, eds, nsq, tick, done, late); });
    snprintf(n, sizeof n, "xcd queues nt, %u WG", wg);
    run(n, [&] { hipLaunchKernelGGL(k_xcd<true>, dim3(wg), dim3(256), 0, 0, eds, nsq, tick, done, late); });
  }
  CK(hipFree(eds));
  return 0;
}
