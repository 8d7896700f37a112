// Throughput of the four GF(2^8) product forms the RS kernels choose between (VERDICT r3
// ask 3: wave-uniform products with SGPR masks against per-lane v_perm tables), one
// "x ^= c * y" per dword, on 128 register dwords per lane at 3 waves per SIMD (the
// encoders' occupancy), no memory traffic:
//   vperm_lane : 3+3+2-bit v_perm product, table = compile-time table XOR the lane's table
//                (rs_gf16x.hip layers 0-4: the twiddle has a per-lane part), 2 dwords per table
//   vperm_const: the same with compile-time tables only (rs_axis.hip layers D = 1, 2, 4)
//   plane_sgpr : 8 dwords as 8 bit planes, product by a RUN-TIME wave-uniform twiddle: its
//                64 matrix entries are 0 / ~0 mask words loaded into SGPRs and each (i, j)
//                is one v_bitop3 x ^ (mask & y) (rs_decode_gf16.hip's form, whose masks come
//                from s_bfe of packed bits instead)
//   plane_const: 8 bit planes, compile-time matrix: an xor3 network (rs_axis.hip D >= 8)
// The plane forms exclude the 8x8 bit transposes that put bytes into planes (48 VALU per
// 8 dwords, once per run of plane layers).
// Build: hipcc --offload-arch=gfx950 -O3 -I../../celestia-app_amd/csrc -o gf_prod gf_prod.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "bitslice8.hpp"
#include "gf8_constexpr.hpp"
#include "gf8_regs.hpp"

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

using namespace cel;
using cx::kGf8;
using cx::sfor;

constexpr int NL = 8;  // layers per launch iteration

template <uint32_t C>
__device__ __forceinline__ uint32_t vxor(uint32_t v) {
  uint32_t r;
  asm volatile("v_xor_b32 %0, %1, %2" : "=v"(r) : "i"(C), "v"(v));
  return r;
}

// MODE 0 vperm_lane, 1 vperm_const, 2 plane_sgpr, 3 plane_const
template <int MODE>
__global__ __launch_bounds__(256, 3) void k_prod(uint32_t* out, const uint32_t* __restrict__ masks, int iters) {
  uint32_t w[128];
  const uint32_t t = blockIdx.x * 256u + threadIdx.x;
#pragma unroll
  for (int i = 0; i < 128; i++) w[i] = t * 0x9E3779B9u + (uint32_t)i * 0x7F4A7C15u;
  const uint32_t m7 = ax::sconst<0x07070707u>(), m3 = ax::sconst<0x03030303u>();
  // the lane's table part (MODE 0): a lane-dependent table word set
  const uint32_t g0 = t * 0x01010101u, g1 = t * 0x02020202u, g2 = t * 0x03030303u, g3 = t * 0x05050505u,
                 g4 = t * 0x07070707u;
#pragma unroll 1
  for (int it = 0; it < iters; it++) {
    sfor<NL>([&](auto li) {
      constexpr int L = decltype(li)::value;
      if constexpr (MODE <= 1) {
        sfor<32>([&](auto bi) {  // 32 tables x 2 dwords = 64 products per layer
          constexpr int b = decltype(bi)::value;
          constexpr uint32_t lm = (uint32_t)(b * 7 + L * 13 + 1) % 255u;
          constexpr ax::Tab tb = ax::make_tab(lm);
          uint32_t t0l, t0h, t1l, t1h, t2;
          if constexpr (MODE == 0) {
            t0l = vxor<tb.t0l>(g0); t0h = vxor<tb.t0h>(g1); t1l = vxor<tb.t1l>(g2); t1h = vxor<tb.t1h>(g3);
            t2 = vxor<tb.t2>(g4);
          } else {
            t0l = ax::vconst<tb.t0l>(); t0h = ax::sconst<tb.t0h>(); t1l = ax::vconst<tb.t1l>();
            t1h = ax::sconst<tb.t1h>(); t2 = ax::sconst<tb.t2>();
          }
          sfor<2>([&](auto ji) {
            constexpr int x = 2 * b + decltype(ji)::value, y = x + 64;
            ax::pin(w[x], w[y]);
            const uint32_t yv = w[y];
            const uint32_t p0 = __builtin_amdgcn_perm(t0h, t0l, yv & m7);
            const uint32_t p1 = __builtin_amdgcn_perm(t1h, t1l, (yv >> 3) & m7);
            const uint32_t p2 = __builtin_amdgcn_perm(0u, t2, (yv >> 6) & m3);
            w[x] = __builtin_amdgcn_bitop3_b32(w[x], p0, p1, 0x96) ^ p2;
            ax::pin(w[x], w[y]);
          });
          __builtin_amdgcn_sched_barrier(0);
        });
      } else {
        sfor<8>([&](auto gi) {  // 8 plane groups x 8 dwords = 64 products per layer
          constexpr int g = decltype(gi)::value;
          constexpr int xo = 8 * g, yo = xo + 64;
          if constexpr (MODE == 2) {
            // the twiddle's 64 matrix entries as 0 / ~0 mask words, wave-uniform: scalar
            // loads into SGPRs (a VOP3 reads one SGPR)
            uint32_t off = 64u * (L * 8 + g);
            asm volatile("" : "+s"(off));  // loaded where used (no hoisting of 4096 masks)
            const uint32_t* mk = masks + off;
            sfor<8>([&](auto ii) {
              constexpr int i = decltype(ii)::value;
              sfor<8>([&](auto jj) {
                constexpr int j = decltype(jj)::value;
                w[xo + j] = __builtin_amdgcn_bitop3_b32(w[xo + j], mk[8 * i + j], w[yo + i], 0x78);
              });
            });
          } else {
            constexpr uint32_t lm = (uint32_t)(g * 11 + L * 17 + 3) % 255u;
            ax::pmuladd<lm, xo, yo>(w);
          }
          __builtin_amdgcn_sched_barrier(0);
        });
      }
    });
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 128; i++) s ^= w[i];
  out[t] = s;
}

template <int MODE>
static float run(uint32_t* out, const uint32_t* masks, int blocks, int iters) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL(k_prod<MODE>, dim3(blocks), dim3(256), 0, 0, out, masks, 1);
  CK(hipEventRecord(a));
  hipLaunchKernelGGL(k_prod<MODE>, dim3(blocks), dim3(256), 0, 0, out, masks, iters);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms;
}

int main() {
  const int blocks = 256 * 3 * 4, iters = 64;  // 3 waves per SIMD on 256 CUs, 4 rounds
  uint32_t *out, *masks;
  CK(hipMalloc(&out, (size_t)blocks * 256 * 4));
  CK(hipMalloc(&masks, 64 * NL * 8 * 4));
  uint32_t hm[64 * NL * 8];
  for (int i = 0; i < 64 * NL * 8; i++) hm[i] = ((0x9E3779B9u * (uint32_t)(i + 1)) >> 7) & 1u ? 0xFFFFFFFFu : 0u;
  CK(hipMemcpy(masks, hm, sizeof hm, hipMemcpyHostToDevice));
  const double prods = (double)blocks * 4 * iters * NL * 64;  // wave-level dword products
  const char* names[4] = {"vperm_lane (per-lane tables)", "vperm_const (compile-time tables)",
                          "plane_sgpr (run-time SGPR masks)", "plane_const (compile-time xor3 net)"};
  float t[4];
  for (int rep = 0; rep < 2; rep++) {
    t[0] = run<0>(out, masks, blocks, iters);
    t[1] = run<1>(out, masks, blocks, iters);
    t[2] = run<2>(out, masks, blocks, iters);
    t[3] = run<3>(out, masks, blocks, iters);
  }
  for (int m = 0; m < 4; m++)
    printf("%-38s %8.3f ms  %6.2f ns per 1k wave-dword-products  %5.2f SIMD-cycles per wave-dword-product @2.4GHz\n",
           names[m], t[m], t[m] * 1e6 / (prods / 1e3), t[m] * 1e-3 * 2.4e9 * 1024 / prods);
  return 0;
}
