// Issue rate of 2- and 3-source VALU ops on gfx950 with the operand registers placed
// explicitly: does the VGPR bank of the sources decide the rate? The SHA-256 compression
// is 58 % v_alignbit_b32 / v_add3_u32, which tools/microbench/valu_rate.hip measured at
// 4 cycles per wave64 instruction against 2 for VOP2 (and v_fma_f32 at 4, where
// MI355X_MICROARCH.md gives 2). Here every instruction writes a register nothing reads
// (no dependency chains at all) and reads registers nothing writes, in blocks of 64
// inline-asm instructions, so only the issue of the op and its operand reads remain.
// Sources: "bank0" = three registers of one bank (v64, v68, v72), "banks" = three banks
// (v64, v65, v66), "one" = one register twice (the rotate form v_alignbit_b32 d, s, s, n).
// Build: hipcc --offload-arch=gfx950 -O3 -o vop3_banks vop3_banks.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

#define R8(x) x x x x x x x x
#define R64(x) R8(R8(x))

// 64 instructions, destinations v40..v55 round robin (written, never read)
#define BLK16(I)                                                                             \
  I("v40") I("v41") I("v42") I("v43") I("v44") I("v45") I("v46") I("v47") I("v48") I("v49") \
  I("v50") I("v51") I("v52") I("v53") I("v54") I("v55")
#define BLK64(I) BLK16(I) BLK16(I) BLK16(I) BLK16(I)

#define CLOB                                                                                                 \
  "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", \
      "v55"

#define I_XOR(d) "v_xor_b32 " d ", v64, v65\n"
#define I_ADD(d) "v_add_u32 " d ", v64, v65\n"
#define I_ALIGN_ONE(d) "v_alignbit_b32 " d ", v64, v64, 7\n"
#define I_ALIGN_BANKS(d) "v_alignbit_b32 " d ", v64, v65, 7\n"
#define I_ALIGN_BANK0(d) "v_alignbit_b32 " d ", v64, v68, 7\n"
#define I_ADD3_BANKS(d) "v_add3_u32 " d ", v64, v65, v66\n"
#define I_ADD3_BANK0(d) "v_add3_u32 " d ", v64, v68, v72\n"
#define I_BITOP3_BANKS(d) "v_bitop3_b32 " d ", v64, v65, v66 bitop3:0x96\n"
#define I_BITOP3_BANK0(d) "v_bitop3_b32 " d ", v64, v68, v72 bitop3:0x96\n"
#define I_FMA_BANKS(d) "v_fma_f32 " d ", v64, v65, v66\n"
#define I_FMA_BANK0(d) "v_fma_f32 " d ", v64, v68, v72\n"
#define I_BITOP3_2BANK(d) "v_bitop3_b32 " d ", v64, v65, v68 bitop3:0x96\n"
#define I_BITOP3_SGPR(d) "v_bitop3_b32 " d ", v64, s20, v68 bitop3:0x96\n"
#define I_XOR_BANK0(d) "v_xor_b32 " d ", v64, v68\n"
#define I_ADD_BANK0(d) "v_add_u32 " d ", v64, v68\n"
#define I_LSHR(d) "v_lshrrev_b32 " d ", 7, v64\n"
#define I_ALIGN_SGPR(d) "v_alignbit_b32 " d ", v64, s20, 7\n"
// round 6: the GF(2^8) v_perm product's operand forms (table dword in an SGPR and a VGPR,
// selector in a VGPR) and the bit-sliced network's xor3 with an SGPR
#define I_PERM_SVV_BANKS(d) "v_perm_b32 " d ", s20, v64, v65\n"
#define I_PERM_SVV_BANK0(d) "v_perm_b32 " d ", s20, v64, v68\n"
#define I_PERM_VVV_BANKS(d) "v_perm_b32 " d ", v64, v65, v66\n"
#define I_PERM_VVV_BANK0(d) "v_perm_b32 " d ", v64, v68, v72\n"
#define I_PERM_0SV(d) "v_perm_b32 " d ", 0, s20, v64\n"
#define I_BITOP3_VSV_BANKS(d) "v_bitop3_b32 " d ", v64, s20, v65 bitop3:0x96\n"
#define I_AND_SV(d) "v_and_b32 " d ", s20, v64\n"
#define I_BFI_VSV_BANKS(d) "v_bitop3_b32 " d ", s20, v64, v65 bitop3:0xCA\n"
#define I_PERM_VVS_BANKS(d) "v_perm_b32 " d ", v64, v65, s20\n"

#define KERNEL(NAME, I)                                                                                      \
  __global__ __launch_bounds__(256) void NAME(uint32_t* out, int iters) {                                 \
    uint32_t x = threadIdx.x * 0x9E3779B9u;                                                                  \
    asm volatile("v_mov_b32 v64, %0\n v_mov_b32 v65, %0\n v_mov_b32 v66, %0\n v_mov_b32 v68, %0\n"         \
                 "v_mov_b32 v72, %0\n s_mov_b32 s20, 0x1234567" ::"v"(x)                                     \
                 : "v64", "v65", "v66", "v68", "v72", "s20");                                                \
    for (int it = 0; it < iters; it++) asm volatile(BLK64(I) ::: CLOB);                                     \
    uint32_t r;                                                                                              \
    asm volatile("v_xor_b32 %0, v40, v55" : "=v"(r)::"v40", "v55");                                          \
    out[blockIdx.x * 256 + threadIdx.x] = r;                                                                 \
  }

KERNEL(k_xor, I_XOR)
KERNEL(k_add, I_ADD)
KERNEL(k_lshr, I_LSHR)
KERNEL(k_align_one, I_ALIGN_ONE)
KERNEL(k_align_banks, I_ALIGN_BANKS)
KERNEL(k_align_bank0, I_ALIGN_BANK0)
KERNEL(k_align_sgpr, I_ALIGN_SGPR)
KERNEL(k_add3_banks, I_ADD3_BANKS)
KERNEL(k_add3_bank0, I_ADD3_BANK0)
KERNEL(k_bitop3_banks, I_BITOP3_BANKS)
KERNEL(k_bitop3_bank0, I_BITOP3_BANK0)
KERNEL(k_fma_banks, I_FMA_BANKS)
KERNEL(k_fma_bank0, I_FMA_BANK0)
KERNEL(k_bitop3_2bank, I_BITOP3_2BANK)
KERNEL(k_bitop3_sgpr, I_BITOP3_SGPR)
KERNEL(k_xor_bank0, I_XOR_BANK0)
KERNEL(k_add_bank0, I_ADD_BANK0)
KERNEL(k_perm_svv_banks, I_PERM_SVV_BANKS)
KERNEL(k_perm_svv_bank0, I_PERM_SVV_BANK0)
KERNEL(k_perm_vvv_banks, I_PERM_VVV_BANKS)
KERNEL(k_perm_vvv_bank0, I_PERM_VVV_BANK0)
KERNEL(k_perm_0sv, I_PERM_0SV)
KERNEL(k_bitop3_vsv_banks, I_BITOP3_VSV_BANKS)
KERNEL(k_and_sv, I_AND_SV)
KERNEL(k_bfi_svv_banks, I_BFI_VSV_BANKS)
KERNEL(k_perm_vvs_banks, I_PERM_VVS_BANKS)

typedef void (*kfn)(uint32_t*, int);

static void run(const char* name, kfn k, uint32_t* out, int wg_per_cu) {
  const int blocks = 256 * wg_per_cu, iters = 512;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 4);
  CK(hipEventRecord(a));
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, iters);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  const double winst = (double)blocks * 4 * iters * 64;  // wave-instructions
  // cycles per wave-instruction per SIMD at 2.4 GHz (1024 SIMDs)
  printf("%-18s waves/SIMD %2d  %8.3f ms  %7.2f T lane-ops/s  %5.2f cycles per wave64 instruction @2.4GHz\n", name,
         wg_per_cu, ms, winst * 64 / (ms * 1e-3) / 1e12, ms * 1e-3 * 2.4e9 * 1024 / winst);
}

int main(int argc, char** argv) {
  uint32_t* out;
  CK(hipMalloc(&out, 256 * 16 * 256 * 4));
  struct {
    const char* n;
    kfn k;
  } ks[] = {{"xor", k_xor},
            {"add_u32", k_add},
            {"lshrrev", k_lshr},
            {"align one-reg", k_align_one},
            {"align banks", k_align_banks},
            {"align bank0", k_align_bank0},
            {"align sgpr", k_align_sgpr},
            {"add3 banks", k_add3_banks},
            {"add3 bank0", k_add3_bank0},
            {"bitop3 banks", k_bitop3_banks},
            {"bitop3 bank0", k_bitop3_bank0},
            {"fma banks", k_fma_banks},
            {"fma bank0", k_fma_bank0},
            {"bitop3 2 banks", k_bitop3_2bank},
            {"bitop3 v,s,v b0", k_bitop3_sgpr},
            {"xor bank0", k_xor_bank0},
            {"add_u32 bank0", k_add_bank0},
            {"perm s,v,v banks", k_perm_svv_banks},
            {"perm s,v,v bank0", k_perm_svv_bank0},
            {"perm v,v,v banks", k_perm_vvv_banks},
            {"perm v,v,v bank0", k_perm_vvv_bank0},
            {"perm 0,s,v", k_perm_0sv},
            {"perm v,v,s banks", k_perm_vvs_banks},
            {"bitop3 v,s,v bnks", k_bitop3_vsv_banks},
            {"bfi s,v,v banks", k_bfi_svv_banks},
            {"and s,v", k_and_sv}};
  for (int w : {2, 4})
    for (auto& k : ks) run(k.n, k.k, out, w);
  return 0;
}
