/* ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.h). Internal declarations. */
#ifndef CEL_ORACLE_INTERNAL_H
#define CEL_ORACLE_INTERNAL_H
#include <stdint.h>
#include <stddef.h>

typedef struct {
  int bits;
  uint32_t order, mod;
  uint16_t* exp;
  uint16_t* log;
  uint16_t* skew;
} gf_t;

extern gf_t g_gf8, g_gf16;
extern int g_simd;

uint32_t gf_mul_log(const gf_t* f, uint32_t a, uint32_t log_b);
uint32_t gf_mul(const gf_t* f, uint32_t a, uint32_t b);
uint32_t gf_inv(const gf_t* f, uint32_t a);
const gf_t* field_for(uint32_t n);
void leo_encode_inplace(const gf_t* f, uint32_t m, uint8_t** w, size_t len);

/* SHA-256 streaming over up to three pieces (avoids building messages). */
void sha256_blocks(const uint8_t* blocks, size_t nblk, uint8_t out[32]);
size_t sha256_pad(uint8_t* buf, size_t len);
void sha256_3(const uint8_t* a, size_t la, const uint8_t* b, size_t lb, const uint8_t* c,
              size_t lc, uint8_t out[32]);

#endif
