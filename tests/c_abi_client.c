/*
 * A plain C99 client of include/celestia_eds.h, the way the cgo stub (go/celestiaeds)
 * binds it: compiled by gcc (not hipcc), linked against libcelestia_eds.so, no HIP or
 * torch headers. It runs da.ExtendShares + NewDataAvailabilityHeader on the generateShares
 * square of pkg/da/data_availability_header_test.go:247-263 (k = 2) and checks the DAH
 * known answer of :45, then the DAH-only call shape (eds_out = NULL) and the
 * "not a power of 2" error string of :68. Then the multi-GPU entry points as the Go Group
 * (go/celestiaeds/multi.go) calls them, with two ctxs on device 0: cel_extend_batch_multi on
 * three copies of that square (each DAH = the known answer), and cel_extend_sharded on a
 * k = 256 square (one rank, the "local" plan) against cel_extend_shares on the same shares,
 * then that square through an explicit two-rank plan with CEL_FLAG_SHARD_PEERCOPY (transport
 * "copy", no note) and its all-to-all timed alone (cel_shard_plan_time_exchange).
 * Exit codes: 0 = all checks passed; 2 = no device (CEL_EDEVICE from cel_ctx_create:
 * the library fails loudly, there is no CPU fallback); 1 = a check failed.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "celestia_eds.h"

static const char* kTypicalK2 = "b56e4d251ac266f4b91cc5464b3fc7efcbdc888064647496d13133f0dc65ac25";

static void hex(const uint8_t* b, size_t n, char* out) {
  for (size_t i = 0; i < n; i++) sprintf(out + 2 * i, "%02x", b[i]);
}

int main(void) {
  cel_ctx* ctx = NULL;
  cel_status st = cel_ctx_create(0, &ctx);
  if (st == CEL_EDEVICE) {
    printf("no device: %s\n", cel_strerror(st));
    return 2;
  }
  if (st != CEL_OK) return 1;
  enum { K = 2, N = K * K, W = 2 * K };
  uint8_t* shares = (uint8_t*)malloc((size_t)N * CEL_SHARE_SIZE);
  for (int i = 0; i < N; i++) {
    uint8_t* s = shares + (size_t)i * CEL_SHARE_SIZE;
    memset(s, 0xFF, CEL_SHARE_SIZE);
    memset(s, 0, 19);       /* namespace version 0, 18 zero bytes */
    memset(s + 19, 1, 10);  /* MustNewV0(0x01 * 10) */
  }
  uint8_t* eds = (uint8_t*)malloc((size_t)W * W * CEL_SHARE_SIZE);
  uint8_t rr[W * CEL_NMT_NODE_SIZE], cr[W * CEL_NMT_NODE_SIZE], dah[32];
  char h[65];
  int ok = 1;
  st = cel_extend_shares(ctx, shares, N, CEL_SHARE_SIZE, eds, rr, cr, dah, CEL_FLAG_ORDER_CHECK);
  hex(dah, 32, h);
  printf("ExtendShares: status %d dah %s\n", st, h);
  ok &= st == CEL_OK && strcmp(h, kTypicalK2) == 0;
  ok &= memcmp(eds, shares, CEL_SHARE_SIZE) == 0; /* cell (0,0) is the first share */
  memset(dah, 0, sizeof dah);
  st = cel_extend_shares(ctx, shares, N, CEL_SHARE_SIZE, NULL, rr, cr, dah, CEL_FLAG_ORDER_CHECK);
  hex(dah, 32, h);
  printf("DAH only:     status %d dah %s\n", st, h);
  ok &= st == CEL_OK && strcmp(h, kTypicalK2) == 0;
  st = cel_extend_shares(ctx, shares, 3, CEL_SHARE_SIZE, NULL, rr, cr, dah, 0);
  printf("3 shares:     status %d \"%s\"\n", st, cel_last_error(ctx));
  ok &= st == CEL_ENOTPOW2 && strcmp(cel_last_error(ctx), "number of shares is not a power of 2: got 3") == 0;

  /* config 4 from C: three k = 2 squares split over two ctxs */
  cel_ctx* ctx2 = NULL;
  ok &= cel_ctx_create(0, &ctx2) == CEL_OK;
  cel_ctx* group[2] = {ctx, ctx2};
  uint8_t* ods3 = (uint8_t*)malloc((size_t)3 * N * CEL_SHARE_SIZE);
  for (int i = 0; i < 3; i++) memcpy(ods3 + (size_t)i * N * CEL_SHARE_SIZE, shares, (size_t)N * CEL_SHARE_SIZE);
  uint8_t rr3[3 * W * CEL_NMT_NODE_SIZE], cr3[3 * W * CEL_NMT_NODE_SIZE], dah3[3 * 32];
  int32_t st3[3] = {-1, -1, -1};
  st = cel_extend_batch_multi(group, 2, ods3, 3, K, CEL_SHARE_SIZE, NULL, rr3, cr3, dah3, st3, CEL_FLAG_ORDER_CHECK);
  printf("batch_multi:  status %d statuses %d %d %d\n", st, st3[0], st3[1], st3[2]);
  ok &= st == CEL_OK;
  for (int i = 0; i < 3; i++) {
    hex(dah3 + 32 * i, 32, h);
    ok &= st3[i] == 0 && strcmp(h, kTypicalK2) == 0;
  }
  free(ods3);

  /* config 3 from C: one k = 256 square through cel_extend_sharded vs cel_extend_shares */
  enum { KB = 256, NB = KB * KB, WB = 2 * KB };
  uint8_t* big = (uint8_t*)malloc((size_t)NB * CEL_SHARE_SIZE);
  uint32_t x = 12345u;
  for (size_t i = 0; i < (size_t)NB * CEL_SHARE_SIZE; i++) {
    x = x * 1664525u + 1013904223u;
    big[i] = (uint8_t)(x >> 24);
  }
  for (int i = 0; i < NB; i++) { /* one namespace for every share: push order holds */
    uint8_t* s = big + (size_t)i * CEL_SHARE_SIZE;
    memset(s, 0, 19);
    memset(s + 19, 7, 10);
  }
  uint8_t* rra = (uint8_t*)malloc((size_t)4 * WB * CEL_NMT_NODE_SIZE);
  uint8_t *cra = rra + WB * CEL_NMT_NODE_SIZE, *rrb = cra + WB * CEL_NMT_NODE_SIZE, *crb = rrb + WB * CEL_NMT_NODE_SIZE;
  uint8_t daha[32], dahb[32];
  st = cel_extend_shares(ctx, big, NB, CEL_SHARE_SIZE, NULL, rra, cra, daha, CEL_FLAG_ORDER_CHECK);
  cel_status st2 = cel_extend_sharded(group, 1, big, KB, CEL_SHARE_SIZE, NULL, rrb, crb, dahb, CEL_FLAG_ORDER_CHECK);
  hex(dahb, 32, h);
  printf("sharded k=256: status %d / %d dah %s\n", st, st2, h);
  ok &= st == CEL_OK && st2 == CEL_OK && memcmp(daha, dahb, 32) == 0;
  ok &= memcmp(rra, rrb, (size_t)2 * WB * CEL_NMT_NODE_SIZE) == 0; /* row and column roots */
  /* round 6: the same square through an explicit two-rank plan that never starts RCCL
   * (CEL_FLAG_SHARD_PEERCOPY; both ctxs on device 0, so transport "copy"), its exchange timed
   * alone, and the roots against cel_extend_shares again */
  cel_shard_plan* plan = NULL;
  st = cel_shard_plan_create(group, 2, KB, CEL_FLAG_ORDER_CHECK | CEL_FLAG_SHARD_PEERCOPY, &plan);
  ok &= st == CEL_OK && plan != NULL;
  if (plan) {
    double a2a_us = 0;
    st = cel_shard_plan_upload(plan, big);
    if (st == CEL_OK) st = cel_shard_plan_run(plan);
    if (st == CEL_OK) st = cel_shard_plan_wait(plan, NULL, rrb, crb, dahb);
    cel_status st3x = cel_shard_plan_time_exchange(plan, 3, &a2a_us);
    printf("plan k=256 x2: status %d transport %s note \"%s\" exchange %.1f us (%d)\n", st,
           cel_shard_plan_transport(plan), cel_shard_plan_note(plan), a2a_us, st3x);
    ok &= st == CEL_OK && strcmp(cel_shard_plan_transport(plan), "copy") == 0 && cel_shard_plan_note(plan)[0] == 0;
    ok &= st3x == CEL_OK && a2a_us > 0;
    ok &= memcmp(daha, dahb, 32) == 0 && memcmp(rra, rrb, (size_t)2 * WB * CEL_NMT_NODE_SIZE) == 0;
    cel_shard_plan_destroy(plan);
  }
  free(rra);
  free(big);
  cel_ctx_destroy(ctx2);

  cel_ctx_destroy(ctx);
  free(eds);
  free(shares);
  printf("%s\n", ok ? "ok" : "FAILED");
  return ok ? 0 : 1;
}
