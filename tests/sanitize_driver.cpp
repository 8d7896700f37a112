// Sanitizer driver (SURVEY.md §5 auxiliaries): the host-only product sources
// (celestia-app_amd/csrc/square.cpp, proof.cpp, inclusion_paths.cpp) and the oracle
// (oracle/*.c) built with -fsanitize=address,undefined by `make -C oracle asan`, driven
// over the same inputs the CPU tests use. Test infrastructure, never shipped.
//
//   sanitize_driver <blocks file>
//
// The blocks file (written by tests/test_sanitizers.py) holds tx lists:
//   u32 nblocks, then per block: u32 ntx, u32 len[ntx], the tx bytes back to back.
// Every section prints "<section> <fnv-1a 64 of everything it produced>" so the
// sanitized build can be compared with a plain build of the same driver.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../include/celestia_eds.h"
#include "../oracle/oracle.h"

namespace {

struct Fnv {
  uint64_t h = 1469598103934665603ull;
  void add(const void* p, size_t n) {
    const uint8_t* b = static_cast<const uint8_t*>(p);
    for (size_t i = 0; i < n; i++) h = (h ^ b[i]) * 1099511628211ull;
  }
  template <class T>
  void val(T v) { add(&v, sizeof v); }
};

struct Rng {
  uint64_t s;
  uint64_t next() {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return s;
  }
  void fill(uint8_t* p, size_t n) {
    for (size_t i = 0; i < n; i++) p[i] = (uint8_t)next();
  }
};

// Exact-size heap copies, so that ASan sees any read past the end of an input.
std::vector<uint8_t> exact(const uint8_t* p, size_t n) { return std::vector<uint8_t>(p, p + n); }

void squares(const char* path, Fnv& f) {
  FILE* fp = std::fopen(path, "rb");
  if (!fp) {
    std::perror(path);
    std::exit(2);
  }
  std::vector<uint8_t> all;
  uint8_t buf[1 << 16];
  size_t got;
  while ((got = std::fread(buf, 1, sizeof buf, fp)) > 0) all.insert(all.end(), buf, buf + got);
  std::fclose(fp);
  size_t off = 0;
  auto u32 = [&]() {
    uint32_t v;
    std::memcpy(&v, all.data() + off, 4);
    off += 4;
    return v;
  };
  const uint32_t nblocks = u32();
  for (uint32_t b = 0; b < nblocks; b++) {
    const uint32_t ntx = u32();
    std::vector<uint32_t> lens(ntx);
    size_t total = 0;
    for (uint32_t i = 0; i < ntx; i++) total += lens[i] = u32();
    std::vector<uint8_t> txs = exact(all.data() + off, total);
    off += total;
    std::vector<uint32_t> lens_exact(lens);
    for (uint32_t greedy = 0; greedy < 2; greedy++) {
      uint32_t k = 0;
      std::vector<uint8_t> inc(ntx ? ntx : 1);
      const uint8_t* tp = total ? txs.data() : nullptr;
      cel_status st = cel_square_construct(tp, lens_exact.data(), ntx, 128, 64, greedy, nullptr, 0, &k, inc.data());
      f.val(st);
      f.val(k);
      if (st == CEL_OK) {
        std::vector<uint8_t> out((size_t)k * k * CEL_SHARE_SIZE);
        st = cel_square_construct(tp, lens_exact.data(), ntx, 128, 64, greedy, out.data(), k * k, &k, inc.data());
        f.val(st);
        f.add(out.data(), out.size());
        f.add(inc.data(), ntx);
      } else {
        const char* m = cel_square_last_error();
        f.add(m, std::strlen(m));
      }
    }
    for (uint32_t i = 0; i < ntx; i += (ntx > 16 ? ntx / 16 : 1)) {
      uint32_t s = 0, e = 0;
      const cel_status st = cel_square_tx_range(total ? txs.data() : nullptr, lens_exact.data(), ntx, 128, 64, i, &s, &e);
      f.val(st);
      f.val(s);
      f.val(e);
    }
  }
}

void proofs(Fnv& f) {
  Rng r{0x9E3779B97F4A7C15ull};
  for (uint32_t n = 1; n <= 64; n *= 2) {
    std::vector<uint8_t> tree((2 * (size_t)n - 1) * CEL_NMT_NODE_SIZE);
    r.fill(tree.data(), tree.size());
    std::vector<uint8_t> levels((2 * (size_t)n - 1) * 32);
    r.fill(levels.data(), levels.size());
    std::vector<uint8_t> out(64 * CEL_NMT_NODE_SIZE);
    for (uint32_t s = 0; s <= n; s++)
      for (uint32_t e = 0; e <= n + 1; e++) {
        uint32_t cnt = 0;
        const cel_status st = cel_nmt_prove_range(tree.data(), n, s, e, out.data(), &cnt);
        f.val(st);
        f.val(cnt);
        if (st == CEL_OK) f.add(out.data(), (size_t)cnt * CEL_NMT_NODE_SIZE);
      }
    std::vector<uint8_t> aunts(64 * 32);
    for (uint32_t i = 0; i <= n; i++) {
      uint32_t cnt = 0;
      const cel_status st = cel_merkle_aunts(levels.data(), n, i, aunts.data(), &cnt);
      f.val(st);
      f.val(cnt);
      if (st == CEL_OK) f.add(aunts.data(), (size_t)cnt * 32);
    }
  }
}

void paths(Fnv& f) {
  std::vector<uint32_t> a(4096), b(4096), c(4096);
  for (uint32_t sq = 1; sq <= 128; sq *= 2)
    for (uint32_t start = 0; start < sq * sq; start += (sq > 8 ? sq * sq / 37 + 1 : 1))
      for (uint32_t len = 1; len <= sq * sq + 1; len += (sq > 8 ? sq * sq / 23 + 1 : 1)) {
        uint32_t n = 0;
        const cel_status st = cel_commitment_paths(sq, start, len, 64, a.data(), b.data(), c.data(), 4096, &n);
        f.val(st);
        f.val(n);
        if (st == CEL_OK && n <= 4096) {
          f.add(a.data(), 4 * n);
          f.add(b.data(), 4 * n);
          f.add(c.data(), 4 * n);
        }
      }
  for (uint32_t maxd = 0; maxd <= 7; maxd++)
    for (uint32_t mind = 0; mind <= maxd + 1; mind++)
      for (uint32_t s = 0; s <= (1u << maxd); s++)
        for (uint32_t e = s; e <= (1u << maxd) + 1; e++) {
          uint32_t n = 0;
          const cel_status st = cel_subtree_root_coordinates(maxd, mind, s, e, b.data(), c.data(), 4096, &n);
          f.val(st);
          f.val(n);
          if (st == CEL_OK && n <= 4096) {
            f.add(b.data(), 4 * n);
            f.add(c.data(), 4 * n);
          }
        }
}

// Honest ODS: namespaces non-decreasing in row-major order.
void random_ods(Rng& r, uint32_t k, std::vector<uint8_t>& ods) {
  ods.assign((size_t)k * k * CEL_SHARE_SIZE, 0);
  r.fill(ods.data(), ods.size());
  for (uint32_t i = 0; i < k * k; i++) {
    uint8_t* sh = ods.data() + (size_t)i * CEL_SHARE_SIZE;
    std::memset(sh, 0, CEL_NAMESPACE_SIZE);
    sh[CEL_NAMESPACE_SIZE - 2] = (uint8_t)(i * 251 / (k * k));
    sh[CEL_NAMESPACE_SIZE - 1] = 1;
  }
}

void oracle(Fnv& f) {
  orc_init();
  orc_set_threads(1);
  Rng r{12345};
  for (uint32_t k = 1; k <= 8; k *= 2) {
    std::vector<uint8_t> ods, eds((size_t)4 * k * k * CEL_SHARE_SIZE);
    random_ods(r, k, ods);
    std::vector<uint8_t> rows(2 * (size_t)k * ORC_NODE), cols(2 * (size_t)k * ORC_NODE);
    uint8_t dah[32];
    f.val(orc_extend_and_commit(ods.data(), k, CEL_SHARE_SIZE, eds.data(), rows.data(), cols.data(), dah));
    f.add(eds.data(), eds.size());
    f.add(dah, 32);
    // repair a quarter-erased copy (a solvable mask: Q3 missing)
    std::vector<uint8_t> damaged(eds), present(4 * (size_t)k * k, 1);
    for (uint32_t i = k; i < 2 * k; i++)
      for (uint32_t j = k; j < 2 * k; j++) {
        present[i * 2 * k + j] = 0;
        std::memset(damaged.data() + ((size_t)i * 2 * k + j) * CEL_SHARE_SIZE, 0, CEL_SHARE_SIZE);
      }
    int32_t ba = -1, bi = -1;
    std::vector<uint8_t> bs(2 * (size_t)k * CEL_SHARE_SIZE), bp(2 * k);
    f.val(orc_repair(damaged.data(), present.data(), k, CEL_SHARE_SIZE, rows.data(), cols.data(), &ba, &bi, bs.data(),
                     bp.data()));
    f.val(std::memcmp(damaged.data(), eds.data(), eds.size()) == 0);
    // one corrupt cell in a complete square: byzantine or bad root, with the axis shares
    std::vector<uint8_t> bad(eds), all(4 * (size_t)k * k, 1);
    bad[((size_t)k * 2 * k + k) * CEL_SHARE_SIZE + 100] ^= 0x5A;
    f.val(orc_repair(bad.data(), all.data(), k, CEL_SHARE_SIZE, rows.data(), cols.data(), &ba, &bi, bs.data(),
                     bp.data()));
    f.val(ba);
    f.val(bi);
  }
  for (uint32_t n : {1u, 16u, 128u, 256u}) {
    const size_t len = 128;
    std::vector<uint8_t> data(n * len), shards(2 * n * len), present(2 * n);
    r.fill(data.data(), data.size());
    std::memcpy(shards.data(), data.data(), data.size());
    f.val(orc_rs_encode(n, len, data.data(), shards.data() + n * len));
    f.add(shards.data(), shards.size());
    std::vector<uint8_t> full(shards);
    for (uint32_t i = 0; i < 2 * n; i++) present[i] = (r.next() % 2) || i >= n + n / 2;
    for (uint32_t i = 0; i < 2 * n; i++)
      if (!present[i]) std::memset(shards.data() + i * len, 0, len);
    f.val(orc_rs_decode(n, len, shards.data(), present.data()));
    f.val(std::memcmp(shards.data(), full.data(), full.size()) == 0);
  }
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s <blocks file>\n", argv[0]);
    return 2;
  }
  Fnv a, b, c, d;
  squares(argv[1], a);
  std::printf("square %016llx\n", (unsigned long long)a.h);
  proofs(b);
  std::printf("proof %016llx\n", (unsigned long long)b.h);
  paths(c);
  std::printf("paths %016llx\n", (unsigned long long)c.h);
  oracle(d);
  std::printf("oracle %016llx\n", (unsigned long long)d.h);
  return 0;
}
