// Host unit test of the row-sharded plan's transport selection (csrc/shard_transport.hpp),
// including the fallback taken when RCCL cannot start (rccl_ok = false stands in for a
// failing ncclCommInitAll). Built and run by tests/test_shard_transport.py.
#include <cstdio>
#include <cstring>
#include <vector>

#include "shard_transport.hpp"

using namespace cel;

static int fails = 0;

static void check(const std::vector<int>& devs, bool exchange, bool peercopy, const char* want_ok,
                  const char* want_failed, bool alias) {
  const ShardChoice c = shard_choose(devs.data(), (uint32_t)devs.size(), exchange, peercopy);
  const bool tries_rccl = c.want == ShardTransport::kRccl;
  const char* ok = shard_transport_name(shard_settle(c, true), false);
  const char* failed = shard_transport_name(shard_settle(c, false), tries_rccl);
  if (std::strcmp(ok, want_ok) || std::strcmp(failed, want_failed) || c.alias != alias) {
    std::printf("FAIL n=%zu exchange=%d peercopy=%d: got %s / %s alias %d, want %s / %s alias %d\n", devs.size(),
                exchange, peercopy, ok, failed, c.alias, want_ok, want_failed, alias);
    fails++;
  }
}

int main() {
  // one rank: no collective unless the exchange is asked for
  check({0}, false, false, "local", "local", true);
  check({0}, true, false, "rccl", "copy-fallback", false);
  check({3}, false, true, "local", "local", true);
  // distinct devices: RCCL, peer copies when it cannot start or when asked
  check({0, 1}, false, false, "rccl", "peer-fallback", false);
  check({0, 1, 2, 3, 4, 5, 6, 7}, false, false, "rccl", "peer-fallback", false);
  check({7, 6, 5, 4, 3, 2, 1, 0}, true, false, "rccl", "peer-fallback", false);
  check({0, 1, 2, 3}, false, true, "peer", "peer", false);
  check({0, 1, 2, 3}, true, true, "peer", "peer", false);
  // a repeated device: device copies (RCCL refuses two ranks on one device), tried anyway
  // under CEL_FLAG_SHARD_EXCHANGE and then the copy fallback
  check({0, 0}, false, false, "copy", "copy", false);
  check({0, 1, 0, 1}, false, false, "copy", "copy", false);
  check({0, 0, 0, 0}, true, false, "rccl", "copy-fallback", false);
  check({0, 0}, false, true, "copy", "copy", false);
  if (fails) return 1;
  std::printf("shard transport selection: ok\n");
  return 0;
}
