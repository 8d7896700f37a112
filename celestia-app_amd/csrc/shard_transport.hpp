// How a row-sharded plan moves its all-to-all blocks and record blocks (api_multi.cpp),
// kept free of HIP and RCCL so the selection is unit-tested on the host
// (tests/shard_transport_test.cpp).
//
//   local  one rank, no collective (the row pass writes the slab in place)
//   rccl   grouped ncclSend / ncclRecv + ncclAllGather over one communicator per device
//   copy   the same schedule with device copies, ctxs repeating a device (RCCL refuses two
//          ranks on one device)
//   peer   the same schedule with hipMemcpyPeerAsync between distinct devices (peer access
//          enabled at plan creation): CEL_FLAG_SHARD_PEERCOPY, or the fallback when RCCL cannot
//          start (not loadable, or ncclCommInitAll fails) so a node's first multi-GPU run
//          still produces the square
#pragma once
#include <algorithm>
#include <cstdint>
#include <vector>

namespace cel {

enum class ShardTransport { kLocal, kRccl, kCopy, kPeer };

struct ShardChoice {
  ShardTransport want;  // what the device list and flags ask for
  bool dup;             // the ctxs repeat a device
  bool copies;          // a fallback moves blocks with same-device copies (dup, or one rank)
  bool alias;           // one rank writing the slab in place (no send buffer)
};

// flags: CEL_FLAG_SHARD_EXCHANGE (exchange through RCCL even where the device list would not),
// CEL_FLAG_SHARD_PEERCOPY (never RCCL); values passed in so this header needs no ABI header.
inline ShardChoice shard_choose(const int* devs, uint32_t n, bool exchange, bool peercopy) {
  std::vector<int> s(devs, devs + n);
  std::sort(s.begin(), s.end());
  const bool dup = std::adjacent_find(s.begin(), s.end()) != s.end();
  const bool copies = dup || n == 1;
  if (n == 1 && !exchange) return {ShardTransport::kLocal, false, true, true};
  if (peercopy) return {copies ? ShardTransport::kCopy : ShardTransport::kPeer, dup, copies, false};
  if (dup && !exchange) return {ShardTransport::kCopy, true, true, false};
  return {ShardTransport::kRccl, dup, copies, false};
}

// The transport the plan runs on once RCCL has (rccl_ok) or has not started.
inline ShardTransport shard_settle(const ShardChoice& c, bool rccl_ok) {
  if (c.want != ShardTransport::kRccl || rccl_ok) return c.want;
  return c.copies ? ShardTransport::kCopy : ShardTransport::kPeer;
}

inline const char* shard_transport_name(ShardTransport t, bool fallback) {
  switch (t) {
    case ShardTransport::kLocal: return "local";
    case ShardTransport::kRccl: return "rccl";
    case ShardTransport::kCopy: return fallback ? "copy-fallback" : "copy";
    case ShardTransport::kPeer: return fallback ? "peer-fallback" : "peer";
  }
  return "";
}

}  // namespace cel
