// Data-square construction: a block's txs -> the k*k ODS shares that da.ExtendShares
// receives.
//
// Restates go-square v1.1.0 (go.mod:9, [dep], not in /root/reference) as called by
//   app/extend_block.go:16-25      square.Construct(txs, SquareSizeUpperBound, SubtreeRootThreshold)
//   app/process_proposal.go:121-130 square.Construct(...)
//   app/prepare_proposal.go:48-61   square.Build(...)  (greedy: drops txs that do not fit)
// with the rules of specs/src/specs/shares.md:24-98 (compact and sparse shares),
// namespace.md:77-84 (reserved namespaces), data_square_layout.md:38-62 (blob
// placement) and SURVEY.md Appendix A.4. Host code: pure byte layout, sequential by
// nature and ~1 us per share; the device path starts at the ODS.
//
// Builder (go-square square/builder.go): normal txs first, then BlobTxs. Every append
// is admitted only if the worst-case square still fits maxSquareSize^2:
//   tx shares + PFB shares (index wrappers with worst-case share indexes)
//   + sum over blobs of (shares + SubTreeWidth(shares) - 1).
// Export: square width = RoundUpPow2(ceil(sqrt(worst case))); blobs stably sorted by
// namespace, each placed at the next multiple of its SubTreeWidth; PFB index wrappers
// carry the real start indexes; primary reserved padding up to the first blob,
// namespace padding (previous blob's namespace) between blobs, tail padding to k*k.
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/celestia_eds.h"

namespace cel {
namespace sq {
namespace {  // internal linkage: only the C entry points are exported

constexpr uint32_t kShare = CEL_SHARE_SIZE;
constexpr uint32_t kNs = CEL_NAMESPACE_SIZE;
constexpr uint32_t kNsIdSize = 28;
// compact share payload: first share ns | info | sequence length(4) | reserved(4)
constexpr uint32_t kCompactFirst = kShare - kNs - 1 - 4 - 4;  // 474
constexpr uint32_t kCompactCont = kShare - kNs - 1 - 4;       // 478
// sparse share payload: first share ns | info | sequence length(4)
constexpr uint32_t kSparseFirst = kShare - kNs - 1 - 4;  // 478
constexpr uint32_t kSparseCont = kShare - kNs - 1;       // 482

using Bytes = std::vector<uint8_t>;
using Ns = std::array<uint8_t, kNs>;

static Ns ns_of(uint8_t version, uint8_t last) {
  Ns n{};
  n[0] = version;
  n[kNs - 1] = last;
  return n;
}
static const Ns kTxNs = ns_of(0, 0x01);              // namespace.md:79 TxNamespace
static const Ns kPfbNs = ns_of(0, 0x04);             // PayForBlobNamespace
static const Ns kPrimaryPadNs = ns_of(0, 0xFF);      // PrimaryReservedPaddingNamespace
static Ns tail_pad_ns() {                            // TailPaddingNamespace 0xFF*28 || 0xFE
  Ns n;
  n.fill(0xFF);
  n[kNs - 1] = 0xFE;
  return n;
}

static void put_uvarint(Bytes& out, uint64_t v) {
  while (v >= 0x80) {
    out.push_back((uint8_t)(v | 0x80));
    v >>= 7;
  }
  out.push_back((uint8_t)v);
}
static uint32_t uvarint_len(uint64_t v) {
  uint32_t n = 1;
  while (v >= 0x80) {
    v >>= 7;
    n++;
  }
  return n;
}

// ----------------------------------------------------------- protobuf wire reads
struct Field {
  uint32_t num, wire;
  uint64_t varint;
  const uint8_t* p;
  size_t len;
};

static bool read_uvarint(const uint8_t*& p, const uint8_t* end, uint64_t& v) {
  v = 0;
  for (int shift = 0; shift < 64; shift += 7) {
    if (p >= end) return false;
    const uint8_t b = *p++;
    v |= (uint64_t)(b & 0x7F) << shift;
    if (!(b & 0x80)) return true;
  }
  return false;
}

// Skips the rest of a group whose start key (wire type 3) was just read: nested fields up
// to the matching end-group key. The generated gogoproto skip function (skipBlob) does the
// same for unknown fields; false where it returns an error.
static bool skip_group(const uint8_t*& p, const uint8_t* end) {
  int depth = 1;
  while (p < end) {
    uint64_t key, v;
    if (!read_uvarint(p, end, key)) return false;
    switch (key & 7) {
      case 0:
        if (!read_uvarint(p, end, v)) return false;
        break;
      case 1:
        if (end - p < 8) return false;
        p += 8;
        break;
      case 2:
        if (!read_uvarint(p, end, v) || v > (uint64_t)(end - p)) return false;
        p += v;
        break;
      case 3:
        depth++;
        break;
      case 4:
        if (--depth == 0) return true;
        break;
      case 5:
        if (end - p < 4) return false;
        p += 4;
        break;
      default:
        return false;
    }
  }
  return false;
}

// Decodes one message level; false on malformed wire data (proto.Unmarshal error). The
// field number is the key's bits 3.. taken as an int32, and must be > 0 (gogoproto
// "illegal tag"); an end-group key outside a group is an error; a group (wire type 3) is
// kept as a field of wire type 3 so that a known field number rejects it.
static bool parse_fields(const uint8_t* p, size_t n, std::vector<Field>& out) {
  const uint8_t* end = p + n;
  while (p < end) {
    uint64_t key;
    if (!read_uvarint(p, end, key)) return false;
    Field f{(uint32_t)(key >> 3), (uint32_t)(key & 7), 0, nullptr, 0};
    if ((int32_t)f.num <= 0) return false;
    switch (f.wire) {
      case 0:
        if (!read_uvarint(p, end, f.varint)) return false;
        break;
      case 1:
        if (end - p < 8) return false;
        f.p = p;
        f.len = 8;
        p += 8;
        break;
      case 2: {
        uint64_t ln;
        if (!read_uvarint(p, end, ln) || ln > (uint64_t)(end - p)) return false;
        f.p = p;
        f.len = (size_t)ln;
        p += ln;
        break;
      }
      case 3:
        if (!skip_group(p, end)) return false;
        break;
      case 5:
        if (end - p < 4) return false;
        f.p = p;
        f.len = 4;
        p += 4;
        break;
      default:
        return false;
    }
    out.push_back(f);
  }
  return true;
}

struct Blob {
  Ns ns;
  const uint8_t* data;
  size_t len;
  uint32_t share_version;
};

// blob.UnmarshalBlobTx (go-square v1.1.0 blob/blob.go): BlobTx {1: tx, 2: repeated Blob,
// 3: type_id}; a blob tx iff it parses, type_id == "BLOB", it has blobs and every
// namespace id is 28 bytes. Blob {1: namespace_id, 2: data, 3: share_version,
// 4: namespace_version} (proto/celestia/core/v1/blob/blob.proto).
static bool unmarshal_blob_tx(const uint8_t* tx, size_t n, const uint8_t*& inner, size_t& inner_len,
                              std::vector<Blob>& blobs) {
  std::vector<Field> fs;
  if (!parse_fields(tx, n, fs)) return false;
  bool typed = false;
  inner = nullptr;
  inner_len = 0;
  blobs.clear();
  for (const Field& f : fs) {
    if (f.num == 1) {
      if (f.wire != 2) return false;
      inner = f.p;
      inner_len = f.len;
    } else if (f.num == 2) {
      if (f.wire != 2) return false;
      std::vector<Field> bf;
      if (!parse_fields(f.p, f.len, bf)) return false;
      Blob b{};
      const uint8_t* id = nullptr;
      size_t id_len = 0;
      uint64_t ns_version = 0;
      for (const Field& g : bf) {
        if (g.num == 1) {
          if (g.wire != 2) return false;
          id = g.p;
          id_len = g.len;
        } else if (g.num == 2) {
          if (g.wire != 2) return false;
          b.data = g.p;
          b.len = g.len;
        } else if (g.num == 3) {
          if (g.wire != 0) return false;
          b.share_version = (uint32_t)g.varint;
        } else if (g.num == 4) {
          if (g.wire != 0) return false;
          ns_version = g.varint;
        }
      }
      if (id_len != kNsIdSize) return false;
      b.ns[0] = (uint8_t)ns_version;
      std::memcpy(b.ns.data() + 1, id, kNsIdSize);
      blobs.push_back(b);
    } else if (f.num == 3) {
      if (f.wire != 2) return false;
      typed = f.len == 4 && std::memcmp(f.p, "BLOB", 4) == 0;
    }
  }
  return typed && !blobs.empty();
}

// IndexWrapper {1: tx, 2: packed share_indexes, 3: type_id "INDX"} (gogoproto Marshal).
static Bytes marshal_index_wrapper(const uint8_t* tx, size_t n, const std::vector<uint32_t>& idx) {
  Bytes packed;
  for (uint32_t i : idx) put_uvarint(packed, i);
  Bytes out;
  if (n) {  // proto3 omits empty bytes fields
    out.push_back(0x0A);
    put_uvarint(out, n);
    out.insert(out.end(), tx, tx + n);
  }
  if (!packed.empty()) {
    out.push_back(0x12);
    put_uvarint(out, packed.size());
    out.insert(out.end(), packed.begin(), packed.end());
  }
  out.push_back(0x1A);
  out.push_back(4);
  out.insert(out.end(), {'I', 'N', 'D', 'X'});
  return out;
}

// ------------------------------------------------------------------ share counts
// shares.CompactShareCounter: units are uvarint(len) || unit, packed in one sequence.
static uint32_t compact_shares_for(uint64_t seq_bytes) {
  if (seq_bytes == 0) return 0;
  if (seq_bytes <= kCompactFirst) return 1;
  return 1 + (uint32_t)((seq_bytes - kCompactFirst + kCompactCont - 1) / kCompactCont);
}
// shares.SparseSharesNeeded
static uint32_t sparse_shares_for(uint64_t len) {
  if (len == 0) return 0;
  if (len <= kSparseFirst) return 1;
  return 1 + (uint32_t)((len - kSparseFirst + kSparseCont - 1) / kSparseCont);
}
static uint32_t pow2ceil(uint64_t n) {
  uint32_t r = 1;
  while (r < n) r <<= 1;
  return r;
}
// inclusion.BlobMinSquareSize / SubTreeWidth / NextShareIndex (go-square v1.1.0)
static uint32_t blob_min_square_size(uint64_t shares) {
  return pow2ceil((uint64_t)std::ceil(std::sqrt((double)shares)));
}
static uint32_t subtree_width(uint32_t shares, uint32_t threshold) {
  const uint32_t s = pow2ceil((shares + threshold - 1) / threshold);
  const uint32_t m = blob_min_square_size(shares);
  return s < m ? s : m;
}
static uint32_t next_share_index(uint32_t cursor, uint32_t shares, uint32_t threshold) {
  const uint32_t w = subtree_width(shares, threshold);
  return (cursor + w - 1) / w * w;
}

// ---------------------------------------------------------------- share writers
static void write_compact(const Ns& ns, const std::vector<Bytes>& units, std::vector<uint8_t>& sq) {
  if (units.empty()) return;
  Bytes data;
  std::vector<size_t> starts;
  for (const Bytes& u : units) {
    starts.push_back(data.size());
    put_uvarint(data, u.size());
    data.insert(data.end(), u.begin(), u.end());
  }
  size_t pos = 0, next_unit = 0;
  for (bool first = true; first || pos < data.size(); first = false) {
    uint8_t sh[kShare] = {0};
    std::memcpy(sh, ns.data(), kNs);
    sh[kNs] = first ? 1 : 0;  // share version 0, sequence start
    uint32_t header = kNs + 1;
    if (first) {
      const uint32_t L = (uint32_t)data.size();
      sh[header] = (uint8_t)(L >> 24), sh[header + 1] = (uint8_t)(L >> 16);
      sh[header + 2] = (uint8_t)(L >> 8), sh[header + 3] = (uint8_t)L;
      header += 4;
    }
    const uint32_t cap = kShare - header - 4;
    // reserved bytes: offset (within this share) of the first unit that starts in it
    while (next_unit < starts.size() && starts[next_unit] < pos) next_unit++;
    uint32_t reserved = 0;
    if (next_unit < starts.size() && starts[next_unit] < pos + cap) reserved = header + 4 + (uint32_t)(starts[next_unit] - pos);
    sh[header] = (uint8_t)(reserved >> 24), sh[header + 1] = (uint8_t)(reserved >> 16);
    sh[header + 2] = (uint8_t)(reserved >> 8), sh[header + 3] = (uint8_t)reserved;
    const size_t n = std::min<size_t>(cap, data.size() - std::min(pos, data.size()));
    if (n) std::memcpy(sh + header + 4, data.data() + pos, n);
    sq.insert(sq.end(), sh, sh + kShare);
    pos += cap;
  }
}

static void write_sparse(const Blob& b, std::vector<uint8_t>& sq) {
  size_t pos = 0;
  for (bool first = true; pos < b.len; first = false) {
    uint8_t sh[kShare] = {0};
    std::memcpy(sh, b.ns.data(), kNs);
    sh[kNs] = (uint8_t)((b.share_version << 1) | (first ? 1 : 0));
    uint32_t header = kNs + 1;
    if (first) {
      const uint32_t L = (uint32_t)b.len;
      sh[header] = (uint8_t)(L >> 24), sh[header + 1] = (uint8_t)(L >> 16);
      sh[header + 2] = (uint8_t)(L >> 8), sh[header + 3] = (uint8_t)L;
      header += 4;
    }
    const size_t n = std::min<size_t>(kShare - header, b.len - pos);
    std::memcpy(sh + header, b.data + pos, n);
    sq.insert(sq.end(), sh, sh + kShare);
    pos += n;
  }
}

static void write_padding(const Ns& ns, uint32_t count, std::vector<uint8_t>& sq) {
  for (uint32_t i = 0; i < count; i++) {
    uint8_t sh[kShare] = {0};
    std::memcpy(sh, ns.data(), kNs);
    sh[kNs] = 1;  // share version 0, sequence start; sequence length 0
    sq.insert(sq.end(), sh, sh + kShare);
  }
}

// -------------------------------------------------------------------- builder
struct Pfb {
  const uint8_t* tx;
  size_t len;
  std::vector<uint32_t> idx;
};
struct Element {
  Blob blob;
  uint32_t pfb, index, shares;
};

struct Builder {
  uint32_t max_size, threshold;
  uint64_t max_capacity;
  uint64_t current = 0;        // worst-case share count so far
  uint64_t tx_bytes = 0, pfb_bytes = 0;  // compact sequence lengths (counters)
  std::vector<Bytes> txs;
  std::vector<Pfb> pfbs;
  std::vector<Element> blobs;
  std::vector<Bytes> iws;  // final PFB index wrappers (after export_square)

  Builder(uint32_t m, uint32_t t) : max_size(m), threshold(t), max_capacity((uint64_t)m * m) {}

  // Builder.AppendTx
  bool append_tx(const uint8_t* tx, size_t n) {
    const uint64_t nb = tx_bytes + uvarint_len(n) + n;
    const uint64_t diff = compact_shares_for(nb) - compact_shares_for(tx_bytes);
    if (current + diff > max_capacity) return false;
    current += diff;
    tx_bytes = nb;
    txs.emplace_back(tx, tx + n);
    return true;
  }

  // Builder.AppendBlobTx: the index wrapper is counted with worst-case share indexes
  // (maxSquareSize^2), each blob with its shares plus SubTreeWidth - 1 of padding.
  bool append_blob_tx(const uint8_t* inner, size_t n, const std::vector<Blob>& bl) {
    const std::vector<uint32_t> worst(bl.size(), max_size * max_size);
    const size_t iw = marshal_index_wrapper(inner, n, worst).size();
    const uint64_t nb = pfb_bytes + uvarint_len(iw) + iw;
    uint64_t diff = compact_shares_for(nb) - compact_shares_for(pfb_bytes);
    for (const Blob& b : bl) {
      const uint32_t s = sparse_shares_for(b.len);
      diff += s + subtree_width(s, threshold) - 1;
    }
    if (current + diff > max_capacity) return false;
    current += diff;
    pfb_bytes = nb;
    const uint32_t pi = (uint32_t)pfbs.size();
    pfbs.push_back(Pfb{inner, n, std::vector<uint32_t>(bl.size(), 0)});
    for (uint32_t i = 0; i < bl.size(); i++) blobs.push_back(Element{bl[i], pi, i, sparse_shares_for(bl[i].len)});
    return true;
  }

  // Builder.Export
  uint32_t export_square(std::vector<uint8_t>& sq) {
    sq.clear();
    if (txs.empty() && pfbs.empty()) {  // EmptySquare: one tail padding share
      write_padding(tail_pad_ns(), 1, sq);
      return 1;
    }
    const uint32_t k = blob_min_square_size(current);
    std::stable_sort(blobs.begin(), blobs.end(),
                     [](const Element& a, const Element& b) { return a.blob.ns < b.blob.ns; });
    const uint32_t non_reserved = compact_shares_for(tx_bytes) + compact_shares_for(pfb_bytes);
    uint32_t cursor = non_reserved, end_of_last = non_reserved;
    std::vector<uint8_t> blob_sq;
    for (size_t i = 0; i < blobs.size(); i++) {
      const Element& e = blobs[i];
      cursor = next_share_index(cursor, e.shares, threshold);
      pfbs[e.pfb].idx[e.index] = cursor;
      if (i) write_padding(blobs[i - 1].blob.ns, cursor - end_of_last, blob_sq);
      write_sparse(e.blob, blob_sq);
      cursor += e.shares;
      end_of_last = cursor;
    }
    iws.clear();
    for (const Pfb& p : pfbs) iws.push_back(marshal_index_wrapper(p.tx, p.len, p.idx));
    write_compact(kTxNs, txs, sq);
    write_compact(kPfbNs, iws, sq);
    // WriteSquare: primary reserved padding up to the first blob, the blobs, tail padding
    const uint32_t first_blob = blobs.empty() ? (uint32_t)(sq.size() / kShare) : pfbs[blobs[0].pfb].idx[blobs[0].index];
    write_padding(kPrimaryPadNs, first_blob - (uint32_t)(sq.size() / kShare), sq);
    sq.insert(sq.end(), blob_sq.begin(), blob_sq.end());
    const uint32_t have = (uint32_t)(sq.size() / kShare);
    write_padding(tail_pad_ns(), (uint32_t)((uint64_t)k * k - have), sq);
    return k;
  }

  // Builder.FindTxShareRange (after export_square): the shares [start, end) holding the
  // uvarint(len) || tx unit of normal tx `i` (i < txs.size()) or of the PFB index
  // wrapper i - txs.size() (offset by the tx shares, which precede the PFB shares).
  bool tx_range(size_t i, uint32_t& start, uint32_t& end) const {
    const bool pfb = i >= txs.size();
    const std::vector<Bytes>& units = pfb ? iws : txs;
    const size_t u = pfb ? i - txs.size() : i;
    if (u >= units.size()) return false;
    uint64_t off = 0;
    for (size_t j = 0; j < u; j++) off += uvarint_len(units[j].size()) + units[j].size();
    const uint64_t last = off + uvarint_len(units[u].size()) + units[u].size() - 1;
    auto share_of = [](uint64_t b) -> uint32_t {
      return b < kCompactFirst ? 0u : 1u + (uint32_t)((b - kCompactFirst) / kCompactCont);
    };
    const uint32_t base = pfb ? compact_shares_for(tx_bytes) : 0u;
    start = base + share_of(off);
    end = base + share_of(last) + 1;
    return true;
  }
};

}  // namespace
}  // namespace sq
}  // namespace cel

namespace {
thread_local std::string g_square_error;
}

extern "C" {

const char* cel_square_last_error(void) { return g_square_error.c_str(); }

}  // extern "C"

namespace {

// NewBuilder(txs...) / Build's admission loop; fills included[] (0 / 1 normal / 2 blob).
cel_status build_square(cel::sq::Builder& b, const uint8_t* txs, const uint32_t* tx_lens, uint32_t ntx,
                        uint32_t greedy, uint8_t* included) {
  using namespace cel::sq;
  size_t off = 0;
  bool seen_blob_tx = false;
  std::vector<Blob> blobs;
  for (uint32_t i = 0; i < ntx; i++) {
    const uint8_t* tx = txs + off;
    const size_t n = tx_lens[i];
    off += n;
    const uint8_t* inner;
    size_t inner_len;
    bool ok;
    const bool is_blob = unmarshal_blob_tx(tx, n, inner, inner_len, blobs);
    if (is_blob) {
      seen_blob_tx = true;
      ok = b.append_blob_tx(inner, inner_len, blobs);
    } else {
      if (seen_blob_tx && !greedy) {  // square.Construct requires normal txs first
        g_square_error = "normal transaction at index " + std::to_string(i) + " can not be appended after blob tx";
        return CEL_EINVAL;
      }
      ok = b.append_tx(tx, n);
    }
    if (included) included[i] = ok ? (is_blob ? 2 : 1) : 0;
    if (!ok && !greedy) {
      g_square_error = std::string("not enough space to append ") + (seen_blob_tx ? "blob tx" : "tx") +
                       " at index " + std::to_string(i);
      return CEL_ETOOBIG;
    }
  }
  return CEL_OK;
}

bool args_ok(const uint8_t* txs, const uint32_t* tx_lens, uint32_t ntx, uint32_t max_square_size,
             uint32_t subtree_root_threshold) {
  return !((ntx && (!txs || !tx_lens)) || !max_square_size || !subtree_root_threshold ||
           (max_square_size & (max_square_size - 1)));
}

}  // namespace

extern "C" {

cel_status cel_square_construct(const uint8_t* txs, const uint32_t* tx_lens, uint32_t ntx, uint32_t max_square_size,
                                uint32_t subtree_root_threshold, uint32_t greedy, uint8_t* shares_out,
                                uint32_t cap_shares, uint32_t* k_out, uint8_t* included) {
  using namespace cel::sq;
  g_square_error.clear();
  if (!k_out || !args_ok(txs, tx_lens, ntx, max_square_size, subtree_root_threshold)) {
    g_square_error = "invalid argument";
    return CEL_EINVAL;
  }
  Builder b(max_square_size, subtree_root_threshold);
  cel_status st = build_square(b, txs, tx_lens, ntx, greedy, included);
  if (st) return st;
  std::vector<uint8_t> sq;
  const uint32_t k = b.export_square(sq);
  *k_out = k;
  if (!shares_out) return CEL_OK;  // size query
  if ((uint64_t)k * k > cap_shares) {
    g_square_error = "output buffer holds " + std::to_string(cap_shares) + " shares, square needs " +
                     std::to_string((uint64_t)k * k);
    return CEL_EINVAL;
  }
  std::memcpy(shares_out, sq.data(), sq.size());
  return CEL_OK;
}

cel_status cel_square_tx_range(const uint8_t* txs, const uint32_t* tx_lens, uint32_t ntx, uint32_t max_square_size,
                               uint32_t subtree_root_threshold, uint32_t tx_index, uint32_t* start, uint32_t* end) {
  using namespace cel::sq;
  g_square_error.clear();
  if (!start || !end || !args_ok(txs, tx_lens, ntx, max_square_size, subtree_root_threshold)) {
    g_square_error = "invalid argument";
    return CEL_EINVAL;
  }
  if (tx_index >= ntx) {  // pkg/proof/proof.go:23-25
    g_square_error = "txIndex " + std::to_string(tx_index) + " out of bounds";
    return CEL_EINVAL;
  }
  Builder b(max_square_size, subtree_root_threshold);
  cel_status st = build_square(b, txs, tx_lens, ntx, 0, nullptr);
  if (st) return st;
  std::vector<uint8_t> sq;
  b.export_square(sq);
  if (!b.tx_range(tx_index, *start, *end)) {
    g_square_error = "txIndex " + std::to_string(tx_index) + " out of range";
    return CEL_EINVAL;
  }
  return CEL_OK;
}

}  // extern "C"
