"""ORACLE — TEST INFRASTRUCTURE ONLY.

Restatement of the go-square v1.1.0 square construction (go.mod:9, [dep], not in
/root/reference) for app v1 (SquareSizeUpperBound 128, SubtreeRootThreshold 64;
pkg/appconsts/v1/app_consts.go). It turns a block's txs into the k*k ODS that
da.ExtendShares receives (app/extend_block.go:16-25, app/prepare_proposal.go:50-61).

It exists to turn mainnet block 408 (x/blob/test/testdata/block_response.json) into
a known-answer test for the whole EDS+NMT+DAH path: the block's data_hash pins
GF(2^8) Leopard, the NMT wrapper and the DAH hash together. Rules followed:
  - share format: specs/src/specs/shares.md:24-98 (compact shares with reserved
    bytes, sparse blob shares, padding shares)
  - reserved namespaces: specs/src/specs/namespace.md:77-84
  - layout / blob alignment: specs/src/specs/data_square_layout.md:38-62
  - SURVEY.md Appendix A.4 (the procedure verified against the block's data root).
"""
import base64
import json
import math

SHARE = 512
NS = 29
TX_NS = bytes(28) + b"\x01"
PFB_NS = bytes(28) + b"\x04"
PRIMARY_PAD_NS = bytes(28) + b"\xff"
TAIL_PAD_NS = b"\xff" * 28 + b"\xfe"
MAX_SQUARE = 128           # app v1 SquareSizeUpperBound
SUBTREE_ROOT_THRESHOLD = 64


def uvarint(n: int) -> bytes:
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


class WireError(ValueError):
    """proto.Unmarshal error (the gogoproto generated decoder's error cases)."""


def _read_varint(buf, i):
    """At most 10 bytes (shift < 64); the bits past 64 are dropped, as in Go."""
    val = 0
    for shift in range(0, 64, 7):
        if i >= len(buf):
            raise WireError("unexpected EOF")
        b = buf[i]
        i += 1
        val |= (b & 0x7F) << shift
        if not b & 0x80:
            return val & (2**64 - 1), i
    raise WireError("integer overflow")


def _skip_group(buf, i):
    """The rest of a group after its start key: nested fields up to the matching
    end-group key (gogoproto skipBlob)."""
    depth = 1
    while i < len(buf):
        key, i = _read_varint(buf, i)
        wt = key & 7
        if wt == 0:
            _, i = _read_varint(buf, i)
        elif wt == 1 or wt == 5:
            i += 8 if wt == 1 else 4
            if i > len(buf):
                raise WireError("unexpected EOF")
        elif wt == 2:
            ln, i = _read_varint(buf, i)
            if ln > len(buf) - i:
                raise WireError("unexpected EOF")
            i += ln
        elif wt == 3:
            depth += 1
        elif wt == 4:
            depth -= 1
            if depth == 0:
                return i
        else:
            raise WireError("illegal wire type")
    raise WireError("unexpected EOF")


def parse_proto(buf: bytes):
    """Protobuf wire decoder for one message level -> list of (field, wiretype, value),
    raising WireError where the generated gogoproto Unmarshal fails: truncated data,
    varints over 10 bytes, field number (key >> 3 as int32) <= 0, wire types 4, 6, 7.
    A group (wire type 3) is skipped and listed with value None."""
    i, out = 0, []
    while i < len(buf):
        key, i = _read_varint(buf, i)
        field, wt = key >> 3, key & 7
        f32 = field & 0xFFFFFFFF
        if f32 == 0 or f32 >= 2**31:
            raise WireError("illegal tag")
        if wt == 0:
            v, i = _read_varint(buf, i)
        elif wt == 2:
            ln, i = _read_varint(buf, i)
            if ln > len(buf) - i:
                raise WireError("unexpected EOF")
            v = buf[i:i + ln]
            i += ln
        elif wt == 1 or wt == 5:
            n = 8 if wt == 1 else 4
            if len(buf) - i < n:
                raise WireError("unexpected EOF")
            v = buf[i:i + n]
            i += n
        elif wt == 3:
            i = _skip_group(buf, i)
            v = None
        else:
            raise WireError("illegal wire type")
        out.append((f32, wt, v))
    return out


def unmarshal_blob_tx(tx: bytes):
    """go-square blob.UnmarshalBlobTx (the two-value form the reference calls,
    pkg/proof/proof.go:52): BlobTx {1: tx, 2: repeated Blob, 3: type_id}
    (proto/celestia/core/v1/blob/blob.proto). None (not a blob tx) unless the message
    decodes, its type_id is "BLOB", it has blobs and every namespace id is 28 bytes.
    A known field with another wire type is a decode error; repeated scalar fields keep
    the last value; share_version / namespace_version are uint32 (varint truncated)."""
    try:
        fields = parse_proto(tx)
        inner, type_id, blobs = b"", b"", []
        for f, wt, v in fields:
            if f in (1, 2, 3) and wt != 2:
                return None
            if f == 1:
                inner = bytes(v)
            elif f == 3:
                type_id = bytes(v)
            elif f == 2:
                b = {1: b"", 2: b"", 3: 0, 4: 0}
                for bf, bwt, bv in parse_proto(v):
                    if bf in (1, 2) and bwt != 2 or bf in (3, 4) and bwt != 0:
                        return None
                    if bf in (1, 2, 3, 4):
                        b[bf] = bv if bf in (1, 2) else bv & 0xFFFFFFFF
                blobs.append(b)
    except WireError:
        return None
    if type_id != b"BLOB" or not blobs or any(len(b[1]) != 28 for b in blobs):
        return None
    return inner, [{"ns": bytes([b[4] & 0xFF]) + bytes(b[1]), "data": bytes(b[2]), "share_version": b[3]}
                   for b in blobs]


def index_wrapper(tx: bytes, share_indexes) -> bytes:
    """IndexWrapper {1: tx, 2: packed share_indexes, 3: type_id "INDX"}."""
    packed = b"".join(uvarint(i) for i in share_indexes)
    return (b"\x0a" + uvarint(len(tx)) + tx + b"\x12" + uvarint(len(packed)) + packed +
            b"\x1a\x04INDX")


def compact_shares(ns: bytes, units) -> list:
    """Compact (tx/pfb) share sequence: every unit is uvarint(len) || unit."""
    data = b"".join(uvarint(len(u)) + u for u in units)
    starts = []
    off = 0
    for u in units:
        starts.append(off)
        off += len(uvarint(len(u))) + len(u)
    shares = []
    pos = 0
    first = True
    while pos < len(data) or first:
        header = NS + 1 + (4 if first else 0) + 4
        cap = SHARE - header
        chunk = data[pos:pos + cap]
        # reserved bytes: absolute index in this share of the first unit starting in it
        reserved = 0
        for s in starts:
            if pos <= s < pos + cap:
                reserved = header + (s - pos)
                break
        sh = ns + bytes([1 if first else 0])
        if first:
            sh += len(data).to_bytes(4, "big")
        sh += reserved.to_bytes(4, "big") + chunk
        sh += bytes(SHARE - len(sh))
        shares.append(sh)
        pos += cap
        first = False
    return shares


def compact_share_count(units) -> int:
    total = sum(len(uvarint(len(u))) + len(u) for u in units)
    if total == 0:  # shares.CompactShareCounter.Size() of an empty sequence
        return 0
    if total <= SHARE - NS - 1 - 4 - 4:
        return 1
    rest = total - (SHARE - NS - 1 - 4 - 4)
    return 1 + math.ceil(rest / (SHARE - NS - 1 - 4))


def sparse_shares(blob) -> list:
    ns, data, ver = blob["ns"], blob["data"], blob["share_version"]
    shares, pos, first = [], 0, True
    while pos < len(data) or first:
        head = ns + bytes([((ver << 1) | (1 if first else 0)) & 0xFF])  # the product truncates too
        if first:
            head += len(data).to_bytes(4, "big")
        cap = SHARE - len(head)
        sh = head + data[pos:pos + cap]
        sh += bytes(SHARE - len(sh))
        shares.append(sh)
        pos += cap
        first = False
    return shares


def padding_share(ns: bytes) -> bytes:
    sh = ns + b"\x01" + bytes(4)
    return sh + bytes(SHARE - len(sh))


def pow2ceil(n: int) -> int:
    r = 1
    while r < n:
        r <<= 1
    return r


def subtree_width(share_count: int) -> int:
    s = math.ceil(share_count / SUBTREE_ROOT_THRESHOLD)
    return min(pow2ceil(s), pow2ceil(math.ceil(math.sqrt(share_count))))


def build_square(txs):
    normal, pfbs = [], []
    for tx in txs:
        r = unmarshal_blob_tx(tx)
        if r is None:
            normal.append(tx)
        else:
            pfbs.append(r)
    worst = MAX_SQUARE * MAX_SQUARE
    tx_count = compact_share_count(normal)
    pfb_units_worst = [index_wrapper(t, [worst] * len(b)) for t, b in pfbs]
    pfb_count = compact_share_count(pfb_units_worst) if pfbs else 0
    blobs = [b for _, bl in pfbs for b in bl]
    # blobs are laid out in namespace order (stable)
    order = sorted(range(len(blobs)), key=lambda i: blobs[i]["ns"])
    cursor = tx_count + pfb_count
    starts = {}
    for i in order:
        n = len(sparse_shares(blobs[i]))
        w = subtree_width(n)
        start = ((cursor + w - 1) // w) * w
        starts[i] = start
        cursor = start + n
    # square size: smallest power of two whose square holds everything (with the
    # worst-case padding go-square reserves per blob)
    worst_total = tx_count + pfb_count + sum(len(sparse_shares(b)) + subtree_width(len(sparse_shares(b))) - 1
                                             for b in blobs)
    k = pow2ceil(math.ceil(math.sqrt(max(worst_total, 1))))
    assert cursor <= k * k
    # real PFB units carry the real share indexes
    idx = 0
    pfb_units = []
    for t, bl in pfbs:
        pfb_units.append(index_wrapper(t, [starts[idx + j] for j in range(len(bl))]))
        idx += len(bl)
    square = compact_shares(TX_NS, normal) if normal else []
    if pfbs:
        square += compact_shares(PFB_NS, pfb_units)
    first_blob = min(starts.values()) if starts else len(square)
    while len(square) < first_blob:
        square.append(padding_share(PRIMARY_PAD_NS))
    prev_ns = None
    for i in order:
        while len(square) < starts[i]:
            square.append(padding_share(prev_ns))  # namespace padding
        square += sparse_shares(blobs[i])
        prev_ns = blobs[i]["ns"]
    while len(square) < k * k:
        square.append(padding_share(TAIL_PAD_NS))
    return k, square


def block408_ods(json_path):
    with open(json_path) as f:
        blk = json.load(f)["block"]
    txs = [base64.b64decode(t) for t in blk["data"]["txs"]]
    k, square = build_square(txs)
    data_hash = base64.b64decode(blk["header"]["data_hash"])
    return k, b"".join(square), data_hash, int(blk["header"]["height"])
