"""pkg/proof mirror: share inclusion proofs to the data root.

Construction (NewShareInclusionProofFromEDS, pkg/proof/proof.go:78-140, and
CreateShareToRowRootProofs, :147-202) reads the NMT nodes of the rows that hold the
shares from the device (cel_axis_trees: every node of those row trees, hashed on the
MI355X) and the row-root proofs from the device-built RFC-6962 tree over
rowRoots || colRoots (cel_dah_tree); cel_nmt_prove_range / cel_merkle_aunts pick the
proof nodes (nmt ProveRange, merkle.ProofsFromByteSlices). The reference instead
rebuilds every row tree on the CPU.

Verification (ShareProof.Validate / VerifyProof, share_proof.go:15-82; RowProof,
row_proof.go:12-48) mirrors the reference on the host: nmt VerifyInclusion (nmt
v0.22.0 proof.go [dep]: leaf hashing with the namespace prefix, completeness check,
computeRoot) and go-square merkle Proof.Verify (RFC-6962). Host-side hashing is the
reference's own choice for verifiers (a light client verifies on its CPU).

Wire format (proto/celestia/core/v1/proof/proof.proto:8-49, gogoproto-generated
pkg/proof/proof.pb.go): ShareProof / RowProof / NMTProof / Proof .Marshal() and
Unmarshal(bytes), the bytes QueryTxInclusionProof / QueryShareInclusionProof return
(pkg/proof/querier.go:53-63).
"""
import ctypes
import hashlib
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from . import _lib
from ._lib import CelError

NS = _lib.NAMESPACE_SIZE
NODE = _lib.NMT_NODE_SIZE
PARITY_NS = b"\xff" * NS


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


# --------------------------------------------------------------------- hashing
def _sha(b):
    return hashlib.sha256(b).digest()


def _nmt_leaf(ns, data):
    """nmt HashLeaf: ns || ns || SHA256(0x00 || ns || data) (data without the ns prefix)."""
    return ns + ns + _sha(b"\x00" + ns + data)


def _nmt_node(left, right, nsz=NS):
    """nmt HashNode with IgnoreMaxNamespace (test/util/malicious/hasher.go:186-310 text copy):
    minNs = L.min; maxNs = L.max if R.min is the max namespace (0xFF * nsz) else
    max(L.max, R.max). Children must be ordered (L.max <= R.min). nmt is generic in the
    namespace size: the app uses 29 bytes, nsz follows the verified namespace."""
    lmin, lmax, rmin, rmax = left[:nsz], left[nsz:2 * nsz], right[:nsz], right[nsz:2 * nsz]
    if lmax > rmin:
        raise ValueError("unordered nmt children")
    mx = lmax if rmin == b"\xff" * nsz else (rmax if rmax > lmax else lmax)
    return lmin + mx + _sha(b"\x01" + left + right)


def _split_point(n):
    """largest power of two strictly less than n (n >= 2)"""
    k = 1
    while k * 2 < n:
        k *= 2
    return k


def _rfc_leaf(item):
    return _sha(b"\x00" + item)


def _rfc_inner(left, right):
    return _sha(b"\x01" + left + right)


# ---------------------------------------------------------------- proto3 wire
# gogoproto's generated Marshal / Unmarshal for these four messages (proof.pb.go):
# fields in ascending number; scalars and singular bytes omitted when zero / empty;
# every element of a repeated field written (empty ones too); a set sub-message written
# even when empty; negative int32 / int64 as 10-byte two's-complement varints. Unmarshal
# skips unknown fields by wire type and rejects a known field with the wrong wire type.
def _uvarint(n):
    n &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        out.append(b | (0x80 if n else 0))
        if not n:
            return bytes(out)


def _key(field, wt):
    return _uvarint(field << 3 | wt)


def _w_varint(field, v):
    return _key(field, 0) + _uvarint(v) if v else b""


def _w_bytes(field, b, always=False):
    b = bytes(b) if b is not None else b""
    return _key(field, 2) + _uvarint(len(b)) + b if (b or always) else b""


class _Reader:
    def __init__(self, buf, msg):
        self.buf, self.i, self.msg = bytes(buf), 0, msg

    def _err(self, what):
        return CelError(_lib.EINVAL, f"proto: {self.msg}: {what}")

    def uvarint(self):
        v, shift = 0, 0
        while True:
            if self.i >= len(self.buf):
                raise self._err("unexpected EOF")
            if shift >= 64:
                raise self._err("integer overflow")
            b = self.buf[self.i]
            self.i += 1
            v |= (b & 0x7F) << shift
            if not b & 0x80:
                return v & ((1 << 64) - 1)
            shift += 7

    def fields(self):
        """Yield (field number, wire type) until the end; the caller reads the value."""
        while self.i < len(self.buf):
            key = self.uvarint()
            field, wt = key >> 3, key & 7
            if field <= 0 or key >> 3 > 0x7FFFFFFF:
                raise self._err(f"illegal tag {field} (wire type {wt})")
            yield field, wt

    def lendelim(self):
        n = self.uvarint()
        if n > len(self.buf) - self.i:
            raise self._err("unexpected EOF")
        b = self.buf[self.i:self.i + n]
        self.i += n
        return b

    def skip(self, wt, depth=0):
        if wt == 0:
            self.uvarint()
        elif wt == 1:
            self._need(8)
        elif wt == 2:
            self.lendelim()
        elif wt == 5:
            self._need(4)
        elif wt == 3:  # start group: skip to the matching end group
            if depth > 100:
                raise self._err("nesting too deep")
            while True:
                if self.i >= len(self.buf):
                    raise self._err("unexpected EOF")
                key = self.uvarint()
                if key & 7 == 4:
                    return
                self.skip(key & 7, depth + 1)
        else:  # 4 (end group outside a group), 6, 7
            raise self._err(f"illegal wireType {wt}")

    def _need(self, n):
        if n > len(self.buf) - self.i:
            raise self._err("unexpected EOF")
        self.i += n

    def want(self, wt, need, name):
        if wt != need:
            raise self._err(f"wrong wireType = {wt} for field {name}")


def _int32(v):
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v >= 1 << 31 else v


def _int64(v):
    return v - (1 << 64) if v >= 1 << 63 else v


# -------------------------------------------------------------------- types
@dataclass
class NMTProof:
    """proof.NMTProof (proto/celestia/core/v1/proof/proof.proto): nmt range proof."""
    Start: int
    End: int
    Nodes: List[bytes]
    LeafHash: Optional[bytes] = None

    def Marshal(self):
        out = _w_varint(1, self.Start) + _w_varint(2, self.End)
        for n in self.Nodes:
            out += _w_bytes(3, n, always=True)
        return out + _w_bytes(4, self.LeafHash)

    @classmethod
    def Unmarshal(cls, buf):
        m, r = cls(0, 0, []), _Reader(buf, "NMTProof")
        for f, wt in r.fields():
            if f == 1:
                r.want(wt, 0, "Start")
                m.Start = _int32(r.uvarint())
            elif f == 2:
                r.want(wt, 0, "End")
                m.End = _int32(r.uvarint())
            elif f == 3:
                r.want(wt, 2, "Nodes")
                m.Nodes.append(r.lendelim())
            elif f == 4:
                r.want(wt, 2, "LeafHash")
                m.LeafHash = r.lendelim()
            else:
                r.skip(wt)
        return m

    def VerifyInclusion(self, namespace, leaves, root):
        """nmt Proof.VerifyInclusion: recompute the root from the leaves (all in `namespace`,
        given without the namespace prefix) and the proof nodes. Like nmt, no completeness
        check: the leaves may be a subset of the namespace's leaves (VerifyNamespace is
        the completeness-checking form)."""
        start, end = self.Start, self.End
        nsz = len(namespace)
        if start < 0 or end <= start or len(leaves) != end - start:
            return False
        hashes = [_nmt_leaf(namespace, d) for d in leaves]
        nodes = list(self.Nodes)
        state = {"nodes": nodes, "leaves": hashes}

        def pop(key):
            lst = state[key]
            if not lst:
                return None
            v = lst[0]
            state[key] = lst[1:]
            return v

        def compute(s, e):
            if e - s == 1:
                return pop("leaves") if start <= s < end else pop("nodes")
            if e <= start or s >= end:
                return pop("nodes")
            k = _split_point(e - s)
            lh = compute(s, s + k)
            rh = compute(s + k, e)
            if rh is None:
                return lh
            return _nmt_node(lh, rh, nsz)

        est = max(_split_point(end) * 2 if end > 1 else 1, 1)
        try:
            h = compute(0, est)
            for n in state["nodes"]:
                h = _nmt_node(h, n, nsz)
        except ValueError:
            return False
        return h == root


@dataclass
class Proof:
    """merkle.Proof (RFC-6962) of one item among Total."""
    Total: int
    Index: int
    LeafHash: bytes
    Aunts: List[bytes]

    def Marshal(self):
        out = _w_varint(1, self.Total) + _w_varint(2, self.Index) + _w_bytes(3, self.LeafHash)
        for a in self.Aunts:
            out += _w_bytes(4, a, always=True)
        return out

    @classmethod
    def Unmarshal(cls, buf):
        m, r = cls(0, 0, b"", []), _Reader(buf, "Proof")
        for f, wt in r.fields():
            if f == 1:
                r.want(wt, 0, "Total")
                m.Total = _int64(r.uvarint())
            elif f == 2:
                r.want(wt, 0, "Index")
                m.Index = _int64(r.uvarint())
            elif f == 3:
                r.want(wt, 2, "LeafHash")
                m.LeafHash = r.lendelim()
            elif f == 4:
                r.want(wt, 2, "Aunts")
                m.Aunts.append(r.lendelim())
            else:
                r.skip(wt)
        return m

    def _compute(self, index, total, leaf, aunts):
        if total == 1:
            return leaf if not aunts else None
        if not aunts:
            return None
        k = _split_point(total)
        if index < k:
            lh = self._compute(index, k, leaf, aunts[:-1])
            return None if lh is None else _rfc_inner(lh, aunts[-1])
        rh = self._compute(index - k, total - k, leaf, aunts[:-1])
        return None if rh is None else _rfc_inner(aunts[-1], rh)

    def Verify(self, root, leaf):
        """go-square merkle Proof.Verify: error (CelError) unless leaf is item Index of root."""
        if self.Total < 0 or self.Index < 0:
            raise CelError(_lib.EINVAL, "proof total and index must be non-negative")
        if _rfc_leaf(leaf) != self.LeafHash:
            raise CelError(_lib.EINVAL, "invalid leaf hash")
        if self._compute(self.Index, self.Total, self.LeafHash, list(self.Aunts)) != root:
            raise CelError(_lib.EINVAL, "invalid root hash")


@dataclass
class RowProof:
    RowRoots: List[bytes]
    Proofs: List[Proof]
    StartRow: int
    EndRow: int
    Root: bytes = b""  # proof.proto field 3; NewShareInclusionProofFromEDS leaves it empty

    def Marshal(self):
        out = b"".join(_w_bytes(1, r, always=True) for r in self.RowRoots)
        for p in self.Proofs:
            out += _w_bytes(2, p.Marshal(), always=True)
        return out + _w_bytes(3, self.Root) + _w_varint(4, self.StartRow) + _w_varint(5, self.EndRow)

    @classmethod
    def Unmarshal(cls, buf):
        m, r = cls([], [], 0, 0), _Reader(buf, "RowProof")
        for f, wt in r.fields():
            if f == 1:
                r.want(wt, 2, "RowRoots")
                m.RowRoots.append(r.lendelim())
            elif f == 2:
                r.want(wt, 2, "Proofs")
                m.Proofs.append(Proof.Unmarshal(r.lendelim()))
            elif f == 3:
                r.want(wt, 2, "Root")
                m.Root = r.lendelim()
            elif f == 4:
                r.want(wt, 0, "StartRow")
                m.StartRow = r.uvarint() & 0xFFFFFFFF
            elif f == 5:
                r.want(wt, 0, "EndRow")
                m.EndRow = r.uvarint() & 0xFFFFFFFF
            else:
                r.skip(wt)
        return m

    def Validate(self, root):
        if self.EndRow - self.StartRow + 1 != len(self.RowRoots):
            raise CelError(_lib.EINVAL, f"the number of rows {self.EndRow - self.StartRow + 1} must equal the "
                                        f"number of row roots {len(self.RowRoots)}")
        if len(self.Proofs) != len(self.RowRoots):
            raise CelError(_lib.EINVAL, f"the number of proofs {len(self.Proofs)} must equal the number of row "
                                        f"roots {len(self.RowRoots)}")
        if not self.VerifyProof(root):
            raise CelError(_lib.EINVAL, "row proof failed to verify")

    def VerifyProof(self, root):
        for p, r in zip(self.Proofs, self.RowRoots):
            try:
                p.Verify(root, r)
            except CelError:
                return False
        return True


@dataclass
class ShareProof:
    Data: List[bytes]
    ShareProofs: List[NMTProof]
    NamespaceId: bytes
    RowProof: Optional[RowProof]
    NamespaceVersion: int = 0

    def Marshal(self):
        """gogoproto ShareProof.Marshal (proof.pb.go): the bytes of the ABCI proof queries."""
        out = b"".join(_w_bytes(1, d, always=True) for d in self.Data)
        for p in self.ShareProofs:
            out += _w_bytes(2, p.Marshal(), always=True)
        out += _w_bytes(3, self.NamespaceId)
        if self.RowProof is not None:
            out += _w_bytes(4, self.RowProof.Marshal(), always=True)
        return out + _w_varint(5, self.NamespaceVersion)

    @classmethod
    def Unmarshal(cls, buf):
        m, r = cls([], [], b"", None), _Reader(buf, "ShareProof")
        for f, wt in r.fields():
            if f == 1:
                r.want(wt, 2, "Data")
                m.Data.append(r.lendelim())
            elif f == 2:
                r.want(wt, 2, "ShareProofs")
                m.ShareProofs.append(NMTProof.Unmarshal(r.lendelim()))
            elif f == 3:
                r.want(wt, 2, "NamespaceId")
                m.NamespaceId = r.lendelim()
            elif f == 4:
                r.want(wt, 2, "RowProof")
                m.RowProof = RowProof.Unmarshal(r.lendelim())
            elif f == 5:
                r.want(wt, 0, "NamespaceVersion")
                m.NamespaceVersion = r.uvarint() & 0xFFFFFFFF
            else:
                r.skip(wt)
        return m

    def Validate(self, root):
        if self.RowProof is None:  # the reference dereferences a nil *RowProof (a panic)
            raise CelError(_lib.EINVAL, "share proof has no row proof")
        if not self.Data:
            raise CelError(_lib.EINVAL, "empty share proof")
        n = sum(p.End - p.Start for p in self.ShareProofs)
        if len(self.ShareProofs) != len(self.RowProof.RowRoots):
            raise CelError(_lib.EINVAL, f"the number of share proofs {len(self.ShareProofs)} must equal the "
                                        f"number of row roots {len(self.RowProof.RowRoots)}")
        if len(self.Data) != n:
            raise CelError(_lib.EINVAL, f"the number of shares {len(self.Data)} must equal the number of shares "
                                        f"in share proofs {n}")
        for p in self.ShareProofs:
            if p.Start < 0:
                raise CelError(_lib.EINVAL, "proof index cannot be negative")
            if p.End - p.Start <= 0:
                raise CelError(_lib.EINVAL, "proof total must be positive")
        self.RowProof.Validate(root)
        if not self.VerifyProof():
            raise CelError(_lib.EINVAL, "share proof failed to verify")

    def VerifyProof(self):
        if self.NamespaceVersion > 255:
            return False
        ns = bytes([self.NamespaceVersion]) + bytes(self.NamespaceId)
        cursor = 0
        for i, p in enumerate(self.ShareProofs):
            used = p.End - p.Start
            if not p.VerifyInclusion(ns, self.Data[cursor:cursor + used], self.RowProof.RowRoots[i]):
                return False
            cursor += used
        return True


# ---------------------------------------------------------------- construction
def axis_trees(eds, axis, first, count, ctx=None):
    """All nodes of the NMTs of EDS rows (axis 0) or columns (1) [first, first+count):
    array [count][4k-1][90] (level-major from the leaves), hashed on the device."""
    ctx = ctx or eds.ctx
    cells = np.ascontiguousarray(eds.cells)
    W = cells.shape[0]
    out = np.zeros((count, 2 * W - 1, NODE), np.uint8)
    ctx.check(ctx.lib.cel_axis_trees(ctx.handle, _p(cells), W // 2, _lib.SHARE_SIZE, axis, first, count, _p(out)))
    return out


def dah_tree(eds, ctx=None):
    """RFC-6962 levels over rowRoots || colRoots: array [4w-1][32], root last."""
    ctx = ctx or eds.ctx
    rr = np.ascontiguousarray(np.frombuffer(b"".join(eds.RowRoots()), np.uint8))
    cr = np.ascontiguousarray(np.frombuffer(b"".join(eds.ColRoots()), np.uint8))
    w = len(eds.RowRoots())
    out = np.zeros((4 * w - 1, 32), np.uint8)
    ctx.check(ctx.lib.cel_dah_tree(ctx.handle, _p(rr), _p(cr), w, _p(out)))
    return out


def nmt_prove_range(tree, start, end):
    """nmt ProveRange(start, end) over one tree of axis_trees(): the proof nodes."""
    l = _lib.load()
    tree = np.ascontiguousarray(tree)
    nleaves = (tree.shape[0] + 1) // 2
    cnt = ctypes.c_uint32()
    out = np.zeros((64, NODE), np.uint8)
    st = l.cel_nmt_prove_range(_p(tree), nleaves, start, end, _p(out), ctypes.byref(cnt))
    if st != _lib.OK:
        raise CelError(st, f"invalid proof range [{start}, {end}) over {nleaves} leaves")
    return [out[i].tobytes() for i in range(cnt.value)]


def merkle_aunts(levels, n, index):
    l = _lib.load()
    levels = np.ascontiguousarray(levels)
    cnt = ctypes.c_uint32()
    out = np.zeros((64, 32), np.uint8)
    st = l.cel_merkle_aunts(_p(levels), n, index, _p(out), ctypes.byref(cnt))
    if st != _lib.OK:
        raise CelError(st, f"invalid merkle index {index} of {n}")
    return [out[i].tobytes() for i in range(cnt.value)]


def CreateShareToRowRootProofs(eds, start_row, end_row, start_leaf, end_leaf):
    """pkg/proof/proof.go:147-202 on device-built trees: per row, the nmt range proof of
    the selected shares and the raw shares."""
    k = eds.Width() // 2
    trees = axis_trees(eds, 0, start_row, end_row - start_row + 1)
    share_proofs, raw = [], []
    roots = eds.RowRoots()
    for i, r in enumerate(range(start_row, end_row + 1)):
        if trees[i, -1].tobytes() != roots[r]:
            raise CelError(_lib.EINVAL, "eds row root is different than tree root")
        s = start_leaf if i == 0 else 0
        e = end_leaf if r == end_row else k - 1  # ODS part of the row (proof.go:180-183, squareSize = k)
        raw += [eds.GetCell(r, c) for c in range(s, e + 1)]
        share_proofs.append(NMTProof(Start=s, End=e + 1, Nodes=nmt_prove_range(trees[i], s, e + 1)))
    return share_proofs, raw


def NewShareInclusionProofFromEDS(eds, namespace, share_start, share_end):
    """pkg/proof/proof.go:78-140: ShareProof of ODS shares [share_start, share_end) (all in
    `namespace`, 29 bytes) to the data root of `eds`."""
    k = eds.Width() // 2
    if not 0 <= share_start < share_end <= k * k:
        raise CelError(_lib.EINVAL, f"share range [{share_start}, {share_end}) outside the {k}x{k} square")
    start_row, end_row = share_start // k, (share_end - 1) // k
    start_leaf, end_leaf = share_start % k, (share_end - 1) % k
    levels = dah_tree(eds)
    n = 4 * k
    roots = eds.RowRoots()
    proofs = []
    for r in range(start_row, end_row + 1):
        proofs.append(Proof(Total=n, Index=r, LeafHash=levels[r].tobytes(), Aunts=merkle_aunts(levels, n, r)))
    share_proofs, raw = CreateShareToRowRootProofs(eds, start_row, end_row, start_leaf, end_leaf)
    ns = bytes(namespace)
    return ShareProof(Data=raw, ShareProofs=share_proofs, NamespaceId=ns[1:], NamespaceVersion=ns[0],
                      RowProof=RowProof(RowRoots=[roots[r] for r in range(start_row, end_row + 1)], Proofs=proofs,
                                        StartRow=start_row, EndRow=end_row))


def NewShareInclusionProof(ods_shares, namespace, share_start, share_end):
    """pkg/proof/proof.go:64-76: extend the ODS on the device, then prove."""
    from . import da
    return NewShareInclusionProofFromEDS(da.ExtendShares(ods_shares), namespace, share_start, share_end)


TX_NAMESPACE = bytes(28) + b"\x01"
PFB_NAMESPACE = bytes(28) + b"\x04"


def ParseNamespace(raw_shares, start_share, end_share):
    """pkg/proof/querier.go:134-166: check the end-exclusive share range and that every
    share in it carries the first one's namespace (29 bytes); return that namespace.
    Raises CelError(EINVAL) with the reference's messages."""
    if start_share < 0:
        raise CelError(_lib.EINVAL, f"start share {start_share} should be positive")
    if end_share < 0:
        raise CelError(_lib.EINVAL, f"end share {end_share} should be positive")
    if end_share <= start_share:
        raise CelError(_lib.EINVAL,
                       f"end share {end_share} cannot be lower or equal to the starting share {start_share}")
    if end_share > len(raw_shares):
        raise CelError(_lib.EINVAL, f"end share {end_share} is higher than block shares {len(raw_shares)}")
    first = bytes(raw_shares[start_share][:NS])
    if len(first) < NS:
        raise CelError(_lib.ESHORT, "share is too short to contain a namespace")
    # Each share's length is checked where the reference parses its namespace (querier.go:
    # 157-160, share.Namespace() per share). The mismatch message prints the namespaces in
    # hex; the reference formats them with %v (a byte-slice dump), so only the text before
    # the colon matches it.
    for i, sh in enumerate(raw_shares[start_share:end_share]):
        ns = bytes(sh[:NS])
        if len(ns) < NS:
            raise CelError(_lib.ESHORT, "share is too short to contain a namespace")
        if ns != first:
            raise CelError(_lib.EINVAL, f"shares range contain different namespaces at index {i}: "
                                        f"{first.hex()} and {ns.hex()} ")
    return first


def NewTxInclusionProof(txs, tx_index, max_square_size=128, subtree_root_threshold=64):
    """pkg/proof/proof.go:21-48: square.Construct, FindTxShareRange, then the share proof
    of that range in the tx's namespace (PayForBlob for blob txs, proof.go:50-56)."""
    from . import square
    if tx_index >= len(txs):
        raise CelError(_lib.EINVAL, f"txIndex {tx_index} out of bounds")
    start, end = square.TxShareRange(txs, tx_index, max_square_size, subtree_root_threshold)
    ods = square.Construct(txs, max_square_size, subtree_root_threshold)
    ns = PFB_NAMESPACE if bytes(ods[start][:NS]) == PFB_NAMESPACE else TX_NAMESPACE
    return NewShareInclusionProof(list(ods), ns, start, end)
