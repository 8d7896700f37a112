"""Wire format of the share / row proofs (proto/celestia/core/v1/proof/proof.proto:8-49,
gogoproto-generated pkg/proof/proof.pb.go), the bytes the reference's ABCI proof queries
return (pkg/proof/querier.go:53-63).

The reference holds no marshaled proof, so the encoding is checked against Google's
protobuf runtime (importable here) over a descriptor that restates proof.proto field by
field: same bytes for random messages (proto3: fields in number order, zero scalars and
empty singular bytes omitted, every repeated element kept, negative int32 / int64 as
10-byte varints), and both decoders agree on those bytes and on bytes with unknown fields
interleaved. Then the reference's own valid share proof (share_proof_test.go) round-trips
and still validates. No device is used."""
import random

import pytest

from celestia_eds import CelError
from celestia_eds.proof import NMTProof, Proof, RowProof, ShareProof

pb = pytest.importorskip("google.protobuf")
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory  # noqa: E402


def _classes():
    """proof.proto:8-49 as a FileDescriptorProto (package celestia.core.v1.proof)."""
    F = descriptor_pb2.FieldDescriptorProto
    fd = descriptor_pb2.FileDescriptorProto(name="proof_restated.proto", package="celestia.core.v1.proof",
                                            syntax="proto3")

    def msg(name, fields):
        m = fd.message_type.add(name=name)
        for num, fname, typ, rep, tname in fields:
            f = m.field.add(name=fname, number=num, type=typ,
                            label=F.LABEL_REPEATED if rep else F.LABEL_OPTIONAL)
            if tname:
                f.type_name = ".celestia.core.v1.proof." + tname

    msg("ShareProof", [(1, "data", F.TYPE_BYTES, True, None), (2, "share_proofs", F.TYPE_MESSAGE, True, "NMTProof"),
                       (3, "namespace_id", F.TYPE_BYTES, False, None),
                       (4, "row_proof", F.TYPE_MESSAGE, False, "RowProof"),
                       (5, "namespace_version", F.TYPE_UINT32, False, None)])
    msg("RowProof", [(1, "row_roots", F.TYPE_BYTES, True, None), (2, "proofs", F.TYPE_MESSAGE, True, "Proof"),
                     (3, "root", F.TYPE_BYTES, False, None), (4, "start_row", F.TYPE_UINT32, False, None),
                     (5, "end_row", F.TYPE_UINT32, False, None)])
    msg("NMTProof", [(1, "start", F.TYPE_INT32, False, None), (2, "end", F.TYPE_INT32, False, None),
                     (3, "nodes", F.TYPE_BYTES, True, None), (4, "leaf_hash", F.TYPE_BYTES, False, None)])
    msg("Proof", [(1, "total", F.TYPE_INT64, False, None), (2, "index", F.TYPE_INT64, False, None),
                  (3, "leaf_hash", F.TYPE_BYTES, False, None), (4, "aunts", F.TYPE_BYTES, True, None)])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    get = message_factory.GetMessageClass
    return {n: get(pool.FindMessageTypeByName("celestia.core.v1.proof." + n))
            for n in ("ShareProof", "RowProof", "NMTProof", "Proof")}


PB = _classes()


def _rb(rng, lo=0, hi=96):
    return bytes(rng.getrandbits(8) for _ in range(rng.randint(lo, hi)))


def _rand_share_proof(rng):
    def nmt():
        return NMTProof(rng.choice([0, 1, 5, -3, 2 ** 31 - 1, -2 ** 31]), rng.choice([0, 2, 64, -1]),
                        [_rb(rng, 0, 90) for _ in range(rng.randint(0, 5))],
                        rng.choice([None, b"", _rb(rng, 1, 40)]))

    def proof():
        return Proof(rng.choice([0, 1, 256, -7, 2 ** 62]), rng.choice([0, 3, -1]), _rb(rng, 0, 32),
                     [_rb(rng, 0, 32) for _ in range(rng.randint(0, 4))])

    rp = None if rng.random() < 0.2 else RowProof([_rb(rng, 0, 90) for _ in range(rng.randint(0, 3))],
                                                   [proof() for _ in range(rng.randint(0, 3))],
                                                   rng.choice([0, 7, 2 ** 32 - 1]), rng.choice([0, 9]),
                                                   rng.choice([b"", _rb(rng, 32, 32)]))
    return ShareProof([_rb(rng, 0, 512) for _ in range(rng.randint(0, 4))], [nmt() for _ in range(rng.randint(0, 3))],
                      rng.choice([b"", _rb(rng, 28, 28)]), rp, rng.choice([0, 1, 255, 2 ** 32 - 1]))


def _to_pb(sp):
    m = PB["ShareProof"]()
    m.data.extend(sp.Data)
    for p in sp.ShareProofs:
        n = m.share_proofs.add(start=p.Start, end=p.End, leaf_hash=p.LeafHash or b"")
        n.nodes.extend(p.Nodes)
    m.namespace_id = sp.NamespaceId
    if sp.RowProof is not None:
        r = m.row_proof
        r.SetInParent()
        r.row_roots.extend(sp.RowProof.RowRoots)
        for q in sp.RowProof.Proofs:
            x = r.proofs.add(total=q.Total, index=q.Index, leaf_hash=q.LeafHash)
            x.aunts.extend(q.Aunts)
        r.root, r.start_row, r.end_row = sp.RowProof.Root, sp.RowProof.StartRow, sp.RowProof.EndRow
    m.namespace_version = sp.NamespaceVersion
    return m


def _same(a, b):
    """ShareProof equality as the wire sees it (nil and empty leaf hashes are the same)."""
    assert a.Data == b.Data and a.NamespaceId == b.NamespaceId and a.NamespaceVersion == b.NamespaceVersion
    assert len(a.ShareProofs) == len(b.ShareProofs)
    for x, y in zip(a.ShareProofs, b.ShareProofs):
        assert (x.Start, x.End, x.Nodes, x.LeafHash or b"") == (y.Start, y.End, y.Nodes, y.LeafHash or b"")
    assert (a.RowProof is None) == (b.RowProof is None)
    if a.RowProof is not None:
        ra, rb = a.RowProof, b.RowProof
        assert (ra.RowRoots, ra.Root, ra.StartRow, ra.EndRow) == (rb.RowRoots, rb.Root, rb.StartRow, rb.EndRow)
        assert [(p.Total, p.Index, p.LeafHash, p.Aunts) for p in ra.Proofs] == \
               [(p.Total, p.Index, p.LeafHash, p.Aunts) for p in rb.Proofs]


def test_marshal_matches_protobuf_runtime():
    rng = random.Random(20)
    for _ in range(300):
        sp = _rand_share_proof(rng)
        wire = sp.Marshal()
        assert wire == _to_pb(sp).SerializeToString(deterministic=True)
        back = ShareProof.Unmarshal(wire)
        _same(sp, back)
        assert back.Marshal() == wire
        # the protobuf runtime reads our bytes back to the same message
        assert PB["ShareProof"].FromString(wire) == _to_pb(sp)


def test_unmarshal_skips_unknown_fields_and_rejects_wrong_wire_types():
    sp = _rand_share_proof(random.Random(3))
    sp.RowProof = RowProof([b"r" * 90], [Proof(4, 1, b"h" * 32, [b"a" * 32])], 0, 0)
    wire = sp.Marshal()
    # unknown varint (field 9), fixed64 (10), bytes (11), fixed32 (12) and a group (13)
    junk = bytes([9 << 3, 0x96, 0x01, 10 << 3 | 1]) + bytes(8) + bytes([11 << 3 | 2, 3]) + b"xyz" + \
        bytes([12 << 3 | 5]) + bytes(4) + bytes([13 << 3 | 3, 1 << 3, 5, 13 << 3 | 4])
    _same(ShareProof.Unmarshal(junk + wire + junk), sp)
    for bad in (bytes([1 << 3 | 0, 1]),          # data as a varint
                bytes([5 << 3 | 2, 0]),          # namespace_version as bytes
                bytes([0x0A, 5]) + b"abc",       # length past the end
                bytes([0x00, 0x00]),             # field number 0
                bytes([0x0C])):                  # end group with no group open
        with pytest.raises(CelError):
            ShareProof.Unmarshal(bad)


def test_reference_share_proof_round_trip():
    """The reference's valid share proof (pkg/proof/share_proof_test.go validShareProof,
    tests/golden/proof_fixture.json) survives Marshal / Unmarshal and still validates
    against its data root (row_proof_test.go); the bytes equal the protobuf runtime's."""
    import json
    import os
    here = os.path.dirname(os.path.abspath(__file__))
    with open(os.path.join(here, "golden", "proof_fixture.json")) as f:
        fx = json.load(f)
    s, r = fx["share_proof"], fx["row_proof"]
    sp = ShareProof([bytes.fromhex(d) for d in s["data"]],
                    [NMTProof(s["start"], s["end"], [bytes.fromhex(n) for n in s["nodes"]])],
                    bytes.fromhex(s["namespace_id"]),
                    RowProof([bytes.fromhex(x) for x in r["row_roots"]],
                             [Proof(p["total"], p["index"], bytes.fromhex(p["leaf_hash"]),
                                    [bytes.fromhex(a) for a in p["aunts"]]) for p in r["proofs"]],
                             r["start_row"], r["end_row"]),
                    s["namespace_version"])
    wire = sp.Marshal()
    assert wire == _to_pb(sp).SerializeToString(deterministic=True)
    back = ShareProof.Unmarshal(wire)
    _same(sp, back)
    back.Validate(bytes.fromhex(fx["root"]))
    back.Data[0] = bytes(len(back.Data[0]))
    with pytest.raises(CelError):
        back.Validate(bytes.fromhex(fx["root"]))
