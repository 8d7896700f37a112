"""GPU: share inclusion proofs built from device-exported trees (cel_axis_trees,
cel_dah_tree; pkg/proof/proof.go:78-202) verify under the host verifier that
tests/test_proof.py pins to the reference's own proof vectors."""
import numpy as np
import pytest

from square_inputs import block408_txs, random_block

pytestmark = pytest.mark.gpu


def _ranges(ods):
    """(namespace, start, end) of every maximal run of equal namespaces in the ODS,
    excluding padding namespaces."""
    ns = [bytes(s[:29]) for s in ods]
    out, i = [], 0
    while i < len(ns):
        j = i
        while j < len(ns) and ns[j] == ns[i]:
            j += 1
        if ns[i][-1] not in (0xFF, 0xFE):
            out.append((ns[i], i, j))
        i = j
    return out


def test_block408_share_proofs(ctx, golden):
    from celestia_eds import da, proof, square
    ods = square.Construct(block408_txs())
    eds = da.ExtendShares(list(ods))
    root = bytes.fromhex(golden["block408"]["data_hash"])
    ranges = _ranges(ods)
    assert len(ranges) >= 3
    for ns, s, e in ranges:
        p = proof.NewShareInclusionProofFromEDS(eds, ns, s, e)
        p.Validate(root)
        assert [bytes(x) for x in ods[s:e]] == p.Data
        # a sub-range (first share only) also verifies
        proof.NewShareInclusionProofFromEDS(eds, ns, s, s + 1).Validate(root)


@pytest.mark.parametrize("seed", [1, 2])
def test_random_block_proofs_and_tamper(ctx, seed):
    from celestia_eds import CelError, da, proof, square
    ods = square.Construct(random_block(seed, 20, 12, max_blob=9000))
    eds = da.ExtendShares(list(ods))
    root = da.NewDataAvailabilityHeader(eds).Hash()
    multi_row = 0
    k = eds.Width() // 2
    for ns, s, e in _ranges(ods):
        p = proof.NewShareInclusionProofFromEDS(eds, ns, s, e)
        p.Validate(root)
        multi_row += p.RowProof.EndRow > p.RowProof.StartRow
    assert multi_row > 0, "no range spans rows"
    ns, s, e = _ranges(ods)[-1]
    p = proof.NewShareInclusionProofFromEDS(eds, ns, s, e)
    bad = bytearray(p.Data[0])
    bad[200] ^= 0x40
    p.Data[0] = bytes(bad)
    with pytest.raises(CelError):
        p.Validate(root)
    with pytest.raises(CelError):
        proof.NewShareInclusionProofFromEDS(eds, ns, s, k * k + 1)


def test_exported_trees_match_roots(ctx):
    from celestia_eds import da, proof
    from eds_inputs import random_ods
    k = 16
    eds = da.ExtendShares(list(random_ods(k, 77).reshape(-1, 512)))
    rows = proof.axis_trees(eds, 0, 0, 2 * k)
    cols = proof.axis_trees(eds, 1, 3, 5)
    assert [r[-1].tobytes() for r in rows] == eds.RowRoots()
    assert [c[-1].tobytes() for c in cols] == eds.ColRoots()[3:8]
    levels = proof.dah_tree(eds)
    assert levels[-1].tobytes() == da.NewDataAvailabilityHeader(eds).Hash()
    # every inner node is HashNode of its children (host recomputation of one tree)
    from celestia_eds.proof import _nmt_leaf, _nmt_node
    t = rows[5]
    W = 2 * k
    leaves = [_nmt_leaf(bytes(eds.GetCell(5, j)[:29]) if (5 < k and j < k) else b"\xff" * 29, eds.GetCell(5, j))
              for j in range(W)]
    assert [t[j].tobytes() for j in range(W)] == leaves
    off, n = 0, W
    while n > 1:
        for j in range(n // 2):
            assert t[off + n + j].tobytes() == _nmt_node(t[off + 2 * j].tobytes(), t[off + 2 * j + 1].tobytes())
        off += n
        n //= 2


def test_tx_inclusion_proofs_block408(ctx, golden):
    """NewTxInclusionProof (pkg/proof/proof.go:21-48) for normal and blob txs of block 408
    verifies against the block's data root."""
    from celestia_eds import proof, square
    txs = block408_txs()
    root = bytes.fromhex(golden["block408"]["data_hash"])
    n_normal = sum(1 for t in txs if not square.is_blob_tx(t))
    for i in (0, n_normal - 1, n_normal, len(txs) - 1):
        p = proof.NewTxInclusionProof(txs, i)
        p.Validate(root)
        assert p.NamespaceId[-1] == (0x01 if i < n_normal else 0x04)
