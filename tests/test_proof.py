"""pkg/proof mirror, host-side verification pinned by the
reference's own vectors: pkg/proof/share_proof_test.go (TestShareProofValidate) and
row_proof_test.go (TestRowProofValidate), extracted to tests/golden/proof_fixture.json
by tests/golden/make_proof_fixture.py. (That vector uses 33-byte namespaces: nmt is
generic in the namespace size, the verifier follows the namespace it is given.)"""
import copy
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def fx():
    with open(os.path.join(ROOT, "tests", "golden", "proof_fixture.json")) as f:
        return json.load(f)


def _share_proof(fx):
    from celestia_eds.proof import NMTProof, Proof, RowProof, ShareProof
    sp, rp = fx["share_proof"], fx["row_proof"]
    return ShareProof(
        Data=[bytes.fromhex(d) for d in sp["data"]],
        ShareProofs=[NMTProof(Start=sp["start"], End=sp["end"], Nodes=[bytes.fromhex(n) for n in sp["nodes"]])],
        NamespaceId=bytes.fromhex(sp["namespace_id"]), NamespaceVersion=sp["namespace_version"],
        RowProof=RowProof(RowRoots=[bytes.fromhex(r) for r in rp["row_roots"]],
                          Proofs=[Proof(Total=p["total"], Index=p["index"], LeafHash=bytes.fromhex(p["leaf_hash"]),
                                        Aunts=[bytes.fromhex(a) for a in p["aunts"]]) for p in rp["proofs"]],
                          StartRow=rp["start_row"], EndRow=rp["end_row"]))


def test_valid_share_proof(fx):
    _share_proof(fx).Validate(bytes.fromhex(fx["root"]))


def test_valid_row_proof(fx):
    _share_proof(fx).RowProof.Validate(bytes.fromhex(fx["root"]))


@pytest.mark.parametrize("case", ["empty", "mismatched_share_proofs", "mismatched_shares", "incorrect_root",
                                  "tampered_share", "tampered_node", "row_mismatched_roots", "row_mismatched_proofs",
                                  "row_mismatched_rows"])
def test_invalid_share_proofs(fx, case):
    from celestia_eds import CelError
    sp = _share_proof(fx)
    root = bytes.fromhex(fx["root"])
    if case == "empty":
        sp.Data = []
    elif case == "mismatched_share_proofs":
        sp.ShareProofs = []
    elif case == "mismatched_shares":
        sp.Data = [sp.Data[0], sp.Data[0]]
    elif case == "incorrect_root":
        root = bytes(32)
    elif case == "tampered_share":
        d = bytearray(sp.Data[0])
        d[100] ^= 1
        sp.Data = [bytes(d)]
    elif case == "tampered_node":
        p = copy.deepcopy(sp.ShareProofs[0])
        n = bytearray(p.Nodes[2])
        n[-1] ^= 1
        p.Nodes[2] = bytes(n)
        sp.ShareProofs = [p]
    elif case == "row_mismatched_roots":
        sp.RowProof.RowRoots = []
    elif case == "row_mismatched_proofs":
        sp.RowProof.Proofs = []
    elif case == "row_mismatched_rows":
        sp.RowProof.EndRow = 10
    with pytest.raises(CelError):
        sp.Validate(root)


def test_prove_range_selection():
    """cel_nmt_prove_range picks, left to right, the roots of the maximal subtrees outside
    the range (nmt buildRangeProof), on a synthetic level-major tree table."""
    import numpy as np
    from celestia_eds.proof import nmt_prove_range
    n = 16
    tree = np.zeros((2 * n - 1, 90), np.uint8)
    off, lvl = 0, 0
    ids = {}
    while n >> lvl >= 1:
        for j in range(n >> lvl):
            tree[off + j, 0] = lvl
            tree[off + j, 1] = j
            ids[off + j] = (lvl, j)
        off += n >> lvl
        if n >> lvl == 1:
            break
        lvl += 1
    got = [(b[0], b[1]) for b in nmt_prove_range(tree, 5, 11)]
    assert got == [(2, 0), (0, 4), (0, 11), (2, 3)]
    assert [(b[0], b[1]) for b in nmt_prove_range(tree, 0, 16)] == []
    assert [(b[0], b[1]) for b in nmt_prove_range(tree, 0, 1)] == [(0, 1), (1, 1), (2, 1), (3, 1)]
