"""GPU: GetCommitment over device-built row trees (cel_get_commitment, pkg/inclusion/
get_commit.go:12-30) equals the blob's share commitment computed independently from its
shares (go-square inclusion.CreateCommitment: merkle mountain range of NMT subtree
roots, RFC-6962 over them), restated here with hashlib — as the reference's
TestEDSSubRootCacher (nmt_caching_test.go:117) checks the cacher against the blobs."""
import hashlib
import math

import pytest

from square_inputs import blob_tx, block408_txs, random_block

pytestmark = pytest.mark.gpu
NS = 29


def _sha(b):
    return hashlib.sha256(b).digest()


def _leaf(share):
    ns = share[:NS]
    return ns + ns + _sha(b"\x00" + ns + share)


def _node(l, r):
    lmin, lmax, rmin, rmax = l[:NS], l[NS:2 * NS], r[:NS], r[NS:2 * NS]
    mx = lmax if rmin == b"\xff" * NS else max(lmax, rmax)
    return lmin + mx + _sha(b"\x01" + l + r)


def _nmt_root(shares):
    level = [_leaf(s) for s in shares]
    while len(level) > 1:
        level = [_node(level[2 * i], level[2 * i + 1]) for i in range(len(level) // 2)]
    return level[0]


def _rfc(items):
    if len(items) == 1:
        return _sha(b"\x00" + items[0])
    k = 1
    while k * 2 < len(items):
        k *= 2
    return _sha(b"\x01" + _rfc(items[:k]) + _rfc(items[k:]))


def _subtree_width(n, threshold=64):
    s = 1 << math.ceil(math.log2(-(-n // threshold)))
    m = 1 << math.ceil(math.log2(math.ceil(math.sqrt(n))))
    return min(s, m)


def create_commitment(shares, threshold=64):
    w = _subtree_width(len(shares), threshold)
    sizes, left = [], len(shares)
    while left:
        t = w if left >= w else 1 << (left.bit_length() - 1)
        sizes.append(t)
        left -= t
    roots, c = [], 0
    for t in sizes:
        roots.append(_nmt_root(shares[c:c + t]))
        c += t
    return _rfc(roots)


def _blobs(ods):
    """(start, n_shares) of every blob sequence in the square (sparse shares with the
    sequence-start bit, namespace not reserved)."""
    out = []
    for i, s in enumerate(ods):
        ns = bytes(s[:NS])
        if s[NS] & 1 and ns[0] == 0 and ns[-1] not in (0x01, 0x04, 0xFF, 0xFE) and ns[1:19] == bytes(18):
            length = int.from_bytes(bytes(s[NS + 1:NS + 5]), "big")
            n = 1 if length <= 478 else 1 + -(-(length - 478) // 482)
            out.append((i, n))
    return out


@pytest.mark.parametrize("source", ["block408", "random"])
def test_get_commitment_matches_blob_commitment(ctx, source):
    from celestia_eds import da, inclusion, square
    txs = block408_txs() if source == "block408" else random_block(21, 4, 25, max_blob=70000)
    ods = square.Construct(txs)
    eds = da.ExtendShares(list(ods))
    blobs = _blobs(ods)
    assert blobs
    for start, n in blobs:
        shares = [bytes(ods[start + j]) for j in range(n)]
        assert inclusion.GetCommitment(eds, start, n) == create_commitment(shares)


def test_commitment_out_of_square(ctx):
    from celestia_eds import CelError, da
    from celestia_eds import inclusion
    from eds_inputs import random_ods
    eds = da.ExtendShares(list(random_ods(4, 5).reshape(-1, 512)))
    with pytest.raises(CelError, match="cannot get commitment for blob that doesn't fit in square"):
        inclusion.GetCommitment(eds, 10, 7)
