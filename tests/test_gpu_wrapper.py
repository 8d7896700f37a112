"""GPU: pkg/wrapper behaviour (nmt_wrapper_test.go:19-128) through the device roots."""
import hashlib

import numpy as np
import pytest

from eds_inputs import random_ods

pytestmark = pytest.mark.gpu


def erasured(oracle, k, seed):
    """generateErasuredData (nmt_wrapper_test.go:143-151): k sorted namespaced shares
    and their Leopard parity (k rounded up to a power of two for the codec)."""
    kk = 1 << (k - 1).bit_length()
    data = random_ods(kk, seed).reshape(-1, 512)[:kk]
    par = oracle.rs_encode(np.ascontiguousarray(data))
    return ([d.tobytes() for d in data] + [p.tobytes() for p in par])[: 2 * k] if kk == k else \
        [d.tobytes() for d in data] + [p.tobytes() for p in par]


@pytest.mark.parametrize("k", [8, 128])
def test_push_and_root_matches_oracle(ctx, oracle, k):
    from celestia_eds.wrapper import NewErasuredNamespacedMerkleTree
    cells = erasured(oracle, k, k)
    tree = NewErasuredNamespacedMerkleTree(k, 0)
    for c in cells:
        tree.Push(c)
    rc, exp = oracle.axis_root(np.frombuffer(b"".join(cells), np.uint8).reshape(2 * k, 512), k, 0)
    assert rc == 0 and tree.Root() == exp


def test_root_differs_from_plain_nmt(ctx, oracle):
    from celestia_eds.wrapper import NewErasuredNamespacedMerkleTree
    k = 8
    data = [d.tobytes() for d in random_ods(4, 3).reshape(-1, 512)[:8]]  # 8 of the 16 sorted shares
    t = NewErasuredNamespacedMerkleTree(k, 0)
    for d in data:
        t.Push(d)
    # nmt.New(...).Push(d) hashes d itself (its first 29 bytes are the namespace);
    # the wrapper prefixes the namespace again (nmt_wrapper_test.go:49-73)
    rc, plain = oracle.nmt_root(data)
    assert rc == 0 and t.Root() != plain


def test_empty_root_independent_of_params(ctx):
    from celestia_eds.wrapper import NewErasuredNamespacedMerkleTree
    r1 = NewErasuredNamespacedMerkleTree(1, 0).Root()
    r2 = NewErasuredNamespacedMerkleTree(2, 1).Root()
    assert r1 == r2 == bytes(58) + hashlib.sha256(b"").digest()


def test_push_errors(ctx, oracle):
    from celestia_eds import CelError
    from celestia_eds.wrapper import NewErasuredNamespacedMerkleTree
    k = 16
    over = erasured(oracle, k + 1, 1)
    t = NewErasuredNamespacedMerkleTree(k, 0)
    with pytest.raises(CelError, match="pushed past predetermined square size"):
        for d in over:
            t.Push(d)
    rev = sorted(erasured(oracle, k, 2), reverse=True)
    t = NewErasuredNamespacedMerkleTree(k, 0)
    with pytest.raises(CelError):
        for d in rev:
            t.Push(d)
    t = NewErasuredNamespacedMerkleTree(k, 0)
    with pytest.raises(CelError, match="data is too short to contain namespace ID"):
        t.Push(b"\x01")


def test_partial_tree_root(ctx, oracle):
    """Root over fewer than 2k pushes goes through the generic device NMT."""
    from celestia_eds.wrapper import NewErasuredNamespacedMerkleTree
    data = [d.tobytes() for d in random_ods(4, 9).reshape(-1, 512)[:5]]
    t = NewErasuredNamespacedMerkleTree(8, 0)
    for d in data:
        t.Push(d)
    rc, exp = oracle.nmt_root([d[:29] + d for d in data])
    assert rc == 0 and t.Root() == exp


@pytest.mark.parametrize("k", [8, 64])
def test_prove_range_verifies(ctx, oracle, k):
    """ErasuredNamespacedMerkleTree.ProveRange (nmt_wrapper.go:127-130) on full axes: the
    device's axis tree (cel_axis_tree) and the picked proof nodes verify every parity-
    namespaced range against the tree's root with the nmt verifier pinned by the
    reference's proof vectors (tests/test_proof.py); a tampered share or node fails;
    empty / reversed / out-of-range ranges raise; a partial tree proves over its pushed
    leaves."""
    from celestia_eds import CelError
    from celestia_eds.wrapper import PARITY_NAMESPACE, NewErasuredNamespacedMerkleTree
    cells = erasured(oracle, k, 300 + k)
    for axis, ranges in ((0, [(k, 2 * k), (k + 2, k + 5), (2 * k - 1, 2 * k)]),
                         (k + 1, [(0, 3), (5, 2 * k), (0, 2 * k), (k - 1, k + 1)])):
        tree = NewErasuredNamespacedMerkleTree(k, axis)
        for c in cells:
            tree.Push(c)
        root = tree.Root()
        for s, e in ranges:
            p = tree.ProveRange(s, e)
            assert (p.Start, p.End) == (s, e)
            assert p.VerifyInclusion(PARITY_NAMESPACE, cells[s:e], root), (axis, s, e)
            bad = list(cells[s:e])
            bad[0] = bytes([bad[0][0] ^ 1]) + bad[0][1:]
            assert not p.VerifyInclusion(PARITY_NAMESPACE, bad, root)
            if p.Nodes:
                p.Nodes[0] = bytes(len(p.Nodes[0]))
                assert not p.VerifyInclusion(PARITY_NAMESPACE, cells[s:e], root)
        for s, e in ((3, 3), (4, 2), (0, 2 * k + 1)):
            with pytest.raises(CelError):
                tree.ProveRange(s, e)
    # a partial tree proves over what was pushed (nmt keeps no width), past it raises
    partial = NewErasuredNamespacedMerkleTree(k, 0)
    for c in cells[:3]:
        partial.Push(c)
    p = partial.ProveRange(1, 2)
    assert p.VerifyInclusion(cells[1][:29], [cells[1]], partial.Root())
    with pytest.raises(CelError):
        partial.ProveRange(0, 4)


def test_axis_tree_abi_errors(ctx):
    """cel_axis_tree validates before any device work: axis index past the square
    (EPUSHPAST, nmt_wrapper.go:94-96), non-power-of-two width (ENOTPOW2), share size other
    than 512 (ECHUNK), nil pointers (EINVAL)."""
    import ctypes
    from celestia_eds import _lib
    k = 8
    cells = np.zeros((2 * k, 512), np.uint8)
    out = np.zeros((4 * k - 1, 90), np.uint8)
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    f = ctx.lib.cel_axis_tree
    assert f(ctx.handle, P(cells), k, 2 * k, 512, P(out)) == _lib.EPUSHPAST
    assert f(ctx.handle, P(cells), 6, 0, 512, P(out)) == _lib.ENOTPOW2
    assert f(ctx.handle, P(cells), k, 0, 256, P(out)) == _lib.ECHUNK
    assert f(ctx.handle, None, k, 0, 512, P(out)) == _lib.EINVAL
    assert f(ctx.handle, P(cells), k, 0, 512, None) == _lib.EINVAL
    assert f(ctx.handle, P(cells), k, 2 * k - 1, 512, P(out)) == _lib.OK


def test_prove_range_every_leaf(ctx, oracle):
    """nmt_wrapper_test.go:152-180 TestErasuredNamespacedMerkleTree_ProveRange: square sizes
    1..16 (odd widths included), axis 0, the k raw shares and their k parity shares; for
    every leaf i ProveRange(i, i+1) is a non-empty proof that verifies against the tree's
    root under the leaf's namespace (its own for i < k, the parity namespace otherwise).
    Power-of-two widths take the cel_axis_tree path, the rest the subtree-root path; both
    give nmt's node order."""
    from celestia_eds.wrapper import PARITY_NAMESPACE, NewErasuredNamespacedMerkleTree
    for k in range(1, 17):
        data = erasured(oracle, k, 700 + k)[: 2 * k]
        tree = NewErasuredNamespacedMerkleTree(k, 0)
        for d in data:
            tree.Push(d)
        root = tree.Root()
        for i in range(2 * k):
            p = tree.ProveRange(i, i + 1)
            assert p.Nodes, (k, i)
            ns = data[i][:29] if i < k else PARITY_NAMESPACE
            assert p.VerifyInclusion(ns, [data[i]], root), (k, i)


def test_out_of_order_nmt_like_the_malicious_tree(ctx, oracle):
    """test/util/malicious/app_test.go:23-62 TestOutOfOrderNMT through the C ABI: over 64
    namespaced shares (square size 64, axis 0) the order-checking root (the honest wrapper)
    and the unchecked root (the malicious tree's hasher, malicious/hasher.go) agree on
    ordered data; shuffled, the honest path refuses (CEL_EORDER) and the unchecked one
    returns a 90-byte root that differs from the ordered one and equals the oracle's NMT
    over the same shuffled leaves."""
    import ctypes
    from celestia_eds import _lib
    rng = np.random.default_rng(62)
    data = [bytes(d) for d in random_ods(8, 64).reshape(-1, 512)[:64]]
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731

    def root(shares, flags):
        leaves = np.frombuffer(b"".join(s[:29] + s for s in shares), np.uint8).copy()  # Q0: ns || share
        out = np.zeros(90, np.uint8)
        st = ctx.lib.cel_nmt_root(ctx.handle, P(leaves), len(shares), 29 + 512, P(out), flags)
        return st, out.tobytes()

    st_good, good = root(data, _lib.FLAG_ORDER_CHECK)
    st_mal, mal = root(data, 0)
    assert st_good == st_mal == _lib.OK and good == mal
    shuffled = [data[i] for i in rng.permutation(64)]
    st, _ = root(shuffled, _lib.FLAG_ORDER_CHECK)
    assert st == _lib.EORDER
    st, bad = root(shuffled, 0)
    assert st == _lib.OK and len(bad) == 90 and bad != good
    rc, exp = oracle.nmt_root([s[:29] + s for s in shuffled], check_order=False)
    assert rc == 0 and bad == exp
