"""Host logic of the Python rsmt2d mirror (no device): custom tree constructors are
honoured the way rsmt2d honours them (pkg/inclusion/nmt_caching.go:96-104,
test/util/malicious/tree.go:36-71 pass their own TreeConstructorFn), and a codec other
than Leopard is refused instead of being silently replaced by the device codec."""
import hashlib

import numpy as np
import pytest


class CountingTree:
    """A stand-in TreeConstructorFn tree: its root is sha256 over what was pushed."""

    calls = []

    def __init__(self, axis, index):
        self.axis, self.index, self.h = axis, index, hashlib.sha256()
        CountingTree.calls.append((axis, index))

    def Push(self, data):
        self.h.update(bytes(data))

    def Root(self):
        return self.h.digest()


def test_custom_tree_constructor_is_honoured():
    from celestia_eds.rsmt2d import Col, ImportExtendedDataSquare, Row
    w = 4
    rng = np.random.default_rng(1)
    cells = rng.integers(0, 256, (w, w, 512), dtype=np.uint8)
    CountingTree.calls = []
    eds = ImportExtendedDataSquare([cells[r, c].tobytes() for r in range(w) for c in range(w)],
                                   tree_constructor=CountingTree)
    rows, cols = eds.RowRoots(), eds.ColRoots()
    assert rows[1] == hashlib.sha256(cells[1].tobytes()).digest()
    assert cols[2] == hashlib.sha256(cells[:, 2].tobytes()).digest()
    assert sorted(CountingTree.calls) == sorted([(Row, i) for i in range(w)] + [(Col, i) for i in range(w)])


def test_default_wrapper_constructor_is_recognised():
    from celestia_eds import wrapper
    from celestia_eds.rsmt2d import _default_constructor
    assert _default_constructor(None, 8)
    assert _default_constructor(wrapper.NewConstructor(4), 8)
    assert not _default_constructor(CountingTree, 8)
    # a wrapper constructor for another square size is the caller's own trees
    assert not _default_constructor(wrapper.NewConstructor(2), 8)
    assert not _default_constructor(wrapper.NewConstructor(8), 8)


def test_foreign_codec_is_refused():
    from celestia_eds import CelError, _lib
    from celestia_eds.rsmt2d import ComputeExtendedDataSquare, ImportExtendedDataSquare

    class RSGF8Codec:  # e.g. rsmt2d.NewRSGF8Codec()
        pass

    with pytest.raises(CelError) as ei:
        ImportExtendedDataSquare([bytes(512)] * 4, codec=RSGF8Codec())
    assert ei.value.status == _lib.EINVAL
    with pytest.raises(CelError):
        ComputeExtendedDataSquare([bytes(512)], codec=RSGF8Codec())


@pytest.mark.parametrize("fn", ["ExtendShares", "ComputeDataAvailabilityHeader"])
def test_share_inputs_checked_before_the_device(fn):
    """ExtendShares / ComputeDataAvailabilityHeader hand the C side only n and the share
    size, so every share must be that size before the buffer is joined: unequal shares get
    rsmt2d's uneven-chunks error, a non-power-of-two count the reference's ENOTPOW2, and a
    wrongly shaped array EINVAL, all raised before any device is touched (this runs with no
    GPU)."""
    from celestia_eds import CelError, _lib, da
    f = getattr(da, fn)
    shares = [bytes(512)] * 3 + [bytes(511)]
    with pytest.raises(CelError) as ei:
        f(shares)
    assert ei.value.status == _lib.ECHUNK and "equal size" in str(ei.value)
    with pytest.raises(CelError) as ei:
        f([bytes(512)] * 3)
    assert ei.value.status == _lib.ENOTPOW2 and "got 3" in str(ei.value)
    with pytest.raises(CelError) as ei:
        f(np.zeros((4, 2, 256), np.uint8))
    assert ei.value.status == _lib.EINVAL


def test_min_shares_are_one_tail_padding_share():
    """MinShares = shares.ToBytes(EmptySquareShares()) = one tail-padding share
    (pkg/da/data_availability_header.go:192-201; go-square TailPaddingShares: the
    tail-padding namespace, version 0xFF and ID 0xFF*27 || 0xFE, the sequence-start info
    byte 0x01, a zero sequence length, zeros), as the reference's MinDataAvailabilityHeader
    extends it (its DAH known answer is checked on the device in test_gpu_square.py). No
    device."""
    from celestia_eds import da
    ms, es = da.MinShares(), da.EmptySquareShares()
    assert ms == es and len(ms) == 1 and len(ms[0]) == 512
    s = ms[0]
    assert s[:29] == b"\xff" * 28 + b"\xfe"
    assert s[29] == 0x01 and s[30:] == bytes(482)
    assert da.SquareSize(len(ms)) == 1


def test_flattened_ods_is_q0_row_major():
    """ExtendedDataSquare.FlattenedODS (rsmt2d, used by pkg/proof/proof.go:84 to size the
    square): the k x k original quadrant, row-major; Flattened is the whole 2k x 2k square.
    Host bookkeeping only, no device."""
    from celestia_eds.rsmt2d import ExtendedDataSquare
    k = 4
    cells = np.zeros((2 * k, 2 * k, 512), np.uint8)
    for r in range(2 * k):
        for c in range(2 * k):
            cells[r, c, :2] = (r, c)
    eds = ExtendedDataSquare(cells)
    ods = eds.FlattenedODS()
    assert len(ods) == k * k and len(eds.Flattened()) == 4 * k * k
    assert [o[:2] for o in ods] == [bytes((r, c)) for r in range(k) for c in range(k)]
