"""GPU rsmt2d Repair (config 5 shape) vs the original EDS, with the masks of
SURVEY.md §8(d): Q0 only, single quadrants, random p=0.55 / p=0.25, one corrupt cell."""
import numpy as np
import pytest

from eds_inputs import random_ods

pytestmark = pytest.mark.gpu


def setup(oracle, k, seed=7):
    eds, rr, cr, _ = oracle.extend_and_commit(random_ods(k, seed))
    return eds, [r.tobytes() for r in rr], [c.tobytes() for c in cr]


def repair(ctx, eds, present, rr, cr):
    from celestia_eds.rsmt2d import ExtendedDataSquare
    damaged = eds.copy()
    damaged[present == 0] = 0
    sq = ExtendedDataSquare(damaged, ctx=ctx)
    sq.Repair(rr, cr, present=present)
    return sq.cells


@pytest.mark.parametrize("k", [4, 32, 128])
@pytest.mark.parametrize("quadrant", [0, 1, 2, 3])
def test_single_quadrant(ctx, oracle, k, quadrant):
    eds, rr, cr = setup(oracle, k)
    w = 2 * k
    present = np.zeros((w, w), np.uint8)
    r0, c0 = (quadrant // 2) * k, (quadrant % 2) * k
    present[r0:r0 + k, c0:c0 + k] = 1
    assert np.array_equal(repair(ctx, eds, present, rr, cr), eds)


@pytest.mark.parametrize("k", [8, 128])
def test_random_055(ctx, oracle, k):
    eds, rr, cr = setup(oracle, k)
    w = 2 * k
    present = (np.random.default_rng(7).random((w, w)) < 0.55).astype(np.uint8)
    assert np.array_equal(repair(ctx, eds, present, rr, cr), eds)


def test_random_025_unrepairable(ctx, oracle):
    from celestia_eds.rsmt2d import ErrUnrepairableDataSquare
    k = 32
    eds, rr, cr = setup(oracle, k)
    w = 2 * k
    present = (np.random.default_rng(7).random((w, w)) < 0.25).astype(np.uint8)
    with pytest.raises(ErrUnrepairableDataSquare):
        repair(ctx, eds, present, rr, cr)


def test_corrupt_cell_byzantine(ctx, oracle):
    from celestia_eds.rsmt2d import ErrByzantineData
    k = 16
    eds, rr, cr = setup(oracle, k)
    w = 2 * k
    present = np.ones((w, w), np.uint8)
    present[3, 5] = 0
    bad = eds.copy()
    bad[0, 1, 200] ^= 0x40
    from celestia_eds.rsmt2d import ExtendedDataSquare
    sq = ExtendedDataSquare(bad, ctx=ctx)
    with pytest.raises(ErrByzantineData) as ei:
        sq.Repair(rr, cr, present=present)
    assert ei.value.Axis in (0, 1) and ei.value.Index >= 0


def test_gf16_repair_k256(ctx, oracle):
    k = 256
    eds, rr, cr = setup(oracle, k, seed=9)
    w = 2 * k
    present = np.zeros((w, w), np.uint8)
    present[k:, :k] = 1  # Q2 only
    assert np.array_equal(repair(ctx, eds, present, rr, cr), eds)


def _dev_repair(ctx, eds, present, rr, cr):
    """cel_dev_repair over a device-resident damaged copy; returns (status, cells, bad)."""
    import ctypes
    from hipmem import DeviceBuffer
    w = eds.shape[0]
    k = w // 2
    damaged = eds.copy()
    damaged[present == 0] = 0
    d = DeviceBuffer(damaged.nbytes)
    d.upload(damaged)
    pres = np.ascontiguousarray(present, np.uint8).copy()
    rra = np.ascontiguousarray(np.frombuffer(b"".join(rr), np.uint8))
    cra = np.ascontiguousarray(np.frombuffer(b"".join(cr), np.uint8))
    ba, bi = ctypes.c_int32(-1), ctypes.c_int32(-1)
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    st = ctx.lib.cel_dev_repair(ctx.handle, d.ptr, P(pres), k, P(rra), P(cra), ctypes.byref(ba), ctypes.byref(bi))
    return st, d.download(eds.shape), (ba.value, bi.value)


@pytest.mark.parametrize("k,p", [(64, 0.55), (128, 0.55), (32, 0.25)])
def test_dev_repair_matches_oracle(ctx, oracle, k, p):
    """Device-resident repair (cel_dev_repair): same outcome as the host entry point and
    the oracle's crossword restatement (filled EDS, or ErrUnrepairable at p = 0.25)."""
    from celestia_eds import _lib
    eds, rr, cr = setup(oracle, k)
    w = 2 * k
    present = (np.random.default_rng(11).random((w, w)) < p).astype(np.uint8)
    st, cells, _ = _dev_repair(ctx, eds, present, rr, cr)
    damaged = eds.copy()
    damaged[present == 0] = 0
    rc, _, _, _ = oracle.repair(damaged, present, np.stack([np.frombuffer(r, np.uint8) for r in rr]),
                                np.stack([np.frombuffer(c, np.uint8) for c in cr]))
    if rc == 0:
        assert st == _lib.OK and np.array_equal(cells, eds)
    else:
        assert st == _lib.EUNREPAIRABLE


def test_dev_repair_byzantine_in_final_verification(ctx, oracle):
    """Row roots of a square whose ODS differs in one cell (r0, c0), column roots of the
    original: the rows solve consistently, so the inconsistency surfaces only in the final
    all-axes check, which must report column c0 like the oracle's restatement."""
    from celestia_eds import _lib
    k, r0, c0 = 32, 5, 9
    ods = random_ods(k, 21)
    eds, rr, cr, _ = oracle.extend_and_commit(ods)
    ods2 = ods.copy()
    ods2[r0, c0, 100] ^= 0x5A
    eds2, rr2, _, _ = oracle.extend_and_commit(ods2)
    w = 2 * k
    present = np.zeros((w, w), np.uint8)
    present[:k, :k] = 1
    st, _, bad = _dev_repair(ctx, eds2, present, [r.tobytes() for r in rr2], [c.tobytes() for c in cr])
    damaged = eds2.copy()
    damaged[present == 0] = 0
    rc, _, _, obad = oracle.repair(damaged, present, rr2, cr)
    assert st == _lib.EBYZANTINE and rc == _lib.EBYZANTINE
    assert bad == obad == (1, c0)


@pytest.mark.parametrize("mask", ["all_but_one", "q0_only", "random_070", "left_half"])
def test_byzantine_axis_matches_oracle(ctx, oracle, mask):
    """A corrupted cell under several presence masks: the device repair reports the same
    status and the same first failing axis as the oracle's rsmt2d restatement
    (prerepairSanityCheck, crossword passes with encoding and root checks, final check)."""
    from celestia_eds import _lib
    k = 32
    w = 2 * k
    eds, rr, cr = setup(oracle, k, seed=31)
    rng = np.random.default_rng(5)
    if mask == "all_but_one":
        present = np.ones((w, w), np.uint8)
        present[3, 5] = 0
    elif mask == "q0_only":
        present = np.zeros((w, w), np.uint8)
        present[:k, :k] = 1
    elif mask == "left_half":
        present = np.zeros((w, w), np.uint8)
        present[:, :k] = 1
    else:
        present = (rng.random((w, w)) < 0.7).astype(np.uint8)
    bad = eds.copy()
    r, c = 7, 11  # a present cell in every mask
    present[r, c] = 1
    bad[r, c, 300] ^= 0x21
    st, _, dbad = _dev_repair(ctx, bad, present, rr, cr)
    damaged = bad.copy()
    damaged[present == 0] = 0
    rc, _, _, obad = oracle.repair(damaged, present, np.stack([np.frombuffer(x, np.uint8) for x in rr]),
                                   np.stack([np.frombuffer(x, np.uint8) for x in cr]))
    assert st == rc
    if rc == _lib.EBYZANTINE:
        assert dbad == obad
