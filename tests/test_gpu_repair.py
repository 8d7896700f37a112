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
