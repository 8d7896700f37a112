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


@pytest.mark.parametrize("k", [1, 2, 4, 32, 128])
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
    from celestia_eds import _lib
    from celestia_eds.rsmt2d import ErrByzantineData
    k = 16
    eds, rr, cr = setup(oracle, k)
    w = 2 * k
    present = np.ones((w, w), np.uint8)
    present[3, 5] = 0
    present[0, 7] = 0  # row 0 and column 1 incomplete: their decode meets the bad cell
    present[9, 1] = 0
    bad = eds.copy()
    bad[0, 1, 200] ^= 0x40
    st, axis, bs, bp = _assert_same_outcome(ctx, oracle, bad, present, rr, cr)
    assert st == _lib.EBYZANTINE
    from celestia_eds.rsmt2d import ExtendedDataSquare
    sq = ExtendedDataSquare(np.where(present[..., None] == 1, bad, 0).astype(np.uint8), ctx=ctx)
    with pytest.raises(ErrByzantineData) as ei:
        sq.Repair(rr, cr, present=present)
    assert (ei.value.Axis, ei.value.Index) == axis


def test_gf16_repair_k256(ctx, oracle):
    k = 256
    eds, rr, cr = setup(oracle, k, seed=9)
    w = 2 * k
    present = np.zeros((w, w), np.uint8)
    present[k:, :k] = 1  # Q2 only
    assert np.array_equal(repair(ctx, eds, present, rr, cr), eds)


def test_gf16_repair_k512(ctx, oracle):
    """The largest square the device repairs: k = 512 (GF(2^16), 1024-shard axes through
    gather -> LDS decoder -> scatter, 512 MiB EDS), Q0 only and a random p = 0.55 mask;
    the repaired square is the original (the codeword is unique)."""
    from celestia_eds import _lib
    k = 512
    eds, rr, cr = setup(oracle, k, seed=12)
    w = 2 * k
    q0 = np.zeros((w, w), np.uint8)
    q0[:k, :k] = 1
    rnd = (np.random.default_rng(12).random((w, w)) < 0.55).astype(np.uint8)
    for present in (q0, rnd):
        st, cells, _ = _dev_repair(ctx, eds, present, rr, cr)
        assert st == _lib.OK and np.array_equal(cells, eds)


def _dev_repair(ctx, eds, present, rr, cr, want_shares=False):
    """cel_dev_repair over a device-resident damaged copy; returns (status, cells, bad)
    (+ (byz_shares, byz_present, mask after) with want_shares)."""
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
    bs = np.zeros((w, 512), np.uint8)
    bp = np.zeros(w, np.uint8)
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    st = ctx.lib.cel_dev_repair(ctx.handle, d.ptr, P(pres), k, P(rra), P(cra), ctypes.byref(ba), ctypes.byref(bi),
                                P(bs), P(bp))
    cells = d.download(eds.shape)
    if want_shares:
        return st, cells, (ba.value, bi.value), (bs, bp, pres)
    return st, cells, (ba.value, bi.value)


def _stack(roots):
    return np.stack([np.frombuffer(r, np.uint8) if isinstance(r, bytes) else r for r in roots])


def _oracle_repair(oracle, eds, present, rr, cr):
    damaged = eds.copy()
    damaged[present == 0] = 0
    return oracle.repair(damaged, present, _stack(rr), _stack(cr), want_shares=True)


def _assert_same_outcome(ctx, oracle, eds, present, rr, cr):
    """Device repair == oracle restatement: status, failing axis, ErrByzantineData.Shares
    (and which of them were known), the mask left behind, and the filled square."""
    from celestia_eds import _lib
    st, cells, bad, (bs, bp, pres) = _dev_repair(ctx, eds, present, rr, cr, want_shares=True)
    rc, ocells, opres, obad, (obs, obp) = _oracle_repair(oracle, eds, present, rr, cr)
    assert st == rc, (st, rc)
    if rc in (_lib.EBYZANTINE, _lib.EBADROOT):
        assert bad == obad
    if rc == _lib.EBYZANTINE:
        assert np.array_equal(bp, obp)
        assert np.array_equal(bs[bp == 1], obs[obp == 1])
    assert np.array_equal(pres, opres)
    if rc == _lib.OK:
        assert np.array_equal(cells, eds)
    else:  # cells the mask vouches for equal the oracle's
        assert np.array_equal(cells[pres == 1], ocells[opres == 1])
    return st, bad, bs, bp


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
    rc, _, _, _ = oracle.repair(damaged, present, _stack(rr), _stack(cr))
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
    st, dbad, _, _ = _assert_same_outcome(ctx, oracle, bad, present, rr, cr)
    assert st in (_lib.EBYZANTINE, _lib.OK, _lib.EBADROOT)


# --- config 5 at its own size (k = 128): (iv) p = 0.25 unrepairable, (v) one corrupt cell


def test_k128_p025_unrepairable(ctx, oracle):
    from celestia_eds import _lib
    k = 128
    eds, rr, cr = setup(oracle, k)
    present = (np.random.default_rng(7).random((2 * k, 2 * k)) < 0.25).astype(np.uint8)
    st, _, _, _ = _assert_same_outcome(ctx, oracle, eds, present, rr, cr)
    assert st == _lib.EUNREPAIRABLE


@pytest.mark.parametrize("p", [0.55, 0.9])
def test_k128_one_corrupt_cell(ctx, oracle, p):
    """One corrupted cell in the k = 128 EDS under random masks: a decoded axis fails its
    re-encoding or root check (a complete axis holding it would be rsmt2d's "bad root
    input" instead, test_sanity_check_bad_root)."""
    from celestia_eds import _lib
    from celestia_eds.rsmt2d import ErrByzantineData, ExtendedDataSquare
    k = 128
    w = 2 * k
    eds, rr, cr = setup(oracle, k)
    present = (np.random.default_rng(7).random((w, w)) < p).astype(np.uint8)
    r, c = 40, 77
    present[r, c] = 1
    present[r, 3] = present[200, c] = 0  # neither axis through the bad cell is complete
    bad = eds.copy()
    bad[r, c, 300] ^= 0x21
    st, axis, bs, bp = _assert_same_outcome(ctx, oracle, bad, present, rr, cr)
    assert st == _lib.EBYZANTINE
    # the host entry point raises rsmt2d's error with the same Shares
    sq = ExtendedDataSquare(np.where(present[..., None] == 1, bad, 0).astype(np.uint8), ctx=ctx)
    mask_in = present.copy()
    with pytest.raises(ErrByzantineData) as ei:
        sq.Repair(rr, cr, present=present)
    assert np.array_equal(present, mask_in)  # the caller's mask is not written through
    e = ei.value
    assert (e.Axis, e.Index) == axis
    assert [s is not None for s in e.Shares] == [bool(x) for x in bp]
    assert all(s == bs[j].tobytes() for j, s in enumerate(e.Shares) if s is not None)


@pytest.mark.parametrize("k", [16, 32, 64, 128, 256, 512])
@pytest.mark.parametrize("in_q1", [True, False])
def test_sanity_check_bad_encoding(ctx, oracle, k, in_q1):
    """Every cell present, one parity cell changed, and roots computed over that square:
    every root matches, so only rsmt2d's re-encoding of complete axes in
    preRepairSanityCheck catches it (ErrByzantineData with all the axis's shares). Cell
    (3, k+1) breaks row 3 and column k+1, reported as row 3; cell (k+1, 3) breaks row k+1
    and column 3, reported as column 3 (rsmt2d checks row i, then column i). k >= 32:
    the in-place check kernel in both directions; k = 16: gather -> encode -> compare;
    k = 256, 512: the GF(2^16) register encoder in check mode, in place on the square (rows
    at the cell stride, columns at the row stride)."""
    from celestia_eds import _lib
    w = 2 * k
    eds, _, _ = setup(oracle, k, seed=3)
    r, c = (3, k + 1) if in_q1 else (k + 1, 3)
    eds[r, c, 100] ^= 0x77
    _, rr, cr = oracle.roots(eds, check_order=False)
    present = np.ones((w, w), np.uint8)
    st, bad, bs, bp = _assert_same_outcome(ctx, oracle, eds, present, [x.tobytes() for x in rr],
                                           [x.tobytes() for x in cr])
    assert st == _lib.EBYZANTINE and bad == ((0, 3) if in_q1 else (1, 3))
    assert bp.all() and np.array_equal(bs, eds[3] if in_q1 else eds[:, 3])


def test_sanity_check_bad_root(ctx, oracle):
    """A complete row whose root differs: rsmt2d's "bad root input", not ErrByzantineData."""
    from celestia_eds import CelError, _lib
    from celestia_eds.rsmt2d import ExtendedDataSquare
    k = 8
    eds, rr, cr = setup(oracle, k)
    rr = list(rr)
    rr[5] = bytes(90)
    present = np.ones((2 * k, 2 * k), np.uint8)
    present[0, 0] = 0
    st, bad, _, _ = _assert_same_outcome(ctx, oracle, eds, present, rr, cr)
    assert st == _lib.EBADROOT and bad == (0, 5)
    with pytest.raises(CelError) as ei:
        ExtendedDataSquare(eds.copy(), ctx=ctx).Repair(rr, cr, present=present)
    assert ei.value.status == _lib.EBADROOT and "bad root input" in str(ei.value)


@pytest.mark.parametrize("k", [16, 256])
def test_orthogonal_completion_then_stuck(ctx, oracle, k):
    """Row r0 decodes and completes column c, whose known cell (r1, c) is corrupted (the
    roots were computed over the corrupted square, so every root matches); nothing else is
    solvable. rsmt2d's check of the newly completed column reports ErrByzantineData(Col, c)
    although the repair is stuck afterwards."""
    from celestia_eds import _lib
    w = 2 * k
    r0, r1, c = 2, 9, 5
    eds, _, _ = setup(oracle, k, seed=4)
    eds[r1, c, 200] ^= 0x10
    _, rr, cr = oracle.roots(eds, check_order=False)
    present = np.zeros((w, w), np.uint8)
    present[:, c] = 1
    present[r0, :] = 0
    present[r0, k:] = 1  # k cells of row r0, not column c
    st, bad, bs, bp = _assert_same_outcome(ctx, oracle, eds, present, [x.tobytes() for x in rr],
                                           [x.tobytes() for x in cr])
    assert st == _lib.EBYZANTINE and bad == (1, c)
    assert bp.all() and np.array_equal(bs, eds[:, c])


@pytest.mark.parametrize("k", [16, 256])
def test_solved_axis_bad_encoding(ctx, oracle, k):
    """An axis that a solve completes, with more than k known cells one of which is
    corrupted (roots computed over the corrupted square, so no root check can fire first):
    row 0 holds k + 1 cells, row 1 only k - 1, so rsmt2d's sweep solves row 0 first, and its
    decode over every known shard is no codeword: verifyEncoding after the solve reports
    ErrByzantineData(Row, 0). k = 256: the dense GF(2^16) path (gather -> LDS decoder ->
    encoding check on the dense buffer)."""
    from celestia_eds import _lib
    w = 2 * k
    eds, _, _ = setup(oracle, k, seed=5)
    eds[0, k + 3, 50] ^= 0x3C
    _, rr, cr = oracle.roots(eds, check_order=False)
    present = np.ones((w, w), np.uint8)
    present[0, :k - 1] = 0
    present[1, k - 1:] = 0
    st, bad, _, _ = _assert_same_outcome(ctx, oracle, eds, present, [x.tobytes() for x in rr],
                                         [x.tobytes() for x in cr])
    assert st == _lib.EBYZANTINE and bad == (0, 0)


def _crossword_passes(present, k):
    """Passes of rsmt2d's crossword loop over a presence mask alone (an axis with at least
    k of its 2k cells gets all of them): (passes, solvable)."""
    m = present.astype(bool).copy()
    w, n = 2 * k, 0
    while True:
        progress = False
        for ax in (0, 1):
            cnt = m.sum(axis=1 - ax)
            s = (cnt >= k) & (cnt < w)
            if s.any():
                if ax == 0:
                    m[s, :] = True
                else:
                    m[:, s] = True
                progress = True
                n += 1
        if m.all():
            return n, True
        if not progress:
            return n, False


@pytest.mark.parametrize("k,p,seed,npass,ok", [
    (32, 0.40, 13, 9, True),     # register decoder in the square, nine alternating passes
    (32, 0.40, 15, 3, False),    # stuck after three passes
    (128, 0.44, 1, 5, True),
    (256, 0.46, 2, 4, True),     # GF(2^16): gather -> LDS decoder -> scatter, both dense buffers
    (256, 0.44, 25, 5, False),
])
def test_dev_repair_many_passes(ctx, oracle, k, p, seed, npass, ok):
    """Masks whose crossword takes several row/column passes (the two-stream schedule:
    solve chain on the main stream, encoding checks on the side stream, alternating dense
    buffers for the LDS decoder): a solvable mask gives back the original EDS (the
    codeword is unique), a stuck one EUNREPAIRABLE with every cell the final mask vouches
    for equal to the original; k = 32 also against the oracle's restatement."""
    from celestia_eds import _lib
    eds, rr, cr = setup(oracle, k, seed=3)
    w = 2 * k
    present = (np.random.default_rng(seed).random((w, w)) < p).astype(np.uint8)
    assert _crossword_passes(present, k) == (npass, ok)
    st, cells, _, (_, _, after) = _dev_repair(ctx, eds, present, rr, cr, want_shares=True)
    if ok:
        assert st == _lib.OK and np.array_equal(cells, eds)
    else:
        assert st == _lib.EUNREPAIRABLE
        assert np.array_equal(cells[after == 1], eds[after == 1])
        assert (after >= present).all() and after.sum() > present.sum()
    if k == 32:
        damaged = eds.copy()
        damaged[present == 0] = 0
        rc, ocells, opres, _ = oracle.repair(damaged, present, _stack(rr), _stack(cr))
        assert rc == st
        assert np.array_equal(after, opres)


@pytest.mark.parametrize("k", [128, 256])
def test_dev_repair_random_masks(ctx, oracle, k):
    """18 random masks near the repair threshold (2-5 crossword passes): every outcome as
    the mask's crossword predicts (solvable -> OK and the original EDS, stuck ->
    EUNREPAIRABLE), through the two-stream schedule (k=128: in-square register decoder,
    k=256: gather -> LDS decoder -> scatter with alternating dense buffers)."""
    from celestia_eds import _lib
    eds, rr, cr = setup(oracle, k, seed=3)
    w = 2 * k
    for seed in range(6):
        for p in (0.44, 0.46, 0.5):
            present = (np.random.default_rng(seed).random((w, w)) < p).astype(np.uint8)
            _, ok = _crossword_passes(present, k)
            st, cells, _ = _dev_repair(ctx, eds, present, rr, cr)
            if ok:
                assert st == _lib.OK and np.array_equal(cells, eds), (seed, p)
            else:
                assert st == _lib.EUNREPAIRABLE, (seed, p, st)


@pytest.mark.parametrize("k", [8, 32, 256])
def test_missing_cells_hold_garbage(ctx, oracle, k):
    """The Repair ABI lets missing cells hold anything: random bytes there must not reach
    the decoders (k = 8 and 256: the LDS decoder, which zeroes erased points at its load;
    k = 32: the in-square register decoder, whose erased points scale by zero)."""
    from celestia_eds import _lib
    eds, rr, cr = setup(oracle, k, seed=5)
    w = 2 * k
    rng = np.random.default_rng(k)
    present = (rng.random((w, w)) < 0.6).astype(np.uint8)
    junk = np.where(present[..., None] == 1, eds, rng.integers(0, 256, eds.shape, dtype=np.uint8))
    import ctypes
    from hipmem import DeviceBuffer
    d = DeviceBuffer(junk.nbytes)
    d.upload(np.ascontiguousarray(junk))
    pres = present.copy()
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    rra, cra = _stack(rr), _stack(cr)
    st = ctx.lib.cel_dev_repair(ctx.handle, d.ptr, P(pres), k, P(rra), P(cra), None, None, None, None)
    assert st == _lib.OK and np.array_equal(d.download(eds.shape), eds)


def test_codec_decode_ignores_erased_bytes(ctx, oracle):
    """cel_codec_decode / cel_dev_decode: erased shards' bytes are not inputs (n = 8 and
    1024: the LDS decoder; n = 64: the register decoder)."""
    import ctypes
    from celestia_eds import _lib
    for n in (8, 64, 1024):
        rng = np.random.default_rng(n)
        data = rng.integers(0, 256, (n, 128), dtype=np.uint8)
        cw = np.concatenate([data, oracle.rs_encode(data)])
        present = np.ones(2 * n, np.uint8)
        present[rng.choice(2 * n, n, replace=False)] = 0
        buf = np.where(present[:, None] == 1, cw, rng.integers(0, 256, cw.shape, dtype=np.uint8)).astype(np.uint8)
        P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
        assert ctx.lib.cel_codec_decode(ctx.handle, P(buf), P(present), n, 128) == _lib.OK
        assert np.array_equal(buf, cw), n


def test_decode_inconsistent_shards_matches_oracle(ctx, oracle):
    """Shards that are not a codeword (byzantine input): the device decoders compute
    Leopard's error-locator formula over every present shard, erased data and parity alike
    (klauspost reconstruct, recoverAll), like the oracle's restatement; Gauss-Jordan over
    any k of them would differ. Parity unpinned (no reference vector decodes such input)."""
    import ctypes
    from celestia_eds import _lib
    for n in (8, 16, 32, 128, 256, 512):
        rng = np.random.default_rng(100 + n)
        data = rng.integers(0, 256, (n, 128), dtype=np.uint8)
        cw = np.concatenate([data, oracle.rs_encode(data)])
        present = np.ones(2 * n, np.uint8)
        present[rng.choice(2 * n, n // 2, replace=False)] = 0
        bad = cw.copy()
        for j in rng.choice(np.flatnonzero(present), 3, replace=False):
            bad[j, rng.integers(0, 128)] ^= 0x3C
        bad[present == 0] = 0
        exp = oracle.rs_decode(bad, present)
        buf = bad.copy()
        P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
        assert ctx.lib.cel_codec_decode(ctx.handle, P(buf), P(present), n, 128) == _lib.OK
        assert np.array_equal(buf, exp), n
        assert not np.array_equal(buf, cw)


# --- rsmt2d's sweep order (row i, then column i) decides which byzantine axis is reported


def _byz_case(oracle, k, seed):
    """A random mask (p = 0.5 / 0.6 / 0.7 by seed) with two corrupted present cells."""
    eds, rr, cr = setup(oracle, k, seed=3)
    w = 2 * k
    rng = np.random.default_rng(seed)
    p = [0.5, 0.6, 0.7][seed % 3]
    present = (rng.random((w, w)) < p).astype(np.uint8)
    bad = eds.copy()
    for _ in range(2):
        r, c = rng.integers(0, w, 2)
        present[r, c] = 1
        bad[r, c, rng.integers(0, 512)] ^= 0x5A
    return bad, present, rr, cr


@pytest.mark.parametrize("k,seed", [(8, 0), (32, 0), (32, 2), (128, 0), (256, 2)])
def test_sweep_order_byzantine(ctx, oracle, k, seed):
    """Cases where rsmt2d's sweep (row i, then column i) reports a different byzantine axis
    than all-rows-then-all-columns passes would: the device (pass-parallel schedule, then
    the exact replay in rsmt2d's order) reports the oracle's sweep-order outcome, Shares
    and mask included. k = 8: gather -> LDS decoder; k = 32, 128: the in-square register
    decoder (a level's rows and columns in one launch); k = 256: GF(2^16), gather -> LDS
    decoder -> scatter per direction."""
    from celestia_eds import _lib
    bad, present, rr, cr = _byz_case(oracle, k, seed)
    damaged = np.where(present[..., None] == 1, bad, 0).astype(np.uint8)
    o_sweep = oracle.repair(damaged, present, _stack(rr), _stack(cr), order=0)
    o_pass = oracle.repair(damaged, present, _stack(rr), _stack(cr), order=1)
    assert o_sweep[0] == o_pass[0] == _lib.EBYZANTINE
    assert o_sweep[3] != o_pass[3]  # the case tells the orders apart
    st, axis, _, _ = _assert_same_outcome(ctx, oracle, bad, present, rr, cr)
    assert axis == o_sweep[3]


@pytest.mark.parametrize("k", [32, 128, 256])
def test_repair_schedule_fuzz(ctx, oracle, k):
    """The repair's two streams with a random idle kernel (0..max us) in front of every
    operation either stream enqueues (cel_debug_schedule_fuzz), over several seeds: any
    missing cross-stream dependency (a check reading a buffer the chain is still writing,
    a decode reusing a buffer a check still reads) would change an outcome. Multi-pass
    solvable and stuck masks, and a byzantine square (exact replay)."""
    from celestia_eds import _lib
    eds, rr, cr = setup(oracle, k, seed=3)
    w = 2 * k
    masks = [(np.random.default_rng(s).random((w, w)) < p).astype(np.uint8)
             for s, p in ((1, 0.44), (2, 0.46), (25, 0.44))]
    try:
        for fseed in range(6):  # idle kernels of up to 60 us, then up to 250 us
            assert ctx.lib.cel_debug_schedule_fuzz(ctx.handle, 1000 + fseed, 60 if fseed < 3 else 250) == _lib.OK
            for present in masks:
                _, ok = _crossword_passes(present, k)
                st, cells, _ = _dev_repair(ctx, eds, present, rr, cr)
                if ok:
                    assert st == _lib.OK and np.array_equal(cells, eds), fseed
                else:
                    assert st == _lib.EUNREPAIRABLE, (fseed, st)
            bad, present, brr, bcr = _byz_case(oracle, k, 0 if k <= 128 else 2)
            _assert_same_outcome(ctx, oracle, bad, present, brr, bcr)
    finally:
        ctx.lib.cel_debug_schedule_fuzz(ctx.handle, 0, 0)
