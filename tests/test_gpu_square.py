"""GPU parity: da.ExtendShares + NewDataAvailabilityHeader through the C ABI vs the
CPU oracle (bit-exact EDS bytes, 4k roots, DAH), the reference's DAH known answers
and mainnet block 408."""
import hashlib

import numpy as np
import pytest

from eds_inputs import constant_ods, random_ods, tail_padding_share

pytestmark = pytest.mark.gpu


def run_device(ctx, ods):
    from celestia_eds import da
    eds = da._extend(np.ascontiguousarray(ods).reshape(-1, 512), ctx=ctx)
    return eds


@pytest.mark.parametrize("k", [1, 2, 4, 8, 16, 32, 64, 128])
def test_extend_commit_matches_oracle(ctx, oracle, k):
    ods = random_ods(k, 1000 + k)
    dev = run_device(ctx, ods)
    eds, rr, cr, dah = oracle.extend_and_commit(ods)
    assert np.array_equal(dev.cells, eds), "EDS bytes differ"
    assert np.array_equal(dev._row_roots, rr), "row roots differ"
    assert np.array_equal(dev._col_roots, cr), "column roots differ"
    assert dev._dah == dah


def test_block408(ctx, golden, block408_ods):
    dev = run_device(ctx, block408_ods)
    g = golden["block408"]
    assert dev._dah.hex() == g["data_hash"]
    assert hashlib.sha256(dev.cells.tobytes()).hexdigest() == g["eds_sha256"]


def test_dah_known_answers(ctx, golden):
    from celestia_eds import da
    kat = golden["dah_known_answers"]
    assert da.NilDataAvailabilityHeaderHash().hex() == kat["empty"]
    assert da.MinDataAvailabilityHeader().Hash().hex() == kat["min"]
    for k, key in ((2, "typical_k2"), (128, "max_k128")):
        eds = da.ExtendShares(list(constant_ods(k).reshape(-1, 512)))
        dah = da.NewDataAvailabilityHeader(eds)
        assert len(dah.RowRoots) == 2 * k and len(dah.ColumnRoots) == 2 * k
        assert dah.Hash().hex() == kat[key]
        assert eds._dah.hex() == kat[key]


def test_compute_dah_without_eds(ctx, golden, block408_ods):
    """ComputeDataAvailabilityHeader (no EDS copied back, the PrepareProposal /
    ProcessProposal shape) equals NewDataAvailabilityHeader(ExtendShares(...)): the DAH known
    answers, block 408's data root, and the same error as ExtendShares."""
    import pytest as _pytest
    from celestia_eds import CelError, _lib, da
    kat = golden["dah_known_answers"]
    for k, key in ((2, "typical_k2"), (128, "max_k128")):
        dah = da.ComputeDataAvailabilityHeader(list(constant_ods(k).reshape(-1, 512)))
        assert dah.Hash().hex() == kat[key] and len(dah.RowRoots) == 2 * k
        dah.hash = b""  # recomputed from the returned roots
        assert dah.Hash().hex() == kat[key]
    ods = random_ods(32, 9)
    ref = da.NewDataAvailabilityHeader(da.ExtendShares(list(ods.reshape(-1, 512))))
    got = da.ComputeDataAvailabilityHeader(list(ods.reshape(-1, 512)))
    assert got.RowRoots == ref.RowRoots and got.ColumnRoots == ref.ColumnRoots and got.Hash() == ref.Hash()
    assert da.ComputeDataAvailabilityHeader(block408_ods.reshape(-1, 512)).Hash().hex() == golden["block408"]["data_hash"]
    with _pytest.raises(CelError) as ei:
        da.ComputeDataAvailabilityHeader([bytes(512)] * 5)
    assert ei.value.status == _lib.ENOTPOW2 and "got 5" in str(ei.value)


def test_min_dah_validate_and_square_size(ctx):
    from celestia_eds import da
    dah = da.MinDataAvailabilityHeader()
    dah.ValidateBasic()
    assert dah.SquareSize() == 1


def test_extend_shares_errors(ctx):
    from celestia_eds import CelError, da
    with pytest.raises(CelError, match="number of shares is not a power of 2: got 5"):
        da.ExtendShares([bytes(512)] * 5)
    with pytest.raises(CelError):  # 129*129 shares (data_availability_header_test.go:77-80)
        da.ExtendShares([bytes(512)] * (129 * 129))
    # equal shares of another size: the library's ECHUNK (it never reads past n x 512 B)
    from celestia_eds import _lib
    for f in (da.ExtendShares, da.ComputeDataAvailabilityHeader):
        with pytest.raises(CelError) as ei:
            f([bytes(256)] * 4)
        assert ei.value.status == _lib.ECHUNK


def test_order_violation_reported(ctx):
    from celestia_eds import CelError, _lib
    ods = random_ods(8, 77)
    ods[2, 3], ods[2, 4] = ods[2, 4].copy(), ods[2, 3].copy()
    with pytest.raises(CelError) as ei:
        run_device(ctx, ods)
    assert ei.value.status == _lib.EORDER


def test_batch_matches_single(ctx, oracle):
    """cel_extend_batch over several independent squares (config 4 shape, small)."""
    import ctypes
    from celestia_eds import _lib
    k, n = 16, 5
    odss = np.stack([random_ods(k, 50 + i) for i in range(n)])
    rr = np.zeros((n, 2 * k, 90), np.uint8)
    cr = np.zeros_like(rr)
    dah = np.zeros((n, 32), np.uint8)
    eds = np.zeros((n, 2 * k, 2 * k, 512), np.uint8)
    st = np.zeros(n, np.int32)
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    ctx.check(ctx.lib.cel_extend_batch(ctx.handle, P(odss), n, k, 512, P(eds), P(rr), P(cr), P(dah), P(st),
                                       _lib.FLAG_ORDER_CHECK))
    for i in range(n):
        e, r, c, d = oracle.extend_and_commit(odss[i])
        assert np.array_equal(eds[i], e) and np.array_equal(rr[i], r) and np.array_equal(cr[i], c)
        assert dah[i].tobytes() == d


def test_gf16_square_k256(ctx, oracle):
    """k = 256: 512 shards per axis -> Leopard GF(2^16) (parity unpinned by the reference;
    checked against the oracle restatement)."""
    k = 256
    ods = random_ods(k, 256)
    dev = run_device(ctx, ods)
    eds, rr, cr, dah = oracle.extend_and_commit(ods)
    assert np.array_equal(dev.cells, eds)
    assert np.array_equal(dev._row_roots, rr) and np.array_equal(dev._col_roots, cr)
    assert dev._dah == dah


def _pinned(ctx, shape):
    import ctypes
    nbytes = int(np.prod(shape))
    p = ctx.lib.cel_host_alloc(nbytes)
    assert p, "cel_host_alloc failed"
    return p, np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p)).reshape(shape)


@pytest.mark.parametrize("k", [32, 64, 128, 256, 512])
def test_pinned_single_square(ctx, oracle, k):
    """One square from page-locked memory (cel_extend_batch, n = 1). At the GF(2^16) widths
    the ODS goes up by DMA into Q0 (at k = 512 in four row chunks whose rows and leaves are
    processed while the next chunk crosses PCIe); at k = 32..128 the GF(2^8) row pass reads
    the ODS straight from the mapped host pages and the top rows download early into the
    page-locked EDS (api.cpp's one-square path, which the Go shim's staged ODS always
    takes). Full EDS, parity only and roots only against the oracle; a push-order
    violation between the rows on either side of a chunk boundary (rows 127 / 128; k / 2
    - 1 / k / 2 below k = 256) is reported with the reference's error."""
    import ctypes
    from celestia_eds import CelError, _lib
    ods_ref = random_ods(k, 600 + k)
    e_ref, rr_ref, cr_ref, dah_ref = oracle.extend_and_commit(ods_ref)
    w = 2 * k
    p_ods, ods = _pinned(ctx, (k, k, 512))
    p_eds, eds = _pinned(ctx, (w, w, 512))
    P = lambda x: x.ctypes.data_as(ctypes.c_void_p)
    rr, cr, dah, st = np.zeros((w, 90), np.uint8), np.zeros((w, 90), np.uint8), np.zeros(32, np.uint8), np.zeros(1, np.int32)
    try:
        ods[...] = ods_ref
        for fl, want_eds in ((0, True), (_lib.FLAG_PARITY_ONLY, True), (0, False)):
            eds[...] = 0
            ctx.check(ctx.lib.cel_extend_batch(ctx.handle, ctypes.c_void_p(p_ods), 1, k, 512,
                                               ctypes.c_void_p(p_eds) if want_eds else None, P(rr), P(cr), P(dah),
                                               P(st), _lib.FLAG_ORDER_CHECK | fl))
            assert np.array_equal(rr, rr_ref) and np.array_equal(cr, cr_ref) and dah.tobytes() == dah_ref
            if want_eds:
                got = eds.copy()
                if fl:
                    assert not got[:k, :k].any(), "Q0 written under CEL_FLAG_PARITY_ONLY"
                    got[:k, :k] = ods_ref
                assert np.array_equal(got, e_ref), "EDS differs"
        # column order broken only across the chunk boundary: row 128 takes row 0's
        # namespaces (still sorted along the row, below row 127's in every column)
        b = 128 if k >= 256 else k // 2
        bad = ods_ref.copy()
        bad[b, :, :29] = bad[0, :, :29]
        assert (bad[b, :, :29].tobytes() < bad[b - 1, :, :29].tobytes())
        ods[...] = bad
        with pytest.raises(CelError) as e:
            ctx.check(ctx.lib.cel_extend_batch(ctx.handle, ctypes.c_void_p(p_ods), 1, k, 512, None, P(rr), P(cr),
                                               P(dah), P(st), _lib.FLAG_ORDER_CHECK))
        assert e.value.status == _lib.EORDER
    finally:
        ctx.lib.cel_host_free(p_ods)
        ctx.lib.cel_host_free(p_eds)


def test_gf16_square_k512(ctx, oracle):
    """k = 512 (config 3's square, here on one GPU): GF(2^16) register kernel, 2k = 1024
    trees. Roots, DAH and the EDS bytes (by digest) against the oracle restatement."""
    import hashlib
    k = 512
    ods = random_ods(k, 512)
    dev = run_device(ctx, ods)
    eds, rr, cr, dah = oracle.extend_and_commit(ods)
    assert hashlib.sha256(dev.cells.tobytes()).digest() == hashlib.sha256(eds.tobytes()).digest()
    assert np.array_equal(dev._row_roots, rr) and np.array_equal(dev._col_roots, cr)
    assert dev._dah == dah


@pytest.mark.parametrize("k,n", [(32, 3), (64, 9), (64, 40), (128, 5), (128, 17)])
def test_batch_extension_uneven(ctx, oracle, k, n):
    """Batches of the wave-per-axis kernel sizes (k = 32..128) with odd square counts:
    (64, 40) and (128, 17) split into the two pipeline chunks of cel_dev_extend_batch
    with a short last chunk; the host path places each ODS in Q0 and extends it in
    place (cel_dev_place_ods). EDS bytes, roots and DAH against the oracle for every square."""
    import ctypes
    from celestia_eds import _lib
    odss = np.stack([random_ods(k, 900 + 7 * i + k) for i in range(n)])
    rr = np.zeros((n, 2 * k, 90), np.uint8)
    cr = np.zeros_like(rr)
    dah = np.zeros((n, 32), np.uint8)
    eds = np.zeros((n, 2 * k, 2 * k, 512), np.uint8)
    st = np.zeros(n, np.int32)
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    ctx.check(ctx.lib.cel_extend_batch(ctx.handle, P(odss), n, k, 512, P(eds), P(rr), P(cr), P(dah), P(st),
                                       _lib.FLAG_ORDER_CHECK))
    for i in range(n):
        e, r, c, d = oracle.extend_and_commit(odss[i])
        assert np.array_equal(eds[i], e), f"square {i}: EDS differs"
        assert np.array_equal(rr[i], r) and np.array_equal(cr[i], c) and dah[i].tobytes() == d


def test_extend_block_408_from_txs(ctx, golden):
    """app.ExtendBlock (app/extend_block.go:14-26) end to end through the product:
    block 408's txs -> square.Construct (cel_square_construct) -> da.ExtendShares ->
    NewDataAvailabilityHeader on the device == the block header's data_hash."""
    from celestia_eds import da, square
    from square_inputs import block408_txs
    ods = square.Construct(block408_txs())
    eds = da.ExtendShares(list(ods))
    assert da.NewDataAvailabilityHeader(eds).Hash().hex() == golden["block408"]["data_hash"]


def test_extend_empty_block(ctx, golden):
    """An empty block's square is one tail-padding share: its DAH is the reference's
    MinDataAvailabilityHeader hash (data_availability_header_test.go:27-32)."""
    from celestia_eds import da, square
    eds = da.ExtendShares(list(square.Construct([])))
    assert da.NewDataAvailabilityHeader(eds).Hash().hex() == golden["dah_known_answers"]["min"]


def test_dah_proto_conversion(ctx):
    """TestDataAvailabilityHeaderProtoConversion (data_availability_header_test.go:101-133):
    min and max (k = 128) DAHs survive ToProto / DataAvailabilityHeaderFromProto."""
    from celestia_eds import da
    big = da.NewDataAvailabilityHeader(da.ExtendShares(list(random_ods(128, 5).reshape(-1, 512))))
    for dah in (da.MinDataAvailabilityHeader(), big):
        res = da.DataAvailabilityHeaderFromProto(dah.ToProto())
        assert res.RowRoots == dah.RowRoots and res.ColumnRoots == dah.ColumnRoots
        assert res.Hash() == dah.Hash()
    raw = da.MinDataAvailabilityHeader().ToProto()
    assert raw[0] == 0x0A and raw[1] == 90 and raw[92] == 0x0A and raw[184] == 0x12  # 2 rows, then 2 columns


def test_dah_validate_basic_cases(ctx):
    """Test_DAHValidateBasic (data_availability_header_test.go:135-215)."""
    from celestia_eds import CelError, da
    big = da.NewDataAvailabilityHeader(da.ExtendShares(list(random_ods(128, 6).reshape(-1, 512))))
    big.ValidateBasic()
    da.MinDataAvailabilityHeader().ValidateBasic()
    max_size = 128 * 128
    too_big = da.DataAvailabilityHeader(big.RowRoots + [b"\x01" * 32] * (max_size - 256 + 1),
                                        big.ColumnRoots + [b"\x01" * 32] * (max_size - 256 + 1))
    too_small = da.DataAvailabilityHeader([b"\x02" * 32], [b"\x02" * 32])
    bad_hash = da.MinDataAvailabilityHeader()
    bad_hash.hash = bytes([1, 2, 3, 4])
    mismatch = da.MinDataAvailabilityHeader()
    mismatch.ColumnRoots = mismatch.ColumnRoots + [b"\x02" * 32]
    for dah, msg in ((too_big, "maximum valid DataAvailabilityHeader has at most"),
                     (too_small, "minimum valid DataAvailabilityHeader has at least"),
                     (bad_hash, "wrong hash"), (mismatch, "unequal number of row and column roots")):
        with pytest.raises(CelError, match=msg):
            dah.ValidateBasic()


@pytest.mark.parametrize("inplace", [True, False])
@pytest.mark.parametrize("k,n", [(32, 5), (64, 3), (128, 13), (256, 2)])
def test_device_batch(ctx, oracle, k, n, inplace):
    """Device-resident batch (cel_dev_*). inplace: the ODS placed in Q0 of each EDS
    buffer by cel_dev_place_ods and extended in place (d_ods = NULL, the bench's input
    layout); otherwise a separate ODS buffer whose rows the row pass copies into Q0.
    EDS bytes, roots and DAH against the oracle for every square; a second
    extend_only over the same buffers is idempotent."""
    import ctypes
    from celestia_eds import _lib
    from hipmem import DeviceBuffer, synchronize
    odss = np.stack([random_ods(k, 4000 + 11 * i + k) for i in range(n)])
    w = 2 * k
    d_eds = DeviceBuffer(n * w * w * 512, fill=0xA5)  # Q1..Q3 must be fully overwritten
    d_rr, d_cr = DeviceBuffer(n * w * 90), DeviceBuffer(n * w * 90)
    d_dah, d_st = DeviceBuffer(n * 32), DeviceBuffer(n * 4, fill=0x7F)
    d_work = DeviceBuffer(ctx.lib.cel_dev_workspace_size(k, n))
    if inplace:
        d_ods = None
        ctx.check(ctx.lib.cel_dev_place_ods(ctx.handle, odss.ctypes.data_as(ctypes.c_void_p), n, k, d_eds.ptr, None))
    else:
        ods_buf = DeviceBuffer(odss.nbytes)
        ods_buf.upload(odss)
        d_ods = ods_buf.ptr
    ctx.check(ctx.lib.cel_dev_extend_batch(ctx.handle, d_ods, n, k, d_eds.ptr, d_rr.ptr, d_cr.ptr, d_dah.ptr,
                                           d_st.ptr, d_work.ptr,
                                           None, _lib.FLAG_ORDER_CHECK))
    synchronize()
    eds = d_eds.download((n, w, w, 512))
    rr, cr = d_rr.download((n, w, 90)), d_cr.download((n, w, 90))
    dah, st = d_dah.download((n, 32)), d_st.download((n,), np.int32)
    assert (st == 0).all()
    for i in range(n):
        e, r, c, d = oracle.extend_and_commit(odss[i])
        assert np.array_equal(eds[i], e), f"square {i}: EDS differs"
        assert np.array_equal(rr[i], r) and np.array_equal(cr[i], c) and dah[i].tobytes() == d
    ctx.check(ctx.lib.cel_dev_extend_only(ctx.handle, d_ods, n, k, d_eds.ptr, None))
    synchronize()
    assert np.array_equal(d_eds.download((n, w, w, 512)), eds)


@pytest.mark.parametrize("k,n", [(128, 3), (256, 2), (16, 5)])
def test_device_batch_caller_stream(ctx, oracle, k, n):
    """CEL_FLAG_CALLER_STREAM at GF(2^8) and GF(2^16) widths and below the axis kernel's
    range (k=16): the whole batch as one chunk on the ctx's stream (NULL caller stream),
    twice in a row (the second call waits for the first one's extension), bit-exact."""
    import ctypes
    from celestia_eds import _lib
    from hipmem import DeviceBuffer, synchronize
    odss = np.stack([random_ods(k, 5100 + 7 * i + k) for i in range(n)])
    w = 2 * k
    d_eds = DeviceBuffer(n * w * w * 512, fill=0x3C)
    d_rr, d_cr = DeviceBuffer(n * w * 90), DeviceBuffer(n * w * 90)
    d_dah, d_st = DeviceBuffer(n * 32), DeviceBuffer(n * 4, fill=0x7F)
    d_work = DeviceBuffer(ctx.lib.cel_dev_workspace_size(k, n))
    ctx.check(ctx.lib.cel_dev_place_ods(ctx.handle, odss.ctypes.data_as(ctypes.c_void_p), n, k, d_eds.ptr, None))
    for _ in range(2):
        ctx.check(ctx.lib.cel_dev_extend_batch(ctx.handle, None, n, k, d_eds.ptr, d_rr.ptr, d_cr.ptr, d_dah.ptr,
                                               d_st.ptr, d_work.ptr, None,
                                               _lib.FLAG_ORDER_CHECK | _lib.FLAG_CALLER_STREAM))
    synchronize()
    eds = d_eds.download((n, w, w, 512))
    rr, cr = d_rr.download((n, w, 90)), d_cr.download((n, w, 90))
    dah, st = d_dah.download((n, 32)), d_st.download((n,), np.int32)
    assert (st == 0).all()
    for i in range(n):
        e, r, c, d = oracle.extend_and_commit(odss[i])
        assert np.array_equal(eds[i], e), f"square {i}: EDS differs"
        assert np.array_equal(rr[i], r) and np.array_equal(cr[i], c) and dah[i].tobytes() == d


@pytest.mark.parametrize("k,region", [(32, "quarter3"), (64, "quarter3"), (128, "quarter3"), (64, "all")])
def test_parity_namespace_in_ods(ctx, oracle, k, region):
    """ODS shares that carry the parity namespace 0xFF*29 themselves. Their subtrees
    start with the same 0x01 || 0xFF*55 node prefix as Q1-Q3 subtrees, so the inner-node
    midstate path (nmt_kernels.hip hash_node) runs on Q0 data too; the IgnoreMaxNamespace
    rule (nmt hasher.go HashNode) applies to them by value. Rows and columns stay
    namespace-ordered."""
    ods = random_ods(k, 7000 + k)
    if region == "all":
        ods[:, :, :29] = 0xFF
    else:  # every cell outside the top-left quarter of the ODS
        h = k // 2
        ods[h:, :, :29] = 0xFF
        ods[:, h:, :29] = 0xFF
    dev = run_device(ctx, ods)
    eds, rr, cr, dah = oracle.extend_and_commit(ods)
    assert np.array_equal(dev.cells, eds), "EDS bytes differ"
    assert np.array_equal(dev._row_roots, rr), "row roots differ"
    assert np.array_equal(dev._col_roots, cr), "column roots differ"
    assert dev._dah == dah


def test_dah_hash_any_root_length(ctx):
    """DataAvailabilityHeader.Hash over roots of any length and unequal row / column
    counts (data_availability_header.go:92-108: rowsCount row roots, then the first
    rowsCount column roots, nil slices where there are fewer) against a hashlib
    merkle.HashFromByteSlices; 90-byte roots keep going through cel_dah_hash."""
    import hashlib
    from celestia_eds import da

    def sha(b):
        return hashlib.sha256(b).digest()

    def rfc(items):
        if not items:
            return sha(b"")
        if len(items) == 1:
            return sha(b"\x00" + items[0])
        k = 1
        while k * 2 < len(items):
            k *= 2
        return sha(b"\x01" + rfc(items[:k]) + rfc(items[k:]))

    rng = np.random.default_rng(7)
    cases = [([], []), ([b"a"], [b"b"]), ([b"x" * 32] * 3, [b"y" * 32] * 3), ([b""] * 2, [b"z"] * 2),
             ([bytes(rng.integers(0, 256, int(n), np.uint8)) for n in rng.integers(0, 300, 7)],
              [bytes(rng.integers(0, 256, int(n), np.uint8)) for n in rng.integers(0, 300, 5)]),
             ([b"r" * 90] * 4, [b"c" * 90] * 6),
             ([bytes(rng.integers(0, 256, 90, np.uint8)) for _ in range(8)],
              [bytes(rng.integers(0, 256, 90, np.uint8)) for _ in range(8)])]
    for rows, cols in cases:
        w = len(rows)
        want = rfc(rows + (cols[:w] + [b""] * max(0, w - len(cols))))
        assert da.DataAvailabilityHeader(rows, cols).Hash() == want, (len(rows), len(cols))


@pytest.mark.parametrize("k,n", [(16, 3), (128, 5)])
def test_batch_parity_only(ctx, oracle, k, n):
    """CEL_FLAG_PARITY_ONLY: the host path copies back Q1, Q2, Q3 only (Q1 as one strided
    copy per square); the caller's Q0 bytes stay untouched, every parity cell, root and
    DAH equals the oracle's."""
    import ctypes
    from celestia_eds import _lib
    odss = np.stack([random_ods(k, 300 + 5 * i + k) for i in range(n)])
    rr = np.zeros((n, 2 * k, 90), np.uint8)
    cr = np.zeros_like(rr)
    dah = np.zeros((n, 32), np.uint8)
    eds = np.full((n, 2 * k, 2 * k, 512), 0xA5, np.uint8)
    st = np.zeros(n, np.int32)
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    ctx.check(ctx.lib.cel_extend_batch(ctx.handle, P(odss), n, k, 512, P(eds), P(rr), P(cr), P(dah), P(st),
                                       _lib.FLAG_ORDER_CHECK | _lib.FLAG_PARITY_ONLY))
    for i in range(n):
        e, r, c, d = oracle.extend_and_commit(odss[i])
        assert (eds[i, :k, :k] == 0xA5).all(), f"square {i}: Q0 was written"
        assert np.array_equal(eds[i, :k, k:], e[:k, k:]) and np.array_equal(eds[i, k:], e[k:]), f"square {i}: parity"
        assert np.array_equal(rr[i], r) and np.array_equal(cr[i], c) and dah[i].tobytes() == d


@pytest.mark.parametrize("k,n", [(32, 3), (64, 4)])
def test_batches_in_flight_on_two_streams(ctx, oracle, k, n):
    """Independent batches issued back to back on two caller streams (bench --inflight 2):
    with CEL_FLAG_CALLER_STREAM each batch runs as one chunk on its caller's stream, so the
    batches overlap on the device; a third batch on the internal two-chunk pipeline runs
    beside them. Each batch's buffers are rewritten by every one of its calls; after
    alternating calls, and again after one batch's input is reloaded on its own stream
    between calls, every EDS, root and DAH equals the oracle's."""
    import ctypes
    from celestia_eds import _lib
    from hipmem import DeviceBuffer, Stream, synchronize
    w = 2 * k

    class Batch:
        def __init__(self, seed, flags):
            self.s, self.flags = Stream(), flags
            self.eds = DeviceBuffer(n * w * w * 512, fill=0)
            self.rr, self.cr = DeviceBuffer(n * w * 90), DeviceBuffer(n * w * 90)
            self.dah, self.st = DeviceBuffer(n * 32), DeviceBuffer(n * 4, fill=0x7F)
            self.work = DeviceBuffer(ctx.lib.cel_dev_workspace_size(k, n))
            self.load(seed)

        def load(self, seed):
            self.odss = np.stack([random_ods(k, seed + i) for i in range(n)])
            ctx.check(ctx.lib.cel_dev_place_ods(ctx.handle, self.odss.ctypes.data_as(ctypes.c_void_p), n, k,
                                                self.eds.ptr, self.s.ptr))

        def step(self):
            ctx.check(ctx.lib.cel_dev_extend_batch(ctx.handle, None, n, k, self.eds.ptr, self.rr.ptr, self.cr.ptr,
                                                   self.dah.ptr, self.st.ptr, self.work.ptr, self.s.ptr,
                                                   _lib.FLAG_ORDER_CHECK | self.flags))

        def check(self):
            self.s.synchronize()
            eds = self.eds.download((n, w, w, 512))
            rr, cr = self.rr.download((n, w, 90)), self.cr.download((n, w, 90))
            dah, st = self.dah.download((n, 32)), self.st.download((n,), np.int32)
            assert (st == 0).all()
            for i in range(n):
                e, r, c, d = oracle.extend_and_commit(self.odss[i])
                assert np.array_equal(eds[i], e) and np.array_equal(rr[i], r) and np.array_equal(cr[i], c)
                assert dah[i].tobytes() == d

    a, b = Batch(7100, _lib.FLAG_CALLER_STREAM), Batch(7200, _lib.FLAG_CALLER_STREAM)
    c = Batch(7400, 0)
    for _ in range(3):
        a.step()
        b.step()
        c.step()
    a.check()
    b.check()
    c.check()
    # a's input is reloaded on a's stream while b's batch may still run
    b.step()
    a.load(7300)
    a.step()
    b.step()
    a.check()
    b.check()
    synchronize()


def test_bench_shape_batches_in_flight(ctx, oracle):
    """The bench's batch shape (BASELINE config 2) through the raw C ABI: 256 k=128
    squares per batch, two batches in flight on two caller streams (CEL_FLAG_CALLER_STREAM),
    steps alternating (the bench's default four batches through SquareBatch:
    tests/test_gpu_bench_shapes.py). Size-independent properties against the oracle: every square's
    DAH and its 512 roots equal those of its source (4 distinct ODSs, as the bench
    replicates them), a sampled square's whole EDS is bit-exact, and every status is 0."""
    import ctypes
    from celestia_eds import _lib
    from hipmem import DeviceBuffer, Stream, synchronize
    k, n, w = 128, 256, 256
    distinct = [random_ods(k, 9100 + i) for i in range(4)]
    expect = [oracle.extend_and_commit(d) for d in distinct]
    host = np.stack([distinct[i % 4] for i in range(n)])

    class Batch:
        def __init__(self, shift):
            self.s = Stream()
            self.eds = DeviceBuffer(n * w * w * 512)
            self.rr, self.cr = DeviceBuffer(n * w * 90), DeviceBuffer(n * w * 90)
            self.dah, self.st = DeviceBuffer(n * 32), DeviceBuffer(n * 4, fill=0x7F)
            self.work = DeviceBuffer(ctx.lib.cel_dev_workspace_size(k, n))
            self.src = host if shift == 0 else np.ascontiguousarray(np.roll(host, shift, axis=0))
            self.shift = shift
            ctx.check(ctx.lib.cel_dev_place_ods(ctx.handle, self.src.ctypes.data_as(ctypes.c_void_p), n, k,
                                                self.eds.ptr, self.s.ptr))

        def step(self):
            ctx.check(ctx.lib.cel_dev_extend_batch(ctx.handle, None, n, k, self.eds.ptr, self.rr.ptr, self.cr.ptr,
                                                   self.dah.ptr, self.st.ptr, self.work.ptr, self.s.ptr,
                                                   _lib.FLAG_ORDER_CHECK | _lib.FLAG_CALLER_STREAM))

    a, b = Batch(0), Batch(1)
    for _ in range(2):
        a.step()
        b.step()
    synchronize()
    for bt in (a, b):
        dah, st = bt.dah.download((n, 32)), bt.st.download((n,), np.int32)
        rr, cr = bt.rr.download((n, w, 90)), bt.cr.download((n, w, 90))
        assert (st == 0).all()
        for i in range(n):
            e = expect[(i - bt.shift) % 4]
            assert dah[i].tobytes() == e[3], f"square {i}: DAH differs"
            assert np.array_equal(rr[i], e[1]) and np.array_equal(cr[i], e[2]), f"square {i}: roots differ"
        for sq in (0, 137, n - 1):
            eds = bt.eds.download_at(sq * w * w * 512, (w, w, 512))
            assert np.array_equal(eds, expect[(sq - bt.shift) % 4][0]), f"square {sq}: EDS differs"


@pytest.mark.parametrize("seed,n_normal,n_blob", [(31, 3, 0), (32, 30, 8), (33, 120, 40), (34, 0, 90), (35, 400, 5)])
def test_prepare_process_consistency(ctx, oracle, seed, n_normal, n_blob):
    """app/test/fuzz_abci_test.go:26-160 in spirit (PrepareProposal's data root must be what
    ProcessProposal recomputes, across square sizes): random blocks of normal and blob txs
    -> the product's square.Construct -> device ExtendShares + DAH, against an independent
    path: the oracle's square layout (oracle/square_layout.py) -> the oracle's extension
    and DAH. Both the square and the data root must agree."""
    import square_layout
    from celestia_eds import da, square
    from square_inputs import random_block
    txs = random_block(seed, n_normal, n_blob)
    ods = square.Construct(txs)
    k_o, shares_o = square_layout.build_square(txs)
    assert np.array_equal(ods, np.frombuffer(b"".join(shares_o), np.uint8).reshape(-1, 512))
    k = int(round(len(ods) ** 0.5))
    assert k == k_o
    dah = da.ComputeDataAvailabilityHeader(list(ods))
    _, _, _, d = oracle.extend_and_commit(np.ascontiguousarray(ods).reshape(k, k, 512))
    assert dah.Hash() == d
