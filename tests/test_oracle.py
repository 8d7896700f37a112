"""CPU: pin the oracle against the reference's own known answers before trusting it.

- DAH known answers: pkg/da/data_availability_header_test.go:15-68
- mainnet block 408 data root: x/blob/test/testdata/block_response.json (GF(2^8) pin)
- Leopard table debug values and model digests: SURVEY.md Appendix A.2, A.3, A.5
- Leopard = Lagrange RS over Cantor-basis points (tests/lagrange_rs.py): pinned on block
  408 at GF(2^8), then equal to the oracle at k=128 and in GF(2^16) (k=256/512)
- scalar vs SIMD oracle paths, decode round trips, repair semantics
"""
import hashlib

import numpy as np
import pytest

from eds_inputs import constant_ods, model_shards, random_ods, tail_padding_share


def test_gf8_debug_values(oracle):
    l = oracle.lib()
    assert [l.orc_gf_exp(8, i) for i in range(8)] == [1, 104, 92, 100, 114, 240, 86, 18]
    assert [l.orc_gf_log(8, i) for i in range(8)] == [255, 0, 85, 170, 17, 68, 34, 136]
    assert [l.orc_gf_skew(8, i) for i in range(16)] == [255, 255, 85, 255, 17, 85, 34, 255, 153, 17, 102, 85,
                                                        51, 34, 187, 255]
    assert [l.orc_gf_skew(8, i) for i in range(127, 135)] == [255, 160, 241, 29, 196, 167, 254, 144]
    assert l.orc_gf_mul(8, 2, 3) == 1 and l.orc_gf_mul(8, 0x53, 0xCA) == 2


def test_gf16_debug_values(oracle):
    l = oracle.lib()
    assert [l.orc_gf_exp(16, i) for i in range(8)] == [1, 18064, 26072, 25296, 22324, 17904, 21432, 7736]
    assert [l.orc_gf_log(16, i) for i in range(8)] == [65535, 0, 21845, 43690, 17476, 4369, 34952, 8738]
    assert [l.orc_gf_skew(16, i) for i in range(8)] == [65535, 65535, 21845, 65535, 17476, 21845, 34952, 65535]


@pytest.mark.parametrize("k", [2, 32, 128, 256, 512])
def test_leopard_model_digest(oracle, golden, k):
    exp = golden["leopard_model"][str(k)]
    for simd in (False, True):
        oracle.set_simd(simd)
        p = oracle.rs_encode(model_shards(k))
        assert hashlib.sha256(p.tobytes()).hexdigest() == exp["parity_sha256"]
        assert p[0, :8].tobytes().hex() == exp["parity0_head"]
    oracle.set_simd(True)


def test_sha256_paths(oracle):
    rng = np.random.default_rng(0)
    for n in [0, 1, 55, 56, 63, 64, 65, 181, 542, 1000]:
        m = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        for simd in (False, True):
            oracle.set_simd(simd)
            assert oracle.sha256(m) == hashlib.sha256(m).digest()
    oracle.set_simd(True)


def test_dah_empty(oracle, golden):
    z = np.zeros((0, 90), np.uint8)
    assert oracle.dah_hash(z, z).hex() == golden["dah_known_answers"]["empty"]


def test_dah_min(oracle, golden):
    ods = np.frombuffer(tail_padding_share(), np.uint8).reshape(1, 1, 512)
    assert oracle.extend_and_commit(ods)[3].hex() == golden["dah_known_answers"]["min"]


@pytest.mark.parametrize("k,key", [(2, "typical_k2"), (128, "max_k128")])
def test_dah_typical_and_max(oracle, golden, k, key):
    _, _, _, dah = oracle.extend_and_commit(constant_ods(k), want_eds=False)
    assert dah.hex() == golden["dah_known_answers"][key]


def test_block408_data_root(oracle, golden, block408_ods):
    g = golden["block408"]
    assert hashlib.sha256(block408_ods.tobytes()).hexdigest() == g["ods_sha256"]
    eds, rr, cr, dah = oracle.extend_and_commit(block408_ods)
    assert dah.hex() == g["data_hash"]
    assert hashlib.sha256(eds.tobytes()).hexdigest() == g["eds_sha256"]
    assert rr[0].tobytes().hex() == g["row_root_0"] and cr[0].tobytes().hex() == g["col_root_0"]
    assert rr[-1].tobytes().hex() == g["row_root_last"] and cr[-1].tobytes().hex() == g["col_root_last"]


def test_lagrange_rs_is_block408_code(oracle, golden, block408_ods):
    """Leopard GF(2^8) = Lagrange RS over Cantor points (tests/lagrange_rs.py), on mainnet
    block 408: Q1 of rows 0, 17 and Q2 of column 5 of the EDS whose sha256 the golden
    fixture pins, at three byte positions each."""
    import lagrange_rs as L
    eds = oracle.extend(block408_ods)
    assert hashlib.sha256(eds.tobytes()).hexdigest() == golden["block408"]["eds_sha256"]
    f, k = L.Field(8, L.POLY8, L.CANTOR8), 32
    for axis in (eds[0], eds[17], eds[:, 5]):
        for b in (0, 200, 511):
            assert L.encode(f, [int(v) for v in axis[:k, b]]) == [int(v) for v in axis[k:, b]]


@pytest.mark.parametrize("m", [256, 512])
def test_lagrange_rs_equals_gf16_oracle(oracle, m):
    """GF(2^16), where the reference holds no vector: the oracle's FFT encoder equals the
    same Lagrange statement (pinned at GF(2^8) above) with klauspost's GF(2^16) POLY and
    Cantor basis; symbols are sym[j] = b[j] | b[j + 32] << 8 per 64-byte block."""
    import lagrange_rs as L
    f = L.Field(16, L.POLY16, L.CANTOR16)
    for i in range(1, 16):  # the basis satisfies beta_i^2 + beta_i = beta_{i-1}
        bi = L.CANTOR16[i]
        assert f.mul(bi, bi) ^ bi == L.CANTOR16[i - 1]
    data = np.random.default_rng(m).integers(0, 256, (m, 128), np.uint8)
    par = oracle.rs_encode(data)
    for blk, j in ((0, 0), (0, 31), (1, 9)):
        sym = lambda a: [int(a[i, 64 * blk + j]) | int(a[i, 64 * blk + 32 + j]) << 8 for i in range(m)]
        assert L.encode(f, sym(data)) == sym(par)


def test_lagrange_rs_equals_gf8_oracle_k128(oracle):
    """The k=128 code (256 shards, the last GF(2^8) width; block 408 is k=32)."""
    import lagrange_rs as L
    f, m = L.Field(8, L.POLY8, L.CANTOR8), 128
    data = np.random.default_rng(128).integers(0, 256, (m, 64), np.uint8)
    par = oracle.rs_encode(data)
    for j in (0, 33, 63):
        assert L.encode(f, [int(v) for v in data[:, j]]) == [int(v) for v in par[:, j]]


def test_q3_both_ways(oracle):
    """specs/src/specs/data_structures.md:305: Q3 is the same extended from Q1 or Q2."""
    k = 8
    eds = oracle.extend(random_ods(k, 3))
    q3_cols = np.stack([oracle.rs_encode(np.ascontiguousarray(eds[:k, k + c])) for c in range(k)], axis=1)
    assert np.array_equal(q3_cols, eds[k:, k:])


@pytest.mark.parametrize("n", [1, 2, 4, 16, 64, 128, 256])
def test_decode_round_trip(oracle, n):
    rng = np.random.default_rng(n)
    ln = 64 if n >= 128 else 128
    data = rng.integers(0, 256, (n, ln), dtype=np.uint8)
    cw = np.concatenate([data, oracle.rs_encode(data)])
    for trial in range(3):
        present = np.ones(2 * n, np.uint8)
        lost = rng.choice(2 * n, n, replace=False) if trial else np.arange(n)
        present[lost] = 0
        sh = cw.copy()
        sh[present == 0] = 0
        assert np.array_equal(oracle.rs_decode(sh, present), cw)


def _leopard_decode_py(oracle, shards, present):
    """Pure-Python catid/leopard erasure decoder over GF(2^8) (klauspost leopard8.go
    reconstruct with recoverAll), with the error locator as the direct sum
    err[i] = sum_{e erased} log(i ^ e) instead of the oracle's FWHTs, and radix-2 layers
    instead of its loops: an independent statement of the same formula."""
    lib = oracle.lib()
    exp = [lib.orc_gf_exp(8, i) for i in range(256)]
    log = [lib.orc_gf_log(8, i) for i in range(256)]
    skew = [lib.orc_gf_skew(8, i) for i in range(255)]
    mod = 255

    def mul(a, lm):  # mulLog with klauspost's partial reduction
        if a == 0:
            return 0
        s = log[a] + lm
        return exp[(s + (s >> 8)) & mod]

    n2, ln = shards.shape
    n = n2 // 2
    er = [p for p in range(n2) if not present[p ^ n]]
    err = [sum(log[i ^ e] % mod for e in er) % mod for i in range(n2)]
    w = [[mul(int(b), err[p]) for b in shards[p ^ n]] if present[p ^ n] else [0] * ln for p in range(n2)]
    d = 1
    while d < n2:
        for b in range(0, n2, 2 * d):
            lm = skew[b + d - 1]
            for j in range(d):
                x, y = w[b + j], w[b + d + j]
                y = [a ^ c for a, c in zip(y, x)]
                if lm != mod:
                    x = [a ^ mul(c, lm) for a, c in zip(x, y)]
                w[b + j], w[b + d + j] = x, y
        d *= 2
    old = [row[:] for row in w]
    for x in range(n2):
        t = 1
        while t < n2:
            if not x & t and x + t < n2:
                w[x] = [a ^ c for a, c in zip(w[x], old[x + t])]
            t *= 2
    d = n2 // 2
    while d >= 1:
        for b in range(0, n2, 2 * d):
            lm = skew[b + d - 1]
            for j in range(d):
                x, y = w[b + j], w[b + d + j]
                if lm != mod:
                    x = [a ^ mul(c, lm) for a, c in zip(x, y)]
                y = [a ^ c for a, c in zip(y, x)]
                w[b + j], w[b + d + j] = x, y
        d //= 2
    out = shards.copy()
    for p in er:
        out[p ^ n] = [mul(v, (mod - err[p]) % mod) for v in w[p]]
    return out


@pytest.mark.parametrize("n", [1, 2, 4, 8, 16])
def test_decode_formula_on_inconsistent_shards(oracle, n):
    """The oracle's decoder is Leopard's formula (not any decoder of the code): on shards
    that are not a codeword it equals an independent pure-Python statement of the
    formula, and differs from the codeword a subset decode would give."""
    rng = np.random.default_rng(40 + n)
    data = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    cw = np.concatenate([data, oracle.rs_encode(data)])
    for simd in (False, True):
        oracle.set_simd(simd)
        for trial in range(3):
            present = np.ones(2 * n, np.uint8)
            present[rng.choice(2 * n, max(1, n // 2), replace=False)] = 0
            bad = cw.copy()
            j = rng.choice(np.flatnonzero(present))
            bad[j, rng.integers(0, 16)] ^= 0x81
            bad[present == 0] = 0
            got = oracle.rs_decode(bad, present)
            assert np.array_equal(got, _leopard_decode_py(oracle, bad, present))
            good = cw.copy()
            good[present == 0] = 0
            assert np.array_equal(oracle.rs_decode(good, present), cw)
    oracle.set_simd(False)


def test_decode_too_few(oracle):
    n = 4
    sh = np.zeros((2 * n, 64), np.uint8)
    present = np.zeros(2 * n, np.uint8)
    present[: n - 1] = 1
    with pytest.raises(ValueError):
        oracle.rs_decode(sh, present)


def test_repair_semantics(oracle):
    k = 4
    eds, rr, cr, _ = oracle.extend_and_commit(random_ods(k, 11))
    w = 2 * k
    # Q0 only (exactly 25%): always repairable
    present = np.zeros((w, w), np.uint8)
    present[:k, :k] = 1
    damaged = eds.copy()
    damaged[present == 0] = 0
    rc, fixed, _, _ = oracle.repair(damaged, present, rr, cr)
    assert rc == oracle.OK and np.array_equal(fixed, eds)
    # too few cells: unrepairable
    present = np.zeros((w, w), np.uint8)
    present[0, :k - 1] = 1
    rc, _, _, _ = oracle.repair(damaged, present, rr, cr)
    assert rc == oracle.EUNREPAIRABLE
    # one corrupted cell of a complete row: rsmt2d's "bad root input" (a plain error)
    present = np.ones((w, w), np.uint8)
    present[1, 1] = 0
    bad = eds.copy()
    bad[0, 0, 100] ^= 1
    rc, _, _, (ba, bi) = oracle.repair(bad, present, rr, cr)
    assert rc == oracle.EBADROOT and (ba, bi) == (0, 0)
    # the corrupted cell inside an incomplete row: the decoded row fails -> byzantine,
    # Shares = that row before the solve
    present[0, 3] = 0
    present[5, 0] = 0  # column 0 incomplete as well
    rc, _, pres, (ba, bi), (bs, bp) = oracle.repair(bad, present, rr, cr, want_shares=True)
    assert rc == oracle.EBYZANTINE and (ba, bi) == (0, 0)
    assert np.array_equal(bp, present[0]) and np.array_equal(bs[0], bad[0, 0])
    assert np.array_equal(pres, present)  # nothing solved before row 0


def test_repair_sanity_encoding_check(oracle):
    """rsmt2d preRepairSanityCheck re-encodes complete axes: a square whose row 3 is not a
    codeword, with roots computed over it, is ErrByzantineData(Row, 3)."""
    k = 8
    w = 2 * k
    eds, _, _, _ = oracle.extend_and_commit(random_ods(k, 12))
    eds[3, k + 2, 50] ^= 0x80
    _, rr, cr = oracle.roots(eds, check_order=False)
    rc, _, _, bad, (bs, bp) = oracle.repair(eds, np.ones((w, w), np.uint8), rr, cr, want_shares=True)
    assert rc == oracle.EBYZANTINE and bad == (0, 3) and bp.all() and np.array_equal(bs, eds[3])


def test_repair_orthogonal_completion(oracle):
    """The orthogonal axis a solve completes is checked at once (root and encoding), so a
    square that is stuck afterwards still reports ErrByzantineData for that column."""
    k = 8
    w = 2 * k
    r0, r1, c = 1, 6, 4
    eds, _, _, _ = oracle.extend_and_commit(random_ods(k, 13))
    eds[r1, c, 100] ^= 0x04
    _, rr, cr = oracle.roots(eds, check_order=False)
    present = np.zeros((w, w), np.uint8)
    present[:, c] = 1
    present[r0, :] = 0
    present[r0, k:] = 1
    rc, _, pres, bad, (bs, bp) = oracle.repair(eds, present, rr, cr, want_shares=True)
    assert rc == oracle.EBYZANTINE and bad == (1, c) and bp.all() and np.array_equal(bs, eds[:, c])
    assert np.array_equal(pres, present)  # the mask before row r0's solve
    # without the corruption the same mask is simply unrepairable
    eds2, rr2, cr2, _ = oracle.extend_and_commit(random_ods(k, 13))
    rc, _, _, _ = oracle.repair(eds2, present, rr2, cr2)
    assert rc == oracle.EUNREPAIRABLE


def test_nmt_empty_root(oracle):
    rc, r = oracle.nmt_root([])
    assert rc == 0 and r == bytes(58) + hashlib.sha256(b"").digest()


def test_nmt_order_check(oracle):
    a = b"\x00" * 28 + b"\x02" + b"x" * 10
    b_ = b"\x00" * 28 + b"\x01" + b"y" * 10
    assert oracle.nmt_root([a, b_])[0] == oracle.EORDER
    assert oracle.nmt_root([b_, a])[0] == 0


def test_roots_order_violation(oracle):
    k = 4
    ods = random_ods(k, 5)
    ods[0, 0], ods[0, 1] = ods[0, 1].copy(), ods[0, 0].copy()
    eds = oracle.extend(ods)
    rc, _, _ = oracle.roots(eds, check_order=True)
    assert rc == oracle.EORDER


def test_cpu_baseline_entry_points_match_checker(oracle):
    """bench.py's CPU baseline (independent squares / repairs per thread, SIMD block
    functions) gives the checker's DAHs and repair outcomes bit for bit, SHA-NI and GFNI
    paths against the scalar ones."""
    k = 16
    ods = np.stack([random_ods(k, s) for s in range(5)])
    oracle.set_simd(False)
    ref = [oracle.extend_and_commit(o, want_eds=False)[3] for o in ods]
    oracle.set_simd(True)
    oracle.set_threads(3)
    got = oracle.extend_commit_many(ods)
    assert [g.tobytes() for g in got] == ref
    eds, rr, cr, _ = oracle.extend_and_commit(ods[0])
    w = 2 * k
    present = (np.random.default_rng(3).random((w, w)) < 0.6).astype(np.uint8)
    damaged = np.where(present[..., None] == 1, eds, 0).astype(np.uint8)
    st = oracle.repair_many(damaged, present, rr, cr, 4)
    assert (st == oracle.repair(damaged, present, rr, cr)[0]).all()
    oracle.set_simd(False)
