"""GPU parity of the multi-GPU entry points inside the library (include/celestia_eds.h,
"multi-GPU" section), through the C ABI:

- cel_extend_sharded / cel_shard_plan_* (config 3): one square row-sharded over the ctxs'
  devices, collectives issued by the library. On the box's one GPU: one rank with no
  collective (transport "local"), one rank on a real RCCL communicator (CEL_FLAG_SHARD_EXCHANGE:
  transport "rccl", the all-to-all through ncclSend / ncclRecv to self and the records through
  ncclAllGather), and N = 2..8 ranks as N ctxs on the same device (transport
  "copy": RCCL refuses two ranks on one device, the plan moves the same blocks with device
  copies in the same schedule). Every EDS byte, root and DAH against the whole-square oracle.
- cel_extend_batch_multi (config 4): squares split over two ctxs on device 0, one host
  thread per ctx in the library, every square against the oracle.
- cel_probe_*: the same-run ceilings bench.py reports.
"""
import numpy as np
import pytest

from celestia_eds.testfactory import random_ods

pytestmark = pytest.mark.gpu

_ORACLE = {}


def expected(oracle, k, seed):
    key = (k, seed)
    if key not in _ORACLE:
        _ORACLE[key] = oracle.extend_and_commit(random_ods(k, seed))
    return _ORACLE[key]


def assert_square(got, want, eds=True):
    g_eds, g_rr, g_cr, g_dah = got
    w_eds, w_rr, w_cr, w_dah = want
    if eds:
        assert np.array_equal(g_eds, w_eds), "EDS bytes differ"
    assert np.array_equal(g_rr, w_rr), "row roots differ"
    assert np.array_equal(g_cr, w_cr), "column roots differ"
    assert g_dah == w_dah, "DAH differs"


@pytest.fixture(scope="module")
def ctxs():
    """Eight contexts on device 0 (ctx[0] is the session's default one)."""
    from celestia_eds import Context, default_context
    cs = [default_context(0)] + [Context(0) for _ in range(7)]
    yield cs
    for c in cs[1:]:
        c.close()


@pytest.mark.parametrize("k", [256, 512])
def test_extend_sharded_one_rank(ctxs, oracle, k):
    """cel_extend_sharded at ngpu = 1: no collective is needed (transport "local": the row
    pass writes the slab in place, the finish reads the rank's own records), bit-exact
    against the oracle."""
    from celestia_eds.multi import ShardPlan, extend_sharded
    got = extend_sharded(ctxs[:1], random_ods(k, 900 + k))
    assert_square(got, expected(oracle, k, 900 + k))
    plan = ShardPlan(ctxs[:1], k)
    assert plan.transport == "local"
    plan.close()


@pytest.mark.parametrize("k", [256, 512])
def test_shard_plan_rccl_exchange(ctxs, oracle, k):
    """One rank with CEL_FLAG_SHARD_EXCHANGE, on a real one-rank RCCL communicator: the
    all-to-all is grouped ncclSend / ncclRecv (to itself) and the records go through
    ncclAllGather; two squares through the same plan."""
    from celestia_eds import _lib
    from celestia_eds.multi import ShardPlan
    plan = ShardPlan(ctxs[:1], k, _lib.FLAG_ORDER_CHECK | _lib.FLAG_SHARD_EXCHANGE)
    assert plan.transport == "rccl"
    for seed in (910, 911):
        plan.upload(random_ods(k, seed))
        plan.run()
        assert_square(plan.wait(want_eds=True), expected(oracle, k, seed))
    plan.close()


@pytest.mark.parametrize("k,n", [(256, 2), (256, 4), (256, 8), (512, 2), (512, 4), (512, 8)])
def test_shard_plan_copy_transport(ctxs, oracle, k, n):
    """N ranks as N ctxs on one device: the plan's N-rank schedule (blocked row pass,
    transpose, slab commits, record gather, finish) with device copies for the collectives;
    two squares back to back with no wait between them (cross-run buffer reuse)."""
    from celestia_eds.multi import ShardPlan
    plan = ShardPlan(ctxs[:n], k)
    assert plan.transport == "copy"
    plan.upload(random_ods(k, 920))
    plan.run()
    plan.upload(random_ods(k, 921))
    plan.run()
    assert_square(plan.wait(want_eds=True), expected(oracle, k, 921))
    plan.close()


def test_shard_plan_rccl_refused_falls_back(ctxs, oracle):
    """RCCL that cannot start leaves the plan on device copies instead of failing: two ranks
    on the box's one device with CEL_FLAG_SHARD_EXCHANGE make ncclCommInitAll refuse them
    (duplicate GPU, profiles/r3_rccl_probe.txt), the plan reports "copy-fallback" with RCCL's
    message, and the square is bit-exact (the path distinct devices take as "peer-fallback")."""
    from celestia_eds import _lib
    from celestia_eds.multi import ShardPlan
    k = 256
    plan = ShardPlan(ctxs[:2], k, _lib.FLAG_ORDER_CHECK | _lib.FLAG_SHARD_EXCHANGE)
    assert plan.transport == "copy-fallback", plan.transport
    assert "ncclCommInitAll" in plan.note or "RCCL" in plan.note, plan.note
    plan.upload(random_ods(k, 925))
    plan.run()
    assert_square(plan.wait(want_eds=True), expected(oracle, k, 925))
    assert plan.time_exchange(3) > 0
    plan.close()


@pytest.mark.parametrize("n", [2, 4])
def test_shard_plan_peercopy_flag(ctxs, oracle, n):
    """CEL_FLAG_SHARD_PEERCOPY never starts RCCL: repeated devices take the copy transport
    (distinct devices would take "peer"), no note, bit-exact; the exchange times alone."""
    from celestia_eds import _lib
    from celestia_eds.multi import ShardPlan
    k = 256
    plan = ShardPlan(ctxs[:n], k, _lib.FLAG_ORDER_CHECK | _lib.FLAG_SHARD_PEERCOPY)
    assert plan.transport == "copy" and plan.note == ""
    plan.upload(random_ods(k, 926))
    plan.run()
    assert_square(plan.wait(want_eds=True), expected(oracle, k, 926))
    assert plan.time_exchange(3) > 0
    plan.close()
    local = ShardPlan(ctxs[:1], k, _lib.FLAG_ORDER_CHECK | _lib.FLAG_SHARD_PEERCOPY)
    assert local.transport == "local" and local.time_exchange() is None
    local.close()


def test_shard_plans_in_flight(ctxs, oracle):
    """Two plans (own streams and communicators) with squares in flight at once."""
    from celestia_eds.multi import ShardPlan
    k = 256
    plans = [ShardPlan(ctxs[:1], k), ShardPlan(ctxs[1:3], k)]
    for i, p in enumerate(plans):
        p.upload(random_ods(k, 930 + i))
    for p in plans:
        p.run()
    for i, p in enumerate(plans):
        assert_square(p.wait(), expected(oracle, k, 930 + i), eds=False)
        p.close()


def test_extend_sharded_parity_only_and_cache(ctxs, oracle):
    """CEL_FLAG_PARITY_ONLY leaves Q0 of eds_out unwritten; the cached plan is rebuilt when
    the device list changes (1 rank -> 4 ranks -> 1 rank) and every result stays exact."""
    from celestia_eds import _lib
    from celestia_eds.multi import extend_sharded
    k = 256
    want = expected(oracle, k, 940)
    for group in (ctxs[:1], ctxs[:4], ctxs[:1]):
        eds, rr, cr, dah = extend_sharded(group, random_ods(k, 940),
                                          flags=_lib.FLAG_ORDER_CHECK | _lib.FLAG_PARITY_ONLY)
        assert not eds[:k, :k].any(), "Q0 written under CEL_FLAG_PARITY_ONLY"
        mask = np.ones((2 * k, 2 * k), bool)
        mask[:k, :k] = False
        assert np.array_equal(eds[mask], want[0][mask])
        assert_square((None, rr, cr, dah), want, eds=False)


@pytest.mark.parametrize("n", [1, 4])
def test_extend_sharded_order_error(ctxs, n):
    """Shares out of namespace order (two cells of one row swapped across rank slabs): the
    push-order check fails with the reference's error, and the next square is fine again."""
    from celestia_eds import CelError, _lib
    from celestia_eds.multi import extend_sharded
    k = 256
    ods = random_ods(k, 950).copy()
    ods[3, 0], ods[3, k - 1] = ods[3, k - 1].copy(), ods[3, 0].copy()
    with pytest.raises(CelError) as e:
        extend_sharded(ctxs[:n], ods, want_eds=False)
    assert e.value.status == _lib.EORDER
    extend_sharded(ctxs[:n], random_ods(k, 951), want_eds=False)


def test_extend_sharded_rejects(ctxs):
    from celestia_eds import CelError, _lib
    from celestia_eds.multi import ShardPlan
    with pytest.raises(CelError) as e:
        ShardPlan(ctxs[:1], 128)
    assert e.value.status == _lib.EINVAL and "k = 256 or 512" in str(e.value)
    with pytest.raises(CelError) as e:
        ShardPlan(ctxs[:3], 256)
    assert e.value.status == _lib.EINVAL


@pytest.mark.parametrize("k,n,g", [(64, 5, 2), (128, 3, 2), (32, 8, 2), (32, 13, 4), (64, 3, 8)])
def test_extend_batch_multi_two_ctxs(ctxs, oracle, k, n, g):
    """cel_extend_batch_multi over g ctxs on device 0 (one host thread each): every square
    of an uneven split equals the oracle, including more ctxs than squares (g = 8, n = 3)."""
    from celestia_eds.multi import extend_batch_multi
    ods = np.stack([random_ods(k, 960 + i) for i in range(n)])
    eds, rr, cr, dah, st = extend_batch_multi(ctxs[:g], ods)
    assert (st == 0).all()
    for i in range(n):
        w_eds, w_rr, w_cr, w_dah = oracle.extend_and_commit(ods[i])
        assert np.array_equal(eds[i], w_eds) and np.array_equal(rr[i], w_rr) and np.array_equal(cr[i], w_cr)
        assert dah[i].tobytes() == w_dah


@pytest.mark.parametrize("k,n,g", [(64, 5, 4), (128, 3, 2), (32, 6, 4)])
def test_extend_batch_multi_pinned_ods(ctxs, oracle, k, n, g):
    """cel_extend_batch_multi over an ODS batch in page-locked memory (cel_host_alloc, as
    the Go shim stages it): the parts that get one square take api.cpp's one-square path
    (the GF(2^8) row pass reading the mapped host pages), the others the batch upload.
    Every square against the oracle."""
    import ctypes
    from celestia_eds.multi import extend_batch_multi
    c0 = ctxs[0]
    nbytes = n * k * k * 512
    p = c0.lib.cel_host_alloc(nbytes)
    assert p, "cel_host_alloc failed"
    try:
        ods = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p)).reshape(n, k, k, 512)
        ods[...] = np.stack([random_ods(k, 980 + i) for i in range(n)])
        eds, rr, cr, dah, st = extend_batch_multi(ctxs[:g], ods)
        assert (st == 0).all()
        for i in range(n):
            w_eds, w_rr, w_cr, w_dah = oracle.extend_and_commit(np.array(ods[i]))
            assert np.array_equal(eds[i], w_eds) and np.array_equal(rr[i], w_rr) and np.array_equal(cr[i], w_cr)
            assert dah[i].tobytes() == w_dah
    finally:
        c0.lib.cel_host_free(p)


def test_extend_batch_multi_status(ctxs):
    """A bad square in the second ctx's range: its status is CEL_EORDER, the others 0, and the
    call returns CEL_EORDER with the reference's message."""
    from celestia_eds import CelError, _lib
    from celestia_eds.multi import extend_batch_multi
    k, n = 32, 4
    ods = np.stack([random_ods(k, 970 + i) for i in range(n)])
    ods[3, 1, 0], ods[3, 1, 5] = ods[3, 1, 5].copy(), ods[3, 1, 0].copy()
    with pytest.raises(CelError) as e:
        extend_batch_multi(ctxs[:2], ods, want_eds=False)
    assert e.value.status == _lib.EORDER and "push order" in str(e.value)


def test_probes(ctx):
    """The same-run ceilings: SHA-256 in registers near the measured 29.4 G/s class, a shader
    clock in the MI355X's range, a streaming copy below the 8 TB/s spec."""
    from celestia_eds.multi import probe
    p = probe(ctx, 1 << 30)
    print(p)
    assert 10 < p["sha256_gcomp_per_s"] < 60
    assert 800 < p["shader_mhz"] < 3000
    assert 1000 < p["hbm_copy_gbps"] < 8000
    # round 6: the read-only and write-only streams (writes stream slower than reads on
    # MI355X, profiles/r6_hbm_write.txt)
    assert 1000 < p["hbm_write_gbps"] < p["hbm_read_gbps"] < 8000
    # the transform alone at k = 128: round 2 measured 8.47 us per square (profiles/r2_gf8_transform_only.log)
    assert 4 < p["rs_transform_us_k128"] < 16 and p["rs_transform_us_k64"] < p["rs_transform_us_k128"]
    # GF(2^16) k = 512: round 2 measured 278.5 us per square (profiles/r2_gf16_transform_only.txt)
    assert 150 < p["rs_transform_us_k512"] < 500
