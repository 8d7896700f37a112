"""Property-based GPU parity (hypothesis), beside the fixed-seed tests of test_gpu_square.py:

- namespace layouts the reference's squares can hold: runs of one namespace, reserved
  namespaces before the blobs, tail padding (0xFF*28 || 0xFE, namespace.md:83) and the parity
  namespace (0xFF*29) at the end of Q0 (shares sorted row-major, as Square.Build lays them
  out); EDS bytes, 4k roots and DAH against the oracle;
- the extension is GF(2^8)- / GF(2^16)-linear, so at the benchmark's full widths (k = 128
  and 512, where the oracle takes seconds per square) EDS(a ^ b) == EDS(a) ^ EDS(b) for random
  squares, through the device batch entry point (cel_dev_extend_only).
"""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

pytestmark = pytest.mark.gpu

SHARE, NS = 512, 29
PARITY_NS = b"\xff" * NS
TAIL_NS = b"\xff" * 28 + b"\xfe"


def layout_ods(k, seed, n_ns, reserved, tail, parity):
    """k*k shares: `reserved` shares in reserved namespaces 0x00 || 0*27 || i, then blobs over
    n_ns random v0 namespaces, then `tail` tail-padding and `parity` parity-namespace shares
    (capped so at least one blob share remains), sorted row-major by namespace."""
    rng = np.random.default_rng(seed)
    n = k * k
    tail = min(tail, n - 1)
    parity = min(parity, n - 1 - tail)
    reserved = min(reserved, n - 1 - tail - parity)
    nblob = n - tail - parity - reserved
    pool = [b"\x00" + bytes(18) + rng.integers(0, 256, 10, dtype=np.uint8).tobytes() for _ in range(n_ns)]
    pool = [p if p[19:] != bytes(10) else p[:28] + b"\x01" for p in pool]
    nss = [b"\x00" + bytes(27) + bytes([1 + (i % 250)]) for i in range(reserved)]
    nss += [pool[int(rng.integers(0, n_ns))] for _ in range(nblob)]
    nss += [TAIL_NS] * tail + [PARITY_NS] * parity
    nss.sort()
    ods = rng.integers(0, 256, (n, SHARE), dtype=np.uint8)
    for i, ns in enumerate(nss):
        ods[i, :NS] = np.frombuffer(ns, np.uint8)
    return ods.reshape(k, k, SHARE)


@settings(max_examples=30, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(lk=st.integers(0, 6), seed=st.integers(0, 2**31), n_ns=st.integers(1, 40), reserved=st.integers(0, 5),
       tail=st.integers(0, 40), parity=st.integers(0, 8))
def test_namespace_layouts(ctx, oracle, lk, seed, n_ns, reserved, tail, parity):
    from celestia_eds import da
    k = 1 << lk
    ods = layout_ods(k, seed, n_ns, reserved, tail, parity)
    dev = da._extend(np.ascontiguousarray(ods).reshape(-1, SHARE), ctx=ctx)
    eds, rr, cr, dah = oracle.extend_and_commit(ods)
    assert np.array_equal(dev.cells, eds), "EDS bytes differ"
    assert np.array_equal(dev._row_roots, rr) and np.array_equal(dev._col_roots, cr), "roots differ"
    assert dev._dah == dah


def _extend_resident(ctx, k, odss):
    """cel_dev_place_ods + cel_dev_extend_only over device buffers of the library's own HIP
    runtime (tests/hipmem.py), the bench's in-place layout; the EDSs back on the host."""
    import ctypes
    from hipmem import DeviceBuffer, synchronize
    odss = np.ascontiguousarray(np.stack(odss))
    n, w = len(odss), 2 * k
    d_eds = DeviceBuffer(n * w * w * SHARE, fill=0xA5)
    ctx.check(ctx.lib.cel_dev_place_ods(ctx.handle, odss.ctypes.data_as(ctypes.c_void_p), n, k, d_eds.ptr, None))
    ctx.check(ctx.lib.cel_dev_extend_only(ctx.handle, None, n, k, d_eds.ptr, None))
    synchronize()
    out = d_eds.download((n, w, w, SHARE))
    d_eds.free()
    return out


@settings(max_examples=4, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(seed=st.integers(0, 2**31))
@pytest.mark.parametrize("k", [128, 512])
def test_extension_linear_full_width(ctx, k, seed):
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 256, (k, k, SHARE), dtype=np.uint8)
    b = rng.integers(0, 256, (k, k, SHARE), dtype=np.uint8)
    ea, eb, ex = _extend_resident(ctx, k, [a, b, a ^ b])
    assert np.array_equal(ex, ea ^ eb), "EDS(a ^ b) != EDS(a) ^ EDS(b)"
    assert np.array_equal(ea[:k, :k], a), "Q0 is not the input"
