"""GPU parity of the rsmt2d.Codec surface (Leopard encode/decode) against the oracle."""
import hashlib

import numpy as np
import pytest

from eds_inputs import model_shards

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("k", [1, 2, 32, 128, 256, 512])
def test_model_digest(ctx, golden, k):
    from celestia_eds.rsmt2d import LeoRSCodec
    codec = LeoRSCodec(ctx)
    data = model_shards(k)
    par = codec.Encode([d.tobytes() for d in data])
    got = b"".join(par)
    if k == 1:
        # one data shard: the Leopard transform is empty and the parity equals the data
        # (SURVEY.md A.2 "k=1 reduces to parity=data")
        assert got == data.tobytes()
    else:
        assert hashlib.sha256(got).hexdigest() == golden["leopard_model"][str(k)]["parity_sha256"]


@pytest.mark.parametrize("n,ln", [(1, 64), (4, 64), (8, 192), (64, 512), (128, 512), (256, 128), (256, 512), (512, 512),
                                  (512, 1024), (1024, 64), (2048, 64)])
def test_encode_matches_oracle(ctx, oracle, n, ln):
    from celestia_eds.rsmt2d import LeoRSCodec
    rng = np.random.default_rng(n * 7 + ln)
    data = rng.integers(0, 256, (n, ln), dtype=np.uint8)
    par = LeoRSCodec(ctx).Encode([d.tobytes() for d in data])
    assert np.array_equal(np.frombuffer(b"".join(par), np.uint8).reshape(n, ln), oracle.rs_encode(data))


@pytest.mark.parametrize("n", [1, 2, 8, 64, 128, 256, 512, 1024])
def test_decode_random_erasures(ctx, oracle, n):
    from celestia_eds.rsmt2d import LeoRSCodec
    codec = LeoRSCodec(ctx)
    rng = np.random.default_rng(n)
    ln = 512 if n <= 128 else 64
    data = rng.integers(0, 256, (n, ln), dtype=np.uint8)
    cw = np.concatenate([data, oracle.rs_encode(data)])
    for trial in range(3):
        lost = set(rng.choice(2 * n, n, replace=False).tolist()) if trial else set(range(n))
        shards = [None if i in lost else cw[i].tobytes() for i in range(2 * n)]
        out = codec.Decode(shards)
        assert np.array_equal(np.frombuffer(b"".join(out), np.uint8).reshape(2 * n, ln), cw)


@pytest.mark.parametrize("n,ln", [(16, 64), (128, 64), (128, 192), (64, 320)])
def test_decode_chunk_tails(ctx, oracle, n, ln):
    """GF(2^8) decode works on 128-byte chunks; shard sizes that end in a 64-byte half
    chunk (zero-padded columns) decode like any other."""
    from celestia_eds.rsmt2d import LeoRSCodec
    codec = LeoRSCodec(ctx)
    rng = np.random.default_rng(1000 + n + ln)
    data = rng.integers(0, 256, (n, ln), dtype=np.uint8)
    cw = np.concatenate([data, oracle.rs_encode(data)])
    lost = set(rng.choice(2 * n, n, replace=False).tolist())
    out = codec.Decode([None if i in lost else cw[i].tobytes() for i in range(2 * n)])
    assert np.array_equal(np.frombuffer(b"".join(out), np.uint8).reshape(2 * n, ln), cw)


def test_decode_too_few(ctx):
    from celestia_eds import CelError, _lib
    from celestia_eds.rsmt2d import LeoRSCodec
    shards = [bytes(64)] * 3 + [None] * 5
    with pytest.raises(CelError) as ei:
        LeoRSCodec(ctx).Decode(shards)
    assert ei.value.status == _lib.ETOOFEW


def test_device_limits(ctx):
    """The device codec's shard-count limits fail loudly with exactly ETOOBIG, the status
    the Go shim keys its fallback to the reference LeoRSCodec on:
    encode takes n <= 2048 data shards (the LDS image), decode n <= 1024; a square wider
    than k = 512 is ETOOBIG too (ExtendSquare's fallback to rsmt2d). Zero-length shards
    are klauspost's ErrShardNoData ("no shard data")."""
    from celestia_eds import CelError, _lib
    from celestia_eds.rsmt2d import LeoRSCodec
    codec = LeoRSCodec(ctx)
    with pytest.raises(CelError) as ei:
        codec.Encode([bytes(64)] * 4096)
    assert ei.value.status == _lib.ETOOBIG
    with pytest.raises(CelError) as ei:
        codec.Decode([bytes(64)] * 2048 + [None] * 2048)
    assert ei.value.status == _lib.ETOOBIG
    with pytest.raises(CelError) as ei:
        codec.Encode([b""] * 4)
    assert ei.value.status == _lib.ENODATA and "no shard data" in str(ei.value)
    with pytest.raises(CelError) as ei:
        codec.Decode([b""] * 4 + [None] * 4)
    assert ei.value.status == _lib.ENODATA
    import ctypes
    k = 1024  # status only: the size check precedes any copy (small stand-in buffers)
    z = np.zeros(64, np.uint8).ctypes.data_as(ctypes.c_void_p)
    st = ctx.lib.cel_extend_shares(ctx.handle, z, k * k, 512, None, z, z, z, 0)
    assert st == _lib.ETOOBIG


@pytest.mark.parametrize("n", [256, 512, 1024])
def test_dev_decode_gf16_axes(ctx, oracle, n):
    """cel_dev_decode over many GF(2^16) axes at once (the bit-plane decoder, 2n = 512..2048
    points, 512-byte shards = 8 chunks per axis), each axis with its own erasure pattern:
    one cell lost, exactly n lost, all data lost, all parity lost, and random counts in
    between, so the present/erased point order of every workgroup takes every shape."""
    import ctypes
    from hipmem import DeviceBuffer, synchronize
    from celestia_eds import _lib
    rng = np.random.default_rng(7 * n)
    ln = 512 if n <= 512 else 128
    naxes = 6 if n <= 512 else 3
    cws, masks = [], []
    for a in range(naxes):
        data = rng.integers(0, 256, (n, ln), dtype=np.uint8)
        cws.append(np.concatenate([data, oracle.rs_encode(data)]))
        present = np.ones(2 * n, np.uint8)
        kind = a % 6
        if kind == 0:
            present[rng.integers(0, 2 * n)] = 0
        elif kind == 1:
            present[rng.choice(2 * n, n, replace=False)] = 0
        elif kind == 2:
            present[:n] = 0
        elif kind == 3:
            present[n:] = 0
        else:
            present[rng.choice(2 * n, int(rng.integers(1, n + 1)), replace=False)] = 0
        masks.append(present)
    cw = np.stack(cws)
    pres = np.stack(masks)
    buf = np.where(pres[..., None] == 1, cw, rng.integers(0, 256, cw.shape, dtype=np.uint8)).astype(np.uint8)
    d, dp = DeviceBuffer(buf.nbytes), DeviceBuffer(pres.nbytes)
    d.upload(np.ascontiguousarray(buf))
    dp.upload(np.ascontiguousarray(pres))
    assert ctx.lib.cel_dev_decode(ctx.handle, d.ptr, dp.ptr, naxes, n, ln, None) == _lib.OK
    synchronize()
    out = d.download(buf.shape)
    for a in range(naxes):
        assert np.array_equal(out[a], cw[a]), (n, a)
