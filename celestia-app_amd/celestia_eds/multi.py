"""Multi-GPU inside the library (include/celestia_eds.h, "multi-GPU" section).

One process drives several devices through the C ABI; the collectives are RCCL calls the
library issues itself (ncclCommInitAll, grouped ncclSend / ncclRecv, ncclAllGather), so a
host that is not Python (the Go node behind da.ExtendShares, pkg/da/
data_availability_header.go:65-75) reaches configs 3 and 4 without torchrun:

  ShardPlan / extend_sharded    config 3: one square row-sharded over the ctxs' devices
  extend_batch_multi            config 4: independent squares split over the ctxs, one host
                                thread per ctx inside the library

sharded.py keeps the per-rank steps for drivers that own their processes (torchrun).
"""
import ctypes

import numpy as np

from . import _lib

_NODE = _lib.NMT_NODE_SIZE


def _handles(ctxs):
    arr = (ctypes.c_void_p * len(ctxs))(*[c.handle.value for c in ctxs])
    return arr


def _ptr(x):
    if x is None:
        return None
    if isinstance(x, np.ndarray):
        return x.ctypes.data_as(ctypes.c_void_p)
    return ctypes.c_void_p(x.data_ptr())  # a torch tensor (device memory)


class ShardPlan:
    """cel_shard_plan: buffers, streams and communicators of one square of width k
    row-sharded over len(ctxs) devices (one rank per ctx, rank order = ctxs order)."""

    def __init__(self, ctxs, k, flags=_lib.FLAG_ORDER_CHECK):
        self.ctxs, self.k, self.flags = list(ctxs), k, flags
        self.lib = self.ctxs[0].lib
        h = ctypes.c_void_p()
        st = self.lib.cel_shard_plan_create(_handles(self.ctxs), len(self.ctxs), k, flags, ctypes.byref(h))
        self.ctxs[0].check(st)
        self.handle = h

    @property
    def transport(self):
        return self.lib.cel_shard_plan_transport(self.handle).decode()

    @property
    def note(self):
        """Why RCCL was not used ("" when it was, or was not asked for)."""
        return self.lib.cel_shard_plan_note(self.handle).decode()

    def time_exchange(self, reps=10):
        """Microseconds per all-to-all alone (slowest rank), or None for a one-rank plan in place."""
        if self.transport == "local":
            return None
        us = ctypes.c_double()
        self.check(self.lib.cel_shard_plan_time_exchange(self.handle, reps, ctypes.byref(us)))
        return us.value

    def check(self, st):
        if st != _lib.OK:
            raise _lib.CelError(st, self.lib.cel_shard_plan_last_error(self.handle).decode()
                                or self.lib.cel_strerror(st).decode())

    def upload(self, ods):
        """ods: [k][k][512] uint8, a host array or a device tensor."""
        if isinstance(ods, np.ndarray):
            ods = np.ascontiguousarray(ods, dtype=np.uint8)
            assert ods.size == self.k * self.k * _lib.SHARE_SIZE
        self._ods = ods  # alive until the copy is done (the run orders after it)
        self.check(self.lib.cel_shard_plan_upload(self.handle, _ptr(ods)))

    def run(self):
        self.check(self.lib.cel_shard_plan_run(self.handle))

    def wait(self, want_eds=False):
        w = 2 * self.k
        eds = np.zeros((w, w, _lib.SHARE_SIZE), np.uint8) if want_eds else None
        rr = np.zeros((w, _NODE), np.uint8)
        cr = np.zeros_like(rr)
        dah = np.zeros(32, np.uint8)
        self.check(self.lib.cel_shard_plan_wait(self.handle, _ptr(eds), _ptr(rr), _ptr(cr), _ptr(dah)))
        return eds, rr, cr, dah.tobytes()

    def close(self):
        if getattr(self, "handle", None):
            self.lib.cel_shard_plan_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def extend_sharded(ctxs, ods, want_eds=True, flags=_lib.FLAG_ORDER_CHECK):
    """cel_extend_sharded: ods [k][k][512] host bytes -> (eds or None, row roots, col roots,
    dah) for the whole square, computed row-sharded over the ctxs' devices."""
    ods = np.ascontiguousarray(ods, dtype=np.uint8)
    k = ods.shape[0]
    w = 2 * k
    eds = np.zeros((w, w, _lib.SHARE_SIZE), np.uint8) if want_eds else None
    rr = np.zeros((w, _NODE), np.uint8)
    cr = np.zeros_like(rr)
    dah = np.zeros(32, np.uint8)
    c0 = ctxs[0]
    c0.check(c0.lib.cel_extend_sharded(_handles(ctxs), len(ctxs), _ptr(ods), k, _lib.SHARE_SIZE, _ptr(eds),
                                       _ptr(rr), _ptr(cr), _ptr(dah), flags))
    return eds, rr, cr, dah.tobytes()


def extend_batch_multi(ctxs, ods, want_eds=True, flags=_lib.FLAG_ORDER_CHECK):
    """cel_extend_batch_multi: ods [n][k][k][512] host bytes split over the ctxs (one host
    thread per ctx in the library) -> (eds or None, row roots, col roots, dahs, status)."""
    ods = np.ascontiguousarray(ods, dtype=np.uint8)
    n, k = ods.shape[0], ods.shape[1]
    w = 2 * k
    eds = np.zeros((n, w, w, _lib.SHARE_SIZE), np.uint8) if want_eds else None
    rr = np.zeros((n, w, _NODE), np.uint8)
    cr = np.zeros_like(rr)
    dah = np.zeros((n, 32), np.uint8)
    st = np.zeros(n, np.int32)
    c0 = ctxs[0]
    c0.check(c0.lib.cel_extend_batch_multi(_handles(ctxs), len(ctxs), _ptr(ods), n, k, _lib.SHARE_SIZE, _ptr(eds),
                                           _ptr(rr), _ptr(cr), _ptr(dah), _ptr(st), flags))
    return eds, rr, cr, dah, st


def probe(ctx, hbm_bytes=4 << 30, rs_k=(64, 128, 512)):
    """Same-run ceilings on ctx's device: SHA-256 G compressions/s in registers, the
    sustained shader clock over that launch (MHz), streaming-copy HBM GB/s (and the
    read-only / write-only stream rates), and the
    microseconds of VALU one k-square's extension takes with no HBM traffic
    (`rs_transform_us_k<k>`, each k in rs_k; GF(2^8) up to k = 128, GF(2^16) at 256 / 512)."""
    g, mhz, bw, rd, wr = (ctypes.c_double() for _ in range(5))
    ctx.check(ctx.lib.cel_probe_sha256(ctx.handle, ctypes.byref(g), ctypes.byref(mhz)))
    ctx.check(ctx.lib.cel_probe_hbm_stream(ctx.handle, hbm_bytes, ctypes.byref(bw), ctypes.byref(rd), ctypes.byref(wr)))
    out = {"sha256_gcomp_per_s": g.value, "shader_mhz": mhz.value, "hbm_copy_gbps": bw.value,
           "hbm_read_gbps": rd.value, "hbm_write_gbps": wr.value}
    for k in rs_k:
        us = ctypes.c_double()
        ctx.check(ctx.lib.cel_probe_rs_transform(ctx.handle, k, ctypes.byref(us)))
        out[f"rs_transform_us_k{k}"] = us.value
    return out
