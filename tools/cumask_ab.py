"""A/B of the headline step's stream structure (one MI355X):

  shipped   M batches in flight, each batch's extension + commit on its own stream
            (CEL_FLAG_CALLER_STREAM), extensions chained (bench.py's default)
  split     the extensions on one stream, each batch's commit on its own stream
            (event hand-offs), no CU masks: the same overlap, other queue mapping
  mask<f>   as split, the extension stream restricted to a fraction f of the CUs and the
            commit streams to the rest (hipExtStreamCreateWithCUMask): the HBM-bound,
            VALU-light RS pass and the VALU-bound hashing on disjoint CUs all the time

Data content does not change the time of either kernel (RS and SHA-256 are data-independent),
so the squares are random bytes and the push-order check is off in every variant.
  python tools/cumask_ab.py <k> <batch> <inflight> <steps> <variant>...
"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))

import torch  # noqa: E402

from celestia_eds import default_context  # noqa: E402
from celestia_eds.device import SquareBatch  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")


def ck(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what}: hip error {rc}")


def stream(mask=None, ncu=256):
    s = ctypes.c_void_p()
    if mask is None:
        ck(hip.hipStreamCreateWithFlags(ctypes.byref(s), 1), "stream")
    else:
        words = (ncu + 31) // 32
        arr = (ctypes.c_uint32 * words)()
        for i in mask:
            arr[i // 32] |= 1 << (i % 32)
        ck(hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), words, arr), "cu-mask stream")
    return s


def event():
    e = ctypes.c_void_p()
    ck(hip.hipEventCreateWithFlags(ctypes.byref(e), 2), "event")  # hipEventDisableTiming
    return e


def main():
    k, B, M, steps = (int(x) for x in sys.argv[1:5])
    variants = sys.argv[5:]
    ctx = default_context(0)
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    sbs = [SquareBatch(B, k, 0, ctx, ods_in_eds=True) for _ in range(M)]
    for sb in sbs:
        sb.eds.random_(0, 256)
    lib, h = ctx.lib, ctx.handle
    P = ctypes.c_void_p

    def run_shipped(n):
        for i in range(n):
            sbs[i % M].extend_and_commit(order_check=False, caller_stream=True)

    def make_split(frac):
        if frac is None:
            rs, nm = stream(), [stream() for _ in range(M)]
        else:
            rs_cus = [i for i in range(ncu) if int((i + 1) * frac) > int(i * frac)]
            other = [i for i in range(ncu) if i not in set(rs_cus)]
            rs, nm = stream(rs_cus, ncu), [stream(other, ncu) for _ in range(M)]
        ev_rs, ev_nm = [event() for _ in range(M)], [event() for _ in range(M)]
        pending = [False] * M

        def run(n):
            for i in range(n):
                b = i % M
                sb = sbs[b]
                if pending[b]:  # the batch's buffers are free once its previous commit is done
                    ck(hip.hipStreamWaitEvent(rs, ev_nm[b], 0), "wait")
                ck(lib.cel_dev_extend_only(h, None, B, k, P(sb.eds.data_ptr()), rs), "extend")
                ck(hip.hipEventRecord(ev_rs[b], rs), "record")
                ck(hip.hipStreamWaitEvent(nm[b], ev_rs[b], 0), "wait")
                ck(lib.cel_dev_commit_only(h, P(sb.eds.data_ptr()), B, k, P(sb.row_roots.data_ptr()),
                                           P(sb.col_roots.data_ptr()), P(sb.dah.data_ptr()),
                                           P(sb.status.data_ptr()), P(sb.work.data_ptr()), nm[b], 0), "commit")
                ck(hip.hipEventRecord(ev_nm[b], nm[b]), "record")
                pending[b] = True
        return run

    runs = {"shipped": run_shipped}
    for v in variants:
        if v == "split":
            runs[v] = make_split(None)
        elif v.startswith("mask"):
            runs[v] = make_split(float(v[4:]))
    dahs = {}
    for rep in range(2):
        for v in variants:
            fn = runs[v]
            fn(2 * M)
            ck(hip.hipDeviceSynchronize(), "sync")
            t0 = time.perf_counter()
            fn(steps)
            ck(hip.hipDeviceSynchronize(), "sync")
            dt = time.perf_counter() - t0
            dahs[v] = sbs[0].dah.cpu().clone()
            print(f"k={k} B={B} inflight {M} {v:10s} {B * steps / dt:9.0f} squares/s  "
                  f"{dt / steps * 1e3:7.3f} ms/step  {dt / (B * steps) * 1e6:6.2f} us/square", flush=True)
    ref = dahs[variants[0]]
    for v in variants[1:]:
        assert torch.equal(dahs[v], ref), f"{v}: DAHs differ from {variants[0]}"
    print("DAHs equal across variants", flush=True)


if __name__ == "__main__":
    main()
