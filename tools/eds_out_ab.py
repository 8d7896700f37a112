"""One square with its EDS copied back through the host entry point (cel_extend_batch, n = 1)
into host memory of different kinds (dev aid): pageable numpy, cel_host_alloc, and
hipHostMalloc with the coherent / non-coherent flags, alternated, full EDS and parity only:
  python tools/eds_out_ab.py <k> [reps]"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))

import numpy as np  # noqa: E402

from celestia_eds import _lib, default_context  # noqa: E402
from celestia_eds.testfactory import random_ods  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 128
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
ctx = default_context(0)
hip = ctypes.CDLL("libamdhip64.so.7")
hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
w = 2 * k
P = lambda x: x.ctypes.data_as(ctypes.c_void_p)


def host(kind, shape):
    nbytes = int(np.prod(shape))
    if kind == "pageable":
        return np.zeros(shape, np.uint8)
    if kind == "cel_host_alloc":
        p = ctx.lib.cel_host_alloc(nbytes)
    else:
        v = ctypes.c_void_p()
        flags = {"coherent": 0x40000000, "noncoherent": 0x80000000}[kind]
        assert hip.hipHostMalloc(ctypes.byref(v), nbytes, flags) == 0
        p = v.value
    return np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p)).reshape(shape)


ods = host("cel_host_alloc", (k, k, 512))
ods[...] = random_ods(k, 5)
rr, cr = np.zeros((w, 90), np.uint8), np.zeros((w, 90), np.uint8)
dah, st = np.zeros(32, np.uint8), np.zeros(1, np.int32)
kinds = ["pageable", "cel_host_alloc", "coherent", "noncoherent"]
outs = {kd: host(kd, (w, w, 512)) for kd in kinds}
for rnd in range(2):
    for fl, fname in ((0, "full EDS"), (_lib.FLAG_PARITY_ONLY, "parity only")):
        for kd in kinds:
            e = outs[kd]

            def call():
                ctx.check(ctx.lib.cel_extend_batch(ctx.handle, P(ods), 1, k, 512, P(e), P(rr), P(cr), P(dah), P(st),
                                                   _lib.FLAG_ORDER_CHECK | fl))
            for _ in range(5):
                call()
            t0 = time.perf_counter()
            for _ in range(reps):
                call()
            ms = (time.perf_counter() - t0) / reps * 1e3
            print(f"k={k} {fname:11s} into {kd:15s}: {ms:7.3f} ms", flush=True)
