"""One square's header through the host entry point (cel_extend_batch, n = 1, eds_out = NULL,
page-locked ODS): ms per call at k = 128, 256, 512 and the DAH (dev aid; CEL_EDS_LIB picks a
library build, so variants can be compared on one box):
  python tools/header_lat.py [reps] [pageable]   (pageable: the ODS in ordinary host memory)"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))

import numpy as np  # noqa: E402

from celestia_eds import _lib, default_context  # noqa: E402
from celestia_eds.testfactory import random_ods  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
pageable = len(sys.argv) > 2 and sys.argv[2] == "pageable"
ctx = default_context(0)
P = lambda x: x.ctypes.data_as(ctypes.c_void_p)
for k in (128, 256, 512):
    nbytes = k * k * 512
    if pageable:
        ods = np.ascontiguousarray(random_ods(k, 31 + k))
        p = ods.ctypes.data
    else:
        p = ctx.lib.cel_host_alloc(nbytes)
        ods = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p)).reshape(k, k, 512)
        ods[...] = random_ods(k, 31 + k)
    rr, cr = np.zeros((2 * k, 90), np.uint8), np.zeros((2 * k, 90), np.uint8)
    dah, st = np.zeros(32, np.uint8), np.zeros(1, np.int32)

    def call():
        ctx.check(ctx.lib.cel_extend_batch(ctx.handle, ctypes.c_void_p(p), 1, k, 512, None, P(rr), P(cr), P(dah),
                                           P(st), _lib.FLAG_ORDER_CHECK))
    call()
    call()
    t0 = time.perf_counter()
    for _ in range(reps):
        call()
    ms = (time.perf_counter() - t0) / reps * 1e3
    print(f"k={k:4d}: {ms:7.3f} ms per header  dah {dah.tobytes().hex()[:16]}", flush=True)
    if not pageable:
        ctx.lib.cel_host_free(p)
