"""PCIe-inclusive rate of the host-buffer entry point (cel_extend_batch): pageable host
ODS in, EDS + roots + DAH out, as the Go shim behind da.ExtendShares would call it.
  python tools/host_io.py --k 128 --batch 16 --reps 5 [--no-eds]"""
import argparse
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
import numpy as np  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--k", type=int, default=128)
ap.add_argument("--batch", type=int, default=16)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--no-eds", action="store_true", help="roots + DAH only (no EDS copy back)")
ap.add_argument("--pinned", action="store_true", help="ODS / EDS buffers from cel_host_alloc (page-locked)")
ap.add_argument("--parity-only", action="store_true", help="CEL_FLAG_PARITY_ONLY: Q1..Q3 of the EDS back, not Q0")
a = ap.parse_args()
from celestia_eds import _lib  # noqa: E402
from celestia_eds.testfactory import random_ods  # noqa: E402

ctx = _lib.default_context(0)
k, n = a.k, a.batch
w = 2 * k
src = np.stack([random_ods(k, 100 + i) for i in range(n)])


def host_array(shape):
    if not a.pinned:
        return np.zeros(shape, np.uint8)
    nbytes = int(np.prod(shape))
    p = ctx.lib.cel_host_alloc(nbytes)
    assert p, "cel_host_alloc failed"
    return np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p)).reshape(shape)


ods = host_array(src.shape)
ods[...] = src
eds = None if a.no_eds else host_array((n, w, w, 512))
rr = np.zeros((n, w, 90), np.uint8)
cr = np.zeros_like(rr)
dah = np.zeros((n, 32), np.uint8)
st = np.zeros(n, np.int32)
P = lambda x: x.ctypes.data_as(ctypes.c_void_p) if x is not None else None


def once():
    ctx.check(ctx.lib.cel_extend_batch(ctx.handle, P(ods), n, k, 512, P(eds), P(rr), P(cr), P(dah), P(st),
                                       _lib.FLAG_ORDER_CHECK | (_lib.FLAG_PARITY_ONLY if a.parity_only else 0)))


once()
t0 = time.perf_counter()
for _ in range(a.reps):
    once()
dt = (time.perf_counter() - t0) / a.reps
mode = ("ODS in, roots+DAH out" if a.no_eds else
        "ODS in, parity quadrants+roots+DAH out" if a.parity_only else "ODS in, EDS+roots+DAH out") + (", pinned" if a.pinned else ", pageable")
print(f"host-buffer cel_extend_batch k={k} batch={n} ({mode}): {dt * 1e3:.2f} ms per call = "
      f"{n / dt:.0f} squares/s; bytes over PCIe {(ods.nbytes + (0 if eds is None else eds.nbytes)) / dt / 1e9:.1f} GB/s")
