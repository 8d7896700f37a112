"""RS extension throughput vs chunking (rows+cols per chunk of C squares), one stream.
  python tools/rs_chunks.py --k 128 --batch 32 --chunks 1 2 4 8 32"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--k", type=int, default=128)
ap.add_argument("--batch", type=int, default=32)
ap.add_argument("--chunks", type=int, nargs="+", default=[1, 2, 4, 8, 32])
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--streams", type=int, default=1)
ap.add_argument("--inplace", action="store_true", help="Q0 already in the EDS (d_ods = NULL)")
a = ap.parse_args()
from celestia_eds.device import SquareBatch  # noqa: E402
from celestia_eds.testfactory import random_ods  # noqa: E402

# --inplace: the random ODS sits in Q0 of every EDS (as in bench.py); the kernels'
# power draw, and so the clock, depends on the data, so never time all-zero squares.
sb = SquareBatch(a.batch, a.k, ods_in_eds=a.inplace)
ods = random_ods(a.k, 1)
sb.load_ods(torch.from_numpy(np.stack([ods] * a.batch)))
c = sb.ctx
k, B = a.k, a.batch
ods_sq, eds_sq = k * k * 512, 4 * k * k * 512


streams = [torch.cuda.Stream() for _ in range(a.streams)]


def run(cs):
    ev = torch.cuda.Event()
    ev.record(sb.hip_stream)
    for st in streams:
        st.wait_event(ev)
    for i, s0 in enumerate(range(0, B, cs)):
        n = min(cs, B - s0)
        st = streams[i % len(streams)] if a.streams > 1 else sb.hip_stream
        c.check(c.lib.cel_dev_extend_only(c.handle, None if a.inplace else ctypes.c_void_p(sb.ods.data_ptr() + s0 * ods_sq), n, k,
                                          ctypes.c_void_p(sb.eds.data_ptr() + s0 * eds_sq),
                                          ctypes.c_void_p(st.cuda_stream)))
    for st in streams:
        e2 = torch.cuda.Event()
        e2.record(st)
        sb.hip_stream.wait_event(e2)


for cs in a.chunks:
    run(cs)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(sb.hip_stream)
    for _ in range(a.reps):
        run(cs)
    e1.record(sb.hip_stream)
    e1.synchronize()
    us = e0.elapsed_time(e1) / a.reps * 1e3 / B
    print(f"{os.environ.get('CEL_RS_IMPL', 'default'):9s} dbg={os.environ.get('CEL_RS_DEBUG', '0')} inplace={int(a.inplace)} streams={a.streams} k={k} chunk={cs:3d}: {us:6.2f} us/square "
          f"= {2048 * k * k / us / 1e3:7.1f} GB/s algorithmic ({2048 * k * k / us / 1e3 / 8000 * 100:4.1f} %)")

if os.environ.get("CEL_COPY_REF"):
    dst = torch.empty_like(sb.eds)
    dst.copy_(sb.eds)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(sb.hip_stream):
        e0.record(sb.hip_stream)
        for _ in range(a.reps):
            dst.copy_(sb.eds)
        e1.record(sb.hip_stream)
    e1.synchronize()
    us = e0.elapsed_time(e1) / a.reps * 1e3
    nbytes = 2 * sb.eds.numel()
    print(f"reference D2D copy of the EDS batch: {nbytes / us / 1e3:7.1f} GB/s (read+write)")
