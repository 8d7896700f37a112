"""Time cel_dev_decode alone (dev aid): the row pass of a k=128 p=0.55 mask, as bench.py
--mode repair's roofline. python tools/dec_time.py [--k 128] [--reps 20]"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
from celestia_eds import default_context  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--k", type=int, default=128)
ap.add_argument("--p", type=float, default=0.55)
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()
k, w = a.k, 2 * a.k
rng = np.random.default_rng(7)
present = (rng.random((w, w)) < a.p).astype(np.uint8)
rows = [i for i in range(w) if k <= int(present[i].sum()) < w]
data = torch.from_numpy(rng.integers(0, 256, (len(rows), w, 512), dtype=np.uint8)).cuda()
mask = torch.from_numpy(np.ascontiguousarray(present[rows])).cuda()
ctx = default_context(0)
s = torch.cuda.Stream()
sp = ctypes.c_void_p(s.cuda_stream)


def dec():
    ctx.check(ctx.lib.cel_dev_decode(ctx.handle, ctypes.c_void_p(data.data_ptr()), ctypes.c_void_p(mask.data_ptr()),
                                     len(rows), k, 512, sp))


dec()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(s)
for _ in range(a.reps):
    dec()
e1.record(s)
e1.synchronize()
print(f"k={k} axes={len(rows)}: {e0.elapsed_time(e1) / a.reps * 1e3:.1f} us per decode launch")
