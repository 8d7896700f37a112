"""Per-rank phase latency of the row-sharded square (config 3) at a simulated world size,
on one GPU: rank 0's device steps with the collectives left out (dev aid).

python tools/rank_latency.py [--k 512] [--n 8] [--reps 20]

Prints the median of `reps` HIP-event timings of each phase on the device-steps stream:
rows (k/N ODS rows -> all-to-all send layout), cols (column-encode + slab commit), finish
(combine of the N subtree roots + DAH), and the three back to back.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--k", type=int, default=512)
ap.add_argument("--n", type=int, default=8)
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()
from celestia_eds import default_context  # noqa: E402
from celestia_eds.sharded import DeviceSteps, ShardedSquare  # noqa: E402
from celestia_eds.testfactory import random_ods  # noqa: E402

torch.cuda.set_device(0)
steps = DeviceSteps(default_context(0), 0)
sq = ShardedSquare(a.k, 0, a.n, steps)
lo, hi = sq.row_range()
sq.ods_rows.copy_(torch.from_numpy(np.ascontiguousarray(random_ods(a.k, 512)[lo:hi])))
sq.slab.copy_(torch.from_numpy(np.ascontiguousarray(random_ods(2 * a.k, 5)[:, : sq.w])))  # stand-in slab
sq.gathered.zero_()
cur = steps.stream


def timed(fn):
    ts = []
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(cur)
        fn()
        e1.record(cur)
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return sorted(ts)[len(ts) // 2]


def chain():
    sq.phase_rows()
    sq.phase_cols()
    sq.phase_finish()


with sq.scope():
    for f in (sq.phase_rows, sq.phase_cols, sq.phase_finish):
        f()
    torch.cuda.synchronize()
    res = {name: timed(f) for name, f in (("rows", sq.phase_rows), ("cols", sq.phase_cols),
                                          ("finish", sq.phase_finish), ("chain", chain))}
print(f"k={a.k} n={a.n} rank 0 (us, median of {a.reps}): " + " ".join(f"{k}={v:.1f}" for k, v in res.items()))
