"""Run one phase of the pipeline on a single stream, for clean per-kernel profiles:
  python tools/prof_phase.py --phase extend|commit --k 128 --batch 8 --reps 5"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--phase", default="extend")
ap.add_argument("--k", type=int, default=128)
ap.add_argument("--batch", type=int, default=8)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--input", default="eds", choices=["eds", "ods"], help="ODS in Q0 of the EDS (in place) or separate")
a = ap.parse_args()
from celestia_eds.device import SquareBatch  # noqa: E402
from celestia_eds.testfactory import random_ods  # noqa: E402

sb = SquareBatch(a.batch, a.k, ods_in_eds=(a.input == "eds"))
ods = random_ods(a.k, 1)
sb.load_ods(torch.from_numpy(np.stack([ods] * a.batch)))
sb.extend_and_commit()
torch.cuda.synchronize()
fn = sb.extend_only if a.phase == "extend" else sb.commit_only
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(sb.hip_stream)
for _ in range(a.reps):
    fn()
e1.record(sb.hip_stream)
e1.synchronize()
print(f"{a.phase} input={a.input} k={a.k} batch={a.batch}: {e0.elapsed_time(e1) / a.reps * 1e3:.1f} us per call "
      f"({e0.elapsed_time(e1) / a.reps * 1e3 / a.batch:.2f} us per square)")
