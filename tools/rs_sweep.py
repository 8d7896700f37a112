"""RS extension per square against batch size, beside the same library's transform-only
probe (cel_probe_rs_transform), for the library CEL_EDS_LIB names (default: the shipped one):
  python tools/rs_sweep.py --k 128 --batches 16,64,256 [--reps 10]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--k", type=int, default=128)
ap.add_argument("--batches", default="16,64,256")
ap.add_argument("--reps", type=int, default=10)
a = ap.parse_args()
from celestia_eds import multi  # noqa: E402
from celestia_eds.device import SquareBatch  # noqa: E402
from celestia_eds.testfactory import random_ods  # noqa: E402

tag = os.path.basename(os.environ.get("CEL_EDS_LIB", "shipped"))
out = []
for b in [int(x) for x in a.batches.split(",")]:
    sb = SquareBatch(b, a.k, ods_in_eds=True)
    ods = random_ods(a.k, 1)
    sb.load_ods(torch.from_numpy(np.stack([ods] * b)))
    sb.extend_only()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(sb.hip_stream)
    for _ in range(a.reps):
        sb.extend_only()
    e1.record(sb.hip_stream)
    e1.synchronize()
    us = e0.elapsed_time(e1) / a.reps * 1e3 / b
    out.append(f"B={b}:{us:.2f}")
    ctx = sb.ctx
    del sb
    torch.cuda.empty_cache()
pr = multi.probe(ctx, hbm_bytes=1 << 30, rs_k=(a.k,))
print(f"{tag} k={a.k} us/square {' '.join(out)}  transform-only {pr[f'rs_transform_us_k{a.k}']:.2f}  "
      f"sha {pr['sha256_gcomp_per_s']:.2f} G/s  {pr['shader_mhz']:.0f} MHz  copy {pr['hbm_copy_gbps']:.0f} GB/s")
