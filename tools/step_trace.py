"""Batch steps separated by idle gaps, for a kernel timeline of one step (dev aid):

  rocprofv3 --kernel-trace -d <dir> -o s --output-format csv -- \
      python3 tools/step_trace.py --k 64 --batch 128 --steps 4
  python3 tools/timeline.py <dir> 1000 -2

Each step is cel_dev_extend_batch over B resident squares (as bench.py's timed steps),
followed by a synchronize and a 3 ms sleep so the trace splits into one burst per step.
--inflight M: a burst is M steps issued back to back on M batches (own buffers and
stream each), as bench.py --inflight M times them."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--k", type=int, default=64)
ap.add_argument("--batch", type=int, default=128)
ap.add_argument("--steps", type=int, default=4)
ap.add_argument("--inflight", type=int, default=1)
ap.add_argument("--chain", type=int, default=0, help="steps per burst, round-robin over the batches (default: one per batch)")
a = ap.parse_args()
from celestia_eds.device import SquareBatch  # noqa: E402
from celestia_eds.testfactory import random_ods  # noqa: E402

sbs = []
for j in range(max(1, a.inflight)):
    sb = SquareBatch(a.batch, a.k, ods_in_eds=True)
    sb.load_ods(torch.from_numpy(np.stack([random_ods(a.k, 3 + ((i + j) % 4)) for i in range(a.batch)])))
    sbs.append(sb)
for i in range(a.steps):
    t0 = time.perf_counter()
    for j in range(a.chain or len(sbs)):
        sbs[j % len(sbs)].extend_and_commit(caller_stream=len(sbs) > 1)
    torch.cuda.synchronize()
    print(f"burst {i}: {(time.perf_counter() - t0) * 1e3:.3f} ms for {a.chain or len(sbs)} step(s) (host, synchronized)",
          flush=True)
    time.sleep(0.003)
for sb in sbs:
    assert (sb.status.cpu().numpy() == 0).all()
