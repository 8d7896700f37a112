"""Repeat device repairs of multi-pass masks and count outcomes (dev aid for the two-stream
repair schedule): python tools/repair_stress.py <k> <reps>"""
import sys
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for d in ("celestia-app_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, d))
import numpy as np  # noqa: E402

import celestia_eds  # noqa: E402
import oracle  # noqa: E402
from eds_inputs import random_ods  # noqa: E402
from test_gpu_repair import _crossword_passes, _dev_repair  # noqa: E402

k, reps = int(sys.argv[1]), int(sys.argv[2])
ctx = celestia_eds.default_context(0)
oracle.set_simd(True)
eds, rr, cr, _ = oracle.extend_and_commit(random_ods(k, 3))
rr = [r.tobytes() for r in rr]
cr = [c.tobytes() for c in cr]
w = 2 * k
counts = {}
for seed in range(reps):
    for p in (0.44, 0.46, 0.5):
        present = (np.random.default_rng(seed).random((w, w)) < p).astype(np.uint8)
        npass, ok = _crossword_passes(present, k)
        st, cells, bad = _dev_repair(ctx, eds, present, rr, cr)
        good = (st == 0) == ok and (not ok or np.array_equal(cells, eds))
        key = ("ok" if good else "BAD", npass)
        counts[key] = counts.get(key, 0) + 1
        if not good:
            print("mismatch", seed, p, npass, ok, st, bad, flush=True)
print(sorted(counts.items()))
