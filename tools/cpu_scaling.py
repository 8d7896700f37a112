"""CPU-baseline scaling on the host it runs on (dev aid for bench.py's cpu_baseline).

Prints the host (bench.cpu_info), which physical core each allowed CPU sits on, then the
C restatement's k=128 squares/s (extend + roots + DAH, one square per thread) and its two
parts measured alone (RS extension GB/s, NMT SHA-256 compressions/s, each on every thread
at once) at 1, 2, 4, ... threads up to the granted share, so measured-vs-linear can be
split into SMT siblings, memory bandwidth and the rest.
usage: python tools/cpu_scaling.py [seconds per point]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import bench  # noqa: E402
import oracle  # noqa: E402
from concurrent.futures import ThreadPoolExecutor  # noqa: E402

sec = float(sys.argv[1]) if len(sys.argv) > 1 else 3.0
info = bench.cpu_info()
print("host", info)
cpu_core = {}
with open("/proc/cpuinfo") as f:
    cur = {}
    for line in f:
        k, _, v = line.partition(":")
        if k.strip() in ("processor", "physical id", "core id"):
            cur[k.strip()] = v.strip()
        if not line.strip() and "processor" in cur:
            cpu_core[int(cur["processor"])] = (cur.get("physical id"), cur.get("core id"))
            cur = {}
allowed = sorted(os.sched_getaffinity(0))
print("allowed cpus -> (package, core):", [(c, cpu_core.get(c)) for c in allowed])

oracle.set_simd(True)
lib, P = oracle.lib(), oracle._p
k = 128
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
from celestia_eds.testfactory import random_ods  # noqa: E402
sq = np.stack([random_ods(k, 7 + i) for i in range(2)])
granted = info["granted_threads"]
points = sorted({t for t in (1, 2, 4, 8, 12, 16, 24, 32) if t <= granted} | {granted})


def rate(fn, n_per_call):
    fn()
    done, t = 0, 0.0
    while t < sec:
        t0 = time.perf_counter()
        fn()
        t += time.perf_counter() - t0
        done += n_per_call
    return done / t


for th in points:
    oracle.set_threads(th)
    batch = np.stack([sq[i % 2] for i in range(2 * th)])
    full = rate(lambda: oracle.extend_commit_many(batch), 2 * th)
    # the parts on every thread at once (one private square per thread, python threads
    # release the GIL inside the ctypes calls)
    oracle.set_threads(1)
    eds = [np.ones((2 * k, 2 * k, 512), np.uint8) for _ in range(th)]
    rr = [np.zeros((2 * k, 90), np.uint8) for _ in range(th)]
    cr = [np.zeros((2 * k, 90), np.uint8) for _ in range(th)]
    with ThreadPoolExecutor(th, initializer=lambda: oracle.set_threads(1)) as ex:  # OpenMP's thread count is per OS thread
        def each(fn):
            list(ex.map(fn, range(th)))
        rs = rate(lambda: each(lambda i: lib.orc_extend(P(sq[i % 2]), k, 512, P(eds[i]))), th)
        nmt = rate(lambda: each(lambda i: lib.orc_roots(P(eds[i]), k, 512, P(rr[i]), P(cr[i]), 0, None)), th)
    print(f"threads={th:3d} squares/s={full:8.1f} per_thread={full / th:6.2f}  "
          f"rs_GBps={rs * 2048 * k * k / 1e9:7.1f} ({rs * 2048 * k * k / 1e9 / th:5.2f}/thread)  "
          f"nmt_Mcomp/s={nmt * (96 * k * k - 12 * k) / 1e6:8.1f} ({nmt * (96 * k * k - 12 * k) / 1e6 / th:5.2f}/thread)",
          flush=True)
