"""Socket power and shader clock while one pipeline phase runs back to back (rocm-smi
sampled from a thread), to tell a power-capped phase from an issue- or HBM-bound one:
  python tools/power_probe.py --phase extend|commit|probe|step --k 128 --batch 256 [--secs 6]
CEL_EDS_LIB picks a variant build. 'probe' loops cel_probe_rs_transform (VALU only); 'step'
the bench's step (four batches in flight, each extended and committed in turn)."""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--phase", default="extend")
ap.add_argument("--k", type=int, default=128)
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--secs", type=float, default=6.0)
a = ap.parse_args()
from celestia_eds.device import SquareBatch  # noqa: E402
from celestia_eds.testfactory import random_ods  # noqa: E402

sb = SquareBatch(a.batch, a.k, ods_in_eds=True)
sb.load_ods(torch.from_numpy(np.stack([random_ods(a.k, 1)] * a.batch)))
sb.extend_and_commit()
torch.cuda.synchronize()
if a.phase == "step":  # the bench's step: 4 batches in flight, each extended and committed in turn
    sbs = [sb] + [SquareBatch(a.batch, a.k, ods_in_eds=True) for _ in range(3)]
    for b in sbs[1:]:
        b.load_ods(torch.from_numpy(np.stack([random_ods(a.k, 2)] * a.batch)))
    it = [0]

    def fn():
        sbs[it[0] % 4].extend_and_commit(caller_stream=True)
        it[0] += 1
elif a.phase == "probe":
    us = ctypes.c_double()
    fn = lambda: sb.ctx.lib.cel_probe_rs_transform(sb.ctx.handle, a.k, ctypes.byref(us))  # noqa: E731
else:
    fn = sb.extend_only if a.phase == "extend" else sb.commit_only

samples, stop = [], threading.Event()


def sampler():
    time.sleep(1.0)
    while not stop.is_set():
        try:
            out = subprocess.run(["rocm-smi", "-P", "-c", "--json"], capture_output=True, text=True, timeout=10).stdout
            samples.append(json.loads(out[out.index("{"):]))
        except Exception as e:  # noqa: BLE001
            samples.append({"error": repr(e)})
        time.sleep(0.3)


th = threading.Thread(target=sampler, daemon=True)
th.start()
t0, n = time.time(), 0
while time.time() - t0 < a.secs:
    fn()
    n += 1
    if n % 4 == 0:
        torch.cuda.synchronize()
torch.cuda.synchronize()
stop.set()
th.join()
el = time.time() - t0
pw, sclk = [], []
for s in samples:
    for card, v in s.items():
        if not isinstance(v, dict):
            continue
        for key, val in v.items():
            kl = key.lower()
            if "power" in kl and "(w)" in kl:
                try:
                    pw.append(float(val))
                except ValueError:
                    pass
            if kl.startswith("sclk"):
                try:
                    sclk.append(float(str(val).strip("()Mhz ")))
                except ValueError:
                    pass
tag = os.path.basename(os.environ.get("CEL_EDS_LIB", "shipped"))
print(f"{tag} {a.phase} k={a.k} B={a.batch}: {el / n * 1e3:.3f} ms per call, {len(samples)} samples, "
      f"power W {[round(x) for x in pw]} sclk MHz {[round(x) for x in sclk]}")
if not pw and samples:
    print(json.dumps(samples[0])[:600])
