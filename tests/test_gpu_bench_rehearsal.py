"""The N-rank bench path on the one-GPU box: `bench.py --gpus 2 --rehearse` relaunches
itself under torch.distributed.run, both ranks drive the HIP library on cuda:0 and the
collectives go through gloo with host staging. It runs the same code the driver's 8-GPU
line runs (launcher, barriers, max over ranks, the k64 and rowshard512 riders, the row-
sharded square's all-to-all and record gathers), RCCL aside, so a shape or protocol
error in the multi-rank path shows up here rather than in the round-end scaling run."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_two_rank_rehearsal():
    env = dict(os.environ)
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(v, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rehearse", "--steps", "2", "--warmup",
           "1", "--batch", "16", "--k512-batch", "2", "--k512-steps", "2", "--rider-steps", "2", "--phase-reps", "2",
           "--no-host-io", "--no-cpu"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    r = lines[0]
    assert r["n_gpus"] == 2 and "rehearsal" in r["config"]
    assert r["value"] > 0 and r["k512"]["value"] > 0
    assert r["k64"]["n_gpus"] == 2 and r["k64"]["squares_per_step_per_gpu"] == 512 and r["k64"]["value"] > 0
    rs = r["rowshard512"]
    assert rs["n_gpus"] == 2 and rs["value"] > 0
    assert rs["a2a_bytes_per_peer"] == 2 * 512 * 512 * 512 // 4 and rs["a2a_us"] > 0
