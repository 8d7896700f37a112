"""bench.py --gpus N relaunches itself under torch.distributed.run with N ranks (the
driver's N-GPU line); the distcheck mode runs that same launcher,
rendezvous (gloo, 127.0.0.1), barrier + MAX-over-ranks timing and rank-0 JSON path on
CPU ranks."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, timeout=240):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    env["OMP_NUM_THREADS"] = "1"
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    return [json.loads(l) for l in lines]


def test_launcher_two_ranks():
    out = _run(["--gpus", "2", "--mode", "distcheck", "--steps", "3", "--warmup", "1"])
    assert len(out) == 1, out
    r = out[0]
    assert r["n_gpus"] == 2 and r["steps"] == 3 and r["warmup"] == 1
    assert r["value"] > 0 and r["scaling"] == "weak" and r["config"]["parallelism"] == "batch2"


def test_single_rank_no_relaunch():
    out = _run(["--mode", "distcheck", "--steps", "2", "--warmup", "0"])
    assert len(out) == 1 and out[0]["n_gpus"] == 1


def test_riders_in_multi_rank_line():
    """One N-rank command carries configs 4 and 3 as riders (k64: 1024/N squares per rank;
    rowshard512: the row-sharded square's all_to_all_single, timed alone, beside SURVEY
    §8e's one-link estimate), with n_gpus = N. Here over gloo with CPU stand-in steps."""
    out = _run(["--gpus", "4", "--mode", "distcheck", "--steps", "2", "--warmup", "1"])
    assert len(out) == 1, out
    r = out[0]
    assert r["n_gpus"] == 4
    assert r["k64"]["n_gpus"] == 4 and r["k64"]["squares_per_step_per_gpu"] == 256
    rs = r["rowshard512"]
    assert rs["n_gpus"] == 4 and rs["scaling"] == "strong"
    assert rs["a2a_bytes_per_peer"] == 2 * 64 * 64 * 512 // 16
    assert rs["a2a_us"] > 0 and rs["a2a_survey_estimate_us"] > 0
    # the library riders: rank 0 alone drives every device (here a CPU stand-in) while the
    # other ranks wait on the gloo idle group; both reach the line with all N devices
    for name in ("rowshard512_lib", "k64_lib"):
        assert r[name]["devices"] == [0, 1, 2, 3] and r[name]["value"] > 0


def test_step_ceiling_fields():
    """roofline_step: the square's compressions at the probe's SHA-256 rate plus the
    transform probe, against the measured time per square (bench.step_ceiling)."""
    sys.path.insert(0, ROOT)
    import bench
    probe = {"sha256_gcomp_per_s": 28.0, "rs_transform_us_k128": 7.5}
    s = bench.step_ceiling(128, probe, 45e-6)
    nmt = (60 * 128 * 128 + 4 * 128 - 2) / 28e9 * 1e6
    assert abs(s["nmt_us"] - nmt) < 1e-9 and s["rs_transform_us"] == 7.5
    assert abs(s["peak"] - (nmt + 7.5)) < 1e-9 and abs(s["achieved"] - 45.0) < 1e-9
    assert abs(s["frac"] - (nmt + 7.5) / 45.0) < 1e-12 and s["bound"] == "valu"
    assert bench.step_ceiling(512, probe, 1e-3) is None  # no k = 512 entry in this probe
    assert bench._step_fields(512, probe, 1e-3) == {} and bench._step_fields(128, None, 1e-3) == {}
    f = bench._step_fields(128, probe, 45e-6)
    assert abs(f["step_valu_frac"] - s["frac"]) < 1e-12 and f["step_rs_transform_us"] == 7.5


def test_rs_traffic_and_achievable_mix():
    """roofline.traffic splits the committed PMC profile into read and write bytes per square
    (FETCH_SIZE doubled, WRITE_SIZE), and achievable_mix prices them at the probe's read-only
    and write-only rates (bench.achievable_mix)."""
    sys.path.insert(0, ROOT)
    import bench
    tr = bench._rs_traffic(128, 256, "eds")
    assert tr is not None and tr["bytes"] == tr["per_square"] * 256
    assert abs(tr["read_per_square"] + tr["write_per_square"] - tr["per_square"]) < 0.03 * tr["per_square"]
    assert tr["write_per_square"] > tr["read_per_square"]  # Q1..Q3 written, Q0 + Q1 read
    probe = {"hbm_read_gbps": 7000.0, "hbm_write_gbps": 5000.0}
    mix = bench.achievable_mix(tr, probe, 128)
    t = tr["read_per_square"] / 7e12 + tr["write_per_square"] / 5e12
    assert abs(mix - 2048 * 128 * 128 / t / 1e9) < 1e-6
    assert 4000 < mix < 6000
    assert bench.achievable_mix(tr, {"hbm_copy_gbps": 6000.0}, 128) is None
    assert bench.achievable_mix(None, probe, 128) is None
