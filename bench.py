"""EDS+DAH throughput on MI355X (BASELINE.json metric), one process per GPU.

A step = da.ExtendShares + da.NewDataAvailabilityHeader for a batch of independent
k x k squares already resident in HBM (RS extension to the 2k x 2k EDS, 4k NMT
roots, DAH hash), through the C ABI's device-resident entry point. Multi-GPU runs
are batch/replay mode: every rank extends its own squares, no data-path
collective (weak scaling); the barrier and max-over-ranks timing follow the driver
contract. `--gpus N` without torchrun's environment relaunches this script under
`torch.distributed.run` with N ranks (before anything touches a GPU), so
`python bench.py --gpus 8` and the driver's torchrun line run the same code.

Besides the headline number the JSON line carries:
  roofline      RS extension (both passes) vs HBM: algorithmic 2048 k^2 bytes per
                square / measured average duration (HIP events on the launch stream)
  roofline_nmt  NMT+DAH phase: SHA-256 compressions (60 k^2 + 4k - 2 per square)
                per second vs the measured SHA-256 peak of the same compression code with
                no memory traffic (and, as peak_model, the op-rate model of its mix)
  probe         same-run ceilings (cel_probe_*): SHA-256 in registers, shader clock, a
                streaming copy, and the GF(2^8) encode transform with no HBM traffic
  roofline_step the whole step per square against the VALU time of its two instruction
                streams (NMT compressions at the probe's SHA-256 rate + the transform alone)
  k512          (default --k 128 run) the same measurement on a short batch of k=512
                squares (GF(2^16)), since the metric names k=128 and k=512
  cpu_baseline  the C restatement (oracle/, SIMD + OpenMP) on a bounded sample of the
                same squares, rank 0 at N = 1 only; its DAHs also cross-check the GPU
  host_io       the PCIe-inclusive rate of the host-buffer entry point (cel_extend_batch)
                that the Go shim behind da.ExtendShares calls: EDS copied back, and
                roots + DAH only (rank 0 at N = 1; never the headline value)
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md chip table)
# SHA-256 op-mix ceiling: the compression's ISA (576 v_alignbit_b32, 241 v_add3_u32, 352
# v_bitop3_b32, 245 VOP2 per wave) priced at the dependency-free rate of each op measured
# alone on the same box as the compression itself (tools/microbench/vop3_banks.hip: 32.15T,
# 32.3T, 57.0T with conflict-free sources, 61.0T lane-ops/s) -> 28.1 G compressions/s;
# the compression chained in registers runs 29.2-29.5 G/s on that box, within 5 % of it
# (profiles/r4_sha_ceiling.txt).
SHA_MIX_CEILING = 1.0 / (576 / 32.15e12 + 241 / 32.3e12 + 352 / 57.0e12 + 245 / 61.0e12)
# Measured SHA-256 peak: the NMT kernels' compression (cel::sha256_compress) chained in
# registers on every lane, no memory traffic, 4-32 waves per SIMD: 29.1-29.6 G
# compressions/s on two boxes (tools/microbench/sha_rate.hip, profiles/r2_sha_rate.txt).
SHA_MEASURED_PEAK = 29.4e9
# The MI355X_MICROARCH.md issue model: every wave64 VALU instruction issues over 2 cycles on
# a SIMD-32; the compression is 1414 VALU per wave (ISA of the unrolled compression,
# tools/roofline_crosscheck.py) -> 1024 SIMDs x 2.4 GHz x 64 / (2 x 1414) = 55.6 G/s. The
# measured per-op rates put v_alignbit / v_add3 (58 % of the mix) at ~4.8 nominal cycles,
# hence peak_model and the measured peak below it.
SHA_GUIDE_CEILING = 1024 * 2.4e9 * 64 / (2 * 1414)
# Measured HBM traffic of the RS extension (rocprofv3 FETCH_SIZE/WRITE_SIZE passes).
# (input layout -> profile): ODS in Q0 of the EDS (in place) / separate ODS buffer.
TRAFFIC_PROFILE = {"eds": "r5_rs_traffic_inplace.json", "ods": "r1_rs_traffic.json"}


def _rs_traffic(k, batch, layout):
    """HBM bytes per RS launch pair from the committed PMC profile, scaled to `batch`
    squares (per-square traffic is batch-independent at these sizes), or None."""
    name = TRAFFIC_PROFILE[layout]
    try:
        with open(os.path.join(ROOT, "profiles", name)) as f:
            p = json.load(f)
    except (OSError, ValueError):
        return None
    if p.get("k") != k:
        return None
    sq = p["squares"]
    read = 2 * sum(p["fetch_kib_raw"].values()) * 1024 / sq  # FETCH_SIZE doubled (gfx950)
    write = sum(p["write_kib"].values()) * 1024 / sq
    return {"bytes": p["bytes_per_square"] * batch, "per_square": p["bytes_per_square"],
            "read_per_square": read, "write_per_square": write,
            "vs_algorithmic": p["bytes_per_square"] / p["algorithmic_bytes_per_square"],
            "source": f"profiles/{name} (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, KiB)"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--k", type=int, default=128, help="original square width")
    ap.add_argument("--batch", type=int, default=256, help="squares per step per GPU")
    ap.add_argument("--distinct", type=int, default=4, help="distinct synthetic squares per GPU")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--input", default="eds", choices=["eds", "ods"],
                    help="eds: the upload places each ODS in Q0 of its EDS buffer and the extension "
                         "reads it in place; ods: separate contiguous ODS buffer, the row pass copies Q0")
    ap.add_argument("--phase-reps", type=int, default=10)
    ap.add_argument("--inflight", type=int, default=4,
                    help="batches in flight: steps go round-robin over this many batches, each with its own "
                         "buffers and stream (independent blocks back to back, CEL_FLAG_CALLER_STREAM); "
                         "1 = one batch, each step split in two chunks on the library's internal streams")
    ap.add_argument("--k512-batch", type=int, default=32,
                    help="with --k 128: k=512 squares per step per GPU of the companion line (0 = off)")
    ap.add_argument("--k512-steps", type=int, default=5)
    ap.add_argument("--no-riders", action="store_true",
                    help="with --k 128: skip the config-4 (k64) and config-3 (rowshard512) riders")
    ap.add_argument("--rider-steps", type=int, default=5)
    ap.add_argument("--depth", type=int, default=4,
                    help="row-sharded square (--mode sharded and the rowshard512 rider): squares in flight "
                         "per step of the pipelined measurement (the plain value keeps one in flight)")
    ap.add_argument("--rehearse", action="store_true",
                    help="multi-rank rehearsal on a one-GPU box: every rank on cuda:0, gloo instead of RCCL "
                         "(collectives staged through host memory); exercises the N-rank code path, its "
                         "numbers are not multi-GPU measurements")
    ap.add_argument("--lib-devices", type=int, default=1,
                    help="--mode libriders: devices the one process drives (rank 0's child in an N-GPU run)")
    ap.add_argument("--mode", default="batch", choices=["batch", "sharded", "repair", "distcheck", "libriders"],
                    help="batch: independent squares per GPU (configs 2, 4); sharded: one square "
                         "row-sharded over the ranks (config 3); repair: rsmt2d Repair (config 5); "
                         "distcheck: the launcher / rendezvous / timing contract on CPU ranks over gloo "
                         "(no GPU work; used by the CPU tests)")
    ap.add_argument("--no-host-io", action="store_true", help="skip the host_io (PCIe-inclusive) measurement")
    ap.add_argument("--no-power", action="store_true", help="skip the rocm-smi power / clock reading of the phases")
    ap.add_argument("--repair-p", type=float, default=0.55, help="repair mode: cell survival probability")
    ap.add_argument("--repair-input", default="device", choices=["device", "host"],
                    help="repair mode: EDS resident in HBM (cel_dev_repair) or host buffers (cel_repair, PCIe)")
    return ap.parse_args()


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch(a):
    """--gpus N > 1 without torchrun's environment: run this script under
    torch.distributed.run with N ranks (one per GPU, rendezvous on 127.0.0.1) as a child
    process and return its exit code. Nothing has touched a GPU in this process."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", str(max(1, (os.cpu_count() or 1) // a.gpus)))
    return subprocess.call(cmd, env=env)


def _dist_env():
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def run_distcheck(a):
    """The multi-rank contract without a GPU: gloo rendezvous, W untimed + K timed steps
    bracketed by barriers, MAX over ranks, one JSON line from rank 0 with n_gpus = world.
    A step is a fixed CPU hash of a rank-local buffer (a stand-in for the batch step)."""
    import hashlib
    import torch.distributed as dist
    global IDLE_GROUP
    world, rank, _ = _dist_env()
    if world > 1:
        dist.init_process_group("gloo")
        IDLE_GROUP = dist.new_group(backend="gloo")
    buf = np.random.default_rng(rank).integers(0, 256, 1 << 20, dtype=np.uint8).tobytes()

    def step():
        hashlib.sha256(buf).digest()

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(a.warmup):
        step()
    barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # the riders' assembly with CPU stand-ins: the k64 split and, for the row-sharded
    # square, the same all_to_all_single shape (k = 64 here) over gloo, timed the same way
    riders = {}
    if not a.no_riders:
        riders["k64"] = _k64_fields(world, elapsed, a.steps)
        k = 64
        per_peer = 2 * k * k * 512 // (world * world)
        inp = torch.full((world * per_peer,), rank, dtype=torch.uint8)
        out = torch.empty_like(inp)
        t_a2a = 0.0
        if world > 1:
            barrier()
            t1 = time.perf_counter()
            dist.all_to_all_single(out, inp)
            t_a2a = time.perf_counter() - t1
            assert all(int(out[h * per_peer]) == h for h in range(world))
            t = torch.tensor([t_a2a], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            t_a2a = float(t.item())
        riders["rowshard512"] = _rowshard_fields(k, world, elapsed, a.steps, t_a2a)

        # the library riders' assembly: rank 0 alone runs them (a CPU stand-in here) while
        # the other ranks wait on the gloo idle group
        def stand_in(name):
            def fn():
                t1 = time.perf_counter()
                for _ in range(a.steps):
                    step()
                return {"driver": "library (CPU stand-in)", "devices": list(range(world)),
                        "value": a.steps / (time.perf_counter() - t1), "unit": "steps/s", "name": name}
            return fn
        _library_riders(riders, a, world, rank, dist if world > 1 else None,
                        {"rowshard512_lib": stand_in("rowshard512_lib"), "k64_lib": stand_in("k64_lib")})
    if rank == 0:
        print(json.dumps({"metric": "distcheck steps/sec", "value": world * a.steps / elapsed, "unit": "steps/s",
                          "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
                          "ms_per_step": elapsed / a.steps * 1e3, "higher_is_better": True, "scaling": "weak",
                          "vs_baseline": None, "dtype": "u8", "data": "synthetic (CPU stand-in step, gloo)",
                          "config": {"workload": "launcher / rendezvous / timing contract check",
                                     "parallelism": f"batch{world}"}, **riders}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def _cpu_cores():
    cores = os.cpu_count() or 1
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        pass
    # the GPU box grants a CPU share (OMP_NUM_THREADS) far below the visible core count
    return min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))


def cpu_info():
    """The host the CPU baseline ran on (every report prints the core count
    and the CPU model): model name, the machine's logical CPUs and physical cores (distinct
    (package, core id) pairs in /proc/cpuinfo), the CPUs this process may run on and how many
    physical cores they span, and the thread count the baseline used (the granted share)."""
    model, cpu_core, cur = None, {}, {}
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                key, _, val = line.partition(":")
                key, val = key.strip(), val.strip()
                if key == "model name" and model is None:
                    model = val
                if key in ("processor", "physical id", "core id"):
                    cur[key] = val
                if not line.strip() and "processor" in cur:
                    cpu_core[int(cur["processor"])] = (cur.get("physical id", "0"), cur.get("core id", cur["processor"]))
                    cur = {}
        if "processor" in cur:
            cpu_core[int(cur["processor"])] = (cur.get("physical id", "0"), cur.get("core id", cur["processor"]))
    except OSError:
        pass
    try:
        allowed = sorted(os.sched_getaffinity(0))
    except AttributeError:
        allowed = list(range(os.cpu_count() or 1))
    return {"cpu_model": model, "logical_cpus": os.cpu_count(),
            "physical_cores": len(set(cpu_core.values())) or None,
            "allowed_cpus": len(allowed),
            "allowed_physical_cores": len({cpu_core[c] for c in allowed if c in cpu_core}) or None,
            "granted_threads": _cpu_cores()}


def run_sharded(a):
    """Config 3: one k x k square per step, row-sharded over all ranks (strong scaling).
    Rank r row-encodes k/N rows straight into the all-to-all layout, one RCCL
    all_to_all_single transposes them into column slabs, each rank column-encodes and
    hashes its slab, one all-gather of 96-byte records and a combine give the roots
    and the DAH on every rank. At N = 1 the same schedule runs without collectives."""
    world, rank, local = _dist_env()
    local = _rank_device(local)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    from celestia_eds.sharded import LocalComm, run_pipelined
    dist = None
    if world > 1:
        dist = _init_dist(dev)
    k = a.k
    sqs = _sharded_squares(k, world, rank, local, max(1, a.depth))
    sq = sqs[0]
    steps = sq.steps
    comm = _comm() if dist is not None else None

    def step():
        if comm is not None:
            sq.run(comm)
        else:
            LocalComm.run([sq])

    def barrier():
        if dist is not None:
            dist.barrier()

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = _max_over_ranks(time.perf_counter() - t0, dist, dev)
    sq.check_status()
    piped = None
    if a.depth > 1:
        e_p = _timed_steps(lambda: run_pipelined(sqs, comm), a.steps, a.warmup, barrier, dist, dev)
        for s in sqs:
            s.check_status()
        piped = {"squares_in_flight": a.depth, "value": a.depth * a.steps / e_p, "unit": "squares/s",
                 "ms_per_square": e_p / (a.depth * a.steps) * 1e3}
    # rank-local phase timing (HIP events on the launch stream of the device steps)
    cur = steps.stream

    def timed(fn, reps):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        fn()
        e0.record(cur)
        for _ in range(reps):
            fn()
        e1.record(cur)
        e1.synchronize()
        return e0.elapsed_time(e1) / reps / 1e3

    with sq.scope():
        t_rows = timed(sq.phase_rows, a.phase_reps)
        t_cols = timed(sq.phase_cols, a.phase_reps)
    value = a.steps / elapsed
    rows_bytes = 1024 * k * k // world  # read k/N ODS rows + write their k parity shards
    result = {
        "metric": "EDS+DAH squares/sec (k=%d, row-sharded)" % k,
        "value": value,
        "unit": "squares/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": elapsed / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (testfactory-style sorted random namespaced shares)",
        "ods_gbps": value * 512 * k * k / 1e9,
        "config": {
            "workload": f"k={k} ODS -> EDS + 4k NMT roots + DAH, one square row-sharded over {world} GPU(s)",
            "k": k,
            "share_size": 512,
            "field": "GF(2^16)",
            "parallelism": f"rowshard{world}",
            "collectives": "all_to_all_single (data), one all_gather (records)" if world > 1
            else "none (N=1)",
        },
        "roofline": {
            "bound": "hbm",
            "kernel": "k_rs_gf16x (row pass of this rank, blocked all-to-all layout)",
            "achieved": rows_bytes / t_rows / 1e9,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": rows_bytes / t_rows / 1e9 / HBM_PEAK_GBS,
            "traffic": None,
            "avg_launch_us": t_rows * 1e6,
        },
        "phase_us": {"rows": t_rows * 1e6, "cols_and_commit": t_cols * 1e6},
        "pipelined": piped,
    }
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def run_repair(a):
    """Config 5: rsmt2d Repair of a k x k EDS from a random sample (cells kept with
    probability --repair-p, seed 7): crossword erasure decode on the device, re-encode
    checks and root re-verification. --repair-input device (default): the damaged EDS
    resident in HBM (cel_dev_repair); the fresh damaged copy each step needs is made
    before the step's clock starts. host: host buffers in and out (cel_repair), PCIe
    copies included. Single rank.
    roofline: the decoder alone (cel_dev_decode over the row pass's axes of the same
    mask: k_rs_decode_axis, register-resident GF(2^8); k >= 256: k_rs_decode_gf16, bit planes
    in LDS), algorithmic bytes = every shard of
    every decoded axis read once + every missing shard written once, against HBM; the
    decoder is VALU-bound (~15K VALU per wave, one wave per SIMD at 239 axes), so the
    fraction says how far from streaming."""
    torch.cuda.set_device(0)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from celestia_eds import default_context
    from celestia_eds.rsmt2d import ExtendedDataSquare
    from celestia_eds.testfactory import random_ods
    oracle.set_simd(True)
    oracle.set_threads(_cpu_cores())
    k, w = a.k, 2 * a.k
    eds, rr, cr, _ = oracle.extend_and_commit(random_ods(k, 7))
    present = (np.random.default_rng(7).random((w, w)) < a.repair_p).astype(np.uint8)
    damaged = eds.copy()
    damaged[present == 0] = 0
    ctx = default_context(0)
    rrl, crl = [r.tobytes() for r in rr], [c.tobytes() for c in cr]
    import ctypes
    P = lambda x: x.ctypes.data_as(ctypes.c_void_p)

    if a.repair_input == "host":
        def prepare():
            return ExtendedDataSquare(damaged.copy(), ctx=ctx)

        def once(sq):
            sq.Repair(rrl, crl, present=present)
            return sq.cells
    else:
        d_damaged = torch.from_numpy(damaged).cuda()
        d_work = torch.empty_like(d_damaged)
        rra, cra = np.ascontiguousarray(rr), np.ascontiguousarray(cr)

        def prepare():
            d_work.copy_(d_damaged)  # 32 MiB D2D at k = 128, outside the step's clock
            torch.cuda.synchronize()
            return present.copy()

        def once(pres):
            ctx.check(ctx.lib.cel_dev_repair(ctx.handle, ctypes.c_void_p(d_work.data_ptr()), P(pres), k, P(rra),
                                             P(cra), None, None, None, None))
            return d_work

    for _ in range(a.warmup):
        once(prepare())
    torch.cuda.synchronize()
    elapsed = 0.0
    for _ in range(a.steps):
        arg = prepare()
        t0 = time.perf_counter()
        out = once(arg)  # cel_dev_repair / cel_repair are synchronous
        torch.cuda.synchronize()
        elapsed += time.perf_counter() - t0
    cells = out if isinstance(out, np.ndarray) else out.cpu().numpy()
    assert np.array_equal(cells, eds), "repaired EDS differs"
    # decode roofline: the row pass's decode (every row with >= k and < 2k known cells)
    rows = [i for i in range(w) if k <= int(present[i].sum()) < w]
    dense = torch.from_numpy(np.ascontiguousarray(damaged[rows])).cuda()
    dmask = torch.from_numpy(np.ascontiguousarray(present[rows])).cuda()
    scratch = torch.empty_like(dense)
    stream = torch.cuda.Stream()
    sp = ctypes.c_void_p(stream.cuda_stream)

    def decode():
        ctx.check(ctx.lib.cel_dev_decode(ctx.handle, ctypes.c_void_p(scratch.data_ptr()),
                                         ctypes.c_void_p(dmask.data_ptr()), len(rows), k, 512, sp))

    reps = max(3, a.phase_reps)
    scratch.copy_(dense)
    torch.cuda.synchronize()
    decode()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        decode()  # re-decoding a decoded axis repeats the same work
    e1.record(stream)
    e1.synchronize()
    t_dec = e0.elapsed_time(e1) / reps / 1e3
    missing = int((present[rows] == 0).sum())
    dec_bytes = len(rows) * w * 512 + missing * 512
    # CPU baseline: the crossword restatement with Leopard's O(n log n) decoder, one repair
    # per thread over the granted cores (independent damaged squares), bounded sample
    rc, fixed, _, _ = oracle.repair(damaged, present, rr, cr)
    assert rc == 0 and np.array_equal(fixed, eds)
    cores = _cpu_cores()
    oracle.set_threads(1)
    t1 = time.perf_counter()
    oracle.repair(damaged, present, rr, cr)
    t_one = time.perf_counter() - t1
    oracle.set_threads(cores)
    n_cpu, t_cpu = 0, 0.0
    while t_cpu < min(a.cpu_seconds, 10.0) or n_cpu == 0:
        t1 = time.perf_counter()
        st = oracle.repair_many(damaged, present, rr, cr, 2 * cores)
        t_cpu += time.perf_counter() - t1
        n_cpu += len(st)
        assert (st == 0).all()
    byz = measure_byzantine_repair(ctx, eds, rr, cr, present, k) if a.repair_input == "device" else None
    value = a.steps / elapsed
    print(json.dumps({
        "metric": "rsmt2d Repair squares/sec (k=%d, p=%.2f)" % (k, a.repair_p),
        "value": value, "unit": "squares/s", "n_gpus": 1, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": elapsed / a.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8", "data": "synthetic (testfactory-style ODS, random survival mask)",
        "config": {"workload": f"Repair k={k} EDS from {present.mean():.3f} of its cells "
                               + ("(host buffers, PCIe included)" if a.repair_input == "host"
                                  else "(EDS resident in HBM; the damaged-copy restore runs before each step's "
                                       "clock)"),
                   "k": k, "parallelism": "single"},
        "roofline": {"bound": "hbm",
                     "kernel": ("k_rs_decode_axis" if k <= 128 else "k_rs_decode_gf16 (bit planes)")
                     + " (cel_dev_decode, the row pass's axes)",
                     "achieved": dec_bytes / t_dec / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": dec_bytes / t_dec / 1e9 / HBM_PEAK_GBS, "traffic": None,
                     "avg_launch_us": t_dec * 1e6, "axes": len(rows),
                     "bytes_per_launch": dec_bytes,
                     "bytes_basis": "every shard of each decoded axis read once + each missing shard written once"},
        "cpu_baseline": {"value": n_cpu / t_cpu, "unit": "squares/s", "cores": cores,
                         "kind": "port",
                         "sample": f"{n_cpu} repairs of the same damaged square, one per thread (C restatement: "
                                   "crossword sweeps, Leopard FWHT decoder, re-encode and root checks)",
                         "one_thread_ms_per_repair": t_one * 1e3, **cpu_info()},
        "byzantine": byz,
    }), flush=True)


def measure_byzantine_repair(ctx, eds, rr, cr, present, k, reps=3):
    """Config 5 (v): the same mask with one corrupted known cell whose row and column are
    both incomplete, so a decode meets it: the pass-parallel schedule finds a failing check
    and the square is replayed in rsmt2d's sweep order. Time per repair
    (EDS resident, damaged copy restored outside the clock) and the reported axis."""
    import ctypes
    w = 2 * k
    pres = present.copy()
    r, c = 40, 77
    pres[r, c] = 1
    pres[r, 3] = pres[200, c] = 0
    bad = eds.copy()
    bad[r, c, 300] ^= 0x21
    bad[pres == 0] = 0
    d_bad = torch.from_numpy(bad).cuda()
    d_work = torch.empty_like(d_bad)
    rra, cra = np.ascontiguousarray(rr), np.ascontiguousarray(cr)
    P = lambda x: x.ctypes.data_as(ctypes.c_void_p)
    ts, axis = [], None
    for i in range(reps + 1):
        d_work.copy_(d_bad)
        torch.cuda.synchronize()
        m = pres.copy()
        ba, bi = ctypes.c_int32(-1), ctypes.c_int32(-1)
        t0 = time.perf_counter()
        st = ctx.lib.cel_dev_repair(ctx.handle, ctypes.c_void_p(d_work.data_ptr()), P(m), k, P(rra), P(cra),
                                    ctypes.byref(ba), ctypes.byref(bi), None, None)
        if i:
            ts.append(time.perf_counter() - t0)
        axis = (ba.value, bi.value)
        assert st == 7, st  # CEL_EBYZANTINE
    del d_bad, d_work
    return {"workload": f"the same k={k} mask with one corrupted known cell (rsmt2d sweep-order replay)",
            "ms_per_repair": sorted(ts)[len(ts) // 2] * 1e3, "status": "ErrByzantineData",
            "axis": axis[0], "index": axis[1]}


def _oracle():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    oracle.set_simd(True)
    return oracle


def cpu_component_rates(oracle, k):
    """Single-thread rates of the CPU restatement's pieces (buffers reused, warm):
    RS extension (GF(2^8) GFNI / GF(2^16) AVX2 Leopard) in algorithmic GB/s, the NMT roots
    in SHA-256 compressions/s (the reference's count: each cell hashed once per axis,
    96 k^2 - 12 k per square), and the Leopard decode of one 2k-shard axis with k erased."""
    oracle.set_threads(1)
    lib, P = oracle.lib(), oracle._p
    rng = np.random.default_rng(1)
    ods = rng.integers(0, 256, (k, k, 512), dtype=np.uint8)
    eds = np.ones((2 * k, 2 * k, 512), np.uint8)
    rr = np.zeros((2 * k, 90), np.uint8)
    cr = rr.copy()
    lib.orc_extend(P(ods), k, 512, P(eds))

    def best(fn, reps=3):
        t = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            t.append(time.perf_counter() - t0)
        return min(t)

    t_rs = best(lambda: lib.orc_extend(P(ods), k, 512, P(eds)))
    t_nmt = best(lambda: lib.orc_roots(P(eds), k, 512, P(rr), P(cr), 0, None))
    axis = np.ascontiguousarray(eds[0])
    present = np.ones(2 * k, np.uint8)
    present[rng.choice(2 * k, k, replace=False)] = 0
    damaged = np.where(present[:, None] == 1, axis, 0).astype(np.uint8)
    t_dec = best(lambda: oracle.rs_decode(damaged, present), reps=5)
    return {"rs_extend_gbps": 2048 * k * k / t_rs / 1e9, "sha_mcompressions_per_s": (96 * k * k - 12 * k) / t_nmt / 1e6,
            "decode_us_per_axis": t_dec * 1e6, "threads": 1}


def cpu_baseline_batch(k, distinct, dah_dev, seconds):
    """The CPU restatement over the host cores the process is granted: independent squares
    on independent threads (orc_extend_commit_many), batches of 2 x cores squares until
    `seconds` of CPU wall time, DAHs checked against the device's; plus single-thread
    component rates. Returns (cpu_baseline dict, parity)."""
    oracle = _oracle()
    rates = cpu_component_rates(oracle, k)
    cores = _cpu_cores()
    oracle.set_threads(cores)
    nd = len(distinct)
    n = max(2 * cores, nd)
    idx = [i % nd for i in range(n)]
    batch = np.stack([distinct[i] for i in idx])
    oracle.extend_commit_many(batch[:cores])  # warm: threads, pages, tables
    done, t_cpu, parity = 0, 0.0, True
    while t_cpu < seconds or done == 0:
        t0 = time.perf_counter()
        dahs = oracle.extend_commit_many(batch)
        t_cpu += time.perf_counter() - t0
        done += n
        parity &= all(dahs[j].tobytes() == dah_dev[idx[j]].tobytes() for j in range(n))
    per_sq = 1.0 / (rates["rs_extend_gbps"] * 1e9 / (2048 * k * k)) + \
        (96 * k * k - 12 * k) / (rates["sha_mcompressions_per_s"] * 1e6)
    return {
        "value": done / t_cpu,
        "unit": "squares/s",
        "cores": cores,
        "kind": "port",
        "sample": f"{done} k={k} squares ({n} per call, one square per thread; extend + roots + DAH, "
                  f"GFNI/AVX2 Leopard + SHA-NI C restatement, reference tree count)",
        "component_rates_1thread": rates,
        "predicted_from_components": cores / per_sq,
        **cpu_info(),
    }, parity


XGMI_LINK_GBS = 153.0  # one xGMI link, per direction


def _k64_fields(world, elapsed, steps, t_ext=None, t_com=None, B=None):
    """Config 4 rider: 1024 independent k=64 squares in total, 1024/N per rank."""
    f = {"workload": "config 4: 1024 independent k=64 squares in total, 1024/N per GPU (batch replay)",
         "value": 1024 * steps / elapsed, "unit": "squares/s", "n_gpus": world, "steps": steps,
         "ms_per_step": elapsed / steps * 1e3, "squares_per_step_per_gpu": 1024 // world, "scaling": "strong"}
    if t_ext is not None:
        f["rs_frac_hbm"] = 2048 * 64 * 64 * B / t_ext / 1e9 / HBM_PEAK_GBS
        f["nmt_frac_sha_peak"] = (60 * 64 * 64 + 4 * 64 - 2) * B / t_com / SHA_MEASURED_PEAK
    return f


def _rowshard_fields(k, world, elapsed, steps, t_a2a):
    """Config 3 rider: one k x k square row-sharded over the N ranks, with the all-to-all
    alone next to SURVEY §8e's one-link estimate (bytes per peer / 153 GB/s)."""
    per_peer = 2 * k * k * 512 // (world * world)  # (k/N rows) x (2k/N columns) x 512 B
    return {"workload": f"config 3: one k={k} square row-sharded over {world} GPU(s), one all_to_all_single "
                        "(column slabs) + one record all_gather",
            "value": steps / elapsed, "unit": "squares/s", "n_gpus": world, "steps": steps,
            "ms_per_step": elapsed / steps * 1e3, "scaling": "strong",
            "a2a_us": t_a2a * 1e6 if world > 1 else None,
            "a2a_bytes_per_peer": per_peer if world > 1 else 0,
            "a2a_gbps_per_peer": per_peer / t_a2a / 1e9 if world > 1 else None,
            "a2a_survey_estimate_us": per_peer / (XGMI_LINK_GBS * 1e9) * 1e6 if world > 1 else None}


REHEARSE = False  # set by main() from --rehearse


def _rank_device(local):
    return 0 if REHEARSE else local


IDLE_GROUP = None  # gloo group: ranks wait here (no GPU work) while rank 0 drives every GPU


def _init_dist(dev):
    global IDLE_GROUP
    import torch.distributed as dist
    if REHEARSE:
        dist.init_process_group("gloo")
    else:
        dist.init_process_group("nccl", device_id=dev)
    IDLE_GROUP = dist.new_group(backend="gloo")
    return dist


def _comm():
    from celestia_eds.sharded import StagedComm, TorchComm
    return StagedComm() if REHEARSE else TorchComm()


def _max_over_ranks(x, dist, dev):
    if dist is None:
        return x
    t = torch.tensor([x], dtype=torch.float64, device="cpu" if REHEARSE else dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _timed_steps(step, steps, warmup, barrier, dist, dev):
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    return _max_over_ranks(time.perf_counter() - t0, dist, dev)


def _sharded_squares(k, world, rank, local, depth):
    """`depth` independent row-sharded squares of this rank, each with its own device
    steps (stream and workspace), loaded with distinct synthetic ODS rows."""
    from celestia_eds import default_context
    from celestia_eds.sharded import DeviceSteps, ShardedSquare
    from celestia_eds.testfactory import random_ods
    ctx = default_context(local)
    sqs = []
    for d in range(depth):
        sq = ShardedSquare(k, rank, world, DeviceSteps(ctx, local))
        lo, hi = sq.row_range()
        sq.ods_rows.copy_(torch.from_numpy(np.ascontiguousarray(random_ods(k, 512 + d)[lo:hi])))
        sqs.append(sq)
    return sqs


def measure_rowshard(k, world, rank, local, dist, dev, steps, warmup, barrier, depth=2):
    """The run_sharded schedule as a rider of the batch line: full steps (barrier-bracketed,
    max over ranks) with one square in flight, the same with `depth` squares in flight
    (sharded.run_pipelined), then the all-to-all alone (median of 5, max over ranks)."""
    from celestia_eds.sharded import LocalComm, run_pipelined
    comm = _comm() if dist is not None else None
    sqs = _sharded_squares(k, world, rank, local, max(1, depth))
    sq = sqs[0]

    def step():
        if comm is not None:
            sq.run(comm)
        else:
            LocalComm.run([sq])

    elapsed = _timed_steps(step, steps, warmup, barrier, dist, dev)
    sq.check_status()
    piped = None
    if depth > 1:
        e_p = _timed_steps(lambda: run_pipelined(sqs, comm), steps, warmup, barrier, dist, dev)
        for s in sqs:
            s.check_status()
        piped = {"squares_in_flight": depth, "value": depth * steps / e_p, "unit": "squares/s",
                 "ms_per_square": e_p / (depth * steps) * 1e3}
    t_a2a = 0.0
    if comm is not None:
        ts = []
        for _ in range(5):
            torch.cuda.synchronize()
            barrier()
            t1 = time.perf_counter()
            with sq.scope():
                sq.exchange(comm)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t1)
        t_a2a = _max_over_ranks(sorted(ts)[2], dist, dev)
    del sq, sqs
    f = _rowshard_fields(k, world, elapsed, steps, t_a2a)
    f["latency_ms"] = elapsed / steps * 1e3
    if piped:
        f["pipelined"] = piped
    return f


def measure_probe(ctx):
    """Same-run ceilings on this rank's device (cel_probe_sha256 / cel_probe_hbm_copy): the
    SHA-256 compression in registers (G/s) with the sustained shader clock over that launch,
    and a streaming copy's read + write GB/s. The line's fractions use them beside the
    fixed constants, so a box with another clock or HBM shows it in its own denominators."""
    from celestia_eds.multi import probe
    return probe(ctx, 4 << 30)


def achievable_mix(traffic, probe, k):
    """The RS extension's own HBM ceiling, as algorithmic GB/s: its measured read and write
    bytes per square (`traffic`, from the PMC profile) at the box's read-only and write-only
    stream rates (`probe`: HBM writes stream ~25 % slower than reads), i.e. the rate the
    extension would reach if its HBM time were the whole launch. None without the inputs."""
    if not traffic or not probe or not probe.get("hbm_read_gbps") or not probe.get("hbm_write_gbps"):
        return None
    t_sq = traffic["read_per_square"] / (probe["hbm_read_gbps"] * 1e9) + \
        traffic["write_per_square"] / (probe["hbm_write_gbps"] * 1e9)
    return 2048 * k * k / t_sq / 1e9


def step_ceiling(k, probe, secs_per_square):
    """The whole step against the VALU time of its two instruction streams, both same-run:
    the square's NMT compressions at the SHA-256 probe's rate plus its GF(2^8) extension's
    transform alone (cel_probe_rs_transform). Both halves are VALU-issue bound, so their sum
    is the step's floor with these kernels; frac = that floor / the measured time per square
    on one GPU (overlap of the RS's memory time with the other batches' hashing is what
    lets it reach 1)."""
    rs_us = probe.get(f"rs_transform_us_k{k}")
    if rs_us is None:
        return None
    nmt_us = (60 * k * k + 4 * k - 2) / (probe["sha256_gcomp_per_s"] * 1e9) * 1e6
    meas_us = secs_per_square * 1e6
    return {
        "bound": "valu",
        "unit": "us per square per GPU",
        "nmt_us": nmt_us,
        "rs_transform_us": rs_us,
        "peak": nmt_us + rs_us,
        "achieved": meas_us,
        "frac": (nmt_us + rs_us) / meas_us,
        "basis": "(60k^2 + 4k - 2) compressions / cel_probe_sha256 + cel_probe_rs_transform (the encode "
                 "tile with no HBM traffic, 3k axis encodes); both kernels' time is VALU issue",
    }


def _step_fields(k, probe, secs_per_square):
    """A rider's step against its VALU floor (step_ceiling), as flat fields; none without a
    probe of that width."""
    step = step_ceiling(k, probe, secs_per_square) if probe else None
    if not step:
        return {}
    return {"step_valu_us": step["peak"], "step_rs_transform_us": step["rs_transform_us"],
            "step_valu_frac": step["frac"]}


def _lib_devices(world):
    """The devices rank 0 drives in one process for the library riders: one per rank (all on
    cuda:0 in a --rehearse run, where the plan's transport is device copies)."""
    return [_rank_device(r) for r in range(world)]


def _lib_ctxs(devs):
    from celestia_eds import Context, default_context
    return [default_context(d) for d in devs]


def measure_rowshard_lib(k, world, steps, warmup, depth):
    """Config 3 through the library (cel_shard_plan_*): this one process drives the square
    over all N devices, the all-to-all and record all-gather issued by the library over RCCL
    (ncclCommInitAll communicators, grouped ncclSend / ncclRecv, ncclAllGather). One square in
    flight (run + wait: the latency of cel_extend_sharded minus the PCIe upload), then `depth`
    plans in flight (own streams and communicators each). The ODS rows are resident (uploaded
    once before the clock); wait() brings back the roots, the DAH and the status."""
    from celestia_eds.multi import ShardPlan
    from celestia_eds.testfactory import random_ods
    devs = _lib_devices(world)
    ctxs = _lib_ctxs(devs)
    plans = [ShardPlan(ctxs, k) for _ in range(max(1, depth))]
    for i, p in enumerate(plans):
        p.upload(random_ods(k, 512 + i))
    p0 = plans[0]

    def one():
        p0.run()
        p0.wait()

    def piped():
        for p in plans:
            p.run()
        for p in plans:
            p.wait()

    def clock(fn, n):
        for _ in range(warmup):
            fn()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        return time.perf_counter() - t0

    t1 = clock(one, steps)
    tp = clock(piped, steps)
    transport, note = p0.transport, p0.note
    try:
        a2a_us = p0.time_exchange(10)  # the all-to-all alone (None at one rank in place)
    except Exception as e:  # noqa: BLE001  (the rider's throughput stands without it)
        print(f"bench: exchange timing failed: {e!r}", file=sys.stderr, flush=True)
        a2a_us = None
    for p in plans:
        p.close()
    n = len(devs)
    per_peer = 2 * k * k * 512 // (n * n)  # (k/N rows) x (2k/N columns) x 512 B
    return {"workload": f"config 3: one k={k} square row-sharded over {n} GPU(s) by ONE process through "
                        "the C ABI (cel_shard_plan_*: in-library RCCL all-to-all + all-gather)",
            "driver": "library", "transport": transport, "transport_note": note or None, "devices": devs,
            "a2a_us": a2a_us, "a2a_bytes_per_peer": per_peer if a2a_us else 0,
            "a2a_gbps_per_peer": per_peer / (a2a_us * 1e-6) / 1e9 if a2a_us else None,
            "a2a_survey_estimate_us": per_peer / (XGMI_LINK_GBS * 1e9) * 1e6 if a2a_us else None,
            "value": steps / t1, "unit": "squares/s", "latency_ms": t1 / steps * 1e3, "steps": steps,
            "scaling": "strong",
            "pipelined": {"squares_in_flight": len(plans), "value": len(plans) * steps / tp, "unit": "squares/s",
                          "ms_per_square": tp / (len(plans) * steps) * 1e3}}


def measure_k64_lib(world, steps, warmup, inflight):
    """Config 4 through the library from ONE process: 1024 k=64 squares resident in HBM, 1024/N
    per device, every device's batches enqueued by this thread (cel_dev_extend_batch on one
    ctx per device, CEL_FLAG_CALLER_STREAM, `inflight` batches per device); the clock brackets
    every device's synchronize."""
    from celestia_eds.device import SquareBatch
    from celestia_eds.testfactory import random_ods
    devs = _lib_devices(world)
    ctxs = _lib_ctxs(devs)
    B = 1024 // len(devs)
    distinct = [random_ods(64, 7000 + i) for i in range(4)]
    host = torch.from_numpy(np.stack([distinct[i % 4] for i in range(B)]))
    sbs = []
    for d, c in zip(devs, ctxs):
        mine = []
        for _ in range(max(1, inflight)):
            sb = SquareBatch(B, 64, device=d, ctx=c, ods_in_eds=True)
            sb.load_ods(host)
            mine.append(sb)
        sbs.append(mine)
    del host

    def sync():
        for d in sorted(set(devs)):
            torch.cuda.synchronize(d)

    piped = inflight > 1
    for i in range(warmup):
        for mine in sbs:
            mine[i % len(mine)].extend_and_commit(caller_stream=piped)
    sync()
    t0 = time.perf_counter()
    for i in range(steps):
        for mine in sbs:
            mine[i % len(mine)].extend_and_commit(caller_stream=piped)
    sync()
    el = time.perf_counter() - t0
    for mine in sbs:
        for sb in mine:
            assert (sb.status.cpu().numpy() == 0).all()
    del sbs
    return {"workload": f"config 4: 1024 independent k=64 squares, {B} per GPU on {len(devs)} GPU(s), all "
                        "enqueued by ONE process through the C ABI (cel_dev_extend_batch per device ctx)",
            "driver": "library", "devices": devs, "value": 1024 * steps / el, "unit": "squares/s",
            "ms_per_step": el / steps * 1e3, "steps": steps, "squares_per_step_per_gpu": B, "scaling": "strong"}


LIB_RIDER_TIMEOUT_S = 180


def run_libriders(a):
    """--mode libriders: the library riders in a process of their own (rank 0's child in the
    N-GPU line): one process, every device of the job, RCCL inside the library. Prints one
    JSON object {rider name: fields}."""
    global REHEARSE
    REHEARSE = a.rehearse
    world = a.lib_devices
    out = {}
    torch.cuda.set_device(0)
    _rider(out, "rowshard512_lib", lambda: measure_rowshard_lib(512, world, a.rider_steps, 2, a.depth))
    if world > 1:
        _rider(out, "k64_lib", lambda: measure_k64_lib(world, a.rider_steps, 2, a.inflight))
    print(json.dumps(out), flush=True)


def _spawn_libriders(a, world):
    """The library riders in a child process with a time limit, so a hang there (RCCL
    communicator setup over N devices, say) cannot take the headline line with it; rank 0's
    own GPU state is not shared with the child."""
    cmd = [sys.executable, os.path.abspath(__file__), "--mode", "libriders", "--lib-devices", str(world),
           "--rider-steps", str(a.rider_steps), "--depth", str(a.depth), "--inflight", str(a.inflight)]
    if a.rehearse:
        cmd.append("--rehearse")
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "GROUP_RANK",
                                                          "LOCAL_WORLD_SIZE", "ROLE_RANK", "ROLE_WORLD_SIZE")}
    try:
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=LIB_RIDER_TIMEOUT_S, env=env)
    except subprocess.TimeoutExpired:
        err = {"error": f"library riders timed out after {LIB_RIDER_TIMEOUT_S} s"}
        return {"rowshard512_lib": err, "k64_lib": err} if world > 1 else {"rowshard512_lib": err}
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    if p.returncode != 0 or not lines:
        err = {"error": f"library riders exited {p.returncode}: {p.stderr[-300:]}"}
        return {"rowshard512_lib": err}
    return json.loads(lines[-1])


def _library_riders(result, a, world, rank, dist, fns=None):
    """Rank 0 alone drives every GPU of the job through the library (one process, as a Go
    node would): configs 3 and 4, in a child process (_spawn_libriders). The other ranks wait
    on a gloo barrier, which puts no work on their GPUs, so the child's kernels and RCCL have
    the devices to themselves. fns: CPU stand-ins by name, run in rank 0 itself (distcheck)."""
    if rank == 0:
        if fns is None:
            result.update(_spawn_libriders(a, world))
        else:
            for name, fn in fns.items():
                result[name] = fn()
    if dist is not None:
        dist.barrier(group=IDLE_GROUP)


def _rider(result, name, fn):
    """result[name] = fn(), a part of the line beside the headline batch. A part that
    raises is reported as {"error": ...} instead of losing the whole line (every rank runs
    the same parts with the same shapes, so a failure is symmetric)."""
    try:
        result[name] = fn()
    except Exception as e:  # noqa: BLE001
        result[name] = {"error": f"{type(e).__name__}: {e}"[:400]}
        print(f"bench: {name} failed: {e!r}", file=sys.stderr, flush=True)
    torch.cuda.empty_cache()


def _measure_batch(ctx, local, rank, k, B, steps, warmup, n_distinct, layout, phase_reps, barrier, dist, dev,
                   inflight=1):
    """Time `steps` batch steps of B k x k squares resident in HBM (barrier + synchronize
    on both sides, max over ranks), then the RS and NMT phases alone with HIP events on
    the batch's launch stream. inflight > 1: that many batches (own buffers and stream
    each) take the steps in turn, each step as one chunk on its batch's stream
    (CEL_FLAG_CALLER_STREAM), so one step's latency-bound tree tops and DAH run beside the
    next step's bulk (independent blocks replayed back to back); every step still extends
    and commits all B squares."""
    from celestia_eds.device import SquareBatch
    from celestia_eds.testfactory import random_ods

    sbs = []
    distinct = [random_ods(k, 1_000_003 * rank + i) for i in range(min(n_distinct, B))]
    for j in range(max(1, inflight)):
        sb = SquareBatch(B, k, device=local, ctx=ctx, ods_in_eds=(layout == "eds"))
        host = np.stack([distinct[(i + j) % len(distinct)] for i in range(B)])
        sb.load_ods(torch.from_numpy(host))
        del host
        sbs.append(sb)
    torch.cuda.synchronize()
    piped = len(sbs) > 1
    for i in range(warmup):
        sbs[i % len(sbs)].extend_and_commit(caller_stream=piped)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        sbs[i % len(sbs)].extend_and_commit(caller_stream=piped)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = _max_over_ranks(time.perf_counter() - t0, dist, dev)
    for sb in sbs:
        status = sb.status.cpu().numpy()
        assert (status == 0).all(), f"device reported status {status}"
    sb = sbs[0]
    del sbs

    stream = sb.hip_stream  # the stream every launch of `sb` goes to

    def timed(fn, reps):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        fn()
        e0.record(stream)
        for _ in range(reps):
            fn()
        e1.record(stream)
        e1.synchronize()
        return e0.elapsed_time(e1) / reps / 1e3  # seconds per launch

    t_ext = timed(sb.extend_only, phase_reps)
    t_com = timed(sb.commit_only, phase_reps)
    return {"sb": sb, "distinct": distinct, "elapsed": elapsed, "t_ext": t_ext, "t_com": t_com}


def measure_power(fn, secs=1.5):
    """Median socket power (W) and shader clock (MHz) from rocm-smi while fn runs back to back
    for `secs` (synchronised every 4 calls), or None fields when rocm-smi reads nothing."""
    import threading
    samples, stop = [], threading.Event()

    def sampler():
        time.sleep(0.3)
        while not stop.is_set():
            try:
                out = subprocess.run(["rocm-smi", "-P", "-c", "--json"], capture_output=True, text=True,
                                     timeout=10).stdout
                samples.append(json.loads(out[out.index("{"):]))
            except Exception:  # noqa: BLE001  (no rocm-smi, or no JSON: the fields stay None)
                pass
            time.sleep(0.2)

    th = threading.Thread(target=sampler, daemon=True)
    th.start()
    t0, n = time.time(), 0
    while time.time() - t0 < secs:
        fn()
        n += 1
        if n % 4 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    stop.set()
    th.join()
    pw, mhz = [], []
    for smp in samples:
        for card in smp.values():
            if not isinstance(card, dict):
                continue
            for key, val in card.items():
                kl = key.lower()
                try:
                    if "power" in kl and "(w)" in kl:
                        pw.append(float(val))
                    elif kl.startswith("sclk"):
                        f = float(str(val).strip("()Mhz "))
                        if f > 100:  # skip the level index rocm-smi prints beside the clock
                            mhz.append(f)
                except ValueError:
                    pass
    med = lambda v: sorted(v)[len(v) // 2] if v else None  # noqa: E731
    return {"watts": med(pw), "sclk_mhz": med(mhz), "samples": len(samples), "calls": n}


def measure_host_io(ctx, k, n=16, reps=5):
    """cel_extend_batch over page-locked host buffers (cel_host_alloc): n ODSs in, then
    (a) the EDS + roots + DAH out (what rsmt2d.ImportExtendedDataSquare needs) and
    (b) the parity cells only (CEL_FLAG_PARITY_ONLY: the caller holds Q0 already) and
    (c) roots + DAH only (PrepareProposal/ProcessProposal keep only the DAH,
    app/prepare_proposal.go:81-83). PCIe copies included; never the headline value."""
    import ctypes
    from celestia_eds import _lib
    from celestia_eds.testfactory import random_ods
    w = 2 * k

    def pinned(shape):
        nbytes = int(np.prod(shape))
        p = ctx.lib.cel_host_alloc(nbytes)
        assert p, "cel_host_alloc failed"
        return p, np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p)).reshape(shape)

    p_ods, ods = pinned((n, k, k, 512))
    ods[...] = np.stack([random_ods(k, 500 + i) for i in range(n)])
    p_eds, eds = pinned((n, w, w, 512))
    rr = np.zeros((n, w, 90), np.uint8)
    cr = np.zeros_like(rr)
    dah = np.zeros((n, 32), np.uint8)
    st = np.zeros(n, np.int32)
    P = lambda x: x.ctypes.data_as(ctypes.c_void_p)
    out = {}
    try:
        for name, e, fl in (("with_eds", eds, 0), ("parity_only", eds, _lib.FLAG_PARITY_ONLY),
                            ("roots_only", None, 0)):
            def once():
                ctx.check(ctx.lib.cel_extend_batch(ctx.handle, P(ods), n, k, 512, P(e) if e is not None else None,
                                                   P(rr), P(cr), P(dah), P(st), _lib.FLAG_ORDER_CHECK | fl))
            for _ in range(3):  # warm: the first calls after the riders ran 30-40 % slower
                once()
            t0 = time.perf_counter()
            for _ in range(reps):
                once()
            dt = (time.perf_counter() - t0) / reps
            eds_b = 0 if e is None else (eds.nbytes * 3 // 4 if fl else eds.nbytes)
            pcie = ods.nbytes + eds_b + rr.nbytes + cr.nbytes
            out[name] = {"squares_per_s": n / dt, "pcie_gbps": pcie / dt / 1e9, "ms_per_call": dt * 1e3}
        # one square per call: da.ExtendShares as PrepareProposal / ProcessProposal issue it
        # (one block, one square), parity cells back
        def one():
            ctx.check(ctx.lib.cel_extend_batch(ctx.handle, P(ods), 1, k, 512, P(eds), P(rr), P(cr), P(dah), P(st),
                                               _lib.FLAG_ORDER_CHECK | _lib.FLAG_PARITY_ONLY))
        one()
        t0 = time.perf_counter()
        for _ in range(10):
            one()
        out["single_square_parity_only_ms"] = (time.perf_counter() - t0) / 10 * 1e3

        # the header alone (da.ComputeDataAvailabilityHeader): what PrepareProposal /
        # ProcessProposal keep; no EDS copied back
        def dah_only():
            ctx.check(ctx.lib.cel_extend_batch(ctx.handle, P(ods), 1, k, 512, None, P(rr), P(cr), P(dah), P(st),
                                               _lib.FLAG_ORDER_CHECK))
        dah_only()
        t0 = time.perf_counter()
        for _ in range(10):
            dah_only()
        out["single_square_dah_only_ms"] = (time.perf_counter() - t0) / 10 * 1e3
    finally:
        ctx.lib.cel_host_free(p_ods)
        ctx.lib.cel_host_free(p_eds)
    # the same header for one k=512 block (GovMaxSquareSize, test/e2e/benchmark/throughput.go:49)
    # on one GPU: 128 MiB of ODS over PCIe, read by the GF(2^16) row pass from page-locked memory
    k5 = 512
    p5, ods5 = pinned((k5, k5, 512))
    try:
        ods5[...] = random_ods(k5, 77)
        rr5, cr5 = np.zeros((2 * k5, 90), np.uint8), np.zeros((2 * k5, 90), np.uint8)

        def dah5():
            ctx.check(ctx.lib.cel_extend_batch(ctx.handle, P(ods5), 1, k5, 512, None, P(rr5), P(cr5), P(dah), P(st),
                                               _lib.FLAG_ORDER_CHECK))
        dah5()
        t0 = time.perf_counter()
        for _ in range(5):
            dah5()
        out["single_square_k512_dah_only_ms"] = (time.perf_counter() - t0) / 5 * 1e3
    finally:
        ctx.lib.cel_host_free(p5)
    out["squares_per_call"] = n
    out["entry_point"] = "cel_extend_batch (host buffers, page-locked, 4 chunks over the ctx streams)"
    return out


def main():
    global REHEARSE
    a = parse()
    REHEARSE = a.rehearse
    world, rank, local = _dist_env()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch(a))
    if a.mode == "distcheck":
        return run_distcheck(a)
    if a.mode == "sharded":
        return run_sharded(a)
    if a.mode == "repair":
        return run_repair(a)
    if a.mode == "libriders":
        return run_libriders(a)
    local = _rank_device(local)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        dist = _init_dist(dev)

    from celestia_eds import default_context

    ctx = default_context(local)

    def barrier():
        if dist is not None:
            dist.barrier()

    probe = None
    try:
        probe = measure_probe(ctx)
    except Exception as e:  # noqa: BLE001  (the line keeps its fixed-constant fractions)
        print(f"bench: probe failed: {e!r}", file=sys.stderr, flush=True)
    m = _measure_batch(ctx, local, rank, a.k, a.batch, a.steps, a.warmup, a.distinct, a.input,
                       a.phase_reps, barrier, dist, dev, a.inflight)
    k, B, elapsed, t_ext, t_com = a.k, a.batch, m["elapsed"], m["t_ext"], m["t_com"]
    sb, distinct = m["sb"], m["distinct"]
    del m
    squares = world * B * a.steps
    value = squares / elapsed
    ods_bytes = 512 * k * k
    rs_bytes = 2048 * k * k * B  # read ODS + write Q1..Q3, per launch pair
    rs_gbs = rs_bytes / t_ext / 1e9
    compressions = (60 * k * k + 4 * k - 2) * B
    nmt_rate = compressions / t_com

    result = {
        "metric": "EDS+DAH squares/sec (k=%d)" % k,
        "value": value,
        "unit": "squares/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": elapsed / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (testfactory-style sorted random namespaced shares)",
        "ods_gbps": value * ods_bytes / 1e9,
        "config": {
            "workload": f"k={k} ODS -> EDS + 4k NMT roots + DAH, batch replay",
            "k": k,
            "squares_per_step_per_gpu": B,
            "share_size": 512,
            "field": "GF(2^8)" if 2 * k <= 256 else "GF(2^16)",
            "parallelism": f"batch{world}",
            "input_layout": ("ODS in Q0 of the EDS buffer (placed by the upload)" if a.input == "eds"
                             else "contiguous ODS buffer"),
            "batches_in_flight": a.inflight,
        },
        "roofline": {
            "bound": "hbm",
            "kernel": ("rs_extend (k_rs_axis_gf8 rows + cols launches)" if 32 <= k <= 128
                       else "rs_extend (rows + cols launches)"),
            "achieved": rs_gbs,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": rs_gbs / HBM_PEAK_GBS,
            "traffic": _rs_traffic(k, B, a.input),
            "avg_launch_us": t_ext * 1e6,
        },
        "roofline_nmt": {
            "bound": "valu",
            "kernel": "nmt_commit (k_leaf + k_level x log2(2k) + k_merkle)",
            "achieved": nmt_rate / 1e9,
            "unit": "G SHA-256 compressions/s",
            "peak": SHA_MEASURED_PEAK / 1e9,
            "peak_basis": "measured SHA-256 compression rate with no memory traffic (profiles/r2_sha_rate.txt)",
            "frac": nmt_rate / SHA_MEASURED_PEAK,
            "peak_model": SHA_MIX_CEILING / 1e9,
            "frac_model": nmt_rate / SHA_MIX_CEILING,
            "peak_model_basis": "SHA-256 ISA mix at the same box's per-op VALU rates (profiles/r4_sha_ceiling.txt)",
            "peak_guide": SHA_GUIDE_CEILING / 1e9,
            "frac_guide": nmt_rate / SHA_GUIDE_CEILING,
            "peak_guide_basis": "1414 VALU per compression x 2 cycles per wave64 instruction (MI355X_MICROARCH.md "
                                "issue model), 1024 SIMDs, 2.4 GHz",
            "avg_launch_us": t_com * 1e6,
        },
    }
    if probe:
        # same-run denominators (cel_probe_*, before the timed region, this rank's device)
        result["probe"] = {**probe, "basis": "cel_probe_sha256 (NMT compression chained in registers, 16 WG/CU; "
                                             "shader clock = s_memtime ticks per s_memrealtime tick over that "
                                             "launch) and cel_probe_hbm_stream (4 GiB: float4 streaming copy, read + write; "
                                             "read-only and write-only streams)"}
        result["roofline"]["achievable"] = probe["hbm_copy_gbps"]
        result["roofline"]["achievable_basis"] = "cel_probe_hbm_copy: float4 streaming copy, one element per lane"
        result["roofline"]["frac_of_achievable_hbm"] = rs_gbs / probe["hbm_copy_gbps"]
        mix = achievable_mix(result["roofline"]["traffic"], probe, k)
        if mix:
            result["roofline"]["achievable_mix"] = mix
            result["roofline"]["frac_of_achievable_mix"] = rs_gbs / mix
            result["roofline"]["achievable_mix_basis"] = ("algorithmic bytes over the time the measured traffic "
                                                          "(read_per_square, write_per_square) takes at the "
                                                          "probe's read-only and write-only rates")
        result["roofline_nmt"]["peak_same_run"] = probe["sha256_gcomp_per_s"]
        result["roofline_nmt"]["frac_same_run"] = nmt_rate / 1e9 / probe["sha256_gcomp_per_s"]
        result["shader_mhz"] = probe["shader_mhz"]
        step = step_ceiling(k, probe, elapsed / (B * a.steps))
        if step:
            result["roofline_step"] = step
    if world == 1 and not a.no_power:
        # after the timed region: each phase looped ~1.5 s while rocm-smi reads socket power
        # and the shader clock (the path runs in the board's power envelope)
        _rider(result, "power", lambda: {"extend": measure_power(sb.extend_only),
                                         "commit": measure_power(sb.commit_only),
                                         "basis": "rocm-smi -P -c every ~0.3 s while the phase runs back to back "
                                                  "on this batch (outside the timed region)"})

    if a.k == 128 and a.k512_batch > 0:
        # The metric names k=128 and k=512: a short GF(2^16) batch rides along with the
        # headline k=128 line (same contract: barrier + max over ranks, whole job).
        dah128 = sb.dah.cpu().numpy()
        del sb
        torch.cuda.empty_cache()

        def k512():
            m5 = _measure_batch(ctx, local, rank, 512, a.k512_batch, a.k512_steps, 2, 2, a.input,
                                3, barrier, dist, dev, a.inflight)
            B5, t5 = a.k512_batch, m5["elapsed"]
            v5 = world * B5 * a.k512_steps / t5
            rs5 = 2048 * 512 * 512 * B5 / m5["t_ext"] / 1e9
            comp5 = (60 * 512 * 512 + 4 * 512 - 2) * B5 / m5["t_com"]
            return {
                "workload": "k=512 ODS (GF(2^16)) -> EDS + 2048 NMT roots + DAH, batch replay",
                "value": v5, "unit": "squares/s", "ods_gbps": v5 * 512 * 512 * 512 / 1e9,
                "squares_per_step_per_gpu": B5, "steps": a.k512_steps,
                "ms_per_step": t5 / a.k512_steps * 1e3,
                "rs_frac_hbm": rs5 / HBM_PEAK_GBS, "rs_avg_launch_us": m5["t_ext"] * 1e6,
                "nmt_frac_sha_peak": comp5 / SHA_MEASURED_PEAK, "nmt_frac_sha_mix": comp5 / SHA_MIX_CEILING,
                "nmt_frac_same_run": comp5 / 1e9 / probe["sha256_gcomp_per_s"] if probe else None,
                "nmt_avg_launch_us": m5["t_com"] * 1e6,
                **_step_fields(512, probe, t5 / (B5 * a.k512_steps)),
            }

        _rider(result, "k512", k512)
        sb = None
    else:
        dah128 = None
    if a.k == 128 and not a.no_riders:
        # Configs 4 and 3 in the same run, so one driver N-GPU command measures configs 2, 3
        # and 4: 1024 k=64 squares split over the ranks, and one k=512 square row-sharded
        # over all ranks through RCCL (all_to_all_single) with its exchange timed alone.
        def k64():
            m4 = _measure_batch(ctx, local, rank, 64, 1024 // world, a.rider_steps, 2, 4, a.input, 3, barrier,
                                dist, dev, a.inflight)
            f = _k64_fields(world, m4["elapsed"], a.rider_steps, m4["t_ext"], m4["t_com"], 1024 // world)
            f.update(_step_fields(64, probe, m4["elapsed"] / (a.rider_steps * (1024 // world))))
            return f

        _rider(result, "k64", k64)
        if world > 1:  # per-rank processes, torch.distributed's RCCL (at N = 1: rowshard512_lib alone)
            _rider(result, "rowshard512", lambda: measure_rowshard(512, world, rank, local, dist, dev, a.rider_steps,
                                                                   2, barrier, a.depth))
        _library_riders(result, a, world, rank, dist)
    if rank == 0 and world == 1 and a.k == 128 and not a.no_host_io:
        _rider(result, "host_io", lambda: measure_host_io(ctx, a.k))
    if rank == 0 and world == 1 and not a.no_cpu:
        dah_dev = dah128 if dah128 is not None else sb.dah.cpu().numpy()

        def cpu():
            base, parity = cpu_baseline_batch(k, distinct, dah_dev, a.cpu_seconds)
            result["parity_vs_cpu"] = bool(parity)
            return base

        _rider(result, "cpu_baseline", cpu)
    if REHEARSE:
        result["config"]["rehearsal"] = "all ranks on cuda:0, gloo with host staging: not a multi-GPU measurement"
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
