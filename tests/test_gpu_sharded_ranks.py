"""The row-sharded square (config 3) with real processes and a real collective: two
ranks, each driving the HIP device steps (cel_dev_shard_*) on the box's GPU, exchanging
the all-to-all blocks and the record all-gather through torch.distributed (gloo over
TCP, the device tensors staged through host memory because gloo has no all_to_all for
device tensors). The result must equal the oracle's whole-square roots and DAH. On the
8-GPU node the same ShardedSquare.run drives RCCL (bench.py --mode sharded)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, k, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist
    from celestia_eds import default_context
    from celestia_eds.sharded import DeviceSteps, ShardedSquare, StagedComm
    from celestia_eds.testfactory import random_ods
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    steps = DeviceSteps(default_context(0), 0)
    sq = ShardedSquare(k, rank, world, steps)
    lo, hi = sq.row_range()
    sq.ods_rows.copy_(torch.from_numpy(np.ascontiguousarray(random_ods(k, 77)[lo:hi])))
    sq.run(StagedComm())
    torch.cuda.synchronize()
    sq.check_status()
    np.savez(os.path.join(outdir, f"r{rank}.npz"), rr=sq.row_roots.cpu().numpy(), cr=sq.col_roots.cpu().numpy(),
             dah=sq.dah.cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_processes_gloo(oracle, tmp_path):
    import torch.multiprocessing as mp
    from celestia_eds.testfactory import random_ods
    k, world = 256, 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_worker, args=(world, port, k, str(tmp_path)), nprocs=world, join=True)
    _, rr, cr, dah = oracle.extend_and_commit(random_ods(k, 77), want_eds=False)
    for r in range(world):
        got = np.load(tmp_path / f"r{r}.npz")
        assert np.array_equal(got["rr"], rr) and np.array_equal(got["cr"], cr)
        assert got["dah"].tobytes() == dah


def _rccl_one_rank(rank, port, k, outdir):
    """One rank on a real RCCL communicator (the box has one GPU, and RCCL refuses two
    ranks on one device: "Duplicate GPU detected", profiles/r3_rccl_probe.txt). Runs the
    collectives TorchComm issues on device tensors of the shapes the sharded square
    uses, then a whole n=1 square through TorchComm on the square's HIP stream."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    import torch
    import torch.distributed as dist
    from celestia_eds import default_context
    from celestia_eds.sharded import RECORD, DeviceSteps, ShardedSquare, TorchComm
    from celestia_eds.testfactory import random_ods
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    assert dist.get_backend() == "nccl"
    comm = TorchComm()
    steps = DeviceSteps(default_context(0), 0)
    g = torch.Generator(device="cpu").manual_seed(5)
    send = torch.randint(0, 256, (1, k, 2 * k, 512), dtype=torch.uint8, generator=g).to(dev)
    recv = torch.empty_like(send)
    rec = torch.randint(0, 256, (2 * k + 2 * k + 1, RECORD), dtype=torch.uint8, generator=g).to(dev)
    rec_all = torch.empty((1,) + rec.shape, dtype=torch.uint8, device=dev)
    with steps.scope():
        comm.all_to_all(recv.view(-1), send.view(-1))
        comm.all_gather(rec_all.view(-1), rec.view(-1))
    torch.cuda.synchronize()
    ok = bool(torch.equal(recv, send) and torch.equal(rec_all[0], rec))
    sq = ShardedSquare(k, 0, 1, steps)
    sq.ods_rows.copy_(torch.from_numpy(np.ascontiguousarray(random_ods(k, 78))))
    sq.run(comm)
    torch.cuda.synchronize()
    sq.check_status()
    np.savez(os.path.join(outdir, "rccl.npz"), ok=ok, rr=sq.row_roots.cpu().numpy(),
             cr=sq.col_roots.cpu().numpy(), dah=sq.dah.cpu().numpy())
    dist.destroy_process_group()


def test_rccl_one_rank_torchcomm(oracle, tmp_path):
    import torch.multiprocessing as mp
    from celestia_eds.testfactory import random_ods
    k = 256
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_rccl_one_rank, args=(port, k, str(tmp_path)), nprocs=1, join=True)
    got = np.load(tmp_path / "rccl.npz")
    assert bool(got["ok"]), "RCCL collectives on device tensors returned wrong data"
    _, rr, cr, dah = oracle.extend_and_commit(random_ods(k, 78), want_eds=False)
    assert np.array_equal(got["rr"], rr) and np.array_equal(got["cr"], cr)
    assert got["dah"].tobytes() == dah


def _worker_pipelined(rank, world, port, k, seeds, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist
    from celestia_eds import default_context
    from celestia_eds.sharded import DeviceSteps, ShardedSquare, StagedComm, run_pipelined
    from celestia_eds.testfactory import random_ods
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    ctx = default_context(0)
    sqs = []
    for sd in seeds:
        sq = ShardedSquare(k, rank, world, DeviceSteps(ctx, 0))
        lo, hi = sq.row_range()
        sq.ods_rows.copy_(torch.from_numpy(np.ascontiguousarray(random_ods(k, sd)[lo:hi])))
        sqs.append(sq)
    for _ in range(2):  # the second round reuses every buffer
        run_pipelined(sqs, StagedComm())
    torch.cuda.synchronize()
    for i, sq in enumerate(sqs):
        sq.check_status()
        np.savez(os.path.join(outdir, f"r{rank}_{i}.npz"), rr=sq.row_roots.cpu().numpy(),
                 cr=sq.col_roots.cpu().numpy(), dah=sq.dah.cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_pipelined_squares(oracle, tmp_path):
    """Two ranks (processes) with three row-sharded squares in flight each
    (sharded.run_pipelined: own stream and workspace per square, the collectives of all
    squares in one order on both ranks), device steps on the GPU, collectives over gloo
    with host staging: every square's roots and DAH equal its whole-square oracle."""
    import torch.multiprocessing as mp
    from celestia_eds.testfactory import random_ods
    k, world, seeds = 256, 2, (81, 82, 83)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_worker_pipelined, args=(world, port, k, seeds, str(tmp_path)), nprocs=world, join=True)
    for i, sd in enumerate(seeds):
        _, rr, cr, dah = oracle.extend_and_commit(random_ods(k, sd), want_eds=False)
        for r in range(world):
            got = np.load(tmp_path / f"r{r}_{i}.npz")
            assert np.array_equal(got["rr"], rr) and np.array_equal(got["cr"], cr), (r, sd)
            assert got["dah"].tobytes() == dah
