"""Row-sharded square (config 3): the N>1 path.

CPU: world_size 2 and 4 over gloo (torch.distributed, 127.0.0.1), the real
orchestration (celestia_eds.sharded.ShardedSquare + TorchComm) with oracle-backed
per-rank steps; the combined roots and DAH must equal the oracle's whole-square
result. GPU: the device steps (cel_dev_shard_*) for N = 1..8 ranks rehearsed in one
process (LocalComm), bit-exact against the oracle at k = 256 and k = 512.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from eds_inputs import random_ods


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, k, seed, order_check, out_q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "celestia-app_amd"), os.path.join(root, "oracle"), os.path.join(root, "tests")):
        sys.path.insert(0, p)
    import torch.distributed as dist
    from celestia_eds.sharded import ShardedSquare, TorchComm
    from sharded_oracle import OracleSteps
    from eds_inputs import random_ods as rods
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ods = rods(k, seed)
        if not order_check:
            ods = ods[::-1].copy()  # rows out of namespace order
        sq = ShardedSquare(k, rank, world, OracleSteps())
        a, b = sq.row_range()
        sq.ods_rows.copy_(torch.from_numpy(np.ascontiguousarray(ods[a:b])))
        sq.run(TorchComm())
        out_q.put((rank, sq.row_roots.numpy().copy(), sq.col_roots.numpy().copy(), sq.dah.numpy().tobytes(),
                   int(sq.status.item())))
    finally:
        dist.destroy_process_group()


def _run_world(world, k, seed, order_ok=True):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, k, seed, order_ok, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(res)


@pytest.mark.parametrize("world,k", [(2, 8), (4, 16)])
def test_gloo_sharded_matches_whole_square(oracle, world, k):
    res = _run_world(world, k, 77 + k)
    _, rr, cr, dah = oracle.extend_and_commit(random_ods(k, 77 + k), want_eds=False)
    for rank, r_rr, r_cr, r_dah, st in res:
        assert st == 0
        assert np.array_equal(r_rr, rr), f"rank {rank} row roots"
        assert np.array_equal(r_cr, cr), f"rank {rank} col roots"
        assert r_dah == dah


def test_gloo_sharded_order_violation(oracle):
    res = _run_world(2, 8, 5, order_ok=False)
    assert all(st == 5 for _, _, _, _, st in res)


@pytest.mark.parametrize("local", [True, False])
def test_one_rank_aliases_slab(oracle, local):
    """One rank: the row pass writes the slab's top half in place (send aliases it, the
    all-to-all is skipped); the result is the whole square's."""
    from celestia_eds.sharded import LocalComm, ShardedSquare
    from sharded_oracle import OracleSteps
    k = 8
    ods = random_ods(k, 31)
    sq = ShardedSquare(k, 0, 1, OracleSteps())
    assert sq.send.data_ptr() == sq.slab.data_ptr()
    sq.ods_rows.copy_(torch.from_numpy(ods))
    if local:
        LocalComm.run([sq])
    else:
        class NoComm:  # a one-rank communicator: the gathers are identities
            def all_gather(self, out, inp):
                out.copy_(inp)

            def all_to_all(self, out, inp):
                raise AssertionError("one rank must not exchange")
        sq.run(NoComm())
    eds, rr, cr, dah = oracle.extend_and_commit(ods)
    assert np.array_equal(sq.slab.numpy(), eds)
    assert np.array_equal(sq.row_roots.numpy(), rr)
    assert np.array_equal(sq.col_roots.numpy(), cr)
    assert sq.dah.numpy().tobytes() == dah


@pytest.mark.gpu
@pytest.mark.parametrize("k,n", [(256, 1), (256, 2), (256, 8), (512, 4), (512, 8)])
def test_device_sharded_local(ctx, oracle, k, n):
    from celestia_eds.sharded import DeviceSteps, LocalComm, ShardedSquare
    steps = DeviceSteps(ctx)
    ods = random_ods(k, 900 + k + n)
    squares = [ShardedSquare(k, r, n, steps) for r in range(n)]
    for s in squares:
        a, b = s.row_range()
        s.ods_rows.copy_(torch.from_numpy(np.ascontiguousarray(ods[a:b])))
    LocalComm.run(squares)
    steps.stream.synchronize()
    eds, rr, cr, dah = oracle.extend_and_commit(ods)
    w = 2 * k // n
    for r, s in enumerate(squares):
        assert int(s.status.item()) == 0
        assert np.array_equal(s.slab.cpu().numpy(), eds[:, r * w:(r + 1) * w]), f"slab of rank {r}"
        assert np.array_equal(s.row_roots.cpu().numpy(), rr)
        assert np.array_equal(s.col_roots.cpu().numpy(), cr)
        assert s.dah.cpu().numpy().tobytes() == dah


def _worker_pipelined(rank, world, port, k, seeds, out_q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "celestia-app_amd"), os.path.join(root, "oracle"), os.path.join(root, "tests")):
        sys.path.insert(0, p)
    import torch.distributed as dist
    from celestia_eds.sharded import ShardedSquare, TorchComm, run_pipelined
    from sharded_oracle import OracleSteps
    from eds_inputs import random_ods as rods
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sqs = []
        for sd in seeds:
            sq = ShardedSquare(k, rank, world, OracleSteps())
            a, b = sq.row_range()
            sq.ods_rows.copy_(torch.from_numpy(np.ascontiguousarray(rods(k, sd)[a:b])))
            sqs.append(sq)
        run_pipelined(sqs, TorchComm())
        out_q.put((rank, [(s.row_roots.numpy().copy(), s.col_roots.numpy().copy(), s.dah.numpy().tobytes(),
                           int(s.status.item())) for s in sqs]))
    finally:
        dist.destroy_process_group()


def test_gloo_pipelined_squares(oracle):
    """Several squares in flight per rank (sharded.run_pipelined: every rank issues the
    all-to-alls of all squares, then their gathers, in the same order), world 2 over gloo:
    each square's roots and DAH are its own whole-square result."""
    world, k, seeds = 2, 8, (41, 42, 43)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_pipelined, args=(r, world, port, k, seeds, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for sd, i in zip(seeds, range(len(seeds))):
        _, rr, cr, dah = oracle.extend_and_commit(random_ods(k, sd), want_eds=False)
        for rank, outs in res:
            r_rr, r_cr, r_dah, st = outs[i]
            assert st == 0 and np.array_equal(r_rr, rr) and np.array_equal(r_cr, cr) and r_dah == dah, (rank, sd)


@pytest.mark.gpu
def test_device_pipelined_one_rank(ctx, oracle):
    """Three k=256 squares in flight on one GPU (each with its own stream and workspace,
    sharded.run_pipelined without collectives): each equals the oracle's whole square."""
    from celestia_eds.sharded import DeviceSteps, ShardedSquare, run_pipelined
    k, seeds = 256, (61, 62, 63)
    sqs = []
    for sd in seeds:
        sq = ShardedSquare(k, 0, 1, DeviceSteps(ctx))
        sq.ods_rows.copy_(torch.from_numpy(random_ods(k, sd)))
        sqs.append(sq)
    for _ in range(2):  # twice: the second round reuses every buffer
        run_pipelined(sqs, None)
    torch.cuda.synchronize()
    for sd, sq in zip(seeds, sqs):
        eds, rr, cr, dah = oracle.extend_and_commit(random_ods(k, sd))
        assert int(sq.status.item()) == 0
        assert np.array_equal(sq.slab.cpu().numpy(), eds)
        assert np.array_equal(sq.row_roots.cpu().numpy(), rr) and np.array_equal(sq.col_roots.cpu().numpy(), cr)
        assert sq.dah.cpu().numpy().tobytes() == dah


def test_pipelined_one_rank_oracle(oracle):
    """run_pipelined without collectives (one rank): the record block is copied into the
    gathered buffer in place of the all-gather; two squares in flight, each equals its
    whole-square oracle (CPU, oracle-backed steps)."""
    from celestia_eds.sharded import ShardedSquare, run_pipelined
    from sharded_oracle import OracleSteps
    k, seeds = 8, (91, 92)
    sqs = []
    for sd in seeds:
        sq = ShardedSquare(k, 0, 1, OracleSteps())
        sq.ods_rows.copy_(torch.from_numpy(random_ods(k, sd)))
        sqs.append(sq)
    run_pipelined(sqs, None)
    for sd, sq in zip(seeds, sqs):
        eds, rr, cr, dah = oracle.extend_and_commit(random_ods(k, sd))
        assert int(sq.status.item()) == 0
        assert np.array_equal(sq.slab.numpy(), eds)
        assert np.array_equal(sq.row_roots.numpy(), rr) and np.array_equal(sq.col_roots.numpy(), cr)
        assert sq.dah.numpy().tobytes() == dah


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 4, 8])
def test_device_sharded_order_across_slabs(ctx, oracle, n):
    """Each row's two column halves swapped: columns stay sorted and, for n >= 4, every slab
    of Q0 is sorted inside, so the push-order break is only across slab boundaries (the
    finish's check of subtree minNs against the previous slab's maxNs); n = 2 catches it
    inside the slab. Every rank reports EORDER, like the whole-square check."""
    from celestia_eds import _lib
    from celestia_eds.sharded import DeviceSteps, LocalComm, ShardedSquare
    k = 256
    ods = random_ods(k, 700 + n)
    ods = np.concatenate([ods[:, k // 2:], ods[:, :k // 2]], axis=1).copy()
    assert oracle.roots(oracle.extend(ods), check_order=True)[0] != 0  # the oracle sees the break too
    steps = DeviceSteps(ctx)
    squares = [ShardedSquare(k, r, n, steps) for r in range(n)]
    for s in squares:
        a, b = s.row_range()
        s.ods_rows.copy_(torch.from_numpy(np.ascontiguousarray(ods[a:b])))
    LocalComm.run(squares)
    steps.stream.synchronize()
    assert all(int(s.status.item()) == _lib.EORDER for s in squares)
