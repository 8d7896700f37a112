"""Row-sharded extension of one square over several GPUs (config 3).

One process per GPU. Rank r owns ODS rows [r*k/N, (r+1)*k/N) and, after one
all-to-all transpose, EDS columns [r*w, (r+1)*w) with w = 2k/N:

  1. rows    row-encode the local rows straight into the all-to-all send layout
             [N][k/N][w][512] (block h = the cells of rank h's columns)
  2. a2a     all_to_all_single: the received blocks, in rank order, are the top half
             (rows 0..k-1) of this rank's column slab [2k][w][512]
  3. cols    column-encode the slab (rows k..2k-1), hash its leaves once, build its
             w column trees and the 2k row subtrees over its w columns
  4. gather  one all_gather of each rank's record block [2k + w + 1][96]: its row
             subtrees, its column roots and its push-order status
  5. finish  combine the N subtree roots of every row (log2 N levels of HashNode),
             then DataAvailabilityHeader.Hash over rowRoots || colRoots

The result is what da.ExtendShares + da.NewDataAvailabilityHeader
(pkg/da/data_availability_header.go:65-75, :44-63) give for the whole square. The
only data-path collective is the all-to-all (2k*k*512/N^2 bytes per peer); the one
gather moves 96-byte records. `steps` does the per-rank device work (DeviceSteps:
the C ABI cel_dev_shard_*); `comm` the collectives (TorchComm: torch.distributed,
i.e. RCCL over xGMI on the GPU box, gloo in the CPU tests).
"""
import contextlib
import ctypes

from . import _lib

RECORD = 96  # 90-byte NMT node + 6 zero bytes (CEL_NODE_RECORD)


class TorchComm:
    """Collectives over torch.distributed (backend "nccl" = RCCL, or "gloo")."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)

    def all_to_all(self, out, inp):
        self.dist.all_to_all_single(out, inp, group=self.group)

    def all_gather(self, out, inp):
        self.dist.all_gather_into_tensor(out, inp, group=self.group)


class StagedComm:
    """The same collectives over gloo on host copies of device tensors (gloo has no
    all_to_all for device tensors): the multi-rank rehearsal of the RCCL path with every
    rank on one GPU (bench.py --rehearse, the two-rank GPU test)."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group

    def all_to_all(self, out, inp):
        h_out = out.cpu()
        self.dist.all_to_all_single(h_out, inp.cpu(), group=self.group)
        out.copy_(h_out)

    def all_gather(self, out, inp):
        h_out = out.cpu()
        self.dist.all_gather_into_tensor(h_out, inp.cpu(), group=self.group)
        out.copy_(h_out)


class DeviceSteps:
    """Per-rank device steps through the C ABI (device tensors, current HIP stream)."""

    def __init__(self, ctx=None, device=0, order_check=True):
        import torch
        self.torch = torch
        self.dev = torch.device("cuda", device)
        self.ctx = ctx or _lib.default_context(device)
        self.flags = _lib.FLAG_ORDER_CHECK if order_check else 0
        self._work = None
        # A dedicated (non-null) stream: the C ABI maps a NULL stream to the ctx's own
        # stream, so torch's legacy default stream cannot be used to order the kernels
        # with torch copies and collectives. Drivers enter scope() around every phase.
        self.stream = torch.cuda.Stream(device=self.dev)

    def scope(self):
        return self.torch.cuda.stream(self.stream)

    def empty(self, shape, dtype):
        return self.torch.empty(shape, dtype=dtype, device=self.dev)

    @staticmethod
    def _p(t):
        return ctypes.c_void_p(t.data_ptr())

    def _stream(self):
        return ctypes.c_void_p(self.stream.cuda_stream)

    def work(self, k, n):
        size = self.ctx.lib.cel_dev_shard_workspace_size(k, n)
        if self._work is None or self._work.numel() < size:
            self._work = self.empty((size,), self.torch.uint8)
        return self._work

    def rows(self, ods_rows, k, n, send):
        c = self.ctx
        c.check(c.lib.cel_dev_shard_rows(c.handle, self._p(ods_rows), k, n, self._p(send), self._stream()))

    def cols(self, slab, k, n, rank, col_rec, row_sub, status):
        c = self.ctx
        c.check(c.lib.cel_dev_shard_cols(c.handle, self._p(slab), k, n, rank, self._p(col_rec), self._p(row_sub),
                                         self._p(status), self._p(self.work(k, n)), self._stream(), self.flags))

    def finish(self, gathered, k, n, row_roots, col_roots, dah, status):
        c = self.ctx
        c.check(c.lib.cel_dev_shard_finish(c.handle, self._p(gathered), k, n, self._p(row_roots), self._p(col_roots),
                                           self._p(dah), self._p(status), self._p(self.work(k, n)), self._stream(),
                                           self.flags))


class ShardedSquare:
    """Buffers and phases of one rank of a row-sharded square of width k over n ranks."""

    def __init__(self, k, rank, n, steps):
        import torch
        if n < 1 or (n & (n - 1)) or n > k:
            raise ValueError(f"world size must be a power of two <= k: got {n}")
        self.k, self.rank, self.n, self.steps = k, rank, n, steps
        self.rows_per_rank, self.w = k // n, 2 * k // n
        u8, i32 = torch.uint8, torch.int32
        S, W = _lib.SHARE_SIZE, 2 * k
        e = steps.empty
        self.ods_rows = e((self.rows_per_rank, k, S), u8)
        self.slab = e((W, self.w, S), u8)
        # one rank: the all-to-all is the identity, so the row pass writes the slab's top
        # half directly (no 2k x k-cell copy)
        self.send = self.slab[:k].view(1, k, W, S) if n == 1 else e((n, self.rows_per_rank, self.w, S), u8)
        # this rank's record block, the all-gather's send buffer: row subtrees, column
        # roots, then a record whose first int32 is the step-2 status
        S = W + self.w + 1
        self.pack = e((S, RECORD), u8)
        self.row_sub = self.pack[:W]
        self.col_rec = self.pack[W:W + self.w]
        self.status_rec = self.pack[W + self.w].view(i32)[:1]
        self.gathered = e((n, S, RECORD), u8)
        self.status = e((1,), i32)  # the finish's: max over ranks, or EORDER across slabs
        self.row_roots = e((W, _lib.NMT_NODE_SIZE), u8)
        self.col_roots = e((W, _lib.NMT_NODE_SIZE), u8)
        self.dah = e((32,), u8)

    def row_range(self):
        return self.rank * self.rows_per_rank, (self.rank + 1) * self.rows_per_rank

    # -- phases (a driver may interleave them across simulated ranks)
    def phase_rows(self):
        self.steps.rows(self.ods_rows, self.k, self.n, self.send)

    def exchange(self, comm):
        if self.n == 1:  # send aliases the slab's top half
            return
        top = self.slab[: self.k].view(self.n, self.rows_per_rank, self.w, _lib.SHARE_SIZE)
        comm.all_to_all(top.view(-1), self.send.view(-1))

    def phase_cols(self):
        self.steps.cols(self.slab, self.k, self.n, self.rank, self.col_rec, self.row_sub, self.status_rec)

    def gather(self, comm):
        comm.all_gather(self.gathered.view(-1), self.pack.view(-1))

    def phase_finish(self):
        self.steps.finish(self.gathered, self.k, self.n, self.row_roots, self.col_roots, self.dah, self.status)

    def scope(self):
        sc = getattr(self.steps, "scope", None)
        return sc() if sc else contextlib.nullcontext()

    def run(self, comm):
        with self.scope():
            self.phase_rows()
            self.exchange(comm)
            self.phase_cols()
            self.gather(comm)
            self.phase_finish()
        return self

    def check_status(self):
        st = int(self.status.cpu().item())
        if st:
            raise _lib.CelError(st, "invalid push order: leaf namespaces must be non-decreasing")


def run_pipelined(squares, comm):
    """Several independent squares in flight on one rank (each ShardedSquare with its own
    DeviceSteps: own stream and workspace), phases interleaved so one square's
    latency-bound tree levels overlap another's encode and leaf hashing. Every rank issues
    the collectives in the same order (square 0's all-to-all, square 1's, ..., then the
    gathers), as RCCL requires. comm None: one rank, no collectives."""
    for sq in squares:
        with sq.scope():
            sq.phase_rows()
            if comm is not None:
                sq.exchange(comm)
    for sq in squares:
        with sq.scope():
            sq.phase_cols()
            if comm is not None:
                sq.gather(comm)
            else:
                sq.gathered[0].copy_(sq.pack)
    for sq in squares:
        with sq.scope():
            sq.phase_finish()
    return squares


class LocalComm:
    """Collectives among ShardedSquare objects of one process (single-GPU rehearsal of
    the N-rank schedule: same buffers, same layouts, copies instead of RCCL)."""

    @staticmethod
    def run(squares):
        import torch
        with squares[0].scope():
            return LocalComm._run(squares)

    @staticmethod
    def _run(squares):
        import torch
        n = len(squares)
        for s in squares:
            s.phase_rows()
        for h, dst in enumerate(squares):  # block h of every sender -> receiver h, sender order
            top = dst.slab[: dst.k].view(n, dst.rows_per_rank, dst.w, _lib.SHARE_SIZE)
            for r, src in enumerate(squares):
                if top[r].data_ptr() != src.send[h].data_ptr():  # aliased at n = 1
                    top[r].copy_(src.send[h])
        for s in squares:
            s.phase_cols()
        gathered = torch.stack([s.pack for s in squares])
        for s in squares:
            s.gathered.copy_(gathered)
            s.phase_finish()
        return squares
