"""Device-resident batch API (cel_dev_*), for benchmarks and multi-GPU drivers.

PyTorch is used only as plumbing here: device memory (torch.empty on the GPU) and
the current HIP stream are handed to the C ABI as raw pointers.
"""
import ctypes

from . import _lib

NODE = _lib.NMT_NODE_SIZE


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


class SquareBatch:
    """Pre-allocated device buffers for n squares of width k.

    ods_in_eds=True: the ODS lives in quadrant Q0 of the EDS buffer (row pitch 2k
    shares), placed there by the upload (`load_ods`), and the extension reads it in
    place (d_ods = NULL in the C ABI): no separate ODS buffer and no Q0 copy pass.
    """

    def __init__(self, n, k, device=0, ctx=None, ods_in_eds=False, priority=0):
        import torch
        self.torch = torch
        self.n, self.k = n, k
        self.dev = torch.device("cuda", device)
        self.ctx = ctx or _lib.default_context(device)
        w = 2 * k
        self.ods_in_eds = ods_in_eds
        self.eds = torch.empty((n, w, w, _lib.SHARE_SIZE), dtype=torch.uint8, device=self.dev)
        # in-place mode: a strided view of Q0 (never handed to the C ABI)
        self.ods = (self.eds[:, :k, :k] if ods_in_eds else
                    torch.empty((n, k, k, _lib.SHARE_SIZE), dtype=torch.uint8, device=self.dev))
        self.row_roots = torch.empty((n, w, NODE), dtype=torch.uint8, device=self.dev)
        self.col_roots = torch.empty((n, w, NODE), dtype=torch.uint8, device=self.dev)
        self.dah = torch.empty((n, 32), dtype=torch.uint8, device=self.dev)
        self.status = torch.empty((n,), dtype=torch.int32, device=self.dev)
        ws = self.ctx.lib.cel_dev_workspace_size(k, n)
        self.work = torch.empty((ws,), dtype=torch.uint8, device=self.dev)
        # A dedicated (non-null) stream: every launch of this batch goes there, and
        # callers time it with events recorded on self.hip_stream.
        self.hip_stream = torch.cuda.Stream(device=self.dev, priority=priority)

    def load_ods(self, host):
        """Upload [n][k][k][512] host shares (uint8 array or tensor) into the ODS input."""
        t = self.torch.as_tensor(host).reshape(self.n, self.k, self.k, _lib.SHARE_SIZE)
        self.ods.copy_(t)

    def _ods_arg(self):
        return None if self.ods_in_eds else _ptr(self.ods)

    def stream(self):
        return ctypes.c_void_p(self.hip_stream.cuda_stream)

    def extend_and_commit(self, order_check=True, caller_stream=False):
        """caller_stream: the whole batch on self.hip_stream (CEL_FLAG_CALLER_STREAM), for
        callers that keep several batches in flight on their own streams."""
        c = self.ctx
        flags = (_lib.FLAG_ORDER_CHECK if order_check else 0) | (_lib.FLAG_CALLER_STREAM if caller_stream else 0)
        c.check(c.lib.cel_dev_extend_batch(c.handle, self._ods_arg(), self.n, self.k, _ptr(self.eds),
                                           _ptr(self.row_roots), _ptr(self.col_roots), _ptr(self.dah),
                                           _ptr(self.status), _ptr(self.work), self.stream(), flags))

    def extend_only(self):
        c = self.ctx
        c.check(c.lib.cel_dev_extend_only(c.handle, self._ods_arg(), self.n, self.k, _ptr(self.eds), self.stream()))

    def commit_only(self, order_check=True):
        c = self.ctx
        c.check(c.lib.cel_dev_commit_only(c.handle, _ptr(self.eds), self.n, self.k, _ptr(self.row_roots),
                                          _ptr(self.col_roots), _ptr(self.dah), _ptr(self.status),
                                          _ptr(self.work), self.stream(),
                                          _lib.FLAG_ORDER_CHECK if order_check else 0))
