"""rsmt2d v0.14.0 surface over the device library (Codec, ExtendedDataSquare, Repair).

Mirrors the pieces of github.com/celestiaorg/rsmt2d that celestia-app uses
(pkg/da/data_availability_header.go:45-74, pkg/appconsts/global_consts.go:92):
  LeoRSCodec: Encode / Decode / MaxChunks / Name / ValidateChunkSize
  ComputeExtendedDataSquare, ExtendedDataSquare.{RowRoots, ColRoots, Row, Col,
  GetCell, Flattened, Width, Repair}
All arithmetic runs in libcelestia_eds.so (HIP); this module marshals bytes.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import CelError

Row, Col = 0, 1  # rsmt2d.Axis


class ErrByzantineData(CelError):
    def __init__(self, axis, index, message):
        super().__init__(_lib.EBYZANTINE, message)
        self.Axis = axis
        self.Index = index


class ErrUnrepairableDataSquare(CelError):
    def __init__(self, message="failed to solve data square"):
        super().__init__(_lib.EUNREPAIRABLE, message)


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class LeoRSCodec:
    """rsmt2d.NewLeoRSCodec(): Leopard GF(2^8) (<=256 shards) / GF(2^16)."""

    def __init__(self, ctx=None):
        self.ctx = ctx or _lib.default_context()

    def Name(self):
        return _lib.load().cel_codec_name().decode()

    def MaxChunks(self):
        return int(_lib.load().cel_codec_max_chunks())

    def ValidateChunkSize(self, chunk_size):
        if _lib.load().cel_codec_validate_chunk_size(int(chunk_size)) != _lib.OK:
            raise CelError(_lib.ECHUNK, f"chunkSize {chunk_size} must be a multiple of 64 bytes")

    def Encode(self, data):
        """data: list of n equal-length byte strings -> list of n parity shards."""
        arr = np.frombuffer(b"".join(bytes(d) for d in data), np.uint8).copy()
        n = len(data)
        ln = len(data[0]) if n else 0
        par = np.zeros(n * ln, np.uint8)
        self.ctx.check(self.ctx.lib.cel_codec_encode(self.ctx.handle, _p(arr), n, ln, _p(par)))
        return [par[i * ln:(i + 1) * ln].tobytes() for i in range(n)]

    def Decode(self, shards):
        """shards: list of 2n entries (None = missing) -> full list of 2n shards."""
        n2 = len(shards)
        ln = next(len(s) for s in shards if s is not None)
        buf = np.zeros(n2 * ln, np.uint8)
        present = np.zeros(n2, np.uint8)
        for i, s in enumerate(shards):
            if s is not None:
                buf[i * ln:(i + 1) * ln] = np.frombuffer(bytes(s), np.uint8)
                present[i] = 1
        self.ctx.check(self.ctx.lib.cel_codec_decode(self.ctx.handle, _p(buf), _p(present), n2 // 2, ln))
        return [buf[i * ln:(i + 1) * ln].tobytes() for i in range(n2)]


def NewLeoRSCodec():
    return LeoRSCodec()


class ExtendedDataSquare:
    """2k x 2k square of 512-byte cells, row-major (rsmt2d flattened layout)."""

    def __init__(self, cells: np.ndarray, row_roots=None, col_roots=None, ctx=None):
        self.cells = cells  # (W, W, share) uint8
        self._row_roots = row_roots
        self._col_roots = col_roots
        self.ctx = ctx or _lib.default_context()

    def Width(self):
        return self.cells.shape[0]

    def GetCell(self, r, c):
        return self.cells[r, c].tobytes()

    def Row(self, r):
        return [self.cells[r, c].tobytes() for c in range(self.Width())]

    def Col(self, c):
        return [self.cells[r, c].tobytes() for r in range(self.Width())]

    def Flattened(self):
        return [self.cells[r, c].tobytes() for r in range(self.Width()) for c in range(self.Width())]

    def RowRoots(self):
        if self._row_roots is None:
            self._compute_roots()
        return [r.tobytes() for r in self._row_roots]

    def ColRoots(self):
        if self._col_roots is None:
            self._compute_roots()
        return [r.tobytes() for r in self._col_roots]

    def _compute_roots(self):
        w = self.Width()
        rr = np.zeros((w, _lib.NMT_NODE_SIZE), np.uint8)
        cr = np.zeros((w, _lib.NMT_NODE_SIZE), np.uint8)
        for axis, out in ((Row, rr), (Col, cr)):
            for i in range(w):
                cells = np.ascontiguousarray(self.cells[i] if axis == Row else self.cells[:, i])
                self.ctx.check(self.ctx.lib.cel_axis_root(self.ctx.handle, _p(cells), w // 2, i,
                                                          _lib.SHARE_SIZE, _p(out[i]), 0))
        self._row_roots, self._col_roots = rr, cr

    def Repair(self, row_roots, col_roots, present=None):
        """Fill every missing cell (present mask False, or a cell set to None via
        `present`) and verify against the roots. Raises ErrByzantineData /
        ErrUnrepairableDataSquare like rsmt2d."""
        w = self.Width()
        mask = np.ones((w, w), np.uint8) if present is None else np.ascontiguousarray(present, np.uint8)
        rr = np.frombuffer(b"".join(row_roots), np.uint8).copy()
        cr = np.frombuffer(b"".join(col_roots), np.uint8).copy()
        cells = np.ascontiguousarray(self.cells)
        ba, bi = ctypes.c_int32(-1), ctypes.c_int32(-1)
        st = self.ctx.lib.cel_repair(self.ctx.handle, _p(cells), _p(mask), w // 2, _lib.SHARE_SIZE, _p(rr),
                                     _p(cr), ctypes.byref(ba), ctypes.byref(bi))
        if st == _lib.EBYZANTINE:
            raise ErrByzantineData(ba.value, bi.value, self.ctx.lib.cel_last_error(self.ctx.handle).decode())
        if st == _lib.EUNREPAIRABLE:
            raise ErrUnrepairableDataSquare()
        self.ctx.check(st)
        self.cells = cells
        self._row_roots = np.frombuffer(rr.tobytes(), np.uint8).reshape(w, -1).copy()
        self._col_roots = np.frombuffer(cr.tobytes(), np.uint8).reshape(w, -1).copy()
        return mask


def ComputeExtendedDataSquare(data, codec=None, tree_constructor=None, ctx=None):
    """rsmt2d.ComputeExtendedDataSquare with the default wrapper constructor: one device
    pass computes the EDS and all 4k roots."""
    from . import da
    return da._extend(data, ctx=ctx, order_check=True)


def ImportExtendedDataSquare(flattened, codec=None, tree_constructor=None, ctx=None):
    n = len(flattened)
    w = int(round(n ** 0.5))
    cells = np.frombuffer(b"".join(flattened), np.uint8).reshape(w, w, -1).copy()
    return ExtendedDataSquare(cells, ctx=ctx)
