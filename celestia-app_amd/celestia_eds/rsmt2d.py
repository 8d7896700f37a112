"""rsmt2d v0.14.0 surface over the device library (Codec, ExtendedDataSquare, Repair).

Mirrors the pieces of github.com/celestiaorg/rsmt2d that celestia-app uses
(pkg/da/data_availability_header.go:45-74, pkg/appconsts/global_consts.go:92):
  LeoRSCodec: Encode / Decode / MaxChunks / Name / ValidateChunkSize
  ComputeExtendedDataSquare, ImportExtendedDataSquare, ExtendedDataSquare.{RowRoots,
  ColRoots, Row, Col, GetCell, Flattened, Width, Repair}
All arithmetic runs in libcelestia_eds.so (HIP); this module marshals bytes.

Tree constructors. rsmt2d computes each axis root through the TreeConstructorFn it
was given (nmt_wrapper.go:14-17,83). The default constructor (wrapper.NewConstructor)
is served by the device pass that also extends the square. Any other constructor
(pkg/inclusion/nmt_caching.go:96-104's subtree-root cacher, test/util/malicious/
tree.go:36-71's out-of-order tree) is honoured: RowRoots/ColRoots push every cell into
a tree it builds and return that tree's Root(), exactly as rsmt2d does. A codec other
than LeoRSCodec is refused (the device implements Leopard only).
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import CelError

Row, Col = 0, 1  # rsmt2d.Axis


class ErrByzantineData(CelError):
    """rsmt2d *ErrByzantineData{Axis, Index, Shares}: Shares lists the axis's 2k shares,
    None where the repair did not know the cell (celestia-node builds bad-encoding fraud
    proofs from them, specs/src/specs/fraud_proofs.md:3-13)."""

    def __init__(self, axis, index, message, shares=None):
        super().__init__(_lib.EBYZANTINE, message)
        self.Axis = axis
        self.Index = index
        self.Shares = shares


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


def _default_constructor(tree_constructor, width):
    """True for None and for wrapper.NewConstructor(k) with k = width / 2 (served by the
    device pass). A wrapper constructor for another square size builds trees with another
    Q0 boundary (or fails to push, nmt_wrapper.go:93-99) upstream, so it is treated like
    any caller constructor: its own trees give the roots."""
    if tree_constructor is None:
        return True
    return (getattr(tree_constructor, "_cel_wrapper_constructor", False)
            and getattr(tree_constructor, "square_size", None) == width // 2)


class ExtendedDataSquare:
    """2k x 2k square of 512-byte cells, row-major (rsmt2d flattened layout)."""

    def __init__(self, cells: np.ndarray, row_roots=None, col_roots=None, ctx=None, tree_constructor=None):
        self.cells = cells  # (W, W, share) uint8
        self._row_roots = row_roots
        self._col_roots = col_roots
        self._ctx = ctx
        self._tree = None if _default_constructor(tree_constructor, cells.shape[0]) else tree_constructor

    @property
    def ctx(self):
        # bound on first device use: a square whose roots come from a caller's trees
        # needs no device
        if self._ctx is None:
            self._ctx = _lib.default_context()
        return self._ctx

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

    def FlattenedODS(self):
        """The original data square (Q0) row-major, as rsmt2d's FlattenedODS; pkg/proof
        sizes the square from it (pkg/proof/proof.go:84)."""
        k = self.Width() // 2
        return [self.cells[r, c].tobytes() for r in range(k) for c in range(k)]

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
        if self._tree is not None:
            # a caller's TreeConstructorFn: rsmt2d computeRoots pushes each axis's cells
            rr, cr = [], []
            for axis, out in ((Row, rr), (Col, cr)):
                for i in range(w):
                    tree = self._tree(axis, i)
                    for c in (self.Row(i) if axis == Row else self.Col(i)):
                        tree.Push(c)
                    out.append(np.frombuffer(bytes(tree.Root()), np.uint8))
            self._row_roots, self._col_roots = rr, cr
            return
        rr = np.zeros((w, _lib.NMT_NODE_SIZE), np.uint8)
        cr = np.zeros((w, _lib.NMT_NODE_SIZE), np.uint8)
        for axis, out in ((Row, rr), (Col, cr)):
            for i in range(w):
                cells = np.ascontiguousarray(self.cells[i] if axis == Row else self.cells[:, i])
                self.ctx.check(self.ctx.lib.cel_axis_root(self.ctx.handle, _p(cells), w // 2, i,
                                                          _lib.SHARE_SIZE, _p(out[i]), 0))
        self._row_roots, self._col_roots = rr, cr

    def Repair(self, row_roots, col_roots, present=None):
        """Fill every missing cell (present mask False) and verify against the roots.
        Raises ErrByzantineData (with the axis's Shares) / ErrUnrepairableDataSquare like
        rsmt2d, and CelError(EBADROOT) for rsmt2d's "bad root input". Returns the mask the
        square is valid under (all ones on success; the caller's array is not modified)."""
        w = self.Width()
        mask = np.ones((w, w), np.uint8) if present is None else np.array(present, np.uint8, copy=True)
        rr = np.frombuffer(b"".join(row_roots), np.uint8).copy()
        cr = np.frombuffer(b"".join(col_roots), np.uint8).copy()
        cells = np.array(self.cells, np.uint8, copy=True, order="C")
        ba, bi = ctypes.c_int32(-1), ctypes.c_int32(-1)
        bs = np.zeros((w, _lib.SHARE_SIZE), np.uint8)
        bp = np.zeros(w, np.uint8)
        st = self.ctx.lib.cel_repair(self.ctx.handle, _p(cells), _p(mask), w // 2, _lib.SHARE_SIZE, _p(rr),
                                     _p(cr), ctypes.byref(ba), ctypes.byref(bi), _p(bs), _p(bp))
        if st in (_lib.OK, _lib.EBYZANTINE, _lib.EBADROOT, _lib.EUNREPAIRABLE):
            self.cells = cells  # the most-repaired square (valid where mask is set)
            self._mask = mask
        if st == _lib.EBYZANTINE:
            shares = [bs[j].tobytes() if bp[j] else None for j in range(w)]
            raise ErrByzantineData(ba.value, bi.value, self.ctx.lib.cel_last_error(self.ctx.handle).decode(),
                                   shares)
        if st == _lib.EUNREPAIRABLE:
            raise ErrUnrepairableDataSquare()
        self.ctx.check(st)
        self._row_roots = np.frombuffer(rr.tobytes(), np.uint8).reshape(w, -1).copy()
        self._col_roots = np.frombuffer(cr.tobytes(), np.uint8).reshape(w, -1).copy()
        return mask


def _check_codec(codec):
    if codec is not None and not isinstance(codec, LeoRSCodec):
        raise CelError(_lib.EINVAL, f"unsupported codec {type(codec).__name__}: the device path implements "
                                    "rsmt2d's LeoRSCodec only")


def ComputeExtendedDataSquare(data, codec=None, tree_constructor=None, ctx=None):
    """rsmt2d.ComputeExtendedDataSquare(data, codec, treeCreatorFn). One device pass
    extends the square; with the default wrapper constructor it also computes all 4k
    roots, with any other constructor the roots come from the caller's trees."""
    from . import da
    _check_codec(codec)
    eds = da._extend(data, ctx=ctx, order_check=True)
    if not _default_constructor(tree_constructor, eds.Width()):
        eds._row_roots = eds._col_roots = None
        eds._tree = tree_constructor
    return eds


def ImportExtendedDataSquare(flattened, codec=None, tree_constructor=None, ctx=None):
    _check_codec(codec)
    n = len(flattened)
    w = int(round(n ** 0.5))
    cells = np.frombuffer(b"".join(flattened), np.uint8).reshape(w, w, -1).copy()
    return ExtendedDataSquare(cells, ctx=ctx, tree_constructor=tree_constructor)
