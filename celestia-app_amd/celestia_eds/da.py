"""pkg/da surface (pkg/da/data_availability_header.go) over the device library.

  ExtendShares(shares)            :65-75   -> one device pass (RS + NMT roots)
  NewDataAvailabilityHeader(eds)  :44-63
  ComputeDataAvailabilityHeader   both at once with no EDS copy-back (the DAH is all that
                                  app/prepare_proposal.go / process_proposal.go keep)
  DataAvailabilityHeader          :33-41, Hash :92-108, ValidateBasic :134-162,
                                  IsZero :164-170, SquareSize :205-207, Equals :86-88
  MinDataAvailabilityHeader       :179-190, MinShares :193-196
  SquareSize / RoundUpPowerOfTwo  :205-215
"""
import ctypes
import math

import numpy as np

from . import _lib
from ._lib import CelError
from .rsmt2d import ExtendedDataSquare

SHARE_SIZE = _lib.SHARE_SIZE
MIN_SQUARE_SIZE = 1                # appconsts.MinSquareSize
DEFAULT_SQUARE_SIZE_UPPER_BOUND = 128  # appconsts.DefaultSquareSizeUpperBound
MAX_EXTENDED_SQUARE_WIDTH = DEFAULT_SQUARE_SIZE_UPPER_BOUND * 2
MIN_EXTENDED_SQUARE_WIDTH = MIN_SQUARE_SIZE * 2
TAIL_PADDING_NAMESPACE = b"\xff" * 28 + b"\xfe"


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def RoundUpPowerOfTwo(n):
    r = 1
    while r < n:
        r <<= 1
    return r


def SquareSize(n):
    return RoundUpPowerOfTwo(int(math.ceil(math.sqrt(n))))


def _is_pow2(n):
    return n > 0 and (n & (n - 1)) == 0


def _ods_buffer(shares):
    """The share list (or an (n, share_size) array) of ExtendShares as one contiguous
    buffer, with the checks the C side cannot make (it receives only n and the share size):
    data_availability_header.go:67-69's power-of-two count, and rsmt2d's equal chunk sizes
    (newDataSquare [dep]: every chunk as long as the first). A share size other than 512
    then gets the library's own ECHUNK. Returns (ods, n, share_size)."""
    n = len(shares)
    if not _is_pow2(n):
        raise CelError(_lib.ENOTPOW2, f"number of shares is not a power of 2: got {n}")
    if isinstance(shares, np.ndarray):
        if shares.ndim != 2:
            raise CelError(_lib.EINVAL, f"shares must be an (n, share_size) array: got shape {shares.shape}")
        ods = np.ascontiguousarray(shares, np.uint8).reshape(-1)
        size = shares.shape[1]
    else:
        chunks = [bytes(s) for s in shares]
        size = len(chunks[0])
        if any(len(c) != size for c in chunks):
            raise CelError(_lib.ECHUNK, "non-nil chunks not all of equal size")
        ods = np.frombuffer(b"".join(chunks), np.uint8).copy()
    if ods.size != n * size:
        raise CelError(_lib.EINVAL, f"share buffer holds {ods.size} bytes, not {n} x {size}")
    return ods, n, size


def _extend(shares, ctx=None, order_check=True):
    ods, n, size = _ods_buffer(shares)  # input errors before any device is touched
    ctx = ctx or _lib.default_context()
    k = SquareSize(n)
    eds = np.zeros((2 * k, 2 * k, SHARE_SIZE), np.uint8)
    rr = np.zeros((2 * k, _lib.NMT_NODE_SIZE), np.uint8)
    cr = np.zeros((2 * k, _lib.NMT_NODE_SIZE), np.uint8)
    dah = np.zeros(32, np.uint8)
    ctx.check(ctx.lib.cel_extend_shares(ctx.handle, _p(ods), n, size, _p(eds), _p(rr), _p(cr), _p(dah),
                                        _lib.FLAG_ORDER_CHECK if order_check else 0))
    out = ExtendedDataSquare(eds, rr, cr, ctx=ctx)
    out._dah = dah.tobytes()
    return out


def ExtendShares(shares):
    """da.ExtendShares: [][]byte (k*k shares) -> *rsmt2d.ExtendedDataSquare."""
    return _extend(shares)


def ComputeDataAvailabilityHeader(shares, ctx=None):
    """NewDataAvailabilityHeader(ExtendShares(shares)) for callers that keep only the DAH:
    app/prepare_proposal.go:61-92 and app/process_proposal.go:138-156 extend the square,
    build the DAH and use nothing but dah.Hash() ("the eds is not returned here"). One
    device pass with no EDS copied back (cel_extend_shares with eds_out = NULL): the ODS
    goes up, the 4k roots and the hash come down. Same errors as ExtendShares."""
    ods, n, size = _ods_buffer(shares)  # input errors before any device is touched
    ctx = ctx or _lib.default_context()
    k = SquareSize(n)
    rr = np.zeros((2 * k, _lib.NMT_NODE_SIZE), np.uint8)
    cr = np.zeros((2 * k, _lib.NMT_NODE_SIZE), np.uint8)
    dah = np.zeros(32, np.uint8)
    ctx.check(ctx.lib.cel_extend_shares(ctx.handle, _p(ods), n, size, None, _p(rr), _p(cr), _p(dah),
                                        _lib.FLAG_ORDER_CHECK))
    out = DataAvailabilityHeader([r.tobytes() for r in rr], [c.tobytes() for c in cr])
    out.hash = dah.tobytes()
    return out


class DataAvailabilityHeader:
    def __init__(self, RowRoots=None, ColumnRoots=None):
        self.RowRoots = list(RowRoots or [])
        self.ColumnRoots = list(ColumnRoots or [])
        self.hash = b""

    def Hash(self):
        """data_availability_header.go:92-108: merkle.HashFromByteSlices over the
        rowsCount row roots followed by the first rowsCount column roots (nil slices where
        there are fewer columns), roots of any length. 90-byte roots with as many columns
        as rows take the NMT-root kernel (cel_dah_hash), anything else the generic one
        (cel_merkle_hash_slices)."""
        if self.hash:
            return self.hash
        ctx = _lib.default_context()
        w = len(self.RowRoots)
        out = np.zeros(32, np.uint8)
        if w == len(self.ColumnRoots) and all(len(r) == _lib.NMT_NODE_SIZE for r in self.RowRoots + self.ColumnRoots):
            rr = np.frombuffer(b"".join(self.RowRoots), np.uint8).copy() if w else np.zeros(1, np.uint8)
            cr = np.frombuffer(b"".join(self.ColumnRoots), np.uint8).copy() if w else np.zeros(1, np.uint8)
            ctx.check(ctx.lib.cel_dah_hash(ctx.handle, _p(rr), _p(cr), w, _p(out)))
        else:
            cols = list(self.ColumnRoots[:w]) + [b""] * max(0, w - len(self.ColumnRoots))
            slices = [bytes(r) for r in self.RowRoots] + [bytes(c) for c in cols]
            offs = np.zeros(len(slices) + 1, np.uint64)
            offs[1:] = np.cumsum([len(x) for x in slices], dtype=np.uint64) if slices else []
            data = np.frombuffer(b"".join(slices) or b"\0", np.uint8).copy()
            ctx.check(ctx.lib.cel_merkle_hash_slices(ctx.handle, _p(data), _p(offs), len(slices), _p(out)))
        self.hash = out.tobytes()
        return self.hash

    def String(self):
        return self.Hash().hex().upper()

    def Equals(self, other):
        return self.Hash() == other.Hash()

    def IsZero(self):
        return len(self.ColumnRoots) == 0 or len(self.RowRoots) == 0

    def SquareSize(self):
        return len(self.RowRoots) // 2

    def ToProto(self):
        """celestia.core.v1.da.DataAvailabilityHeader wire bytes
        (proto/celestia/core/v1/da/data_availability_header.proto: 1 = repeated bytes
        row_roots, 2 = repeated bytes column_roots; data_availability_header.go:110-119)."""
        out = bytearray()
        for tag, roots in ((0x0A, self.RowRoots), (0x12, self.ColumnRoots)):
            for r in roots:
                out.append(tag)
                out += _uvarint(len(r)) + bytes(r)
        return bytes(out)

    def ValidateBasic(self):
        if len(self.ColumnRoots) < MIN_EXTENDED_SQUARE_WIDTH or len(self.RowRoots) < MIN_EXTENDED_SQUARE_WIDTH:
            raise CelError(_lib.EINVAL, "minimum valid DataAvailabilityHeader has at least "
                                        f"{MIN_EXTENDED_SQUARE_WIDTH} row and column roots")
        if len(self.ColumnRoots) > MAX_EXTENDED_SQUARE_WIDTH or len(self.RowRoots) > MAX_EXTENDED_SQUARE_WIDTH:
            raise CelError(_lib.EINVAL, "maximum valid DataAvailabilityHeader has at most "
                                        f"{MAX_EXTENDED_SQUARE_WIDTH} row and column roots")
        if len(self.ColumnRoots) != len(self.RowRoots):
            raise CelError(_lib.EINVAL, "unequal number of row and column roots: row "
                                        f"{len(self.RowRoots)} col {len(self.ColumnRoots)}")
        if len(self.Hash()) != 32:
            raise CelError(_lib.EINVAL, f"wrong hash: expected size to be 32 bytes, got {len(self.Hash())} bytes")


def _uvarint(n):
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        out.append(b | (0x80 if n else 0))
        if not n:
            return bytes(out)


def DataAvailabilityHeaderFromProto(buf):
    """data_availability_header.go:121-131: decode, then ValidateBasic (raises CelError)."""
    rows, cols, i = [], [], 0
    buf = bytes(buf)
    while i < len(buf):
        key, i = _read_uvarint(buf, i)
        if key & 7 != 2:
            raise CelError(_lib.EINVAL, "proto: wrong wire type for DataAvailabilityHeader")
        ln, i = _read_uvarint(buf, i)
        if i + ln > len(buf):
            raise CelError(_lib.EINVAL, "proto: unexpected EOF")
        if key >> 3 == 1:
            rows.append(buf[i:i + ln])
        elif key >> 3 == 2:
            cols.append(buf[i:i + ln])
        i += ln
    dah = DataAvailabilityHeader(rows, cols)
    dah.ValidateBasic()
    return dah


def _read_uvarint(buf, i):
    v, shift = 0, 0
    while True:
        if i >= len(buf) or shift > 63:
            raise CelError(_lib.EINVAL, "proto: bad varint")
        b = buf[i]
        i += 1
        v |= (b & 0x7F) << shift
        if not b & 0x80:
            return v, i
        shift += 7


def NilDataAvailabilityHeaderHash():
    """(*DataAvailabilityHeader)(nil).Hash() == merkle.HashFromByteSlices(nil)."""
    return DataAvailabilityHeader().Hash()


def NewDataAvailabilityHeader(eds):
    dah = DataAvailabilityHeader(eds.RowRoots(), eds.ColRoots())
    dah.Hash()
    return dah


def EmptySquareShares():
    """shares.TailPaddingShares(appconsts.MinShareCount = 1) (data_availability_header.go:197-201)."""
    share = TAIL_PADDING_NAMESPACE + b"\x01" + b"\x00" * 4
    return [share + b"\x00" * (SHARE_SIZE - len(share))]


def MinShares():
    """One tail-padding share: shares.ToBytes(EmptySquareShares()) (data_availability_header.go:192-195)."""
    return EmptySquareShares()


def MinDataAvailabilityHeader():
    return NewDataAvailabilityHeader(ExtendShares(MinShares()))
