"""go-square v1.1.0 data-square construction, mirrored over the
C ABI's cel_square_construct (host code in csrc/square.cpp, no device needed).

  Construct(txs, max_square_size, subtree_root_threshold)
      square.Construct as called by app/extend_block.go:16-25 and
      app/process_proposal.go:121-130: the exact ordered tx list -> the k*k shares
      handed to da.ExtendShares; raises CelError if a tx does not fit or a normal tx
      follows a blob tx (go-square's error strings).
  Build(txs, max_square_size, subtree_root_threshold)
      square.Build as called by app/prepare_proposal.go:48-61: greedy, drops what does
      not fit; returns (shares, kept txs with normal txs before blob txs).

The defaults are appconsts SquareSizeUpperBound = 128 and SubtreeRootThreshold = 64
(pkg/appconsts/v1,v2/app_consts.go).
"""
import ctypes

import numpy as np

from . import _lib

SQUARE_SIZE_UPPER_BOUND = 128
SUBTREE_ROOT_THRESHOLD = 64


def _call(txs, max_square_size, subtree_root_threshold, greedy):
    l = _lib.load()
    txs = [bytes(t) for t in txs]
    lens = (ctypes.c_uint32 * max(len(txs), 1))(*[len(t) for t in txs])
    blob = b"".join(txs)
    buf = ctypes.create_string_buffer(blob, max(len(blob), 1))
    k = ctypes.c_uint32()
    included = (ctypes.c_uint8 * max(len(txs), 1))()

    def run(out, cap):
        return l.cel_square_construct(buf, lens, len(txs), max_square_size, subtree_root_threshold, greedy,
                                      out, cap, ctypes.byref(k), included)

    st = run(None, 0)
    if st != _lib.OK:
        raise _lib.CelError(st, l.cel_square_last_error().decode())
    n = k.value * k.value
    out = np.zeros((n, _lib.SHARE_SIZE), np.uint8)
    st = run(out.ctypes.data_as(ctypes.c_void_p), n)
    if st != _lib.OK:
        raise _lib.CelError(st, l.cel_square_last_error().decode())
    return out, [int(included[i]) for i in range(len(txs))]


def Construct(txs, max_square_size=SQUARE_SIZE_UPPER_BOUND, subtree_root_threshold=SUBTREE_ROOT_THRESHOLD):
    """-> uint8 array [k*k][512]: the ODS shares (shares.ToBytes of the square)."""
    return _call(txs, max_square_size, subtree_root_threshold, 0)[0]


def Build(txs, max_square_size=SQUARE_SIZE_UPPER_BOUND, subtree_root_threshold=SUBTREE_ROOT_THRESHOLD):
    """-> (shares [k*k][512], kept txs: normal txs first, then blob txs)."""
    out, kept = _call(txs, max_square_size, subtree_root_threshold, 1)
    normal = [bytes(t) for t, s in zip(txs, kept) if s == 1]
    blob = [bytes(t) for t, s in zip(txs, kept) if s == 2]
    return out, normal + blob


def TxShareRange(txs, tx_index, max_square_size=SQUARE_SIZE_UPPER_BOUND,
                 subtree_root_threshold=SUBTREE_ROOT_THRESHOLD):
    """Builder.FindTxShareRange after square.Construct(txs): (start, end) ODS shares of tx
    `tx_index` (its PFB index wrapper for a blob tx)."""
    l = _lib.load()
    txs = [bytes(t) for t in txs]
    lens = (ctypes.c_uint32 * max(len(txs), 1))(*[len(t) for t in txs])
    blob = b"".join(txs)
    buf = ctypes.create_string_buffer(blob, max(len(blob), 1))
    a, b = ctypes.c_uint32(), ctypes.c_uint32()
    st = l.cel_square_tx_range(buf, lens, len(txs), max_square_size, subtree_root_threshold, tx_index,
                               ctypes.byref(a), ctypes.byref(b))
    if st != _lib.OK:
        raise _lib.CelError(st, l.cel_square_last_error().decode())
    return a.value, b.value


def is_blob_tx(tx):
    """blob.UnmarshalBlobTx's verdict, read from a one-tx square.Build (included code 2 =
    kept blob tx; a blob tx too large for a 128 x 128 square reads as not kept)."""
    return _call([tx], SQUARE_SIZE_UPPER_BOUND, SUBTREE_ROOT_THRESHOLD, 1)[1][0] == 2
