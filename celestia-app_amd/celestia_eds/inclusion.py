"""pkg/inclusion mirror: blob share commitments read from the EDS.

  calculate_commitment_paths  paths.go:16-47 (host: cel_commitment_paths)
  gen_subtree_root_path       paths.go:49-63
  GetCommitment               get_commit.go:12-30 over device-built row trees
                              (cel_get_commitment; the reference walks the
                              EDSSubTreeRootCacher of nmt_caching.go filled while rsmt2d
                              computed the row roots)
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import CelError

WALK_LEFT, WALK_RIGHT = False, True
DEFAULT_SUBTREE_ROOT_THRESHOLD = 64


def gen_subtree_root_path(depth, pos):
    """WalkInstructions from a subtree root at (depth, pos) down: the bits of pos, most
    significant first (False = left, True = right)."""
    return [bool(pos & (1 << i)) for i in range(depth - 1, -1, -1)]


def _paths(square_size, start, blob_len, threshold):
    l = _lib.load()
    n = ctypes.c_uint32()
    st = l.cel_commitment_paths(square_size, start, blob_len, threshold, None, None, None, 0, ctypes.byref(n))
    if st != _lib.OK:
        raise CelError(st, "cannot get commitment for blob that doesn't fit in square" if st == _lib.ETOOBIG
                       else "invalid commitment path arguments")
    rows, depths, pos = (np.zeros(max(n.value, 1), np.uint32) for _ in range(3))
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    l.cel_commitment_paths(square_size, start, blob_len, threshold, P(rows), P(depths), P(pos), n.value,
                           ctypes.byref(n))
    return [(int(rows[i]), int(depths[i]), int(pos[i])) for i in range(n.value)]


def calculate_subtree_root_coordinates(max_depth, min_depth, start, end):
    """paths.go:95-173 -> [(depth, position)]"""
    l = _lib.load()
    n = ctypes.c_uint32()
    cap = 64
    d, p = np.zeros(cap, np.uint32), np.zeros(cap, np.uint32)
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    st = l.cel_subtree_root_coordinates(max_depth, min_depth, start, end, P(d), P(p), cap, ctypes.byref(n))
    if st != _lib.OK:
        raise CelError(st, "invalid subtree root coordinate arguments")
    return [(int(d[i]), int(p[i])) for i in range(min(n.value, cap))]


def calculate_commitment_paths(square_size, start, blob_len, threshold=DEFAULT_SUBTREE_ROOT_THRESHOLD):
    """-> [(row, [WalkInstruction...])] inside each row's ODS half (the reference walk
    from the row root prepends one WalkLeft)."""
    return [(r, gen_subtree_root_path(d, p)) for r, d, p in _paths(square_size, start, blob_len, threshold)]


def GetCommitment(eds, start, blob_share_len, subtree_root_threshold=DEFAULT_SUBTREE_ROOT_THRESHOLD, ctx=None):
    """The blob share commitment (32 B) of the blob of blob_share_len shares at share
    index `start` (first aligned index >= start) of the EDS's original square."""
    ctx = ctx or eds.ctx
    cells = np.ascontiguousarray(eds.cells)
    k = cells.shape[0] // 2
    out = np.zeros(32, np.uint8)
    ctx.check(ctx.lib.cel_get_commitment(ctx.handle, cells.ctypes.data_as(ctypes.c_void_p), k, _lib.SHARE_SIZE,
                                         start, blob_share_len, subtree_root_threshold,
                                         out.ctypes.data_as(ctypes.c_void_p)))
    return out.tobytes()
