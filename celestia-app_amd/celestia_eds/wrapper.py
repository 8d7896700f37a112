"""pkg/wrapper surface (pkg/wrapper/nmt_wrapper.go) over the device library.

ErasuredNamespacedMerkleTree keeps the reference's Push-time checks and errors
(:93-114) and computes Root (:118-124) on the device: a full axis (2k pushes)
goes through cel_axis_root, a partial one through cel_nmt_root over the
namespace-prefixed leaves.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import CelError

PARITY_NAMESPACE = b"\xff" * _lib.NAMESPACE_SIZE


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class ErasuredNamespacedMerkleTree:
    def __init__(self, square_size, axis_index, ctx=None):
        if square_size == 0:
            raise ValueError("cannot create a ErasuredNamespacedMerkleTree of squareSize == 0")
        self.squareSize = int(square_size)
        self.axisIndex = int(axis_index)
        self.shareIndex = 0
        self.leaves = []  # namespace-prefixed data
        self.ctx = ctx or _lib.default_context()

    def isQuadrantZero(self):
        return self.shareIndex < self.squareSize and self.axisIndex < self.squareSize

    def Push(self, data):
        data = bytes(data)
        if self.axisIndex + 1 > 2 * self.squareSize or self.shareIndex + 1 > 2 * self.squareSize:
            raise CelError(_lib.EPUSHPAST, "pushed past predetermined square size: boundary at "
                                           f"{2 * self.squareSize} index at {self.axisIndex} {self.shareIndex}")
        if len(data) < _lib.NAMESPACE_SIZE:
            raise CelError(_lib.ESHORT, "data is too short to contain namespace ID")
        ns = data[:_lib.NAMESPACE_SIZE] if self.isQuadrantZero() else PARITY_NAMESPACE
        leaf = ns + data
        if self.leaves and leaf[:_lib.NAMESPACE_SIZE] < self.leaves[-1][:_lib.NAMESPACE_SIZE]:
            raise CelError(_lib.EORDER, "pushed data has to be lexicographically ordered by namespace IDs")
        self.leaves.append(leaf)
        self.shareIndex += 1

    def Root(self):
        n = len(self.leaves)
        out = np.zeros(_lib.NMT_NODE_SIZE, np.uint8)
        full = (n == 2 * self.squareSize and all(len(l) == _lib.NAMESPACE_SIZE + _lib.SHARE_SIZE
                                                  for l in self.leaves))
        if full:
            cells = np.frombuffer(b"".join(l[_lib.NAMESPACE_SIZE:] for l in self.leaves), np.uint8).copy()
            self.ctx.check(self.ctx.lib.cel_axis_root(self.ctx.handle, _p(cells), self.squareSize, self.axisIndex,
                                                      _lib.SHARE_SIZE, _p(out), 0))
        else:
            ln = len(self.leaves[0]) if n else _lib.NAMESPACE_SIZE
            if any(len(l) != ln for l in self.leaves):
                raise CelError(_lib.EINVAL, "device NMT root needs equal-length leaves")
            buf = np.frombuffer(b"".join(self.leaves), np.uint8).copy() if n else np.zeros(1, np.uint8)
            self.ctx.check(self.ctx.lib.cel_nmt_root(self.ctx.handle, _p(buf), n, ln, _p(out), 0))
        return out.tobytes()


    def _subtree_root(self, lo, hi):
        """NMT root over pushed leaves [lo, hi) on the device (cel_nmt_root)."""
        ln = len(self.leaves[lo])
        if any(len(l) != ln for l in self.leaves[lo:hi]):
            raise CelError(_lib.EINVAL, "device NMT root needs equal-length leaves")
        buf = np.frombuffer(b"".join(self.leaves[lo:hi]), np.uint8).copy()
        out = np.zeros(_lib.NMT_NODE_SIZE, np.uint8)
        self.ctx.check(self.ctx.lib.cel_nmt_root(self.ctx.handle, _p(buf), hi - lo, ln, _p(out), 0))
        return out.tobytes()

    def ProveRange(self, start, end):
        """nmt Proof for the leaf range [start, end) over the pushed leaves
        (nmt_wrapper.go:127-130). A full axis of 512-byte shares with 2k a power of two
        takes every node of its tree from the device (cel_axis_tree) and the proof nodes
        picked by cel_nmt_prove_range; any other tree (a partial or odd-width one, as the
        reference test's square sizes 1..16) collects nmt's proof nodes, the roots of the
        maximal subtrees outside the range under its split rule (largest power of two
        below the width), each hashed on the device (cel_nmt_root). start >= end,
        start < 0 or end past the leaves raise, as nmt's validateRange does."""
        from .proof import NMTProof, _split_point, nmt_prove_range
        start, end, n = int(start), int(end), len(self.leaves)
        if start < 0 or start >= end or end > n:
            raise CelError(_lib.EINVAL, f"invalid proof range [{start}, {end}) over {n} leaves")
        W = 2 * self.squareSize
        full = (n == W and W & (W - 1) == 0 and
                all(len(l) == _lib.NAMESPACE_SIZE + _lib.SHARE_SIZE for l in self.leaves))
        if full:
            cells = np.frombuffer(b"".join(l[_lib.NAMESPACE_SIZE:] for l in self.leaves), np.uint8).copy()
            tree = np.zeros((2 * W - 1, _lib.NMT_NODE_SIZE), np.uint8)
            self.ctx.check(self.ctx.lib.cel_axis_tree(self.ctx.handle, _p(cells), self.squareSize, self.axisIndex,
                                                      _lib.SHARE_SIZE, _p(tree)))
            return NMTProof(start, end, nmt_prove_range(tree, start, end))

        def collect(lo, hi):
            if hi <= start or lo >= end:
                return [self._subtree_root(lo, hi)]
            if start <= lo and hi <= end:
                return []
            k = _split_point(hi - lo)
            return collect(lo, lo + k) + collect(lo + k, hi)

        return NMTProof(start, end, collect(0, n))


def NewErasuredNamespacedMerkleTree(square_size, axis_index):
    return ErasuredNamespacedMerkleTree(square_size, axis_index)


def NewConstructor(square_size):
    """wrapper.NewConstructor (nmt_wrapper.go:73-86). Marked as the default constructor:
    rsmt2d.ComputeExtendedDataSquare serves it with the device pass's roots."""
    def NewTree(_axis, axis_index):
        return ErasuredNamespacedMerkleTree(square_size, axis_index)
    NewTree._cel_wrapper_constructor = True
    NewTree.square_size = square_size
    return NewTree
