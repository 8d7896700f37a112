"""Oracle-backed per-rank steps of the row-sharded square (test infrastructure).

Same interface as celestia_eds.sharded.DeviceSteps, computed by the CPU oracle on CPU
tensors, so the CPU tests can drive the real orchestration (ShardedSquare + TorchComm
over gloo, world size > 1) and check its layouts, collective order and subtree
combination against oracle.extend_and_commit of the whole square.
"""
import hashlib

import numpy as np
import torch

import oracle

NS = 29
PARITY_NS = b"\xff" * NS
EORDER = 5


def record(node90: bytes) -> np.ndarray:
    return np.frombuffer(node90 + bytes(6), np.uint8)


def hash_node(left: bytes, right: bytes) -> bytes:
    """nmt HashNode with IgnoreMaxNamespace (test/util/malicious/hasher.go:264-300)."""
    max_ns = left[NS:2 * NS] if right[:NS] == PARITY_NS else right[NS:2 * NS]
    return left[:NS] + max_ns + hashlib.sha256(b"\x01" + left + right).digest()


class OracleSteps:
    def __init__(self, order_check=True):
        self.order_check = order_check

    @staticmethod
    def empty(shape, dtype):
        return torch.zeros(shape, dtype=dtype)

    def rows(self, ods_rows, k, n, send):
        w = 2 * k // n
        for i in range(ods_rows.shape[0]):
            data = ods_rows[i].numpy()
            full = np.concatenate([data, oracle.rs_encode(data)])
            for h in range(n):
                send[h, i] = torch.from_numpy(full[h * w:(h + 1) * w])

    def cols(self, slab, k, n, rank, col_rec, row_sub, status):
        w, c0 = 2 * k // n, rank * (2 * k // n)
        s = slab.numpy()
        for j in range(w):
            s[k:, j] = oracle.rs_encode(np.ascontiguousarray(s[:k, j]))
        bad = False
        for j in range(w):
            rc, root = oracle.axis_root(np.ascontiguousarray(s[:, j]), k, c0 + j, self.order_check)
            bad |= rc != 0
            col_rec[j] = torch.from_numpy(record(root).copy())
        for i in range(2 * k):
            leaves = []
            for j in range(w):
                cell = s[i, j].tobytes()
                ns = cell[:NS] if (i < k and c0 + j < k) else PARITY_NS
                leaves.append(ns + cell)
            rc, root = oracle.nmt_root(leaves, self.order_check)
            bad |= rc != 0
            row_sub[i] = torch.from_numpy(record(root).copy())
        status[0] = EORDER if bad else 0

    def finish(self, gathered, k, n, row_roots, col_roots, dah, status):
        w, W = 2 * k // n, 2 * k
        g = gathered.numpy()
        subs = g[:, :W]
        col_rec_all = torch.from_numpy(np.ascontiguousarray(g[:, W:W + w]).reshape(W, -1))
        st = int(max(np.frombuffer(g[r, W + w, :4].tobytes(), np.int32)[0] for r in range(n)))
        bad = False
        for i in range(2 * k):
            nodes = [subs[r, i, :90].tobytes() for r in range(n)]
            if self.order_check and i < k:
                for r in range(1, n):
                    if r * w < k and nodes[r][:NS] < nodes[r - 1][NS:2 * NS]:
                        bad = True
            while len(nodes) > 1:
                nodes = [hash_node(nodes[2 * j], nodes[2 * j + 1]) for j in range(len(nodes) // 2)]
            row_roots[i] = torch.from_numpy(np.frombuffer(nodes[0], np.uint8).copy())
        col_roots.copy_(col_rec_all[:, :90])
        dah.copy_(torch.from_numpy(np.frombuffer(oracle.dah_hash(row_roots.numpy(), col_roots.numpy()), np.uint8).copy()))
        status[0] = EORDER if bad else st
