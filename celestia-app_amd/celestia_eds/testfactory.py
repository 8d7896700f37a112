"""Synthetic ODS generator (restates test/util/testfactory/common.go:36-50 and
namespace.go:15-28 GenerateRandNamespacedRawData): 512 random bytes per share,
bytes [0:29] overwritten by a random version-0 blob namespace
0x00 || 0x00*18 || rand(10) (primary-reserved IDs re-drawn), all shares sorted
lexicographically, so every row and column of the k x k ODS is namespace-ordered.
"""
import numpy as np

SHARE = 512
NS = 29


def random_ods(k, seed, share=SHARE):
    rng = np.random.default_rng(seed)
    n = k * k
    shares = rng.integers(0, 256, (n, share), dtype=np.uint8)
    shares[:, :19] = 0
    ids = rng.integers(0, 256, (n, 10), dtype=np.uint8)
    reserved = ~ids[:, :9].any(axis=1)
    while reserved.any():
        ids[reserved] = rng.integers(0, 256, (int(reserved.sum()), 10), dtype=np.uint8)
        reserved = ~ids[:, :9].any(axis=1)
    shares[:, 19:29] = ids
    order = np.argsort(shares.view(f"S{share}").ravel(), kind="stable")
    return np.ascontiguousarray(shares[order]).reshape(k, k, share)
