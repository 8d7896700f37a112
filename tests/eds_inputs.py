"""Synthetic inputs shaped like the reference's test factory.

random_ods restates testfactory.GenerateRandNamespacedRawData
(test/util/testfactory/common.go:36-50, namespace.go:15-28): 512 random bytes per
share, bytes [0:29] overwritten with a random version-0 blob namespace
0x00 || 0x00*18 || rand(10) (reserved namespaces rejected), all shares sorted
lexicographically so every row and column of the ODS is namespace-ordered.
"""
import numpy as np

SHARE = 512
NS = 29


from celestia_eds.testfactory import random_ods  # noqa: E402,F401


def constant_ods(k):
    """pkg/da/data_availability_header_test.go:247-263 generateShares: namespace
    MustNewV0(0x01*10) and 0xFF fill."""
    ns = bytes([0]) + bytes(18) + bytes([1]) * 10
    sh = ns + bytes([0xFF]) * (SHARE - NS)
    return np.frombuffer(sh * (k * k), np.uint8).reshape(k, k, SHARE).copy()


def tail_padding_share():
    sh = b"\xff" * 28 + b"\xfe" + b"\x01" + bytes(4)
    return sh + bytes(SHARE - len(sh))


def model_shards(k, length=SHARE):
    """SURVEY.md Appendix A.5 model input: shard j, byte i = (j*131 + i*7 + 1) & 0xFF."""
    j = np.arange(k)[:, None]
    i = np.arange(length)[None, :]
    return ((j * 131 + i * 7 + 1) & 0xFF).astype(np.uint8)
