"""Synthetic block transactions for the data-square construction tests: normal txs
(opaque bytes) and BlobTx protobufs (proto/celestia/core/v1/blob/blob.proto) with v0
blob namespaces (0x00 || 18 zero bytes || 10 random bytes, namespace.go:20-28)."""
import gzip
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def uvarint(n):
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        out.append(b | (0x80 if n else 0))
        if not n:
            return bytes(out)


def field_bytes(num, data):
    return uvarint(num << 3 | 2) + uvarint(len(data)) + data


def blob_msg(ns_id, data, share_version=0, ns_version=0):
    m = field_bytes(1, ns_id) + field_bytes(2, data)
    if share_version:
        m += uvarint(3 << 3) + uvarint(share_version)
    if ns_version:
        m += uvarint(4 << 3) + uvarint(ns_version)
    return m


def blob_tx(inner, blobs):
    """blobs: list of (ns_id (28 B), data)."""
    return field_bytes(1, inner) + b"".join(field_bytes(2, blob_msg(i, d)) for i, d in blobs) + field_bytes(3, b"BLOB")


def random_block(seed, n_normal, n_blob_txs, max_blob=6000, blobs_per_tx=(1, 3)):
    rng = np.random.default_rng(seed)
    txs = [rng.integers(0, 256, int(rng.integers(40, 700)), np.uint8).tobytes() for _ in range(n_normal)]
    for _ in range(n_blob_txs):
        nb = int(rng.integers(blobs_per_tx[0], blobs_per_tx[1] + 1))
        blobs = []
        for _ in range(nb):
            ns_id = bytes(18) + rng.integers(0, 256, 10, np.uint8).tobytes()
            blobs.append((ns_id, rng.integers(0, 256, int(rng.integers(1, max_blob)), np.uint8).tobytes()))
        txs.append(blob_tx(rng.integers(0, 256, int(rng.integers(150, 400)), np.uint8).tobytes(), blobs))
    return txs


def block408_txs():
    raw = gzip.open(os.path.join(GOLDEN, "block408_txs.bin.gz")).read()
    txs, i = [], 0
    while i < len(raw):
        n = int.from_bytes(raw[i:i + 4], "little")
        txs.append(raw[i + 4:i + 4 + n])
        i += 4 + n
    return txs
