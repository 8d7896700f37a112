"""Generates the committed golden fixtures in this directory (run in the build
container, where /root/reference exists; the GPU box only reads the outputs).

Fixtures:
  block408_txs.bin.gz  the 408 block's transactions as in the reference fixture
                       (data, not code): records of u32 little-endian length || tx bytes
  block408_ods.bin.gz  the k=32 ODS of mainnet block 408, built from
                       /root/reference/x/blob/test/testdata/block_response.json by the
                       go-square layout restatement in oracle/square_layout.py
  golden.json          expected hashes:
    - block 408: data root = the block header's data_hash (pinned by the reference),
      plus the oracle's ODS/EDS digests and corner roots
    - DAH known answers of pkg/da/data_availability_header_test.go:15-68
    - Leopard model digests
"""
import base64
import gzip
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402
import square_layout  # noqa: E402

REF_JSON = "/root/reference/x/blob/test/testdata/block_response.json"


def model_data(k):
    j = np.arange(k)[:, None]
    i = np.arange(512)[None, :]
    return ((j * 131 + i * 7 + 1) & 0xFF).astype(np.uint8)


def main():
    oracle.set_simd(True)
    k, ods, data_hash, height = square_layout.block408_ods(REF_JSON)
    with open(REF_JSON) as f:
        txs = [base64.b64decode(t) for t in json.load(f)["block"]["data"]["txs"]]
    with gzip.open(os.path.join(HERE, "block408_txs.bin.gz"), "wb", compresslevel=9) as f:
        for t in txs:
            f.write(len(t).to_bytes(4, "little") + t)
    with gzip.open(os.path.join(HERE, "block408_ods.bin.gz"), "wb", compresslevel=9) as f:
        f.write(ods)
    eds, rr, cr, dah = oracle.extend_and_commit(np.frombuffer(ods, np.uint8).reshape(k, k, 512))
    assert dah == data_hash, "oracle does not reproduce block 408"
    golden = {
        "block408": {
            "height": height, "k": k, "ntx": len(txs),
            "data_hash": data_hash.hex(),
            "ods_sha256": hashlib.sha256(ods).hexdigest(),
            "eds_sha256": hashlib.sha256(eds.tobytes()).hexdigest(),
            "row_root_0": rr[0].tobytes().hex(), "col_root_0": cr[0].tobytes().hex(),
            "row_root_last": rr[-1].tobytes().hex(), "col_root_last": cr[-1].tobytes().hex(),
        },
        "dah_known_answers": {
            "empty": "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855",
            "min": "3d96b7d238e7e0456f6af8e7cdf0a67bd6cf9c2089ecb559c659dcaa1f880353",
            "typical_k2": "b56e4d251ac266f4b91cc5464b3fc7efcbdc888064647496d13133f0dc65ac25",
            "max_k128": "0bd3abeeacfbb0b92dfbdac4a154868e3c4e79666f7fcf6c620bb90dd3a0dcf0",
        },
        "leopard_model": {},
    }
    for kk in (2, 32, 128, 256, 512):
        p = oracle.rs_encode(model_data(kk))
        golden["leopard_model"][str(kk)] = {
            "field": 8 if 2 * kk <= 256 else 16,
            "parity_sha256": hashlib.sha256(p.tobytes()).hexdigest(),
            "parity0_head": p[0, :8].tobytes().hex(),
        }
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(golden, f, indent=1, sort_keys=True)
    print(json.dumps(golden["block408"], indent=1))


if __name__ == "__main__":
    main()
