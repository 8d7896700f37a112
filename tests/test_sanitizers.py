"""ASan + UBSan run of the host-only code (SURVEY.md §5 auxiliaries): `make -C oracle
asan` builds tests/sanitize_driver.cpp against the oracle (oracle/*.c) and the host-only
product sources (csrc/square.cpp, proof.cpp, inclusion_paths.cpp), once with
-fsanitize=address,undefined (no recovery, runtime linked statically) and once plain.
The driver feeds square construction the block-408 txs, synthetic blocks, the error
cases and the malformed-tx corpus of test_square.py, sweeps the proof and inclusion-path
entry points over valid and invalid ranges, and runs the oracle's extend / repair /
codec. The test asserts a clean sanitizer run and identical output hashes in both builds.
CPU only."""
import os
import shutil
import struct
import subprocess

import pytest

from square_inputs import blob_tx, block408_txs, random_block
from test_square import _malformed_corpus

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")


def _blocks():
    import square_layout
    mal = _malformed_corpus()
    blocks = [block408_txs(), [], random_block(1, 0, 1), random_block(3, 12, 4), random_block(6, 200, 2),
              # Construct errors: a normal tx after a blob tx; no space
              [random_block(9, 2, 1)[0], random_block(9, 2, 1)[2], random_block(9, 2, 1)[1]],
              [b"\x07" * 400_000] * 30,
              [blob_tx(b"i", [(bytes(18) + bytes(range(10)), b"\x01" * 100_000)])] * 3]
    blocks += [[t] for t in mal[:120]]
    for i in range(0, len(mal), 25):
        blocks.append(sorted(mal[i:i + 25], key=lambda t: square_layout.unmarshal_blob_tx(t) is not None))
    return blocks


def _write_blocks(path):
    with open(path, "wb") as f:
        bl = _blocks()
        f.write(struct.pack("<I", len(bl)))
        for txs in bl:
            f.write(struct.pack("<I", len(txs)))
            f.write(b"".join(struct.pack("<I", len(t)) for t in txs))
            f.write(b"".join(txs))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_code_sanitizer_clean(tmp_path):
    r = subprocess.run(["make", "-C", ORACLE, "asan"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    blocks = str(tmp_path / "blocks.bin")
    _write_blocks(blocks)
    env = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:detect_leaks=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", OMP_NUM_THREADS="1")
    out = {}
    for name in ("sanitize_driver", "plain_driver"):
        r = subprocess.run([os.path.join(ORACLE, "_asan", name), blocks], capture_output=True, text=True,
                           timeout=900, env=env)
        assert r.returncode == 0, f"{name} exit {r.returncode}:\n{r.stderr[-4000:]}"
        assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
        out[name] = r.stdout.split()
    assert len(out["plain_driver"]) == 8
    assert out["sanitize_driver"] == out["plain_driver"]
