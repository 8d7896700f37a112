"""Shared test setup: import paths, the `gpu` marker, golden fixtures.

`-m "not gpu"` runs the oracle-vs-golden checks, host logic and the C-ABI
load/export checks on CPU; `-m gpu` runs the parity tests through the C ABI on a
real MI355X (the oracle under oracle/ is the checker, never the thing tested).
"""
import gzip
import json
import os
import sys

import numpy as np
import pytest

try:
    # PyTorch before the library: torch brings its own HIP runtime, and the library (loaded
    # by ctypes) then binds to that same runtime, as in bench.py. Loaded the other way
    # round, torch's CUDA init reports "No HIP GPUs are available" in the same process
    # (tests/test_gpu_bench_shapes.py after a ctypes test, profiles/r6_torch_order.txt).
    import torch  # noqa: F401
except ImportError:  # the CPU suite without torch still runs
    pass

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "celestia-app_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP path through the C ABI)")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLDEN_DIR, "golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def block408_ods():
    with gzip.open(os.path.join(GOLDEN_DIR, "block408_ods.bin.gz"), "rb") as f:
        raw = f.read()
    k = 32
    return np.frombuffer(raw, np.uint8).reshape(k, k, 512)


@pytest.fixture(scope="session")
def oracle():
    import oracle as o
    o.lib()
    o.set_simd(True)
    return o


@pytest.fixture(scope="session")
def ctx():
    import celestia_eds
    return celestia_eds.default_context(0)
