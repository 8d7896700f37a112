#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_inclusion.py tests/test_gpu_proof.py tests/test_gpu_square.py -m gpu -v -x --timeout 120 --timeout-method thread > gpurun_out/pytest_new.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|Error|passed|failed" gpurun_out/pytest_new.log | tail -8; exit $rc
