#!/bin/bash
# Two-stream extension schedule (rows(c+1) beside cols(c)): parity, then A/B.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
CEL_RS_OVERLAP=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_square.py -m gpu -x -q -k "device_batch" --timeout 200 --timeout-method thread > gpurun_out/pytest_ovl.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_ovl.log; [ $rc -eq 0 ] || exit $rc
for ov in 0 2 4 8 16; do
  CEL_RS_OVERLAP=$ov timeout -k 10 120 python3 tools/rs_chunks.py --k 128 --batch 256 --chunks 256 --inplace | sed "s/^/overlap=$ov /" || exit 1
done
for ov in 0 4 8; do
  CEL_RS_OVERLAP=$ov timeout -k 10 120 python3 tools/rs_chunks.py --k 64 --batch 256 --chunks 256 --inplace | sed "s/^/overlap=$ov /" || exit 1
done
