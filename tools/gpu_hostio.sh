#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_square.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_hostio.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_hostio.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/hostio.txt
for hc in 1 4 8; do for pin in "" "--pinned"; do
  CEL_HOST_CHUNKS=$hc timeout -k 10 200 python3 tools/host_io.py --k 128 --batch 16 --reps 5 $pin >> gpurun_out/hostio.txt 2>&1 || exit 1
done; done
CEL_HOST_CHUNKS=4 timeout -k 10 200 python3 tools/host_io.py --k 128 --batch 16 --reps 5 --pinned --no-eds >> gpurun_out/hostio.txt 2>&1 || exit 1
grep host-buffer gpurun_out/hostio.txt
