#!/bin/bash
# RS-only A/B of buffer cache-policy bits (CEL_RS_CP) on the hybrid axis kernel.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_square.py -q --timeout 150 --timeout-method thread > gpurun_out/pytest_cp.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_cp.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do for cp in 0 1 2 3; do
  CEL_RS_CP=$cp timeout -k 10 120 python -u tools/rs_chunks.py --k 128 --batch 256 --chunks 256 --inplace --reps 10 > gpurun_out/rs_cp.log 2>&1
  rc=$?; echo -n "r$round cp=$cp: "; tail -1 gpurun_out/rs_cp.log; [ $rc -eq 0 ] || exit $rc
done; done
exit 0
