#!/bin/bash
# Hybrid transform with bfi transposes: GPU parity, then RS-only timings
# (full / memory-only / transform-only) and the Infinity-Cache chunk schedule.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-hyb2}
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu_$TAG.log; [ $rc -eq 0 ] || exit $rc
for cfg in "CEL_RS_DEBUG=0" "CEL_RS_DEBUG=1" "CEL_RS_DEBUG=2" "CEL_RS_HYB=0" "CEL_RS_CHUNK=8" "CEL_RS_CHUNK=16" "CEL_RS_CHUNK=32" "CEL_RS_CHUNK=16 CEL_RS_DEBUG=1"; do
  env $cfg timeout -k 10 120 python -u tools/rs_chunks.py --k 128 --batch 256 --chunks 256 --inplace --reps 10 > gpurun_out/rs_$TAG.log 2>&1
  rc=$?; echo -n "$cfg: "; tail -1 gpurun_out/rs_$TAG.log; [ $rc -eq 0 ] || exit $rc
done
exit 0
