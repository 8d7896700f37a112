#!/bin/bash
# GF(2^16) check: codec + k=256/512 square parity, then phase timings (new vs LDS kernel).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_square.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gf16.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR" gpurun_out/pytest_gf16.log | tail -40; case $rc in 0|1) ;; *) exit $rc ;; esac
for k in 256 512; do
  for impl in reg lds; do
    CEL_GF16_IMPL=$impl timeout -k 10 60 python3 tools/prof_phase.py --phase extend --k $k --batch 2 --reps 5 || exit 1
  done
  timeout -k 10 60 python3 tools/prof_phase.py --phase commit --k $k --batch 2 --reps 3 || exit 1
done
