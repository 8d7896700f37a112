#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 250 python -u -m pytest tests/test_gpu_square.py tests/test_gpu_codec.py tests/test_sharded.py tests/test_gpu_repair.py -m gpu -v -x --timeout 100 --timeout-method thread > gpurun_out/pytest_gf16b.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/pytest_gf16b.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 60 python3 tools/prof_phase.py --phase extend --k 512 --batch 1 --reps 5 || exit 1
timeout -k 10 60 python3 tools/prof_phase.py --phase extend --k 256 --batch 4 --reps 5 || exit 1
timeout -k 10 120 python -u bench.py --mode sharded --k 512 --no-cpu > gpurun_out/b512.log 2>&1 || exit 1
tail -1 gpurun_out/b512.log | cut -c1-600
