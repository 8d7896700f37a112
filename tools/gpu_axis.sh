#!/bin/bash
# A/B of the GF(2^8) encode kernels (tools/rs_chunks.py) + parity of the axis kernel.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
CEL_RS_IMPL=axis timeout -k 10 300 python -u -m pytest tests/test_gpu_square.py tests/test_gpu_codec.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_axis.log 2>&1
rc=$?; echo "pytest(axis) rc=$rc"; tail -3 gpurun_out/pytest_axis.log; [ $rc -eq 0 ] || exit $rc
for impl in perm axis; do
  CEL_RS_IMPL=$impl timeout -k 10 120 python3 tools/rs_chunks.py --k 128 --batch 32 --chunks 32 4 1 || exit 1
done
CEL_RS_IMPL=axis CEL_RS_DEBUG=1 timeout -k 10 120 python3 tools/rs_chunks.py --k 128 --batch 32 --chunks 32 4 1 || exit 1
CEL_RS_IMPL=axis CEL_RS_DEBUG=2 timeout -k 10 120 python3 tools/rs_chunks.py --k 128 --batch 32 --chunks 32 || exit 1
CEL_COPY_REF=1 CEL_RS_IMPL=axis timeout -k 10 120 python3 tools/rs_chunks.py --k 64 --batch 64 --chunks 64 || exit 1
CEL_RS_IMPL=perm timeout -k 10 120 python3 tools/rs_chunks.py --k 64 --batch 64 --chunks 64 || exit 1
