#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
CEL_EDS_LIB=$PWD/build_variants/lib_ILP2.so timeout -k 10 170 python -u -m pytest tests/test_gpu_square.py -m gpu -q -x --timeout 60 --timeout-method thread > gpurun_out/pytest_ilp.log 2>&1
rc=$?; echo "pytest(ILP2) rc=$rc"; tail -1 gpurun_out/pytest_ilp.log; [ $rc -eq 0 ] || exit $rc
for v in default ILP2; do
  if [ $v = default ]; then unset CEL_EDS_LIB; else export CEL_EDS_LIB=$PWD/build_variants/lib_$v.so; fi
  echo "== $v"
  timeout -k 10 60 python3 tools/rs_chunks.py --k 128 --batch 32 --chunks 32 || exit 1
  CEL_RS_DEBUG=2 timeout -k 10 60 python3 tools/rs_chunks.py --k 128 --batch 32 --chunks 32 || exit 1
  timeout -k 10 60 python3 tools/rs_chunks.py --k 64 --batch 64 --chunks 64 || exit 1
done
