#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 170 python -u -m pytest tests/test_gpu_square.py tests/test_gpu_codec.py -m gpu -v -x --timeout 60 --timeout-method thread > gpurun_out/pytest_rs.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_rs.log; [ $rc -eq 0 ] || exit $rc
for p in 0 4 8 16; do
  CEL_RS_PIPE=$p timeout -k 10 60 python3 tools/rs_chunks.py --k 128 --batch 32 --chunks 32 || exit 1
done
CEL_RS_PIPE=8 CEL_RS_DEBUG=1 timeout -k 10 60 python3 tools/rs_chunks.py --k 128 --batch 32 --chunks 32 || exit 1
timeout -k 10 60 python3 tools/rs_chunks.py --k 128 --batch 64 --chunks 64 || exit 1
for p in 0 16; do
  CEL_RS_PIPE=$p timeout -k 10 60 python3 tools/rs_chunks.py --k 64 --batch 64 --chunks 64 || exit 1
done
timeout -k 10 120 python -u bench.py --no-cpu > gpurun_out/b.log 2>&1 || exit 1
python3 -c "
import json; d=json.loads(open('gpurun_out/b.log').read().strip().split('\n')[-1])
print('bench value=%.0f rs_us=%.1f rs_frac=%.3f nmt_us=%.1f' % (d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['roofline_nmt']['avg_launch_us']))"
