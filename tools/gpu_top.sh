#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_square.py tests/test_gpu_wrapper.py tests/test_gpu_repair.py -m gpu -v -x --timeout 60 --timeout-method thread > gpurun_out/pytest_top.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/pytest_top.log | tail -3; [ $rc -eq 0 ] || exit $rc
for t in 0 1; do
  echo "== CEL_NMT_TOP=$t"; CEL_NMT_TOP=$t timeout -k 10 60 python3 tools/prof_phase.py --phase commit --batch 16 --reps 5 || exit 1
done
timeout -k 10 90 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_commit3 -o run --output-format csv -- python3 tools/prof_phase.py --phase commit --batch 16 --reps 5 > /dev/null 2>&1; echo "prof rc=$?"
python3 tools/kstats.py gpurun_out/prof_commit3
for t in 0 1; do
  CEL_NMT_TOP=$t timeout -k 10 120 python -u bench.py --no-cpu > gpurun_out/b.log 2>&1 || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/b.log').read().strip().split('\n')[-1])
print('NMT_TOP=$t bench value=%.0f rs_us=%.1f rs_frac=%.3f nmt_us=%.1f nmt_frac=%.3f' % (d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['roofline_nmt']['avg_launch_us'], d['roofline_nmt']['frac']))"
done
