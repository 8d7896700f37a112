#!/bin/bash
# A/B of library variants (CEL_EDS_LIB) on the same box + one PMC pass.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log; case $rc in 0|1) ;; *) exit $rc ;; esac
for round in 1 2; do
for v in ${VARIANTS:-libcelestia_eds.so}; do
  CEL_EDS_LIB=$PWD/celestia-app_amd/$v timeout -k 10 120 python -u bench.py --no-cpu ${BENCH_ARGS:-} > gpurun_out/ab_$v.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "bench $v rc=$rc"; tail -3 gpurun_out/ab_$v.log; exit $rc; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/ab_$v.log').read().strip().split('\n')[-1])
print('r$round $v value=%.0f rs_us=%.1f rs_frac=%.3f nmt_us=%.1f nmt_frac=%.3f' % (d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['roofline_nmt']['avg_launch_us'], d['roofline_nmt']['frac']))"
done; done
if [ -n "${PMC:-}" ]; then
  timeout -s KILL 90 rocprofv3 --pmc $PMC -d gpurun_out/pmc -o pmc --output-format csv -- python3 bench.py --no-cpu --steps 3 --warmup 1 --phase-reps 2 > gpurun_out/pmc.log 2>&1
  echo "pmc rc=$?"
fi
exit 0
