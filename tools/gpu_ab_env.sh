#!/bin/bash
# A/B of environment settings (e.g. CEL_RS_IMPL) on one box, after the GPU parity tests.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_gpu.log; case $rc in 0|1) ;; *) exit $rc ;; esac
for round in 1 2; do
  for env in ${ENVS:-X=0}; do
    env $env timeout -k 10 120 python -u bench.py --no-cpu ${BENCH_ARGS:-} > gpurun_out/ab.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "bench $env rc=$rc"; tail -3 gpurun_out/ab.log; exit $rc; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/ab.log').read().strip().split('\n')[-1])
print('r$round $env value=%.0f rs_us=%.1f rs_frac=%.3f nmt_us=%.1f' % (d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['roofline_nmt']['avg_launch_us']))"
  done
done
exit 0
