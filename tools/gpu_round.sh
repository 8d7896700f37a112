#!/bin/bash
# Full round check: GPU parity tests -> smoke -> default bench (with CPU baseline)
# -> rocprofv3 kernel-trace stats of the same bench. Each GPU step has its own limit;
# any crash/abort/timeout stops the script.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-run}
timeout -k 10 ${PYTEST_TIMEOUT:-420} python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread \
  ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu_$TAG.log; case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke_$TAG.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 240 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_$TAG.log | cut -c1-1500; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
  python3 bench.py --no-cpu ${BENCH_ARGS:-} > gpurun_out/bench_prof_$TAG.log 2>&1
rc=$?; echo "prof rc=$rc"
python3 tools/kstats.py gpurun_out/prof_$TAG
exit $rc
