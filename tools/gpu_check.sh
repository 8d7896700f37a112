#!/bin/bash
# One GPU session: parity tests -> smoke -> short bench. Every GPU step has its own
# time limit; a crash/abort/timeout stops the script (no further GPU work).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
ok_or_fail() {  # $1 = rc of a test step: 0 pass, 1 test failures (still safe to go on)
  case "$1" in 0|1) return 0 ;; *) echo "step died with rc=$1; stopping"; exit "$1" ;; esac
}
timeout -k 10 ${PYTEST_TIMEOUT:-420} python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread \
  ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log; ok_or_fail $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 240 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
exit $rc
