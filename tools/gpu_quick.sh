#!/bin/bash
# A focused GPU pass: pytest selection ($1, -k expression) then optional bench args ($2..).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
sel="$1"; shift
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$sel" \
  > gpurun_out/quick_pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/quick_pytest.log | tail -60
tail -3 gpurun_out/quick_pytest.log
[ $rc -eq 0 ] || exit $rc
if [ $# -gt 0 ]; then
  timeout -k 10 300 python -u bench.py "$@" > gpurun_out/quick_bench.json 2> gpurun_out/quick_bench.err || { tail -20 gpurun_out/quick_bench.err; exit 1; }
  cat gpurun_out/quick_bench.json
fi
