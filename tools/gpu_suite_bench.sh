#!/bin/bash
# Full -m gpu suite, then one default bench line: gpurun_out/$1_pytest_gpu.log, $1_bench.json.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
tag=${1:-chk}; shift
timeout -k 10 800 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/${tag}_pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/${tag}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py "$@" > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err; rc=$?
tail -3 gpurun_out/${tag}_bench.err; cat gpurun_out/${tag}_bench.json; exit $rc
