#!/bin/bash
# Full -m gpu suite, then the row-sharded rank chain at N = 1 and 8 (tools/rank_latency.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
tag=${1:-chk}
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/${tag}_pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/${tag}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for n in 1 8; do timeout -k 10 120 python3 tools/rank_latency.py --k 512 --n $n 2>&1 | grep -v amdgpu.ids || exit 1; done
