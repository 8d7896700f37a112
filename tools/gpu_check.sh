#!/bin/bash
# Full -m gpu parity suite, then a kernel trace of the extension phase at two shapes.
#   bash tools/gpu_check.sh <tag> [k batch [k2 batch2]]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-chk}
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > gpurun_out/${tag}_pytest_gpu.log 2>&1 || { grep -E "FAILED|ERROR|Error" gpurun_out/${tag}_pytest_gpu.log | head -30; tail -5 gpurun_out/${tag}_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/${tag}_pytest_gpu.log
shift
while [ $# -ge 2 ]; do
  k=$1; b=$2; shift 2
  timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/${tag}_trace_k$k -o t --output-format csv -- \
    python3 tools/prof_phase.py --phase extend --k $k --batch $b --reps 5 > gpurun_out/${tag}_phase_k$k.log 2>&1 || exit 2
  grep -v "amdgpu.ids\|^W20\|^E20" gpurun_out/${tag}_phase_k$k.log
  python3 tools/ktrace.py gpurun_out/${tag}_trace_k$k rs_
done
