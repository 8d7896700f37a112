#!/bin/bash
# Steady-state timeline of k=64 B=128 steps with two batches in flight (8 steps per burst).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
tag=${1:-r4j}
timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/${tag}_trace -o tr -- python3 tools/step_trace.py --k 64 --batch 128 \
  --inflight 2 --chain 8 --steps 3 > gpurun_out/${tag}_trace.log 2>&1 || { tail -20 gpurun_out/${tag}_trace.log; exit 3; }
cat gpurun_out/${tag}_trace.log
python3 tools/timeline.py gpurun_out/${tag}_trace 1000 -2 > gpurun_out/${tag}_timeline.txt && tail -5 gpurun_out/${tag}_timeline.txt
