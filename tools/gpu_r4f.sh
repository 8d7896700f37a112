#!/bin/bash
# Round-4 check of a library change: the whole -m gpu suite on the in-tree build, then the
# latency paths and the batch steps A/B against variants/libbase.so.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
tag=${1:-r4f}; shift
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${tag}_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/${tag}_pytest_gpu.log
bash tools/gpu_latency_ab.sh "$@" > gpurun_out/${tag}_latency_ab.txt 2>&1 || { cat gpurun_out/${tag}_latency_ab.txt; exit 2; }
cat gpurun_out/${tag}_latency_ab.txt
bash tools/gpu_pipe_ab.sh "$@" > gpurun_out/${tag}_pipe_ab.txt 2>&1 || { cat gpurun_out/${tag}_pipe_ab.txt; exit 3; }
cat gpurun_out/${tag}_pipe_ab.txt
