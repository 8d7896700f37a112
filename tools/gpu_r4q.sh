#!/bin/bash
# Latency-path tree levels (k_level_lat): GPU tests of every commit path, then the latency lines (rank chain,
# one header, k=64 B=128 steps, repair) and header timelines against variants/libbase.so.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
tag=${1:-r4q}
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${tag}_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/${tag}_pytest_gpu.log
cp celestia-app_amd/libcelestia_eds.so variants/libnew.so
bash tools/gpu_latency_ab.sh base new base new > gpurun_out/${tag}_latency_ab.txt 2>&1 || { cat gpurun_out/${tag}_latency_ab.txt; exit 2; }
cat gpurun_out/${tag}_latency_ab.txt
bash tools/gpu_trace_header.sh ${tag}_hdr base new || exit 3
