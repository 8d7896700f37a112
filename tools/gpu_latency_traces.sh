#!/bin/bash
# Kernel timelines of the latency-bound single-square paths: rank 0 of a row-sharded
# k=512 square at simulated N=8 (tools/rank_latency.py) and one k=128 header through the
# host entry point (tools/host_io.py --batch 1 --no-eds).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/lat_rank8 -o r --output-format csv -- \
  python3 tools/rank_latency.py --k 512 --n 8 --reps 5 > /dev/null 2>&1 || exit $?
timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/lat_dah128 -o r --output-format csv -- \
  python3 tools/host_io.py --batch 1 --no-eds --pinned --reps 10 > /dev/null 2>&1 || exit $?
echo "== rank 0 of N=8, one chain (rows, cols, finish)"; python3 tools/timeline.py gpurun_out/lat_rank8 60 -2
echo "== one k=128 header (host entry point)"; python3 tools/timeline.py gpurun_out/lat_dah128 200 -2
