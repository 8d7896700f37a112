#!/bin/bash
# Per-kernel durations of the RS extension in memory-only / full modes, in-place, chunk 32 vs 4.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/microbench/ic_reuse > gpurun_out/ic_reuse2.txt 2>&1; rc=$?; [ $rc -eq 0 ] || exit $rc
for dbg in 1 0; do for c in 32 4; do
  CEL_RS_DEBUG=$dbg timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/ic2_d${dbg}_c${c} -o run -- python3 tools/rs_chunks.py --k 128 --batch 32 --chunks $c --inplace > gpurun_out/ic2_d${dbg}_c${c}.log 2>&1 || exit 1
done; done
