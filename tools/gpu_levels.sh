#!/bin/bash
# Per-dispatch durations of the NMT phase at batch 128 (one stream).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/lv128 -o run -- python3 tools/prof_phase.py --phase commit --batch 128 --reps 2 > gpurun_out/lv128.log 2>&1; echo "rc=$?"
grep "commit input" gpurun_out/lv128.log
