#!/bin/bash
# Kernel timelines of the latency-bound paths: one repair (bench --mode repair) and one
# single-square header (host_io --batch 1 --no-eds), rocprofv3 kernel trace + stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r3_prof_repair -o r --output-format csv -- \
  python3 bench.py --mode repair --steps 4 --warmup 2 --cpu-seconds 1 > gpurun_out/r3_prof_repair.json 2>gpurun_out/r3_prof_repair.err || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r3_prof_hostio -o h --output-format csv -- \
  python3 tools/host_io.py --batch 1 --no-eds --pinned --reps 10 > gpurun_out/r3_prof_hostio.txt 2>&1 || exit $?
python3 tools/timeline.py gpurun_out/r3_prof_repair 300 | tail -80
