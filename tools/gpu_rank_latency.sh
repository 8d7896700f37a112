#!/bin/bash
# Per-rank phase latency of the row-sharded k=512 square at simulated N = 1, 2, 4, 8
# (tools/rank_latency.py), then a kernel trace of the N = 8 rank.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for n in 1 2 4 8; do
  timeout -k 10 120 python3 tools/rank_latency.py --k 512 --n $n 2>&1 | grep -v amdgpu.ids || exit 1
done
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r3_prof_rank8 -o r --output-format csv -- \
  python3 tools/rank_latency.py --k 512 --n 8 --reps 5 > /dev/null 2>&1 || exit $?
python3 tools/timeline.py gpurun_out/r3_prof_rank8 100 -2
