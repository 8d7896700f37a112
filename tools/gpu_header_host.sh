#!/bin/bash
# Host-side view of one k=128 header through the host entry point (cel_extend_batch, batch 1,
# roots + DAH only, pinned): kernel + HIP API + roctx trace, then the timeline of the last call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-hh}
timeout -k 10 240 rocprofv3 --kernel-trace --hip-runtime-trace --marker-trace --memory-copy-trace -d gpurun_out/${tag} -o h --output-format csv -- \
  python3 tools/host_io.py --batch 1 --no-eds --pinned --reps 5 > gpurun_out/${tag}.log 2>&1 || { tail -20 gpurun_out/${tag}.log; exit 1; }
python3 tools/host_timeline.py gpurun_out/${tag} nmt.leaf 600 600 -1 > gpurun_out/${tag}_timeline.txt
tail -60 gpurun_out/${tag}_timeline.txt
