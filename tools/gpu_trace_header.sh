#!/bin/bash
# Kernel timelines of one k=128 header (host entry point, batch 1) per library variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-hdr}; shift
for v in "$@"; do
  CEL_EDS_LIB=variants/lib$v.so timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/${tag}_$v -o h --output-format csv -- \
    python3 tools/host_io.py --batch 1 --no-eds --pinned --reps 5 > /dev/null 2>&1 || exit 1
  echo "== $v"; python3 tools/timeline.py gpurun_out/${tag}_$v 300 -2 | tail -22
done
