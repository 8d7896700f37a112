#!/bin/bash
# One k=128 header through the host entry point (page-locked ODS, roots + DAH back) per
# library variant, interleaved: bash tools/gpu_header_ab.sh <variant>... (variants/lib<v>.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
for v in "$@"; do
  echo -n "$v: "
  CEL_EDS_LIB=variants/lib$v.so timeout -k 10 120 python3 tools/host_io.py --batch 1 --no-eds --pinned --reps 50 2>&1 \
    | grep -v amdgpu.ids | tail -1 || exit 1
done
