#!/bin/bash
# Host-buffer batch entry point (cel_extend_batch, 16 k=128 squares per call, page-locked) per
# library variant, interleaved: EDS back, parity quadrants back, roots only.
#   bash tools/gpu_hostio_ab.sh <variant>...   (variants/lib<v>.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
for v in "$@"; do
  for m in "" "--parity-only" "--no-eds"; do
    echo -n "$v $m: "
    CEL_EDS_LIB=variants/lib$v.so timeout -k 10 120 python3 tools/host_io.py --batch 16 --pinned --reps 5 $m 2>&1 \
      | grep -v amdgpu.ids | tail -1 || exit 1
  done
done
