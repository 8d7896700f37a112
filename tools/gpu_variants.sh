#!/bin/bash
# A/B of library variants (variants/lib*.so, built elsewhere) on one pipeline phase:
#   PHASE=extend|commit bash tools/gpu_variants.sh <k> <batch> <variant>...
# Variants run in the order given (repeat names to interleave them against drift).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
k=$1; b=$2; shift 2
for v in "$@"; do
  echo -n "$v: "
  CEL_EDS_LIB=variants/lib$v.so timeout -k 10 120 python3 tools/prof_phase.py --phase ${PHASE:-extend} --k $k --batch $b --reps 10 2>&1 | grep -v amdgpu.ids || exit 1
done
