#!/bin/bash
# A/B of library variants (variants/lib*.so, built elsewhere) on the extension phase:
#   bash tools/gpu_variants.sh <k> <batch> <variant>...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
k=$1; b=$2; shift 2
cp celestia-app_amd/libcelestia_eds.so gpurun_out/lib.orig.so
for v in "$@"; do
  cp variants/lib$v.so celestia-app_amd/libcelestia_eds.so
  echo -n "$v: "
  timeout -k 10 120 python3 tools/prof_phase.py --phase extend --k $k --batch $b --reps 10 2>&1 | grep -v amdgpu.ids || break
done
cp gpurun_out/lib.orig.so celestia-app_amd/libcelestia_eds.so
