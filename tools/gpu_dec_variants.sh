#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
cp celestia-app_amd/libcelestia_eds.so gpurun_out/lib.orig.so
for v in "$@"; do
  cp variants/lib$v.so celestia-app_amd/libcelestia_eds.so
  echo -n "$v: "
  timeout -k 10 120 python3 tools/dec_time.py 2>&1 | grep -v amdgpu.ids || break
done
cp gpurun_out/lib.orig.so celestia-app_amd/libcelestia_eds.so
