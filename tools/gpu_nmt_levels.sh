#!/bin/bash
# Per-launch SHA-256 rates of the NMT commit at k=128 (B=256) and k=512 (B=32): kernel traces
# of prof_phase.py --phase commit, one stream, then tools/nmt_levels.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-lv}
for kb in "128 256" "512 32"; do
  set -- $kb
  timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/${tag}_k$1 -o t --output-format csv -- \
    python3 tools/prof_phase.py --phase commit --k $1 --batch $2 --reps 5 > gpurun_out/${tag}_k$1.log 2>&1 || { tail -5 gpurun_out/${tag}_k$1.log; exit 1; }
  python3 tools/nmt_levels.py gpurun_out/${tag}_k$1 $1 $2 ${PEAK:-29.4} | tee gpurun_out/${tag}_k$1_levels.txt
done
