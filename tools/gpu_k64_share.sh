#!/bin/bash
# Config 4's per-GPU share at N = 8 (128 k=64 squares per step) against one GPU's 1024 per
# step, same box, same call (VERDICT r4 ask 6): bench lines at --inflight 1, 2, 3, or the
# "batch inflight" pairs SHAPES lists (e.g. SHAPES="1024 4,128 4,128 8").
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
out=gpurun_out/${1:-k64share}.txt; : > $out
common="--k 64 --no-cpu --no-host-io --no-riders --steps 20 --warmup 3"
IFS=, read -ra shapes <<< "${SHAPES:-1024 1,1024 2,128 1,128 2,128 3,1024 3}"
for b in "${shapes[@]}"; do
  set -- $b
  line=$(timeout -k 10 200 python -u bench.py $common --batch $1 --inflight $2 2>/dev/null | grep '^{') || exit 1
  python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(f'batch {sys.argv[2]:>5s} inflight {sys.argv[3]}: {d[\"value\"]:9.0f} squares/s  ms/step {d[\"ms_per_step\"]:.3f}')" "$line" $1 $2 | tee -a $out
done
