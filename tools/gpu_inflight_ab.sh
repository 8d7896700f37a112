#!/bin/bash
# Headline step with M batches in flight, alternated (bench.py --inflight M, headline only):
#   bash tools/gpu_inflight_ab.sh <k> <batch> <M>...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
k=$1; b=$2; shift 2
for m in "$@"; do
  line=$(timeout -k 10 200 python -u bench.py --k $k --batch $b --inflight $m --steps 20 --warmup 3 --no-cpu \
    --no-host-io --no-riders --k512-batch 0 2>/dev/null | grep '^{') || exit 1
  python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(f'k {sys.argv[2]} batch {sys.argv[3]} inflight {sys.argv[4]}: {d[\"value\"]:9.0f} squares/s  ms/step {d[\"ms_per_step\"]:.3f}')" "$line" $k $b $m
done
