#!/bin/bash
# Repair A/B of library variants (variants/lib*.so): bench --mode repair per variant, in
# the order given (repeat names to interleave against drift); prints value per run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for v in "$@"; do
  CEL_EDS_LIB=variants/lib$v.so timeout -k 10 120 python3 bench.py --mode repair --steps 40 --warmup 5 --cpu-seconds 0.5 \
    > gpurun_out/ab_$v.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_$v.json')); print('$v', round(d['value'],1), round(d['ms_per_step']*1e3,1), 'us', d['byzantine']['ms_per_repair'])"
done
