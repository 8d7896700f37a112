#!/bin/bash
# Repair-line A/B of library variants (variants/lib*.so): bench.py --mode repair.
#   bash tools/gpu_repair_variants.sh <variant>...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for v in "$@"; do
  CEL_EDS_LIB=variants/lib$v.so timeout -k 10 180 python3 bench.py --mode repair --steps 30 --warmup 3 \
    > gpurun_out/rv.json 2> gpurun_out/rv.err || { tail -5 gpurun_out/rv.err; exit 1; }
  python3 -c "
import json; r = json.load(open('gpurun_out/rv.json'))
print('$v: %.1f repairs/s  %.3f ms/step  decode %.1f us/launch (frac %.3f)' % (r['value'], r['ms_per_step'], r['roofline']['avg_launch_us'], r['roofline']['frac']))"
done
