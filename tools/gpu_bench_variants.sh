#!/bin/bash
# Whole-step A/B of library variants (variants/lib*.so): bench.py batch mode with the
# given k and batch, no CPU / host-io / companion lines; prints value, RS and NMT phases.
#   bash tools/gpu_bench_variants.sh <k> <batch> <steps> <variant>...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
k=$1; b=$2; n=$3; shift 3
for v in "$@"; do
  CEL_EDS_LIB=variants/lib$v.so timeout -k 10 180 python3 bench.py --k $k --batch $b --steps $n --warmup 2 \
    --no-cpu --no-host-io --k512-batch 0 > gpurun_out/bv.json 2> gpurun_out/bv.err || { tail -5 gpurun_out/bv.err; exit 1; }
  python3 -c "
import json; r = json.load(open('gpurun_out/bv.json'))
print('$v k=$k B=$b: %.1f squares/s  %.3f ms/step  rs %.1f us/launch (frac %.3f)  nmt %.1f us/launch' % (r['value'], r['ms_per_step'], r['roofline']['avg_launch_us'], r['roofline']['frac'], r['roofline_nmt']['avg_launch_us']))"
done
