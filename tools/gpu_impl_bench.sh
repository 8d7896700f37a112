#!/bin/bash
# Headline bench (two-chunk pipeline, k=128 B=32) with each GF(2^8) encode implementation.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for impl in axis bitslice perm axis; do
  CEL_RS_IMPL=$impl timeout -k 10 120 python -u bench.py --no-cpu > gpurun_out/b.log 2>&1 || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/b.log').read().strip().split('\n')[-1])
print('$impl value=%.0f rs_us=%.1f rs_frac=%.3f nmt_us=%.1f' % (d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['roofline_nmt']['avg_launch_us']))"
done
