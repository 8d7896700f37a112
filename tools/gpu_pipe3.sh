#!/bin/bash
# Batch pipeline chunks x batch size at k=128 (headline bench, in-place input).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in 128 256; do for pc in 1 2 4; do
  CEL_PIPE_CHUNKS=$pc timeout -k 10 300 python3 bench.py --no-cpu --batch $b --steps 10 > gpurun_out/bench_pc${pc}_b${b}.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_pc${pc}_b${b}.log').read().strip().splitlines()[-1]); print('pipe_chunks=$pc batch=$b', round(d['value']), 'sq/s  rs_frac', round(d['roofline']['frac'],3), 'nmt_us/sq', round(d['roofline_nmt']['avg_launch_us']/$b,2))"
done; done
