#!/bin/bash
# Headline throughput vs batch size and pipeline chunk count (k=128).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "32 2" "64 2" "64 4" "128 2" "128 4" "128 8"; do
  set -- $cfg
  CEL_PIPE_CHUNKS=$2 timeout -k 10 150 python -u bench.py --no-cpu --batch $1 --steps 10 > gpurun_out/b.log 2>&1 || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/b.log').read().strip().split('\n')[-1])
print('B=$1 chunks=$2 value=%.0f ms_per_step=%.3f' % (d['value'], d['ms_per_step']))"
done
