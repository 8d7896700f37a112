#!/bin/bash
# Batch-size sweep of the default bench (k=128, in place, 2 pipeline chunks).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/batch_r1g.txt
: > $out
for b in 256 512 1024 256; do
  timeout -k 10 150 python -u bench.py --no-cpu --k512-batch 0 --batch $b > gpurun_out/batch_$b.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "batch $b rc=$rc" >> $out; exit $rc; }
  python3 - "$b" >> $out <<'PY'
import json, sys
b = sys.argv[1]
d = json.loads(open(f"gpurun_out/batch_{b}.log").read().strip().splitlines()[-1])
print(f"B={b:>5s}: {d['value']:9.1f} squares/s  {d['ms_per_step']:7.2f} ms/step  rs frac {d['roofline']['frac']:.3f}  nmt frac {d['roofline_nmt']['frac']:.3f}")
PY
done
cat $out
