#!/bin/bash
# A/B of the Infinity-Cache chunked RS schedule (CEL_RS_CHUNK) with the hybrid transform:
# bench.py default k=128 B=256 in place; each run has its own time limit.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/rs_ab_${VAR:-CEL_RS_CHUNK}.txt
: > $out
VAR=${VAR:-CEL_RS_CHUNK}
VALS=${VALS:-0 4 8 16 32 0}
for c in $VALS; do
  env $VAR=$c timeout -k 10 120 python -u bench.py --no-cpu --k512-batch 0 > gpurun_out/rschunk_$c.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "chunk $c rc=$rc" >> $out; exit $rc; }
  python3 - "$c" "$VAR" >> $out <<'PY'
import json, sys
c = sys.argv[1]
d = json.loads(open(f"gpurun_out/rschunk_{c}.log").read().strip().splitlines()[-1])
print(f"{sys.argv[2]}={c:>3s}: {d['value']:9.1f} squares/s  rs {d['roofline']['avg_launch_us'] / 256:6.2f} us/square"
      f" (frac {d['roofline']['frac']:.3f})  nmt {d['roofline_nmt']['avg_launch_us'] / 256:6.2f} us/square")
PY
done
cat $out
