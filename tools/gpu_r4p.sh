#!/bin/bash
# Batches in flight, where the next batch starts: shipped (previous extension done), leafstart (previous leaf
# hashing done, variants/libleafstart.so), nostagger (no wait); and 3 in flight; k=64 B=128 / 1024, k=128 B=256.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
tag=${1:-r4p}
out=gpurun_out/${tag}_start_ab.txt
: > $out
for rep in 1 2; do
  for cfg in "64 128" "64 1024" "128 256"; do
    for mode in "1 ship" "2 ship" "3 ship" "2 leafstart" "3 leafstart" "2 nostagger"; do
      set -- $cfg $mode
      lib=celestia-app_amd/libcelestia_eds.so; [ $4 != ship ] && lib=variants/lib$4.so
      CEL_EDS_LIB=$lib timeout -k 10 180 python bench.py --k $1 --batch $2 --steps 20 --warmup 3 --inflight $3 --no-cpu \
        --no-riders --k512-batch 0 --no-host-io > gpurun_out/${tag}_b.json 2> gpurun_out/${tag}_b.err || { cat gpurun_out/${tag}_b.err; exit 2; }
      python - "$1" "$2" "$3" "$4" gpurun_out/${tag}_b.json >> $out <<'PY'
import json, sys
k, B, inf, lib, f = sys.argv[1:]
d = json.loads(open(f).read().strip().splitlines()[-1])
print(f"k {k:>3} B {B:>4} inflight {inf} {lib:>10}: {d['value']:9.1f} squares/s  {d['ms_per_step']:7.3f} ms/step")
PY
    done
  done
done
cat $out
