#!/bin/bash
# (historical: needs the CEL_BENCH_PRIO hook removed from bench.py after this A/B) Batches in flight: stream priority on the first batch (CEL_BENCH_PRIO=1) vs none, k=64 B=128 / 1024, k=128 B=256.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
tag=${1:-r4i}
out=gpurun_out/${tag}_prio_ab.txt
: > $out
for rep in 1 2; do
  for cfg in "64 128" "64 1024" "128 256"; do
    set -- $cfg
    for mode in "1 0" "2 0" "2 1"; do
      set -- $1 $2 $mode
      CEL_BENCH_PRIO=$4 timeout -k 10 180 python bench.py --k $1 --batch $2 --steps 20 --warmup 3 --inflight $3 --no-cpu \
        --no-riders --k512-batch 0 --no-host-io > gpurun_out/${tag}_b.json 2> gpurun_out/${tag}_b.err || { cat gpurun_out/${tag}_b.err; exit 2; }
      python - "$1" "$2" "$3" "$4" gpurun_out/${tag}_b.json >> $out <<'PY'
import json, sys
k, B, inf, prio, f = sys.argv[1:]
d = json.loads(open(f).read().strip().splitlines()[-1])
print(f"k {k:>3} B {B:>4} inflight {inf} prio {prio}: {d['value']:9.1f} squares/s  {d['ms_per_step']:7.3f} ms/step")
PY
      set -- $cfg
    done
  done
done
cat $out
