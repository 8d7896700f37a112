#!/bin/bash
# Latency-path A/B of library variants (variants/lib<v>.so, built by build_variant.sh from a
# tools/variants/*.patch; the shipped sources have no A/B macros): rank-0 chain of
# a row-sharded k=512 square (N = 1, 8), one k=128 header through the host entry point,
# k=64 B=128 batch steps, the k=128 repair.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
for v in "$@"; do
  export CEL_EDS_LIB=variants/lib$v.so
  for n in 1 8; do
    echo -n "$v "; timeout -k 10 120 python3 tools/rank_latency.py --k 512 --n $n 2>&1 | grep -v amdgpu.ids || exit 1
  done
  echo -n "$v "; timeout -k 10 120 python3 tools/host_io.py --batch 1 --no-eds --pinned --reps 30 2>&1 | grep -v amdgpu.ids | tail -1
  timeout -k 10 200 python bench.py --k 64 --batch 128 --steps 10 --warmup 2 --no-cpu --no-host-io --no-riders --k512-batch 0 2>/dev/null \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v k64 B128', round(d['value'],1))" || exit 1
  timeout -k 10 200 python bench.py --mode repair --steps 40 --warmup 5 --cpu-seconds 0.5 2>/dev/null \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v repair', round(d['value'],1))" || exit 1
done
