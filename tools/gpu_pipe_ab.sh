#!/bin/bash
# Batch-pipeline A/B of library variants (variants/lib<v>.so, built by build_variant.sh from a
# tools/variants/*.patch): k=64 B=128 (config 4's per-GPU share at N = 8) and k=128 B=256 (the
# headline step), one batch per step (--inflight 1), so each step runs the library's own
# two-chunk pipeline (pipe_plan) that the variants change. INFLIGHT=2 times the default
# bench shape (CEL_FLAG_CALLER_STREAM batches) instead.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
for v in "$@"; do
  for kb in "64 128" "128 256"; do
    set -- $kb
    CEL_EDS_LIB=variants/lib$v.so timeout -k 10 200 python bench.py --k $1 --batch $2 --steps 10 --warmup 2 --no-cpu --no-host-io \
      --no-riders --k512-batch 0 --inflight ${INFLIGHT:-1} 2>/dev/null \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', 'k', $1, 'B', $2, round(d['value'],1), round(d['ms_per_step'],3), 'ms/step')" || exit 1
  done
done
