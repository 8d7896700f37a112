#!/bin/bash
# Infinity-Cache reuse probe + in-place (Q0 already in the EDS) RS extension A/B.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/microbench/ic_reuse > gpurun_out/ic_reuse.txt 2>&1; rc=$?; cat gpurun_out/ic_reuse.txt; [ $rc -eq 0 ] || exit $rc
for ip in "" "--inplace"; do
  timeout -k 10 120 python3 tools/rs_chunks.py --k 128 --batch 32 --chunks 32 8 4 $ip || exit 1
  CEL_RS_DEBUG=1 timeout -k 10 120 python3 tools/rs_chunks.py --k 128 --batch 32 --chunks 32 8 4 $ip || exit 1
done
