#!/bin/bash
# Instruction-fetch and issue counters of the repair's decode kernel, per library variant
# (variants/lib*.so): one rocprofv3 --pmc pass per counter set and variant.
#   bash tools/gpu_pmc_icache.sh <variant>...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "$@"; do
  i=0
  for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_IFETCH SQ_ACTIVE_INST_VALU SQ_WAIT_ANY" \
             "SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE"; do
    i=$((i+1))
    CEL_EDS_LIB=variants/lib$v.so timeout -s KILL 120 rocprofv3 --pmc $set -d gpurun_out/ic_${v}_p$i -o p --output-format csv -- \
      python3 bench.py --mode repair --steps 2 --warmup 1 > /dev/null 2>&1 || { echo "$v pass $i rc=$?"; exit 3; }
  done
  python3 tools/pmc_dispatch.py gpurun_out/ic_${v}_p1 gpurun_out/ic_${v}_p2 --kernel rs_decode | tail -4
done
