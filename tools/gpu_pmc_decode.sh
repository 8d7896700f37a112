#!/bin/bash
# PMC passes over the repair bench (k_rs_decode and the repair kernels), one pass per set.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-dec}
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY" \
           "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_LDS_ADDR_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_LDS_UNALIGNED_STALL"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d gpurun_out/${tag}_p$i -o p --output-format csv -- \
    python3 bench.py --mode repair --steps 3 --warmup 1 > /dev/null 2>&1 || { echo "pass $i rc=$?"; exit 3; }
done
python3 tools/pmc_dispatch.py gpurun_out/${tag}_p1 gpurun_out/${tag}_p2 --kernel rs_decode | head -8
