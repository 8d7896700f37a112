#!/bin/bash
# PMC of the repair kernels (decode focus).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU -d gpurun_out/pmc_dec1 -o p --output-format csv -- python3 bench.py --mode repair --steps 2 --warmup 1 --cpu-seconds 0.1 > /dev/null 2>&1; echo "pmc1 rc=$?"
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_INSTS_VMEM_RD -d gpurun_out/pmc_dec2 -o p --output-format csv -- python3 bench.py --mode repair --steps 2 --warmup 1 --cpu-seconds 0.1 > /dev/null 2>&1; echo "pmc2 rc=$?"
python3 tools/pmc_summary.py gpurun_out/pmc_dec1 gpurun_out/pmc_dec2 | grep -E "decode|axis_gf8|k_level<f"
