#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 python3 tools/prof_phase.py --phase extend --k 512 --batch 1 --reps 5 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD -d gpurun_out/pmc_gf16 -o p --output-format csv -- python3 tools/prof_phase.py --phase extend --k 512 --batch 1 --reps 2 > /dev/null 2>&1; echo "pmc rc=$?"
python3 tools/pmc_summary.py gpurun_out/pmc_gf16
