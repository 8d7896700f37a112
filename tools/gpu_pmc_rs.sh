#!/bin/bash
# Kernel trace + PMC passes of the RS extension phase alone (tools/prof_phase.py).
#   bash tools/gpu_pmc_rs.sh <tag> <k> <batch>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-rs}; k=${2:-512}; b=${3:-8}
timeout -k 10 120 python3 tools/prof_phase.py --phase extend --k $k --batch $b --reps 5 || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_trace -o t --output-format csv -- \
  python3 tools/prof_phase.py --phase extend --k $k --batch $b --reps 5 > /dev/null 2>&1 || exit 2
python3 tools/kstats.py gpurun_out/${tag}_trace 2>/dev/null | head -20
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD \
  -d gpurun_out/${tag}_pmc1 -o p --output-format csv -- python3 tools/prof_phase.py --phase extend --k $k --batch 2 --reps 2 > /dev/null 2>&1 || exit 3
python3 tools/pmc_summary.py gpurun_out/${tag}_pmc1 | grep -v "copy\|fill"
timeout -s KILL 90 rocprofv3 --pmc SQ_IFETCH SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD \
  -d gpurun_out/${tag}_pmc2 -o p --output-format csv -- python3 tools/prof_phase.py --phase extend --k $k --batch 2 --reps 2 > /dev/null 2>&1 || echo "pmc2 rc=$?"
python3 tools/pmc_summary.py gpurun_out/${tag}_pmc2 | grep -v "copy\|fill"
exit 0
