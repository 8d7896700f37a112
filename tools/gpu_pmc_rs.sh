#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for impl in perm bitslice; do
  CEL_RS_IMPL=$impl timeout -k 10 60 python3 tools/prof_phase.py --phase extend --batch 8 --reps 10 || exit 1
  CEL_RS_IMPL=$impl timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d gpurun_out/pmc_$impl -o p --output-format csv -- python3 tools/prof_phase.py --phase extend --batch 8 --reps 3 > /dev/null 2>&1; echo "pmc $impl rc=$?"
  CEL_RS_IMPL=$impl timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcf_$impl -o p --output-format csv -- python3 tools/prof_phase.py --phase extend --batch 8 --reps 3 > /dev/null 2>&1; echo "fetch $impl rc=$?"
  CEL_RS_IMPL=$impl timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw_$impl -o p --output-format csv -- python3 tools/prof_phase.py --phase extend --batch 8 --reps 3 > /dev/null 2>&1; echo "write $impl rc=$?"
done
