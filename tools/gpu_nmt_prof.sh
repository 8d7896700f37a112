#!/bin/bash
# Clean per-kernel profile of the NMT+DAH phase (single stream) + PMC of its kernels,
# and FETCH/WRITE_SIZE of the RS extension (roofline traffic).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 python3 tools/prof_phase.py --phase commit --batch 16 --reps 5 || exit 1
timeout -k 10 90 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_commit -o run --output-format csv -- python3 tools/prof_phase.py --phase commit --batch 16 --reps 5 > /dev/null 2>&1; echo "prof rc=$?"
python3 tools/kstats.py gpurun_out/prof_commit
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU -d gpurun_out/pmc_commit -o p --output-format csv -- python3 tools/prof_phase.py --phase commit --batch 16 --reps 2 > /dev/null 2>&1; echo "pmc rc=$?"
python3 tools/pmc_summary.py gpurun_out/pmc_commit
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcf_ext -o p --output-format csv -- python3 tools/prof_phase.py --phase extend --batch 32 --reps 3 > /dev/null 2>&1; echo "fetch rc=$?"
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw_ext -o p --output-format csv -- python3 tools/prof_phase.py --phase extend --batch 32 --reps 3 > /dev/null 2>&1; echo "write rc=$?"
python3 tools/pmc_summary.py gpurun_out/pmcf_ext gpurun_out/pmcw_ext
