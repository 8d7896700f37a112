#!/bin/bash
# PMC passes over the wave-per-axis RS kernel (k=128, 32 squares): transform-only
# (CEL_RS_DEBUG=2) and full. One counter group per rocprofv3 run.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/pmc_avail.txt 2>&1; echo "list rc=$?"
grep -oE "SQC?_[A-Z0-9_]*(ICACHE|IFETCH|INST_LEVEL|WAIT_INST|LEVEL_INST)[A-Z0-9_]*" gpurun_out/pmc_avail.txt | sort -u | head -40 || true
for dbg in 2 0; do
  CEL_RS_DEBUG=$dbg timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_IFETCH -d gpurun_out/pmc_ax$dbg -o p --output-format csv -- python3 tools/rs_chunks.py --k 128 --batch 32 --chunks 32 --reps 2 > /dev/null 2>&1; echo "pmc dbg=$dbg rc=$?"
  CEL_RS_DEBUG=$dbg timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_INSTS_SALU SQ_ACTIVE_INST_ANY -d gpurun_out/pmci_ax$dbg -o p --output-format csv -- python3 tools/rs_chunks.py --k 128 --batch 32 --chunks 32 --reps 2 > /dev/null 2>&1; echo "pmci dbg=$dbg rc=$?"
done
python3 tools/pmc_summary.py gpurun_out/pmc_ax2 gpurun_out/pmci_ax2 gpurun_out/pmc_ax0 gpurun_out/pmci_ax0
