#!/bin/bash
# Issue-side PMC of the headline shape's kernels (k=128, 64 squares, one timed call of each phase):
# VALU instructions, VALU-busy and wave cycles, and GRBM_GUI_ACTIVE for the shader clock over a
# dispatch. One counter set per rocprofv3 pass (SQ <= 8, GRBM <= 2 per pass).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r4v}
i=0
for phase in commit extend; do
  for c in "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_BUSY_CYCLES" "SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INST_CYCLES_VMEM" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
    i=$((i + 1))
    timeout -s KILL 90 rocprofv3 --pmc $c -d gpurun_out/${tag}_$i -o p --output-format csv -- \
      python3 tools/prof_phase.py --phase $phase --k 128 --batch 64 --reps 1 > /dev/null 2>&1 || { echo "$phase $c rc=$?"; exit 3; }
    echo "== $phase | $c"
    python3 tools/pmc_dispatch.py gpurun_out/${tag}_$i --kernel k_ | tail -12
  done
done
