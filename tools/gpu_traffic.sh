#!/bin/bash
# HBM traffic (rocprofv3 FETCH_SIZE / WRITE_SIZE, one pass each) of the RS extension:
#   bash tools/gpu_traffic.sh <tag> <k> <batch>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-tr}; k=${2:-512}; b=${3:-2}
for c in FETCH_SIZE WRITE_SIZE TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum; do
  timeout -s KILL 90 rocprofv3 --pmc $c -d gpurun_out/${tag}_$c -o p --output-format csv -- \
    python3 tools/prof_phase.py --phase extend --k $k --batch $b --reps 2 > /dev/null 2>&1 || { echo "$c rc=$?"; exit 3; }
  python3 tools/pmc_dispatch.py gpurun_out/${tag}_$c --kernel rs_
done
