#!/bin/bash
# Config 4 at N = 8 runs 128 k=64 squares per GPU per step: per-square rate against the
# batch size, and a kernel trace of B = 128 steps (what is idle between steps).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for b in 128 256 1024 128; do
  timeout -k 10 200 python bench.py --k 64 --batch $b --steps 10 --warmup 2 --no-cpu --no-host-io --no-riders --k512-batch 0 2>/dev/null \
   | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('k64 B', $b, round(d['value'],1), round(d['ms_per_step'],3), 'ms/step', round(d['roofline']['avg_launch_us'],1), round(d['roofline_nmt']['avg_launch_us'],1))" || exit 1
done
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/k64tail -o r --output-format csv -- \
  python3 bench.py --k 64 --batch 128 --steps 6 --warmup 2 --no-cpu --no-host-io --no-riders --k512-batch 0 --phase-reps 1 > /dev/null 2>&1 || exit $?
python3 tools/timeline.py gpurun_out/k64tail 30 -3 | tail -45
