#!/bin/bash
# Pipeline chunk count A/B of the headline step (hybrid nt RS kernel), then the full
# round check (tests, smoke, bench with CPU baseline, rocprofv3 stats).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for round in 1 2; do for pc in 1 2 4 8; do
  CEL_PIPE_CHUNKS=$pc timeout -k 10 120 python -u bench.py --no-cpu --steps 10 > gpurun_out/ab_pipe.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "bench pc=$pc rc=$rc"; tail -3 gpurun_out/ab_pipe.log; exit $rc; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/ab_pipe.log').read().strip().split('\n')[-1])
print('r$round chunks=$pc value=%.0f rs_us_per_sq=%.2f rs_frac=%.3f nmt_frac=%.3f' % (d['value'], d['roofline']['avg_launch_us']/d['config']['squares_per_step_per_gpu'], d['roofline']['frac'], d['roofline_nmt']['frac']))"
done; done
TAG=${TAG:-r1e} bash tools/gpu_round.sh
