#!/bin/bash
# Hybrid (bit-sliced D >= 8 layers) vs all-v_perm axis transform: GPU parity tests with
# the default (hybrid), RS-only A/B (full, memory-only, transform-only), bench A/B at
# B=256, and rocprofv3 kernel stats of the default bench.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-hyb}
B=${B:-256}
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_gpu_$TAG.log; [ $rc -eq 0 ] || exit $rc
for hyb in 0 1; do for dbg in 0 2; do
  CEL_RS_HYB=$hyb CEL_RS_DEBUG=$dbg timeout -k 10 120 python -u tools/rs_chunks.py --k 128 --batch 128 --chunks 128 --inplace --reps 10 > gpurun_out/rs_$TAG.log 2>&1
  rc=$?; echo -n "hyb=$hyb "; tail -1 gpurun_out/rs_$TAG.log; [ $rc -eq 0 ] || exit $rc
done; done
for round in 1 2; do
  for hyb in 0 1; do
    CEL_RS_HYB=$hyb timeout -k 10 120 python -u bench.py --no-cpu --batch $B --steps 10 > gpurun_out/ab_$TAG.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "bench hyb=$hyb rc=$rc"; tail -3 gpurun_out/ab_$TAG.log; exit $rc; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/ab_$TAG.log').read().strip().split('\n')[-1])
print('r$round hyb=$hyb value=%.0f rs_us_per_sq=%.2f rs_frac=%.3f nmt_us=%.1f' % (d['value'], d['roofline']['avg_launch_us']/$B, d['roofline']['frac'], d['roofline_nmt']['avg_launch_us']))"
  done
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
  python3 bench.py --no-cpu --batch $B > gpurun_out/bench_prof_$TAG.log 2>&1
rc=$?; echo "prof rc=$rc"
python3 tools/kstats.py gpurun_out/prof_$TAG
exit $rc
