#!/bin/bash
# Perf session: GPU parity tests, bench sweep over batch sizes, one rocprofv3 kernel trace.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log; case $rc in 0|1) ;; *) exit $rc ;; esac
for B in ${BATCHES:-8 32}; do
  timeout -k 10 200 python -u bench.py --batch $B --no-cpu ${BENCH_ARGS:-} > gpurun_out/bench_b$B.log 2>&1
  rc=$?; echo "bench B=$B rc=$rc"; tail -1 gpurun_out/bench_b$B.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu ${PROF_ARGS:-} > gpurun_out/bench_prof.log 2>&1
rc=$?; echo "prof rc=$rc"
python3 - <<'PY'
import csv, glob
for f in glob.glob('gpurun_out/prof/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"{r['Name'][:58]:58s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs'])/1e3:9.2f} pct={float(r['Percentage']):6.2f}")
PY
exit $rc
