#!/bin/bash
# Repair: parity tests, device vs host bench, kernel trace of the device repair.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_repair.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_repair.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_repair.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 bench.py --mode repair --steps 10 > gpurun_out/bench_repair_dev.log 2>&1 || exit 1
tail -1 gpurun_out/bench_repair_dev.log
timeout -k 10 200 python3 bench.py --mode repair --steps 5 --repair-input host > gpurun_out/bench_repair_host.log 2>&1 || exit 1
tail -1 gpurun_out/bench_repair_host.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_repair -o run --output-format csv -- python3 bench.py --mode repair --steps 5 --cpu-seconds 0.1 > /dev/null 2>&1; echo "prof rc=$?"
python3 tools/kstats.py gpurun_out/prof_repair
