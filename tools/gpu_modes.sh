#!/bin/bash
# Sharded-mode parity (device steps, N rehearsed in one process) + bench modes for configs 3/4/5.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_sharded.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/pytest_sharded.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|Error" gpurun_out/pytest_sharded.log | tail -20; case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 120 python -u bench.py --mode sharded --k 512 --steps 10 --warmup 2 > gpurun_out/bench_sharded512.log 2>&1
rc=$?; echo "sharded rc=$rc"; tail -2 gpurun_out/bench_sharded512.log | cut -c1-1500; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u bench.py --mode sharded --k 256 --steps 10 --warmup 2 > gpurun_out/bench_sharded256.log 2>&1
rc=$?; echo "sharded256 rc=$rc"; tail -1 gpurun_out/bench_sharded256.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --mode repair --k 128 --steps 5 --warmup 1 > gpurun_out/bench_repair.log 2>&1
rc=$?; echo "repair rc=$rc"; tail -2 gpurun_out/bench_repair.log | cut -c1-1500; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --k 64 --batch 128 --steps 10 --cpu-seconds 5 > gpurun_out/bench_k64.log 2>&1
rc=$?; echo "k64 rc=$rc"; tail -1 gpurun_out/bench_k64.log | cut -c1-1500
exit $rc
