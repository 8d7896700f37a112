#!/bin/bash
# Chunked Q0|Q1 extension pipeline: parity, then CEL_RS_CHUNK A/B and bench in both input layouts.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_square.py tests/test_gpu_codec.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_pipe2.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_pipe2.log; [ $rc -eq 0 ] || exit $rc
for ch in 0 2 4 6 8 12; do
  CEL_RS_CHUNK=$ch timeout -k 10 120 python3 tools/rs_chunks.py --k 128 --batch 48 --chunks 48 --inplace | sed "s/^/chunk=$ch /" || exit 1
done
for ch in 0 6; do
  CEL_RS_CHUNK=$ch CEL_RS_DEBUG=1 timeout -k 10 120 python3 tools/rs_chunks.py --k 128 --batch 48 --chunks 48 --inplace | sed "s/^/chunk=$ch /" || exit 1
  CEL_RS_CHUNK=$ch timeout -k 10 120 python3 tools/rs_chunks.py --k 128 --batch 48 --chunks 48 | sed "s/^/chunk=$ch /" || exit 1
done
for ch in 0 12 24; do
  CEL_RS_CHUNK=$ch timeout -k 10 120 python3 tools/rs_chunks.py --k 64 --batch 96 --chunks 96 --inplace | sed "s/^/chunk=$ch /" || exit 1
done
timeout -k 10 300 python3 bench.py --no-cpu > gpurun_out/bench_pipe2_eds.log 2>&1 || exit 1
tail -1 gpurun_out/bench_pipe2_eds.log
timeout -k 10 300 python3 bench.py --no-cpu --input ods > gpurun_out/bench_pipe2_ods.log 2>&1 || exit 1
tail -1 gpurun_out/bench_pipe2_ods.log
CEL_RS_CHUNK=0 timeout -k 10 300 python3 bench.py --no-cpu > gpurun_out/bench_pipe2_c0.log 2>&1 || exit 1
tail -1 gpurun_out/bench_pipe2_c0.log
