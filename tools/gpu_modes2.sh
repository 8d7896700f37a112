#!/bin/bash
# Secondary configs with the current code: k=64 batch (config 4 per GPU), k=512 row-sharded on 1 GPU (config 3 shape).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python3 bench.py --k 64 --batch 256 --cpu-seconds 5 > gpurun_out/bench_k64_r1c.log 2>&1 || exit 1
tail -1 gpurun_out/bench_k64_r1c.log | cut -c1-900
timeout -k 10 240 python3 bench.py --mode sharded --k 512 > gpurun_out/bench_sh512_r1c.log 2>&1 || exit 1
tail -1 gpurun_out/bench_sh512_r1c.log | cut -c1-900
