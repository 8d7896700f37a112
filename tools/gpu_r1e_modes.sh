#!/bin/bash
# Round-1e refresh: HBM traffic PMC of the hybrid nt RS kernel (k=128, 32 squares),
# config-4 (k=64) and k=512 batch benches, repair bench.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 python3 tools/prof_phase.py --phase extend --batch 32 --reps 3 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcf_r1e -o p --output-format csv -- python3 tools/prof_phase.py --phase extend --batch 32 --reps 3 > /dev/null 2>&1; echo "fetch rc=$?"
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw_r1e -o p --output-format csv -- python3 tools/prof_phase.py --phase extend --batch 32 --reps 3 > /dev/null 2>&1; echo "write rc=$?"
python3 tools/pmc_summary.py gpurun_out/pmcf_r1e gpurun_out/pmcw_r1e
timeout -k 10 240 python3 bench.py --k 64 --batch 256 --cpu-seconds 5 > gpurun_out/bench_k64_r1e.log 2>&1 || exit 1
tail -1 gpurun_out/bench_k64_r1e.log | cut -c1-900
timeout -k 10 240 python3 bench.py --k 512 --batch 8 --steps 5 --cpu-seconds 5 > gpurun_out/bench_k512_r1e.log 2>&1 || exit 1
tail -1 gpurun_out/bench_k512_r1e.log | cut -c1-900
timeout -k 10 240 python3 bench.py --mode repair --steps 10 --cpu-seconds 5 > gpurun_out/bench_repair_r1e.log 2>&1 || exit 1
tail -1 gpurun_out/bench_repair_r1e.log | cut -c1-900
