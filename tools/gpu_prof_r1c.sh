#!/bin/bash
# In-place input: RS traffic PMC (FETCH/WRITE_SIZE passes), kernel stats of the bench.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 python3 tools/prof_phase.py --phase extend --batch 32 --reps 3 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcf_ext_ip -o p --output-format csv -- python3 tools/prof_phase.py --phase extend --batch 32 --reps 3 > /dev/null 2>&1; echo "fetch rc=$?"
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw_ext_ip -o p --output-format csv -- python3 tools/prof_phase.py --phase extend --batch 32 --reps 3 > /dev/null 2>&1; echo "write rc=$?"
python3 tools/pmc_summary.py gpurun_out/pmcf_ext_ip gpurun_out/pmcw_ext_ip
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench_r1c -o run --output-format csv -- python3 bench.py --no-cpu > gpurun_out/bench_prof_r1c.log 2>&1; echo "prof rc=$?"
tail -1 gpurun_out/bench_prof_r1c.log
python3 tools/kstats.py gpurun_out/prof_bench_r1c
