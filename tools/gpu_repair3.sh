#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_repair.py tests/test_gpu_codec.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_repair3.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_repair3.log; [ $rc -eq 0 ] || exit $rc
for c in 1 2 4 8; do
  CEL_DEC_CPW=$c timeout -k 10 200 python3 bench.py --mode repair --steps 20 --cpu-seconds 0.1 > gpurun_out/bench_repair_cpw$c.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_repair_cpw$c.log').read().strip().splitlines()[-1]); print('cpw=$c', round(d['value']), 'repairs/s', round(d['ms_per_step']*1000), 'us')"
done
CEL_DEC_CPW=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_repair3 -o run --output-format csv -- python3 bench.py --mode repair --steps 5 --cpu-seconds 0.1 > /dev/null 2>&1; echo "prof rc=$?"
python3 tools/kstats.py gpurun_out/prof_repair3 | head -4
