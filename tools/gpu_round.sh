#!/bin/bash
# One GPU-box pass: smoke(), the -m gpu parity suite, then the default bench line and the
# repair line. Every step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
tag=${1:-r2}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || { tail -20 gpurun_out/${tag}_smoke.log; exit 1; }
tail -1 gpurun_out/${tag}_smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/${tag}_pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/${tag}_pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || exit $?
cat gpurun_out/${tag}_bench.json
timeout -k 10 300 python -u bench.py --mode repair --steps 20 --warmup 3 \
  > gpurun_out/${tag}_bench_repair.json 2> gpurun_out/${tag}_bench_repair.err || exit $?
cat gpurun_out/${tag}_bench_repair.json
timeout -k 10 300 python -u bench.py --mode repair --k 512 --steps 8 --warmup 2 --cpu-seconds 4 \
  > gpurun_out/${tag}_bench_repair512.json 2> gpurun_out/${tag}_bench_repair512.err || exit $?
cat gpurun_out/${tag}_bench_repair512.json
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --stats -d gpurun_out/${tag}_prof -o b --output-format csv -- \
  python3 bench.py --steps 5 --warmup 2 --no-host-io --k512-batch 8 > gpurun_out/${tag}_bench_prof.json 2>/dev/null || exit $?
python3 tools/kstats.py gpurun_out/${tag}_prof > gpurun_out/${tag}_kstats.txt && head -16 gpurun_out/${tag}_kstats.txt
