#!/bin/bash
# Headline evidence on one GPU box: the default bench line, a rocprofv3 kernel trace of the
# same command (for tools/roofline_crosscheck.py), and the host's CPU-baseline scaling
# (tools/cpu_scaling.py). Every step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
tag=${1:-r4a}
export TMPDIR=/tmp
if [ -n "$GPU_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$GPU_TESTS" \
    > gpurun_out/${tag}_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/${tag}_pytest_gpu.log
fi
timeout -k 10 400 python -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || exit $?
cat gpurun_out/${tag}_bench.json
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o b --output-format csv -- \
  python3 bench.py > gpurun_out/${tag}_bench_prof.json 2> gpurun_out/${tag}_bench_prof.err || exit $?
python3 tools/roofline_crosscheck.py gpurun_out/${tag}_prof gpurun_out/${tag}_bench_prof.json \
  > gpurun_out/${tag}_roofline_crosscheck.txt || exit $?
tail -8 gpurun_out/${tag}_roofline_crosscheck.txt
timeout -k 10 300 python3 -u tools/cpu_scaling.py 2 > gpurun_out/${tag}_cpu_scaling.txt 2>&1 || exit $?
cat gpurun_out/${tag}_cpu_scaling.txt
