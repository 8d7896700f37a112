#!/bin/bash
# One default bench line on the box (+ optional extra bench args) into gpurun_out/$TAG_bench.json.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
tag="${TAG:-r5}"
timeout -k 10 400 python -u bench.py "$@" > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
rc=$?
tail -5 gpurun_out/${tag}_bench.err
cat gpurun_out/${tag}_bench.json
exit $rc
