#!/bin/bash
# Host-side view of one repair: rocprofv3 kernel trace + HIP API trace + roctx markers of
# bench --mode repair (short), then the timeline of the last repair burst.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --hip-runtime-trace --marker-trace -d gpurun_out/r3_prof_rephost -o r --output-format csv -- \
  python3 bench.py --mode repair --steps 4 --warmup 2 --cpu-seconds 1 > gpurun_out/r3_prof_rephost.json 2>gpurun_out/r3_prof_rephost.err || exit $?
ls gpurun_out/r3_prof_rephost/*
