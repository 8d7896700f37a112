#!/bin/bash
# Pipelined row-sharded squares: the sharded GPU tests, --mode sharded at depth 1/2/4
# (N = 1), then the default bench line (its rowshard512 rider carries the pipelined value).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
bash tools/gpu_quick.sh "sharded" || exit 1
for d in 1 2 4; do
  timeout -k 10 200 python bench.py --mode sharded --k 512 --steps 10 --warmup 3 --depth $d 2>/dev/null \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('depth', $d, round(d['value'],1), d['pipelined'])" || exit 1
done
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/pipe_bench.json 2> gpurun_out/pipe_bench.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/pipe_bench.json')); print(d['value'], d['rowshard512'])"
