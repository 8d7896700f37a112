#!/bin/bash
# Batches in flight: the new two-stream test, then bench batch lines with --inflight 1 / 2
# (2n: the library without the bulk-done stagger, variants/libnostagger.so) interleaved (k=64 B=128 and B=1024, k=128 B=256), then a kernel trace of k=64 B=128 with
# two in flight for the timeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
tag=${1:-r4g}
timeout -k 10 300 python -u -m pytest tests/test_gpu_square.py -x -q --timeout 120 --timeout-method thread \
  -k "in_flight or device_batch" > gpurun_out/${tag}_pytest.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest.log; exit 1; }
tail -2 gpurun_out/${tag}_pytest.log
out=gpurun_out/${tag}_inflight_ab.txt
: > $out
for rep in 1 2; do
  for cfg in "64 128" "64 1024" "128 256"; do
    set -- $cfg
    for inf in 1 2 2n; do
      lib=""; [ $inf = 2n ] && lib=variants/libnostagger.so
      CEL_EDS_LIB=${lib:-celestia-app_amd/libcelestia_eds.so} timeout -k 10 180 python bench.py --k $1 --batch $2 --steps 20 --warmup 3 --inflight ${inf%n} --no-cpu --no-riders \
        --k512-batch 0 --no-host-io > gpurun_out/${tag}_b.json 2> gpurun_out/${tag}_b.err || { cat gpurun_out/${tag}_b.err; exit 2; }
      python - "$1" "$2" "$inf" gpurun_out/${tag}_b.json >> $out <<'PY'
import json, sys
k, B, inf, f = sys.argv[1:]
d = json.loads(open(f).read().strip().splitlines()[-1])
print(f"k {k:>3} B {B:>4} inflight {inf}: {d['value']:9.1f} squares/s  {d['ms_per_step']:7.3f} ms/step")
PY
    done
  done
done
cat $out
timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/${tag}_trace -o tr -- python3 tools/step_trace.py --k 64 --batch 128 \
  --inflight 2 --chain 8 --steps 3 > gpurun_out/${tag}_trace.log 2>&1 || { tail -20 gpurun_out/${tag}_trace.log; exit 3; }
python3 tools/timeline.py gpurun_out/${tag}_trace 1000 -2 > gpurun_out/${tag}_timeline.txt && tail -25 gpurun_out/${tag}_timeline.txt
