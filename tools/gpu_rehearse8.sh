#!/bin/bash
# The N = 8 code path on one GPU: 8 ranks over gloo with host staging (bench --rehearse),
# small batches, riders on (config 4 split, config 3 row-sharded incl. the pipelined
# schedule); then the RS traffic PMC passes of this round's build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --rehearse --gpus 8 --batch 64 --k512-batch 8 --steps 3 --warmup 1 --rider-steps 2 \
  --no-cpu --no-host-io > gpurun_out/rehearse8.json 2> gpurun_out/rehearse8.err || { tail -20 gpurun_out/rehearse8.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/rehearse8.json'))
print('n_gpus', d['n_gpus'], 'value', round(d['value']), 'k512', round(d['k512']['value']), 'k64', round(d['k64']['value']))
r=d['rowshard512']; print('rowshard', r['n_gpus'], round(r['value'],1), r.get('pipelined'), r['a2a_bytes_per_peer'])"
bash tools/gpu_traffic.sh r3tr 128 32
