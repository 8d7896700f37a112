set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r3h_pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/r3h_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for n in 1 8; do timeout -k 10 120 python3 tools/rank_latency.py --k 512 --n $n 2>&1 | grep -v amdgpu.ids || exit 1; done
timeout -k 10 200 python bench.py --mode repair --steps 40 --warmup 5 --cpu-seconds 0.5 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('repair', round(d['value'],1), round(d['ms_per_step']*1e3,1),'us')"
timeout -k 10 120 python3 tools/host_io.py --batch 1 --no-eds --pinned --reps 20 2>&1 | grep -v amdgpu.ids | tail -2
bash tools/gpu_latency_traces.sh 2>&1 | grep -E "k_leaf|k_slab_leaf|span"
