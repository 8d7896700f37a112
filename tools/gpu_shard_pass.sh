set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r3f_pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/r3f_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for n in 1 8; do timeout -k 10 120 python3 tools/rank_latency.py --k 512 --n $n 2>&1 | grep -v amdgpu.ids || exit 1; done
timeout -k 10 200 python bench.py --mode sharded --k 512 --steps 10 --warmup 3 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rowshard N=1', round(d['value'],1), d['phase_us'])"
