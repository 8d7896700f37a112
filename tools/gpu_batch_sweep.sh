set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for b in 256 512 256 512 1024; do
  timeout -k 10 200 python bench.py --batch $b --steps 10 --warmup 2 --no-cpu --no-host-io --no-riders --k512-batch 0 2>/dev/null \
   | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('B', $b, round(d['value'],1), round(d['roofline']['frac'],3), round(d['roofline_nmt']['frac'],3))" || exit 1
done
for b in 32 64; do
  timeout -k 10 200 python bench.py --k 512 --batch $b --steps 5 --warmup 2 --no-cpu --no-host-io --no-riders 2>/dev/null \
   | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('k512 B', $b, round(d['value'],1), round(d['roofline']['frac'],3), round(d['roofline_nmt']['frac'],3))" || exit 1
done
