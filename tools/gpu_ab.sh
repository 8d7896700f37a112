#!/bin/bash
# A/B of library builds on one measurement, variants in the order given (repeat names to
# interleave them against drift). A variant is variants/lib<v>.so from build_variant.sh
# (a tools/variants/*.patch on a copy of csrc); "shipped" is the in-tree library.
#   bash tools/gpu_ab.sh <what> <variant>...
# what:
#   extend | commit   one phase alone, K=<k> B=<batch> (default 128 256): tools/prof_phase.py
#   sweep             extend per square at B = 64 and 256 beside the transform-only probe (rs_sweep.py), K=<k>
#   power             socket power and clock while the extend phase loops (power_probe.py), K, B
#   step              the headline line (k=128 B=256, --inflight ${INFLIGHT:-4}, no riders)
#   pipe              batch steps k=64 B=128 and k=128 B=256 at --inflight ${INFLIGHT:-1}
#   header            one k=128 header through the host entry point (page-locked ODS, roots + DAH)
#   hostio            cel_extend_batch, 16 k=128 squares: EDS / parity only / roots only back
#   repair            bench --mode repair at k = ${K:-128} (k = 512 / 256: the GF(2^16) decoder)
#   latency           rank-0 chain of a row-sharded k=512 square (N = 1, 8), one header, k=64 B=128 steps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
what=$1; shift
k=${K:-128}; b=${B:-256}
lib() { [ "$1" = shipped ] && echo celestia-app_amd/libcelestia_eds.so || echo variants/lib$1.so; }
line() {  # value and ms/step of a bench JSON line on stdin
  python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$1', round(d['value'],1), round(d['ms_per_step'],3), 'ms/step')"
}
for v in "$@"; do
  export CEL_EDS_LIB=$(lib $v)
  case $what in
    extend|commit)
      echo -n "$v: "
      timeout -k 10 120 python3 tools/prof_phase.py --phase $what --k $k --batch $b --reps 10 2>&1 | grep -v amdgpu.ids || exit 1 ;;
    sweep)
      timeout -k 10 120 python3 tools/rs_sweep.py --k $k --batches 64,256 2>&1 | grep -v amdgpu.ids || exit 1 ;;
    power)
      timeout -k 10 60 python3 tools/power_probe.py --phase extend --k $k --batch $b 2>&1 | grep -v amdgpu.ids || exit 1 ;;
    step)
      timeout -k 10 200 python bench.py --steps 20 --warmup 5 --inflight ${INFLIGHT:-4} --no-cpu --no-host-io --no-riders \
        --k512-batch 0 2>/dev/null | line "$v step" || exit 1 ;;
    pipe)
      for kb in "64 128" "128 256"; do
        set -- $kb
        timeout -k 10 200 python bench.py --k $1 --batch $2 --steps 10 --warmup 2 --no-cpu --no-host-io --no-riders \
          --k512-batch 0 --inflight ${INFLIGHT:-1} 2>/dev/null | line "$v k $1 B $2" || exit 1
      done ;;
    header)
      echo -n "$v: "
      timeout -k 10 120 python3 tools/host_io.py --batch 1 --no-eds --pinned --reps 50 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1 ;;
    hostio)
      for m in "" "--parity-only" "--no-eds"; do
        echo -n "$v $m: "
        timeout -k 10 120 python3 tools/host_io.py --batch 16 --pinned --reps 5 $m 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
      done ;;
    repair)
      timeout -k 10 200 python3 bench.py --mode repair --k $k --steps 20 --warmup 3 --cpu-seconds 0.5 \
        > gpurun_out/ab_repair_$v.json 2>/dev/null || exit 1
      python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/ab_repair_$v.json') if l.startswith('{')][-1]; print('$v k=$k', round(d['value'],1), 'repairs/s', round(d['ms_per_step'],3), 'ms, decode launch', round(d['roofline']['avg_launch_us'],1), 'us')" ;;
    latency)
      for n in 1 8; do
        echo -n "$v "; timeout -k 10 120 python3 tools/rank_latency.py --k 512 --n $n 2>&1 | grep -v amdgpu.ids || exit 1
      done
      echo -n "$v "; timeout -k 10 120 python3 tools/host_io.py --batch 1 --no-eds --pinned --reps 30 2>&1 | grep -v amdgpu.ids | tail -1
      timeout -k 10 200 python bench.py --k 64 --batch 128 --steps 10 --warmup 2 --no-cpu --no-host-io --no-riders \
        --k512-batch 0 2>/dev/null | line "$v k64 B128" || exit 1 ;;
    *) echo "unknown measurement: $what" >&2; exit 2 ;;
  esac
done
