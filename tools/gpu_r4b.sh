#!/bin/bash
# Round-4 probes: the one-pass extension data flow against the two-pass one (memory only,
# tools/microbench/onepass_mem.hip: timing + L2 / HBM PMC passes, one data flow per pass),
# then kernel timelines of single batch steps at config 4's per-GPU shape (k=64, B=128)
# and at B=1024 (tools/step_trace.py). Each GPU step has its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r4b}
mb=tools/microbench/onepass_mem
timeout -k 10 120 $mb > gpurun_out/${tag}_onepass.txt 2>&1 || { cat gpurun_out/${tag}_onepass.txt; exit 1; }
cat gpurun_out/${tag}_onepass.txt
i=0
for cfg in "two-pass" "S=8 xcd default" "S=8 rr default" "S=32 xcd"; do
  for pmc in "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" "FETCH_SIZE" "WRITE_SIZE TCC_EA0_RDREQ_sum"; do
    i=$((i + 1))
    timeout -s KILL 60 rocprofv3 --pmc $pmc -d gpurun_out/${tag}_pmc_$i -o p --output-format csv -- \
      $mb "$cfg" > /dev/null 2>&1 || { echo "pmc pass $i ($cfg: $pmc) rc=$?"; exit 2; }
    echo "== $cfg | $pmc" >> gpurun_out/${tag}_onepass_pmc.txt
    python3 tools/pmc_summary.py gpurun_out/${tag}_pmc_$i >> gpurun_out/${tag}_onepass_pmc.txt
  done
done
cat gpurun_out/${tag}_onepass_pmc.txt
for b in 128 1024; do
  timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/${tag}_step_k64_b$b -o s --output-format csv -- \
    python3 tools/step_trace.py --k 64 --batch $b --steps 4 > gpurun_out/${tag}_step_k64_b$b.txt 2>&1 || exit 3
  cat gpurun_out/${tag}_step_k64_b$b.txt
  python3 tools/timeline.py gpurun_out/${tag}_step_k64_b$b 1000 -2 > gpurun_out/${tag}_timeline_k64_b$b.txt
  tail -3 gpurun_out/${tag}_timeline_k64_b$b.txt
done
