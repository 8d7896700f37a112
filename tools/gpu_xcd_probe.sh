#!/bin/bash
# tools/microbench/xcd_two_pass.hip, one variant per process under its own time limit.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
out=gpurun_out/xcd_two_pass.txt; : > $out
for v in "two-pass" "default, 256" "nt, 256" "default, 512" "nt, 512"; do
  timeout -k 5 40 ./tools/microbench/xcd_two_pass ${NSQ:-64} "$v" >> $out 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "variant '$v' rc=$rc" >> $out; [ $rc -eq 124 ] || [ $rc -eq 137 ] && break; }
done
cat $out
