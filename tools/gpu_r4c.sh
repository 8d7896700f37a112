set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
( bash tools/gpu_pipe_ab.sh base prio base prio ) > gpurun_out/r4c_pipe_ab.txt 2>&1 || { cat gpurun_out/r4c_pipe_ab.txt; exit 1; }
cat gpurun_out/r4c_pipe_ab.txt
( bash tools/gpu_latency_ab.sh base prio ) > gpurun_out/r4c_latency_ab.txt 2>&1 || { cat gpurun_out/r4c_latency_ab.txt; exit 2; }
cat gpurun_out/r4c_latency_ab.txt
CEL_EDS_LIB=variants/libprio.so timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/r4c_step_prio -o s --output-format csv -- \
    python3 tools/step_trace.py --k 64 --batch 128 --steps 4 > /dev/null 2>&1 || exit 3
python3 tools/timeline.py gpurun_out/r4c_step_prio 1000 -2 > gpurun_out/r4c_timeline_prio.txt
tail -12 gpurun_out/r4c_timeline_prio.txt
