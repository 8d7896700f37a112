#!/bin/bash
# Kernel-time breakdown and decoder PMC counters of the k=512 repair (run on the GPU box).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof512
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof512/stats -o run --output-format csv -- \
  python3 bench.py --mode repair --k 512 --steps 4 --warmup 1 --cpu-seconds 0.5 > gpurun_out/prof512/bench.json
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SMEM \
  -d gpurun_out/prof512/pmc1 -o run --output-format csv -- python3 bench.py --mode repair --k 512 --steps 1 --warmup 0 --cpu-seconds 0.5 > /dev/null
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_WAVE_CYCLES \
  -d gpurun_out/prof512/pmc2 -o run --output-format csv -- python3 bench.py --mode repair --k 512 --steps 1 --warmup 0 --cpu-seconds 0.5 > /dev/null

# keep only the summaries and the decoder's rows (the full traces are large)
python3 - <<'PY'
import csv, glob, os
root = "gpurun_out/prof512"
for f in glob.glob(f"{root}/pmc*/**/*counter_collection.csv", recursive=True):
    rows = [r for r in csv.DictReader(open(f)) if "decode_gf16" in r.get("Kernel_Name", "")]
    per = {}
    for r in rows:
        per.setdefault(r["Dispatch_Id"], {})[r["Counter_Name"]] = float(r["Counter_Value"])
    # the largest launch (the first row pass: 1024 axes)
    big = max(per.values(), key=lambda d: d.get("SQ_WAVES", d.get("SQ_WAVE_CYCLES", 0)))
    with open(f"{root}/{os.path.basename(os.path.dirname(f))}_decode.txt", "w") as o:
        o.write(f"# largest k_rs_decode_gf16 launch of {len(per)}\n")
        for k, v in sorted(big.items()):
            o.write(f"{k} {v:.0f}\n")
    os.remove(f)
for f in glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True):
    os.remove(f)
PY
ls -R gpurun_out/prof512 | head -30
