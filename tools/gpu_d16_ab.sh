#!/bin/bash
# A/B of the GF(2^16) decoder variants (variants/lib*.so) on the k=512 and k=256 repairs.
#   bash tools/gpu_d16_ab.sh name1 name2 ...   (run on the GPU box; "default" = the product .so)
set -e
mkdir -p gpurun_out
out=gpurun_out/d16_ab.txt
: > $out
for v in "$@"; do
  for k in 512 256; do
    if [ "$v" = default ]; then lib=celestia-app_amd/libcelestia_eds.so; else lib=variants/lib$v.so; fi
    CEL_EDS_LIB=$lib timeout -k 10 200 python bench.py --mode repair --k $k --steps 8 --warmup 2 --cpu-seconds 0.5 > gpurun_out/d16_ab_${v}_${k}.json
    python3 - "$v" "$k" gpurun_out/d16_ab_${v}_${k}.json >> $out <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[3]) if l.startswith("{")][-1]
print(f"{sys.argv[1]:>10} k={sys.argv[2]}: {d['ms_per_step']:.3f} ms/repair, decode launch {d['roofline']['avg_launch_us']:.1f} us")
PY
  done
done
cat $out
