#!/bin/bash
# A short default bench line and the presence (or error) of each of its parts.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
tag=${1:-bc}
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --cpu-seconds 3 > gpurun_out/${tag}_bench.json \
  2> gpurun_out/${tag}_bench.err || { tail -20 gpurun_out/${tag}_bench.err; exit 1; }
python3 - gpurun_out/${tag}_bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", round(d["value"]), "inflight", d["config"].get("batches_in_flight"))
for k in ("k512", "k64", "rowshard512", "host_io", "cpu_baseline"):
    v = d.get(k)
    print(k, "missing" if v is None else ("ERROR " + v["error"] if "error" in v else "ok"))
print("parity_vs_cpu", d.get("parity_vs_cpu"))
PY
