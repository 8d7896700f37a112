set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
for v in ${VARIANTS:-dl0 dl1}; do
  CEL_EDS_LIB=variants/lib$v.so timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0,'celestia-app_amd'); sys.argv=['x']
import bench, json
from celestia_eds import default_context
r = bench.measure_host_io(default_context(0), 128)
print('$v', json.dumps({k: (v if not isinstance(v, dict) else round(v['squares_per_s'])) for k, v in r.items() if k != 'entry_point'}))
" 2>&1 | grep -v amdgpu.ids || exit 1
done
