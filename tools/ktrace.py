"""Per-grid-size average durations of kernels in a rocprofv3 --kernel-trace CSV run
(dev aid): python tools/ktrace.py <dir> [kernel-name substring]"""
import collections
import csv
import glob
import sys

pat = sys.argv[2] if len(sys.argv) > 2 else ''
for f in glob.glob(sys.argv[1] + '/**/*kernel_trace.csv', recursive=True):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if pat in r['Kernel_Name']:
            d[(r['Kernel_Name'][:48], int(r['Grid_Size_X']))].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
    for (n, g), v in sorted(d.items()):
        v = v[1:] if len(v) > 2 else v  # drop the first (cold) call
        print(f"{n:48s} grid={g:9d} calls={len(v):3d} avg_us={sum(v) / len(v):9.1f} min_us={min(v):9.1f}")
