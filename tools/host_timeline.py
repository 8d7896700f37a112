"""Merged host/device timeline of a rocprofv3 run with --kernel-trace, --hip-runtime-trace
and --marker-trace (dev aid).

python tools/host_timeline.py <dir> <marker> [before_us] [after_us] [which]

Window: from `before_us` ahead of the start of occurrence `which` (default -1, the last)
of roctx range `marker` to `after_us` past its end. Prints every kernel (K), memory copy
(C), HIP API call (H) and roctx range (M) in the window by start time: start offset and
duration (us).
"""
import csv
import glob
import sys

d, marker = sys.argv[1], sys.argv[2]
before = float(sys.argv[3]) if len(sys.argv) > 3 else 200.0
after = float(sys.argv[4]) if len(sys.argv) > 4 else 400.0
which = int(sys.argv[5]) if len(sys.argv) > 5 else -1


def rows(pattern):
    out = []
    for f in glob.glob(d + '/**/' + pattern, recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


ev = []
for r in rows('*kernel_trace.csv'):
    ev.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), 'K',
               r['Kernel_Name'].split('(')[0].replace('void ', '').replace('cel::', '')[:40]))
for r in rows('*memory_copy_trace.csv'):
    ev.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), 'C',
               (r.get('Direction', '') + ' ' + r.get('Size', '')).strip()[:40]))
for r in rows('*hip_api_trace.csv'):
    ev.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), 'H', r['Function'][:40]))
marks = []
for r in rows('*marker_api_trace.csv'):
    name = r.get('Function') or r.get('Message') or ''
    e = (int(r['Start_Timestamp']), int(r['End_Timestamp']), 'M', name[:40])
    ev.append(e)
    if name == marker:
        marks.append(e)
marks.sort()
if not marks:
    sys.exit(f"no marker {marker!r}")
m = marks[which]
t0, t1 = m[0] - before * 1e3, m[1] + after * 1e3
ev = sorted(e for e in ev if e[1] >= t0 and e[0] <= t1)
for s, e, kind, name in ev:
    print(f"{(s - m[0]) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {kind} {name}")
