"""Kernel timeline of a rocprofv3 --kernel-trace CSV (dev aid).

python tools/timeline.py <dir> [gap_us] [which]

Splits the trace into bursts separated by idle gaps longer than gap_us (default 500) and
prints burst `which` (default: the second-to-last) kernel by kernel: start offset, duration
and gap to the previous kernel end (all in us), queue id and a short kernel name, then the
burst's busy time (union of kernel intervals) against its span.
"""
import csv
import glob
import sys

d = sys.argv[1]
gap_us = float(sys.argv[2]) if len(sys.argv) > 2 else 500.0
which = int(sys.argv[3]) if len(sys.argv) > 3 else -2
rows = []
for f in glob.glob(d + '/**/*kernel_trace.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        q = r.get('Queue_Id') or r.get('Stream_Id') or '?'
        rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), q, r['Kernel_Name']))
for f in glob.glob(d + '/**/*.db', recursive=True):  # rocprofv3's default (rocpd SQLite) output
    import sqlite3
    con = sqlite3.connect(f)
    for s, e, q, st, n in con.execute("select start, end, queue_id, stream_id, name from kernels"):
        rows.append((int(s), int(e), f"{q}/{st}", n))
rows.sort()
bursts, cur, end = [], [], None
for s, e, q, n in rows:
    if cur and s - end > gap_us * 1e3:
        bursts.append(cur)
        cur = []
    cur.append((s, e, q, n))
    end = e if end is None or not cur[:-1] else max(end, e)
if cur:
    bursts.append(cur)
print(f"{len(bursts)} bursts; showing {which}")
b = bursts[which]
t0, prev_end, busy, cov_end = b[0][0], b[0][0], 0, b[0][0]
for s, e, q, n in b:
    name = n.split('(')[0].replace('void ', '').replace('cel::', '')[:44]
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} gap={(s - prev_end) / 1e3:7.1f} q={q:>3} {name}")
    prev_end = max(prev_end, e)
    if e > cov_end:
        busy += e - max(s, cov_end)
        cov_end = e
span = max(e for _, e, _, _ in b) - t0
print(f"span {span / 1e3:.1f} us, busy {busy / 1e3:.1f} us, kernels {len(b)}")
