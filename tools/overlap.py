"""How the RS extension and the NMT commit kernels overlap in a burst of batch steps
(dev aid, rocprofv3 --kernel-trace CSV of tools/step_trace.py):

  python3 tools/overlap.py <dir> [gap_us] [which]

Splits the trace into bursts at idle gaps longer than gap_us (default 1000) and, for burst
`which` (default: the second-to-last), sums the wall time in each state: RS kernels only,
NMT kernels only, both, neither; plus each class's summed kernel time. With both halves
VALU-bound, the time spent with RS alone is where the step leaves VALU idle while the
extension waits on HBM."""
import csv
import glob
import sys

d = sys.argv[1]
gap_us = float(sys.argv[2]) if len(sys.argv) > 2 else 1000.0
which = int(sys.argv[3]) if len(sys.argv) > 3 else -2
rows = []
for f in glob.glob(d + '/**/*kernel_trace.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']))
rows.sort()
bursts, cur, end = [], [], None
for s, e, n in rows:
    if cur and s - end > gap_us * 1e3:
        bursts.append(cur)
        cur, end = [], None
    cur.append((s, e, n))
    end = e if end is None else max(end, e)
if cur:
    bursts.append(cur)
b = bursts[which]


def cls(n):
    if "rs_axis" in n or "rs_gf16" in n or "rs_encode" in n:
        return "rs"
    if "k_leaf" in n or "k_level" in n or "k_merkle" in n or "k_slab" in n:
        return "nmt"
    return "other"


ev = []
tot = {"rs": 0, "nmt": 0, "other": 0}
cnt = {"rs": 0, "nmt": 0, "other": 0}
for s, e, n in b:
    c = cls(n)
    tot[c] += e - s
    cnt[c] += 1
    ev.append((s, 1, c))
    ev.append((e, -1, c))
ev.sort()
live = {"rs": 0, "nmt": 0, "other": 0}
state_t = {"rs only": 0, "nmt only": 0, "both": 0, "neither": 0}
t0, last = ev[0][0], ev[0][0]
for t, dlt, c in ev:
    if t > last:
        r, m = live["rs"] > 0, live["nmt"] > 0
        key = "both" if r and m else "rs only" if r else "nmt only" if m else "neither"
        state_t[key] += t - last
        last = t
    live[c] += dlt
span = last - t0
print(f"burst {which} of {len(bursts)}: {len(b)} kernels, span {span / 1e3:.1f} us")
for c in ("rs", "nmt", "other"):
    print(f"  {c:5s} {cnt[c]:5d} launches, summed kernel time {tot[c] / 1e3:10.1f} us")
for k, v in state_t.items():
    print(f"  {k:9s} {v / 1e3:10.1f} us  ({v / span:.3f} of the span)")
