"""GPU timeline gaps of a rocprofv3 run (dev aid): kernels + copies sorted by start, the
idle gaps between them, and the HIP API calls that overlap the largest gaps.
python tools/gap_trace.py <dir> [--last-us N]  (analyses the last N us of the run)"""
import csv
import glob
import sys


def rows(d, pat):
    out = []
    for f in glob.glob(d + '/**/' + pat, recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def main():
    d = sys.argv[1]
    last = float(sys.argv[sys.argv.index('--last-us') + 1]) if '--last-us' in sys.argv else 3000.0
    ev = []
    for r in rows(d, '*kernel_trace.csv'):
        ev.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), 'K ' + r['Kernel_Name'][:60]))
    for r in rows(d, '*memory_copy_trace.csv'):
        ev.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), 'C ' + r.get('Direction', 'copy')))
    ev.sort()
    api = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Function']) for r in rows(d, '*hip_api_trace.csv'))
    end = ev[-1][1]
    t0 = end - last * 1e3
    win = [e for e in ev if e[0] >= t0]
    busy = 0
    prev_end = win[0][0]
    gaps = []
    for s, e, n in win:
        if s > prev_end:
            gaps.append((s - prev_end, prev_end, s, n))
        busy += e - max(s, prev_end) if e > prev_end else 0
        prev_end = max(prev_end, e)
    span = prev_end - win[0][0]
    print(f"window {span / 1e3:.1f} us, busy {busy / 1e3:.1f} us ({busy / span:.2f}), {len(win)} ops, "
          f"{len(gaps)} gaps, sum {sum(g[0] for g in gaps) / 1e3:.1f} us")
    for g, a, b, n in sorted(gaps, reverse=True)[:12]:
        calls = [c for c in api if c[1] > a and c[0] < b]
        names = {}
        for c in calls:
            names[c[2]] = names.get(c[2], 0) + (min(c[1], b) - max(c[0], a))
        top = sorted(names.items(), key=lambda x: -x[1])[:4]
        print(f"gap {g / 1e3:7.1f} us before {n[:50]:50s} | " + ", ".join(f"{k} {v / 1e3:.1f}" for k, v in top))
    if '--seq' in sys.argv:
        for s, e, n in win:
            print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} {n}")


if __name__ == '__main__':
    main()
