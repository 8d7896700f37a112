"""Per-launch SHA-256 rates of one NMT commit (k_leaf, every k_level, k_merkle) from a
rocprofv3 --kernel-trace of `prof_phase.py --phase commit --k K --batch B` (dev aid):
  python tools/nmt_levels.py <trace dir> <k> <batch> [peak G/s]
Each launch's algorithmic compressions: leaves 9 per cell (4k^2 cells),
a level's nodes 3 each (all 4k trees), the root level 2 more per root (its RFC-6962 leaf
digest), the DAH tree 2 per inner node (4k - 1). Median over the traced calls."""
import collections
import csv
import glob
import statistics
import sys

d, k, B = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
peak = float(sys.argv[4]) if len(sys.argv) > 4 else None
W = 2 * k
runs = collections.defaultdict(list)
for f in glob.glob(d + '/**/*kernel_trace.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        name = r['Kernel_Name']
        if not any(x in name for x in ('k_leaf', 'k_level', 'k_merkle')):
            continue
        runs[(name.split('(')[0].replace('void ', '').replace('cel::', '')[:24], int(r['Grid_Size_X']))].append(
            (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)


def comps(name, grid):
    if 'k_leaf' in name:
        return 9 * W * W * B, 'leaves'
    if 'k_merkle' in name:
        return 2 * (2 * W - 1) * B, 'DAH tree'
    nodes = grid  # threads = nodes rounded up to 256 per square row of the grid
    # k_level: grid x = ceil(trees * nout / 256) * 256 threads, y = squares
    for lv in range(1, 20):
        nout = W >> lv
        if nout < 1:
            break
        if (2 * W * nout + 255) // 256 * 256 == grid:
            extra = 2 * 2 * W * B if nout == 1 else 0
            return 3 * 2 * W * nout * B + extra, f'level {lv} ({nout} nodes/tree)'
    return None, '?'


rows, tot_c, tot_t = [], 0, 0.0
for (name, grid), ts in runs.items():
    ts = ts[1:] if len(ts) > 2 else ts
    c, what = comps(name, grid)
    if c is None:
        continue
    t = statistics.median(ts)
    rows.append((0 if 'leaves' in what else (99 if 'DAH' in what else int(what.split()[1])), what, name, t, c))
    tot_c += c
    tot_t += t
print(f"k={k} batch={B}: per launch (median of traced calls)")
print(f"{'launch':26s} {'kernel':24s} {'us':>9s} {'M comp':>9s} {'G comp/s':>9s} {'share':>6s}" +
      (" frac_peak" if peak else ""))
for _, what, name, t, c in sorted(rows):
    line = f"{what:26s} {name:24s} {t:9.1f} {c / 1e6:9.3f} {c / t / 1e3:9.2f} {t / tot_t:6.1%}"
    if peak:
        line += f" {c / t / 1e3 / peak:8.3f}"
    print(line)
print(f"{'commit':26s} {'':24s} {tot_t:9.1f} {tot_c / 1e6:9.3f} {tot_c / tot_t / 1e3:9.2f}" +
      (f"        {tot_c / tot_t / 1e3 / peak:8.3f}" if peak else ""))
print(f"check: 60k^2 + 4k - 2 per square = {(60 * k * k + 4 * k - 2) * B / 1e6:.3f} M")
