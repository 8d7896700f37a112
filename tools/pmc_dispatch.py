"""Per-dispatch counter values of rocprofv3 --pmc CSV runs (dev aid):
  python tools/pmc_dispatch.py <dir> [<dir> ...] [--kernel substring]"""
import collections
import csv
import glob
import sys

args = [a for a in sys.argv[1:] if not a.startswith('--')]
pat = sys.argv[sys.argv.index('--kernel') + 1] if '--kernel' in sys.argv else ''
if pat in args:
    args.remove(pat)
for d in args:
    for f in glob.glob(d + '/**/*counter_collection.csv', recursive=True):
        vals = collections.defaultdict(dict)
        info = {}
        for r in csv.DictReader(open(f)):
            if pat not in r['Kernel_Name'] or r['Kernel_Name'].startswith('__amd'):
                continue
            k = int(r['Dispatch_Id'])
            vals[k][r['Counter_Name']] = vals[k].get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
            info[k] = (r['Kernel_Name'][:40], int(r['Grid_Size']), (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
        for k in sorted(vals):
            n, g, us = info[k]
            print(f"{d.split('/')[-1]:10s} {k:4d} {n:40s} grid={g:8d} us={us:8.1f} " +
                  ' '.join(f"{c}={v:.3g}" for c, v in sorted(vals[k].items())))
