"""Print the rocprofv3 --stats kernel summary found under a directory."""
import csv
import glob
import sys

for f in glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True):
    print(f)
    for r in csv.DictReader(open(f)):
        print(f"{r['Name'][:60]:60s} calls={r['Calls']:>6s} avg_us={float(r['AverageNs'])/1e3:9.2f} pct={float(r['Percentage']):6.2f}")
