"""Summarise rocprofv3 --pmc CSVs: per kernel, mean counter values per dispatch."""
import csv
import glob
import sys
from collections import defaultdict

for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        agg = defaultdict(lambda: defaultdict(float))
        disp = defaultdict(set)
        dur = defaultdict(dict)
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0][-40:]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
            dur[k][r["Dispatch_Id"]] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
        for k, v in agg.items():
            n = len(disp[k])
            us = sum(dur[k].values()) / n / 1e3
            parts = " ".join(f"{c}={val / n:.4g}" for c, val in sorted(v.items()))
            print(f"{d.split('/')[-1]:14s} {k:40s} n={n} us={us:.1f} {parts}")
