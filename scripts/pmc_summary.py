#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc CSVs (per dispatch, millions).
usage: pmc_summary.py DIR [kernel-substring ...]"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
keys = sys.argv[2:]
for path in sorted(glob.glob(os.path.join(d, "*", "pmc_counter_collection.csv"))):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"]
        if keys and not any(k in n for k in keys):
            continue
        agg[n[:60]][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[n[:60]].add(r["Dispatch_Id"])
    for k, v in agg.items():
        nd = len(disp[k])
        print(os.path.basename(os.path.dirname(path)), k,
              {c: round(x / nd / 1e6, 2) for c, x in sorted(v.items())}, "dispatches", nd)
