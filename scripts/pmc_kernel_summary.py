#!/usr/bin/env python3
"""Average of each counter per kernel from a rocprofv3 --pmc counter_collection.csv (one row per dispatch x counter)."""
import collections
import csv
import glob
import sys

path = sys.argv[1]
files = glob.glob(path + "/**/*counter_collection.csv", recursive=True)
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in files:
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("cc::", "")
        if not name.startswith("k_"):
            continue
        agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(agg.items()):
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:24s} n={len(v):3d} avg={sum(v) / len(v):16.1f}")
