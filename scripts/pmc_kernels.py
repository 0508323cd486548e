#!/usr/bin/env python3
"""Average of every counter per engine kernel (k_*) from a rocprofv3 --pmc counter_collection.csv.
Usage: pmc_kernels.py <dir with *counter_collection.csv> [out.txt]   (then delete the big CSV on the box)"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("cc::", "")
        if n.startswith("k_"):
            agg[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
lines = [f"{n}: " + ", ".join(f"{k}={sum(v) / len(v):.4g}" for k, v in sorted(c.items())) for n, c in sorted(agg.items())]
out = "\n".join(lines)
print(out)
if len(sys.argv) > 2:
    open(sys.argv[2], "w").write(out + "\n")
