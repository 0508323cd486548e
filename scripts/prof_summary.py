#!/usr/bin/env python3
"""Summarize a gpu_round.sh output dir: per-kernel avg duration (kernel trace) and per-launch FETCH/WRITE_SIZE."""
import collections
import csv
import os
import sys


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "").replace("cc::", "")


def main(d):
    stats = list(csv.DictReader(open(os.path.join(d, "kt", "run_kernel_stats.csv"))))
    print(f"{'kernel':40s} {'calls':>6s} {'avg_us':>10s} {'total_ms':>10s}")
    for r in stats:
        print(f"{short(r['Name'])[:40]:40s} {r['Calls']:>6s} {float(r['AverageNs'])/1e3:10.1f} {float(r['TotalDurationNs'])/1e6:10.3f}")
    for c in ("fetch", "write"):
        p = os.path.join(d, c, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(p)):
            agg[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
        print(f"-- {c.upper()}_SIZE per launch (KB, raw counter; gfx950 FETCH_SIZE reads half of wide streaming reads)")
        for k, v in agg.items():
            if k.startswith("k_"):
                print(f"   {k:30s} n={len(v):3d} avg={sum(v)/len(v):12.0f} KB")


if __name__ == "__main__":
    main(sys.argv[1])
