#!/usr/bin/env python3
"""Timeline of the timed window of a kernel trace (bench.py --window-markers): every kernel in launch order with its
duration and the idle gap before it, and a per-gap-kind summary (which kernel pairs the GPU idles between).
   python3 scripts/kt_timeline.py <kernel_trace.csv> [--steps K] [--show N]"""
import collections
import csv
import sys

trace, args = sys.argv[1], sys.argv[2:]
steps = int(args[args.index("--steps") + 1]) if "--steps" in args else 1
show = int(args[args.index("--show") + 1]) if "--show" in args else 120
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(trace)))
marks = [s for s, e, n in rows if "spin_kernel" in n]
w0, w1 = marks[0], marks[-1]
ks = [(s, e, n.split("(")[0].replace("void ", "").replace("cc::", "")[:40]) for s, e, n in rows if w0 < s < w1 and "spin_kernel" not in n]
print(f"window {(w1 - w0) / 1e6:.3f} ms, {len(ks)} kernels, {steps} steps")
end = w0
gaps = collections.Counter()
busy = 0
for i, (s, e, n) in enumerate(ks):
    gap = max(0, s - end)
    if i < show:
        print(f"{(s - w0) / 1e3:10.1f} us  gap {gap / 1e3:8.1f}  dur {(e - s) / 1e3:8.1f}  {n}")
    prev = ks[i - 1][2] if i else "(window start)"
    gaps[(prev, n)] += gap
    busy += e - max(s, end) if e > end else 0
    end = max(end, e)
print(f"busy {busy / 1e6 / steps:.3f} ms/step, idle {((w1 - w0) - busy) / 1e6 / steps:.3f} ms/step")
print("largest idle totals by (before, after) kernel pair, per step:")
for (a, b), g in gaps.most_common(15):
    print(f"  {g / 1e3 / steps:8.1f} us  {a} -> {b}")
