#!/usr/bin/env python3
"""Per-launch HBM-side traffic of every engine kernel from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

Correction (MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE reports half the bytes of wide (16 B/lane)
streaming reads, so reads are doubled; WRITE_SIZE is taken as is.  Both counters are in KiB and count L2 misses
(Infinity-Cache hits included), i.e. an upper bound on HBM bytes.

Usage: pmc_traffic.py <gpurun_out/TAG> <out.json> [workload=c2]   (expects TAG/fetch and TAG/write from scripts/gpu_round.sh)
bench.py reads profiles/traffic_latest.json (a copy of the newest out.json) to fill roofline.traffic.
"""
import collections
import csv
import json
import os
import sys


def per_kernel(path):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("cc::", "")
        name = name.split("<")[0]
        if name.startswith("k_"):
            agg[name].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main(d, out, workload="c2"):
    f = per_kernel(os.path.join(d, "fetch", "run_counter_collection.csv"))
    w = per_kernel(os.path.join(d, "write", "run_counter_collection.csv"))
    res = {}
    for k in sorted(set(f) | set(w)):
        fk, wk = f.get(k, 0.0), w.get(k, 0.0)
        res[k] = {"fetch_kib_raw": round(fk, 1), "write_kib": round(wk, 1),
                  "bytes_per_launch": round((2 * fk + wk) * 1024)}
    json.dump({"source": d, "workload": workload, "correction": "2 x FETCH_SIZE + WRITE_SIZE (KiB -> B), per launch", "kernels": res},
              open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
