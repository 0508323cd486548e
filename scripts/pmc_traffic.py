#!/usr/bin/env python3
"""Per-launch HBM-side traffic of every engine kernel from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

Correction (MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE reports half the bytes of wide (16 B/lane)
streaming reads, so reads are doubled; WRITE_SIZE is taken as is.  Both counters are in KiB and count L2 misses
(Infinity-Cache hits included), i.e. an upper bound on HBM bytes.

Usage: pmc_traffic.py <gpurun_out/TAG> <out.json> [workload=c2] [commits]   (expects TAG/fetch and TAG/write: scripts/gpu_round.sh,
scripts/gpu_profile_wl.sh).  out.json keeps one entry per workload ("workloads": {"c2": ..., "c3": ..., "c5": ...}):
the workload's entry is replaced, the others kept.  bench.py reads profiles/traffic_latest.json to fill
roofline.traffic.  With `commits` (every commit the profiled command applied: (warmup + steps) x commits per step)
each kernel also gets bytes_per_commit (its bytes per launch x its launches / commits) and the workload
bytes_per_commit_total, the whole step's measured HBM bytes per commit.
"""
import collections
import csv
import json
import os
import sys


def per_kernel(path):
    """kernel -> (average counter value per launch, launches)"""
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("cc::", "")
        name = name.split("<")[0]
        if name.startswith("k_"):
            agg[name].append(float(r["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in agg.items()}


def per_kernel_summary(path, counter):
    """scripts/gpu_prof.sh's on-box summary (scripts/pmc_kernel_summary.py output): kernel line, then counter lines."""
    tot, cur = collections.defaultdict(lambda: [0.0, 0]), None  # kernel -> [sum over launches, launches]
    for line in open(path):
        if not line.startswith(" "):
            cur = line.strip().split("<")[0]  # template variants of one kernel add up
        elif cur and line.split()[0] == counter:
            launches = int(line.split("n=")[1].split()[0])
            tot[cur][0] += float(line.split("avg=")[1]) * launches
            tot[cur][1] += launches
    return {k: (v[0] / v[1], v[1]) for k, v in tot.items() if v[1]}


def main(d, out, workload="c2", commits=None):
    if os.path.exists(os.path.join(d, "pmc1_summary.txt")):  # scripts/gpu_prof.sh layout
        f = per_kernel_summary(os.path.join(d, "pmc1_summary.txt"), "FETCH_SIZE")
        w = per_kernel_summary(os.path.join(d, "pmc2_summary.txt"), "WRITE_SIZE")
    else:
        f = per_kernel(os.path.join(d, "fetch", "run_counter_collection.csv"))
        w = per_kernel(os.path.join(d, "write", "run_counter_collection.csv"))
    res = {}
    total = 0.0
    for k in sorted(set(f) | set(w)):
        (fk, nf), (wk, nw) = f.get(k, (0.0, 0)), w.get(k, (0.0, 0))
        res[k] = {"fetch_kib_raw": round(fk, 1), "write_kib": round(wk, 1),
                  "bytes_per_launch": round((2 * fk + wk) * 1024), "launches": max(nf, nw)}
        if commits:
            res[k]["bytes_per_commit"] = round((2 * fk * nf + wk * nw) * 1024 / commits, 3)
            total += res[k]["bytes_per_commit"]
    doc = {"correction": "2 x FETCH_SIZE + WRITE_SIZE (KiB -> B), per launch", "workloads": {}}
    try:
        with open(out) as fh:
            old = json.load(fh)
        if "workloads" in old:
            doc["workloads"] = old["workloads"]
        elif "kernels" in old:  # the single-workload layout of round 1
            doc["workloads"][old.get("workload", "c2")] = {"source": old.get("source"), "kernels": old["kernels"]}
    except (OSError, ValueError):
        pass
    doc["workloads"][workload] = {"source": d, "kernels": res}
    if commits:  # the whole step's measured bytes per commit (bench.py roofline.traffic)
        doc["workloads"][workload]["commits_profiled"] = commits
        doc["workloads"][workload]["bytes_per_commit_total"] = round(total, 2)
    json.dump(doc, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4], int(float(sys.argv[4])) if len(sys.argv) > 4 else None)
