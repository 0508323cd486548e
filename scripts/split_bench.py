"""Single-global-log split rate (cc_split_batch / cc_merge_results, copycat_amd/csrc/split.cpp) on this host's cores.

One c2-shaped global log of N rows over world x 65,536 resources (instance slot = resource slot, owner = slot % world,
DESIGN.md §6), split into `world` per-rank batches with every column, then the per-rank results merged back into log
order.  Output buffers are allocated once and reused (a pipeline reuses its staging buffers); the first call is a
warm-up that also faults the pages in.  Prints one JSON line.  Usage: python scripts/split_bench.py [N] [world] [reps]
"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from copycat_amd import abi, shard  # noqa: E402
from copycat_amd.batch import Batch  # noqa: E402
from copycat_amd.engine import _check, _np, lib  # noqa: E402
from copycat_amd.workload import atomic_long_stream  # noqa: E402


def main():
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 100_000_000
    world = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    threads = shard._threads(0)
    R = 65536 * world
    b = atomic_long_stream(n, R)
    tab = (np.arange(R) % world).astype(np.uint8)
    counts = shard.split_counts(b, tab, world, threads)
    subs = [Batch(int(c)) for c in counts]
    outs = (abi.cc_batch_out * world)()
    for r in range(world):
        for name in Batch.__slots__:
            setattr(outs[r], name, _np(getattr(subs[r], name)))
    cols = abi.cc_batch(**{name: _np(getattr(b, name)) for name in Batch.__slots__})
    cap = counts.copy()
    split_s = []
    for it in range(reps + 1):
        t0 = time.perf_counter()
        _check(lib().cc_split_batch(C.byref(cols), n, _np(tab), R, world, threads, outs, _np(cap), _np(counts), None))
        if it:
            split_s.append(time.perf_counter() - t0)
    # each rank's results (synthetic: status = rank, value = the row's index column) merged back
    res = [(np.full(int(c), r, np.uint8), subs[r].index) for r, c in enumerate(counts)]
    pr = (abi.cc_results * world)()
    for r, (s, v) in enumerate(res):
        pr[r].status, pr[r].value = _np(s), _np(v)
    st, va = np.empty(n, np.uint8), np.empty(n, np.uint64)
    out = abi.cc_results(_np(st), _np(va))
    merge_s = []
    for it in range(reps + 1):
        t0 = time.perf_counter()
        _check(lib().cc_merge_results(_np(b.inst), n, _np(tab), R, world, threads, pr, C.byref(out)))
        if it:
            merge_s.append(time.perf_counter() - t0)
    ok = bool(np.array_equal(va, b.index) and np.array_equal(st, tab[b.inst]))
    for r in range(world):  # stable and complete: rank r's rows are exactly the log's rows of rank r, in order
        m = tab[b.inst] == r
        ok &= bool(np.array_equal(subs[r].index, b.index[m]) and np.array_equal(subs[r].a, b.a[m]))
    ts, tm = min(split_s), min(merge_s)
    print(json.dumps({"split_rows_per_s": n / ts, "split_ms": ts * 1e3, "merge_rows_per_s": n / tm, "merge_ms": tm * 1e3,
                      "rows": n, "world": world, "threads": threads, "bytes_per_row_split": 54, "ok": ok,
                      "split_GBps_copied": n * 54 / ts / 1e9}))


if __name__ == "__main__":
    main()
