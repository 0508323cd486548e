#!/usr/bin/env python3
"""Diagnostics: apply the 20M-row c3 stream on the GPU and on the oracle (as tests/test_gpu_scale.py does) up to
`--tries` times; on a mismatch, print the mismatching rows grouped by (map, key) with each key's full op history
around the first bad row and its share of the first sub-batch."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tries", type=int, default=3)
    ap.add_argument("--n", type=int, default=20_000_000)
    a = ap.parse_args()
    from copycat_amd.workload import map_zipf_rows
    from tests.test_gpu_map import _apply_both, _engines

    maps, pairs = 4096, 1 << 20
    b = map_zipf_rows(0, a.n, maps=maps, pairs=pairs, threads=8)
    for k in range(a.tries):
        E, O = _engines(maps, maps, a.n, pairs)
        gs, gv, os_, ov = _apply_both(E, O, [b])
        bad = np.nonzero((gs != os_) | (gv != ov))[0]
        print(f"try {k}: {len(bad)} bad rows", flush=True)
        if not len(bad):
            continue
        keys = {}
        for r in bad:
            keys.setdefault((int(b.inst[r]), int(b.key[r])), []).append(int(r))
        sub = 16 << 20
        print(f"  distinct keys {len(keys)}; rows by sub-batch {np.bincount(bad // sub).tolist()}")
        ms = sorted(set(m for m, _ in keys))[:4]
        for m in ms:  # final state of the affected maps vs the oracle
            g, o = E.map_entries(m), O.map_entries(m)
            gk = dict(zip(g[1].tolist(), zip(g[2].tolist(), g[3].tolist())))
            ok = dict(zip(o[1].tolist(), zip(o[2].tolist(), o[3].tolist())))
            diff = [k for k in set(gk) | set(ok) if gk.get(k) != ok.get(k)]
            print(f"  map {m}: gpu {len(gk)} entries, oracle {len(ok)}; {len(diff)} keys differ "
                  f"(bad keys among them: {sum(1 for (mm, kk) in keys if mm == m and kk in diff)})")
        for (m, key), rows in list(keys.items())[:6]:
            sel = np.nonzero((b.inst == m) & (b.key == key))[0]
            first = rows[0]
            share = np.count_nonzero(sel < sub) / min(sub, a.n)
            print(f"  map {m} key {key:#x}: {len(rows)} bad of {len(sel)} rows; share of sub-batch 0 {share:.5f}; "
                  f"bad rows {rows[:8]}")
            around = sel[(sel >= first - 20000) & (sel <= first + 2000)][-12:]
            for r in around:
                print(f"    row {r} op {int(b.op[r])} a {int(b.a[r])} flags {int(b.flags[r])} gpu ({int(gs[r])},{int(gv[r])}) "
                      f"oracle ({int(os_[r])},{int(ov[r])})")
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
