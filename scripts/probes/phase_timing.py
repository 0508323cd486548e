#!/usr/bin/env python3
"""Diagnostics: per-phase wall time inside k_part_tile / k_apply_value / k_unpermute on the c2 stream.

  python scripts/probes/phase_timing.py --build        # here (CPU): hipcc the engine with -DCC_PHASE_TIMING
  python scripts/probes/phase_timing.py [--commits N]  # GPU box: run c2 and print the phase table

Thread 0 of every workgroup sums s_memrealtime ticks (10 ns) between phase marks (common.h PH_*); the table
shows the sum over workgroups divided by the number of workgroups (= average time per workgroup per launch).
"""
import argparse
import ctypes as C
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OUT = os.path.join(ROOT, "copycat_amd", "diag", "libcopycat_apply_phase.so")
PHASES = {
    0: ["histogram+row", "rank+wait", "wave-prefix", "exscan", "place", "write-out", "top(clear,issue)", "-"],
    1: ["W walk", "W wait", "L result store", "L rank", "L barriers", "L clear+bases", "L place", "L load issue"],
    2: ["load", "scatter", "-", "-", "-", "-", "-", "-"],
    5: ["setup", "rank+wait", "slot-scan", "gather", "walk", "event-flush", "-", "-"],
    3: ["region-load+list", "chunk-load", "binding", "lookup+orphans", "sort", "scan-apply", "cmp-runs+clear",
        "write-back"],
}


def build():
    sys.path.insert(0, ROOT)
    from copycat_amd import build as b

    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    cmd = [os.environ.get("HIPCC", "/opt/rocm/bin/hipcc"), f"--offload-arch={b.ARCH}", "-O3", "-std=c++17", "-fPIC",
           "-shared", "-DCC_PHASE_TIMING", *os.environ.get("PHASE_DEFS", "").split(), *b.ENGINE_SRCS, "-o", OUT]
    subprocess.run(cmd, cwd=b.CSRC, check=True)
    print(OUT)


def run(args):
    os.environ["CC_ENGINE_SO"] = os.environ.get("PHASE_SO", OUT)
    sys.path.insert(0, ROOT)
    import torch

    from copycat_amd import abi
    from copycat_amd.engine import DeviceBatch, Engine, lib
    from copycat_amd.workload import SEED_C2, atomic_long_stream

    if args.c5:
        return run_c5(args)
    if args.c3:
        return run_c3(args)
    n, R = args.commits, 65536
    b = atomic_long_stream(n, resources=R, seed=SEED_C2, index0=1)
    db = DeviceBatch.upload(b, device="cuda:0", columns=("index", "inst", "op", "flags", "a", "b"))
    st = torch.zeros(n, dtype=torch.uint8, device="cuda:0")
    va = torch.zeros(n, dtype=torch.int64, device="cuda:0")
    E = Engine(R, R, n, device=0, sub_batch=args.sub_batch)
    E.resource_create_range(0, R, abi.CC_RES_VALUE)
    E.instance_open_range(0, R, 0, 1, 1)
    L = lib()
    L.cc_debug_phases.restype = C.c_int
    L.cc_debug_phases.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
    ticks = (C.c_uint64 * 8)()
    E.apply(db, st, va)
    E.sync()
    for k in range(3):
        L.cc_debug_phases(E.h, k, ticks)  # clear the warmup sums
    E.profile(True)
    for _ in range(args.steps):
        E.apply(db, st, va)
    E.sync()
    prof = E.profile_read()
    sub = args.sub_batch or (16 << 20)
    launches = args.steps * ((n + sub - 1) // sub)
    tiles = (n + 16383) // 16384
    if os.environ.get("CC_V3_PHASES"):  # value_path.hip: k_part_v4 (one 1024-thread workgroup per CU, 8192-commit tiles)
        PHASES[0] = ["loads wait+gather+rank", "B1", "wave-0 scan", "B2", "place+cpos+issue next",
                     "B3", "write-out", "-"]
        tiles = (n + 8191) // 8192
    wgs = {0: tiles * args.steps, 1: 256 * launches, 2: min(tiles, 256) * launches}
    names = {0: "k_part_tile", 1: "k_apply_value", 2: "k_unpermute"}
    for k in range(3):
        rc = L.cc_debug_phases(E.h, k, ticks)
        assert rc == 0, rc
        tot = sum(ticks)
        ms, nl = prof.get(names[k], (0.0, 0))
        print(f"{names[k]}: {ms / max(nl, 1) * 1e3:.1f} us/launch, workgroups {wgs[k]}, "
              f"per-WG mean {tot * 10e-3 / wgs[k]:.2f} us")
        for q in range(8):
            if ticks[q]:
                print(f"   {PHASES[k][q]:18s} {ticks[q] * 10e-3 / wgs[k]:9.2f} us/WG  {100.0 * ticks[q] / tot:5.1f} %")


def run_c3(args):
    """The map path on bench.py's c3 stream (Zipf 0.99 over 1M (map, key) pairs in 4,096 maps)."""
    import torch

    from copycat_amd import abi
    from copycat_amd.engine import DeviceBatch, Engine, lib
    from copycat_amd.workload import map_zipf_rows

    n, R = args.commits, 4096
    hb = map_zipf_rows(0, n, maps=R, pairs=1 << 20, threads=8)
    if args.cv_rate or args.clear_rate:  # bench.py's whole-map variant
        sys.path.insert(0, ROOT)
        from bench import c3_whole_map_rows
        from copycat_amd.workload import SEED_C3

        c3_whole_map_rows(hb, 0, args.cv_rate, args.clear_rate, SEED_C3)
    db = DeviceBatch.upload(hb, device="cuda:0")
    st = torch.zeros(n, dtype=torch.uint8, device="cuda:0")
    va = torch.zeros(n, dtype=torch.int64, device="cuda:0")
    E = Engine(R, R, n, device=0, sub_batch=args.sub_batch, map_capacity=1 << 20)
    E.resource_create_range(0, R, abi.CC_RES_MAP)
    E.instance_open_range(0, R, 0, 1, 1)
    L = lib()
    L.cc_debug_phases.restype = C.c_int
    L.cc_debug_phases.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
    ticks = (C.c_uint64 * 8)()
    E.apply(db, st, va)
    E.sync()
    for k in (0, 3):
        L.cc_debug_phases(E.h, k, ticks)
    os.environ["CC_SMALL_PHASES"] = "1"
    L.cc_debug_phases(E.h, 3, ticks)
    del os.environ["CC_SMALL_PHASES"]
    E.profile(True)
    for _ in range(args.steps):
        E.apply(db, st, va)
    E.sync()
    prof = E.profile_read()
    sub = args.sub_batch or (16 << 20)
    launches = args.steps * ((n + sub - 1) // sub)
    tiles = (n + 16383) // 16384
    wgs = {0: tiles * args.steps, 3: 1024 * launches}
    names = {0: "k_part_tile", 3: "k_apply_map"}
    for k in (0, 3):
        assert L.cc_debug_phases(E.h, k, ticks) == 0
        tot = sum(ticks)
        ms, nl = prof.get(names[k], (0.0, 0))
        print(f"{names[k]}: {ms / max(nl, 1) * 1e3:.1f} us/launch, workgroups {wgs[k]}, per-WG mean {tot * 10e-3 / wgs[k]:.2f} us")
        for q in range(8):
            if ticks[q]:
                print(f"   {PHASES[k][q]:18s} {ticks[q] * 10e-3 / wgs[k]:9.2f} us/WG  {100.0 * ticks[q] / tot:5.1f} %")
    print({k: round(v[0] / args.steps, 3) for k, v in prof.items()})
    os.environ["CC_SMALL_PHASES"] = "1"
    assert L.cc_debug_phases(E.h, 3, ticks) == 0
    t = list(ticks)
    print(f"k_small_replay over {args.steps} steps: events applied {t[0]}, max per map {t[1]}, runs {t[2]}, "
          f"lane-0 time {t[3] * 10e-3:.0f} us total, max per map {t[4] * 10e-3:.0f} us, longest run {t[5]} events, "
          f"staging {t[6] * 10e-3:.0f} us total")
    print("counters", E.counters())


PHASES_PARTX = ["route+hist+ttab", "rank", "wave-prefix", "run-start scan", "place", "write-out", "top(clear,issue)", "-"]


def part_ext_report(L, E, ticks, n, steps, prof):
    """k_part_ext's phases (CC_PART_EXT_PHASES=1): one workgroup per 16384-commit tile."""
    assert L.cc_debug_phases(E.h, 0, ticks) == 0
    wgs = (n + 16383) // 16384 * steps
    tot = sum(ticks)
    ms, nl = prof.get("k_part_tile", (0.0, 0))
    print(f"k_part_ext: {ms / max(nl, 1) * 1e3:.1f} us/launch, workgroups {wgs}, per-WG mean {tot * 10e-3 / wgs:.2f} us")
    for q in range(8):
        if ticks[q]:
            print(f"   {PHASES_PARTX[q]:18s} {ticks[q] * 10e-3 / wgs:9.2f} us/WG  {100.0 * ticks[q] / tot:5.1f} %")


def run_c5(args):
    """The coordination kernel on bench.py's c5 stream (32,768 resources, a third each lock/election/group)."""
    import numpy as np
    import torch

    from copycat_amd import abi
    from copycat_amd.engine import DeviceBatch, DeviceEvents, Engine, lib
    n, R = args.commits, 32768
    kinds = {"L": abi.CC_RES_LOCK, "E": abi.CC_RES_ELECTION, "G": abi.CC_RES_GROUP}
    tl = [kinds[c] for c in args.types]
    if args.manager:
        args.interleave = True
    if args.group64:  # the allocator's layout: 64-slot groups of one type, types in turn
        types = np.repeat(np.resize(np.array(tl, np.uint8), R // 64), 64)
    elif args.interleave:
        types = np.resize(np.array(tl, np.uint8), R)
    else:
        types = np.repeat(np.array(tl, np.uint8), (R + len(tl) - 1) // len(tl))[:R]
    types_in = types.copy()
    from copycat_amd.workload import CoordClients

    clients = CoordClients(types, K=1, max_inst=R, seed=0xA700000 + 5)
    dbs = [DeviceBatch.upload(clients.next(n), device="cuda:0") for _ in range(args.steps + 1)]
    db = dbs[0]
    st = torch.zeros(n, dtype=torch.uint8, device="cuda:0")
    va = torch.zeros(n, dtype=torch.int64, device="cuda:0")
    evs = DeviceEvents(2 * n, device="cuda:0")
    # (as bench.py c5: one spare super-bucket, so no 64-slot group has to mix types)
    E = Engine(R + (256 if args.manager else 0), R, n, flags=abi.CC_CFG_TIMERS_DEFERRED, max_events=2 * n)
    if args.manager:  # as bench.py c5: cc_create_resource in turn (the allocator's 64-slot groups)
        for r in range(R):
            E.create_resource(r + 1, int(types[r]), 1, 1000 + r)
        types = np.zeros(R + 256, np.uint8)  # the slot -> type table, for the per-WG report
        for r in range(R):
            types[E.resource_slot(1000 + r)] = tl[r % len(tl)] if args.interleave else types_in[r]
    else:
        for r in range(R):
            E.resource_create(r, int(types[r]))
        E.instance_open_range(0, R, 0, 1000, 1)
    L = lib()
    ticks = (C.c_uint64 * 8)()
    E.apply_events(db, st, va, evs)
    E.sync()
    L.cc_debug_phases(E.h, 5, ticks)
    if os.environ.get("CC_PART_EXT_PHASES"):
        L.cc_debug_phases(E.h, 0, ticks)
    E.profile(True)
    for k in range(args.steps):
        E.apply_events(dbs[k + 1], st, va, evs)
    E.sync()
    prof = E.profile_read()
    L.cc_debug_phases(E.h, 5, ticks)
    sub = args.sub_batch or (16 << 20)
    launches = args.steps * ((n + sub - 1) // sub)
    wgs = ((R + (256 if args.manager else 0)) // 256) * 4 * launches
    tot = sum(ticks)
    ms, nl = prof.get("k_apply_coord", (0.0, 0))
    print(f"[{args.types}] k_apply_coord: {ms / max(nl, 1) * 1e3:.1f} us/launch, workgroups {wgs}, per-WG mean {tot * 10e-3 / wgs:.2f} us")
    for q in range(8):
        if ticks[q]:
            print(f"   {PHASES[5][q]:18s} {ticks[q] * 10e-3 / wgs:9.2f} us/WG  {100.0 * ticks[q] / tot:5.1f} %")
    print({k: round(v[0] / args.steps, 3) for k, v in prof.items()})
    if os.environ.get("CC_PART_EXT_PHASES"):
        part_ext_report(L, E, ticks, n, args.steps, prof)
    wgt = (C.c_uint64 * 16384)()
    if L.cc_debug_phases(E.h, 64, wgt) == 0:  # the last launch's workgroups: start skew and duration spread
        import numpy as np

        a = np.frombuffer(wgt, np.uint64).reshape(-1, 4)[: wgs // max(launches, 1)].astype(np.int64)
        a = a[a[:, 0] > 0]
        t0 = a[:, 0].min()
        st, en = (a[:, 0] - t0) * 10e-3, (a[:, 1] - t0) * 10e-3
        print(f"last launch, {len(a)} WGs: start skew p50 {np.percentile(st, 50):.1f} p90 {np.percentile(st, 90):.1f} "
              f"max {st.max():.1f} us; duration p50 {np.percentile(en - st, 50):.1f} p90 {np.percentile(en - st, 90):.1f} "
              f"max {(en - st).max():.1f} us; last end {en.max():.1f} us")
        dur = en - st
        order = np.argsort(-dur)[:12]
        tn = {int(abi.CC_RES_LOCK): "L", int(abi.CC_RES_ELECTION): "E", int(abi.CC_RES_GROUP): "G"}
        print("   slowest (wg, us, type, records, events):",
              [(int(b), round(float(dur[b]), 1), tn.get(int(types[(b // 4) * 256 + (b % 4) * 64]), "?"), int(a[b, 2]), int(a[b, 3]))
               for b in order])
        print(f"   records per WG: p50 {np.percentile(a[:, 2], 50):.0f} max {a[:, 2].max()}; events per WG: p50 "
              f"{np.percentile(a[:, 3], 50):.0f} max {a[:, 3].max()}")
        for k, nm in tn.items():
            sel = np.array([types[(b // 4) * 256 + (b % 4) * 64] == k for b in range(len(a))])
            if sel.any():
                print(f"   {nm}: p50 {np.percentile(dur[sel], 50):.1f} max {dur[sel].max():.1f} us over {sel.sum()} WGs")
        late = st > 50
        print(f"   WGs starting > 50 us late: {late.sum()} (their blockIdx mod 8: {np.bincount(np.nonzero(late)[0] % 8, minlength=8).tolist()})")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--c3", action="store_true")
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--commits", type=int, default=100_000_000)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--sub-batch", type=int, default=0)
    ap.add_argument("--c5", action="store_true", help="the coordination kernel on the c5 stream")
    ap.add_argument("--cv-rate", type=float, default=0.0, help="--c3: share of containsValue rows (bench.py)")
    ap.add_argument("--clear-rate", type=float, default=0.0, help="--c3: share of clear rows (bench.py)")
    ap.add_argument("--interleave", action="store_true", help="--c5: slot r holds type r %% len(types)")
    ap.add_argument("--group64", action="store_true", help="--c5: 64-slot groups of one type, types in turn")
    ap.add_argument("--manager", action="store_true", help="--c5: resources created through cc_create_resource in turn")
    ap.add_argument("--types", default="LEG", help="--c5: resource types in thirds (L lock, E election, G group)")
    a = ap.parse_args()
    build() if a.build else run(a)
