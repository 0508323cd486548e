#!/usr/bin/env python3
"""Bench: committed ops applied/s on MI355X (BASELINE.json metric), one JSON line on rank 0.

Default workload (BASELINE.json configs[1]): a DistributedAtomicLong client-model stream —
Get(50) + CompareAndSet(52) of java.lang.Long values, ~10% stale CASes — of 100M committed entries over
65,536 AtomicValueState resources per GPU.  A "step" = one cc_apply_batch over the whole 100M-entry batch
with its columns already resident in HBM (state carries over from step to step, as a replica's would).

Multi-GPU (torchrun, one process per GPU, RCCL): resources shard by id (rank r owns global ids
r, r+N, ...; weak scaling: every rank applies its own 100M-entry stream over its own 65,536 resources);
after every batch the applied-index watermark is all-gathered over RCCL — the only
cross-GPU exchange on this path.

roofline: per-kernel device time from HIP events recorded on the launch stream over the timed region
(cc_profile_*), dominant kernel, algorithmic bytes = 39 B/commit x commits per launch.
cpu_baseline: the oracle (C++ restatement of the Java apply path, single thread) timed on this host
over a bounded prefix of the same stream (rank 0, N=1 only).

--workload c3 (BASELINE.json configs[2]): DistributedMap put/get/remove 45/45/10 over 1,048,576 (map, key)
pairs in 4,096 MapState resources, pair rank ~ Zipf(0.99), 1e9 committed entries per step (generated block by
block on the host, uploaded once); algorithmic bytes 34.6 B/commit.

--workload c4 (BASELINE.json configs[3]): leader quorum commit index for 1,048,576 5-replica Raft groups plus
the session expiry sweep over 1,048,576 sessions; a step = one aggregation + one sweep; value = (groups +
sessions) / s; algorithmic bytes 64 B/group and 8.125 B/session.

--workload c5: mixed coordination -- 32,768 resources per GPU (262,144 over 8), a third each LockState,
LeaderElectionState and MembershipGroupState, one instance each; 100M committed lock/unlock (timeouts -1/0/>0),
listen/unlisten/isLeader and join/leave entries per step from the parity-test generator, applied with the
ordered event stream in HBM; algorithmic bytes 48 B/op (26 in, 9 out, ~1 event of 13 B).
"""
import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "committed ops applied/sec (1 and 8 GPUs) + % of HBM GB/s roofline"
B_OP_C2 = 39  # index 8 + res 4 + op 1 + flags 1 + expect 8 + update 8 in, status 1 + value 8 out
B_OP_C3 = 34.6  # put 30 in / get, remove 22 in; 9 out; weighted by the 45/45/10 mix
B_OP_C5 = 48  # 26 in + 9 out + ~1 event x 13 B
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def pmc_traffic(kernel, workload):
    """HBM-side bytes per launch of `kernel` from the committed rocprofv3 FETCH_SIZE/WRITE_SIZE passes of the same
    bench command (scripts/pmc_traffic.py -> profiles/traffic_latest.json; counters cannot be read in-process)."""
    p = os.path.join(ROOT, "profiles", "traffic_latest.json")
    try:
        with open(p) as f:
            d = json.load(f)
        if d.get("workload", "c2") != workload:
            return None
        return d["kernels"][kernel]["bytes_per_launch"] / 1e9
    except (OSError, KeyError, ValueError):
        return None


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def upload_c3(n, maps, pairs, zipf, rank, dev, keep_host, block=1 << 26):
    """Config-3 stream generated block by block on the host and copied into HBM-resident columns.
    Returns (host Batch of the first keep_host rows for the CPU baseline, DeviceBatch)."""
    from copycat_amd.batch import Batch
    from copycat_amd.engine import DeviceBatch
    from copycat_amd.workload import SEED_C3, map_zipf_rows

    names = ("index", "inst", "op", "flags", "key", "a", "b")
    host = Batch(min(n, block))
    dt = {"index": torch.int64, "inst": torch.int32, "op": torch.uint8, "flags": torch.uint8, "key": torch.int64,
          "a": torch.int64, "b": torch.int64}
    cols = {k: torch.empty(n, dtype=dt[k], device=dev) for k in names}
    keep = None
    threads = min(16, os.cpu_count() or 1)
    for lo in range(0, n, block):
        m = min(block, n - lo)
        part = host if m == len(host) else Batch(m)
        map_zipf_rows(lo, m, maps=maps, pairs=pairs, s=zipf, seed=SEED_C3 + rank, threads=threads, out=part)
        if lo == 0:
            keep = part.slice(0, min(keep_host, m))
        for k in names:
            src = torch.from_numpy(getattr(part, k).view(np.dtype(str(dt[k]).replace("torch.", ""))))
            cols[k][lo:lo + m].copy_(src, non_blocking=False)
    return keep, DeviceBatch(cols, n)


def run_c4(args, dev, rank, world, dist):
    """Config 4: quorum commit-index aggregation + session expiry sweep, inputs resident in HBM."""
    from copycat_amd.engine import expire_sweep, quorum_commit
    from copycat_amd.workload import expiry_sessions, quorum_groups

    G = args.commits or (1 << 20)
    S = G
    match, ts, ci = quorum_groups(G, replicas=5, seed=0xA700000 + 4 + rank)
    last, now, timeout = expiry_sessions(S, seed=0xA700000 + 5 + rank)

    def dev_u64(a):
        return torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)

    d_match, d_ts, d_ci, d_last = dev_u64(match), dev_u64(ts), dev_u64(ci), dev_u64(last)
    d_out = torch.zeros(G, dtype=torch.int64, device=dev)
    d_bm = torch.zeros((S + 63) // 64, dtype=torch.int64, device=dev)
    d_cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
           torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]

    def step(k=None):
        if k is not None:
            ev[k][0].record(stream)
        quorum_commit(d_match, d_ts, d_ci, d_out, stream=stream)
        if k is not None:
            ev[k][1].record(stream)
        d_cnt.zero_()
        expire_sweep(d_last, now, timeout, d_bm, d_cnt, stream=stream)
        if k is not None:
            ev[k][2].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(k)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    q_ms = sum(e[0].elapsed_time(e[1]) for e in ev) / args.steps
    x_ms = sum(e[1].elapsed_time(e[2]) for e in ev) / args.steps
    q_gbps = 64 * G / (q_ms * 1e-3) / 1e9
    x_gbps = 8.125 * S / (x_ms * 1e-3) / 1e9
    dom = "k_quorum" if q_ms >= x_ms else "k_expire"
    ach = q_gbps if dom == "k_quorum" else x_gbps
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle.oracle_py import expire_sweep as ox
        from oracle.oracle_py import quorum_commit as oq

        tc = time.perf_counter()
        reps = 0
        while time.perf_counter() - tc < 10 or reps == 0:
            oq(match, ts, ci)
            ox(last, now, timeout)
            reps += 1
        tc = time.perf_counter() - tc
        cpu = {"value": round(reps * (G + S) / tc, 1), "unit": "groups+sessions/s", "cores": 1, "kind": "port",
               "sample": f"{reps} x (quorum over {G:,} groups + sweep over {S:,} sessions), oracle/oracle.cpp, "
                         f"1 thread, {cpu_model()}"}
    if rank == 0:
        ms = elapsed * 1e3 / args.steps
        out = {
            "metric": METRIC, "value": round((G + S) * args.steps * world / elapsed, 1), "unit": "groups+sessions/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic",
            "config": {"workload": f"c4: quorum commit index for {G:,} 5-replica Raft groups + expiry sweep over "
                                   f"{S:,} sessions per GPU", "parallelism": f"shard{world}"},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(ach, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(ach / HBM_PEAK_GBPS, 4), "traffic": None,
                         "per_kernel_ms": {"k_quorum": round(q_ms, 5), "k_expire": round(x_ms, 5)},
                         "per_kernel_gbps": {"k_quorum": round(q_gbps, 1), "k_expire": round(x_gbps, 1)},
                         "bytes_per_unit": {"group": 64, "session": 8.125}},
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def run_c5(args, dev, rank, world, dist):
    """Mixed coordination through cc_apply_batch with the event stream."""
    from copycat_amd import abi
    from copycat_amd.engine import DeviceBatch, DeviceEvents, Engine
    from copycat_amd.workload import coord_random_stream

    n = args.commits or 100_000_000
    R = args.resources or 262_144 // 8  # 262,144 resources sharded res % 8 -> 32,768 per GPU
    third = (R + 2) // 3  # type-major slots: locks, then elections, then groups
    types = np.repeat(np.array([abi.CC_RES_LOCK, abi.CC_RES_ELECTION, abi.CC_RES_GROUP], np.uint8), third)[:R]
    t_gen = time.time()
    batch = coord_random_stream(n, types, 1, R, seed=0xA700000 + 5 + rank)
    db = DeviceBatch.upload(batch, device=dev)
    t_gen = time.time() - t_gen
    status = torch.zeros(n, dtype=torch.uint8, device=dev)
    value = torch.zeros(n, dtype=torch.int64, device=dev)
    evs = DeviceEvents(2 * n, device=dev)
    flags = abi.CC_CFG_TIMERS_DEFERRED
    E = Engine(R, R, n, device=dev.index, sub_batch=args.sub_batch, flags=flags, max_events=2 * n)
    for k, t in enumerate((abi.CC_RES_LOCK, abi.CC_RES_ELECTION, abi.CC_RES_GROUP)):
        E.resource_create_range(k * third, min(third, R - k * third), int(t))
    E.instance_open_range(0, R, 0, 1000, 1 + rank)
    stream = torch.cuda.current_stream(dev)
    wm_all = torch.zeros(world, dtype=torch.int64, device=dev)
    wm_local = db.cols["index"][n - 1:n].view(torch.int64)

    def step():
        E.apply_events(db, status, value, evs, stream=stream)
        if dist is not None:
            dist.all_gather_into_tensor(wm_all, wm_local)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if not args.no_profile:
        E.profile(True)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    E.sync()
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    prof = E.profile_read() if not args.no_profile else {}
    n_events = int(evs.count.item())
    ms_per_step = elapsed * 1e3 / args.steps
    roofline = None
    if prof:
        dom = max(prof, key=lambda k: prof[k][0])
        ms_tot, launches = prof[dom]
        commits_per_launch = n * args.steps / max(launches, 1)
        avg_ms = ms_tot / max(launches, 1)
        achieved = B_OP_C5 * commits_per_launch / (avg_ms * 1e-3) / 1e9
        roofline = {
            "bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": pmc_traffic(dom, "c5"),
            "alg_gb_per_launch": round(B_OP_C5 * commits_per_launch / 1e9, 4), "avg_launch_ms": round(avg_ms, 4),
            "launches": launches, "per_kernel_ms_per_step": {k: round(v[0] / args.steps, 4) for k, v in prof.items()},
            "bytes_per_commit": B_OP_C5,
            "pipeline_frac": round(B_OP_C5 * n / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
        }
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle.oracle_py import Oracle

        m = min(n, args.cpu_sample or 10_000_000)
        O = Oracle(R, R, flags)
        for r in range(R):
            O.resource_create(r, int(types[r]))
            O.instance_open(r, r, 1000 + r, 1)
        tc = time.perf_counter()
        O.apply(batch.slice(0, m))
        tc = time.perf_counter() - tc
        cpu = {"value": round(m / tc, 1), "unit": "ops/s", "cores": 1, "kind": "port",
               "sample": f"first {m:,} commits of the same c5 stream (events included), C++ restatement of the Java "
                         f"apply path (oracle/oracle.cpp), 1 thread, {cpu_model()}"}
    if rank == 0:
        out = {
            "metric": METRIC, "value": round(n * args.steps * world / elapsed, 1), "unit": "ops/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "int64", "data": "synthetic",
            "config": {"workload": f"c5: mixed coordination (lock / election / group, a third each) over {R:,} resources, "
                                   f"{n:,} committed entries per GPU with the ordered event stream",
                       "commits_per_step_per_gpu": n, "resources_per_gpu": R, "parallelism": f"shard{world}",
                       "events_per_step": n_events, "gen_s": round(t_gen, 2)},
            "roofline": roofline, "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=("c2", "c3", "c4", "c5"), default="c2")
    ap.add_argument("--commits", type=int, default=0, help="default: 100M (c2), 1e9 (c3)")
    ap.add_argument("--resources", type=int, default=0, help="default: 65536 resources (c2), 4096 maps (c3)")
    ap.add_argument("--pairs", type=int, default=1 << 20, help="c3: distinct (map, key) pairs")
    ap.add_argument("--zipf", type=float, default=0.99, help="c3: Zipf exponent of the pair rank (0 = uniform)")
    ap.add_argument("--sub-batch", type=int, default=0)
    ap.add_argument("--cpu-sample", type=int, default=0, help="default: 100M (c2), 20M (c3)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--retained", action="store_true", help="c2: also keep the retained value commit per slot (CC_CFG_VALUE_RETAINED)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local if world > 1 else 0)

    from copycat_amd import abi
    from copycat_amd.engine import DeviceBatch, Engine
    from copycat_amd.workload import SEED_C2, atomic_long_stream

    if args.workload == "c4":
        return run_c4(args, dev, rank, world, dist)
    if args.workload == "c5":
        return run_c5(args, dev, rank, world, dist)

    c3 = args.workload == "c3"
    n = args.commits or (1_000_000_000 if c3 else 100_000_000)
    R = args.resources or (4096 if c3 else 65536)
    cpu_sample = args.cpu_sample or (20_000_000 if c3 else 100_000_000)
    B_OP = B_OP_C3 if c3 else B_OP_C2
    t_gen = time.time()
    if c3:
        batch, db = upload_c3(n, R, args.pairs, args.zipf, rank, dev, keep_host=min(n, cpu_sample))
    else:
        batch = atomic_long_stream(n, resources=R, seed=SEED_C2 + rank, index0=1)
        db = DeviceBatch.upload(batch, device=dev, columns=("index", "inst", "op", "flags", "a", "b"))
    t_gen = time.time() - t_gen
    status = torch.zeros(n, dtype=torch.uint8, device=dev)
    value = torch.zeros(n, dtype=torch.int64, device=dev)

    if c3:
        E = Engine(R, R, n, device=dev.index, sub_batch=args.sub_batch, map_capacity=args.pairs)
        E.resource_create_range(0, R, abi.CC_RES_MAP)
    else:
        E = Engine(R, R, n, device=dev.index, sub_batch=args.sub_batch,
                   flags=abi.CC_CFG_TIMERS_DEFERRED | (abi.CC_CFG_VALUE_RETAINED if args.retained else 0))
        E.resource_create_range(0, R, abi.CC_RES_VALUE)
    E.instance_open_range(0, R, 0, 1 + rank, 1 + rank)
    stream = torch.cuda.current_stream(dev)
    wm_all = torch.zeros(world, dtype=torch.int64, device=dev)
    wm_local = db.cols["index"][n - 1:n].view(torch.int64)

    def step():
        E.apply(db, status, value, stream=stream)
        if dist is not None:  # applied-index watermark exchange (RCCL all-gather over xGMI)
            dist.all_gather_into_tensor(wm_all, wm_local)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if not args.no_profile:
        E.profile(True)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    E.sync()  # surfaces device-side errors
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    prof = E.profile_read() if not args.no_profile else {}
    # sanity: the result columns are the real per-commit results (spot-check CAS success share on rank 0)
    st_h = status[: min(n, 1_000_000)].cpu().numpy()
    ok_share = float(np.mean(abi.status_code(st_h) == abi.CC_ST_OK))

    total_commits = n * args.steps * world
    value_ops = total_commits / elapsed
    ms_per_step = elapsed * 1e3 / args.steps

    roofline = None
    if prof:
        dom = max(prof, key=lambda k: prof[k][0])
        ms_tot, launches = prof[dom]
        commits_per_launch = n * args.steps / max(launches, 1)
        avg_ms = ms_tot / max(launches, 1)
        achieved = B_OP * commits_per_launch / (avg_ms * 1e-3) / 1e9
        roofline = {
            "bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": pmc_traffic(dom, args.workload),
            "traffic_unit": "GB per launch (2 x FETCH_SIZE + WRITE_SIZE, profiles/traffic_latest.json)",
            "alg_gb_per_launch": round(B_OP * commits_per_launch / 1e9, 4),
            "avg_launch_ms": round(avg_ms, 4), "launches": launches,
            "per_kernel_ms_per_step": {k: round(v[0] / args.steps, 4) for k, v in prof.items()},
            "bytes_per_commit": B_OP,
            "pipeline_achieved_gbps": round(B_OP * n / (ms_per_step * 1e-3) / 1e9, 1),
            "pipeline_frac": round(B_OP * n / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
        }

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle.oracle_py import Oracle

        m = min(n, cpu_sample)
        sample = batch.slice(0, m)
        O = Oracle(R, R)
        for r in range(R):
            O.resource_create(r, abi.CC_RES_MAP if c3 else abi.CC_RES_VALUE)
            O.instance_open(r, r, 1 + r, 1)
        tc = time.perf_counter()
        O.apply(sample)
        tc = time.perf_counter() - tc
        cpu = {"value": round(m / tc, 1), "unit": "ops/s", "cores": 1, "kind": "port",
               "sample": f"first {m:,} commits of the same {args.workload} stream, C++ restatement of the Java apply "
                         f"path (oracle/oracle.cpp), 1 thread, {cpu_model()}"}

    if c3:
        wl = (f"c3: DistributedMap put/get/remove 45/45/10, Zipf({args.zipf}) over {args.pairs:,} (map, key) pairs in "
              f"{R:,} MapState resources, {n:,} committed entries per GPU")
    else:
        wl = ("c2: DistributedAtomicLong Get/CompareAndSet client-model stream, "
              f"{n:,} committed entries over {R:,} AtomicValueState resources per GPU")
    if rank == 0:
        out = {
            "metric": METRIC, "value": round(value_ops, 1), "unit": "ops/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "int64", "data": "synthetic",
            "config": {"workload": wl,
                       "commits_per_step_per_gpu": n, "resources_per_gpu": R, "parallelism": f"shard{world}",
                       "sub_batch": args.sub_batch or "default(16M)", "ok_status_share": round(ok_share, 4),
                       "gen_s": round(t_gen, 2)},
            "roofline": roofline, "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
