#!/usr/bin/env python3
"""Bench: committed ops applied/s on MI355X (BASELINE.json metric), one JSON line on rank 0.

Default workload (BASELINE.json configs[1]): a DistributedAtomicLong client-model stream —
Get(50) + CompareAndSet(52) of java.lang.Long values, ~10% stale CASes — of 100M committed entries over
65,536 AtomicValueState resources per GPU.  A "step" = one cc_apply_batch over one 100M-entry batch with its
columns already resident in HBM.  Every step applies its OWN batch: the client model continues from the values the
previous steps left (copycat_amd.workload.AtomicLongClients), so every timed step holds the stated ~10% stale CASes
(the per-step CAS success share is reported), and the results of every step stay in HBM.

Parity at full size: the oracle applies step 0's 100M rows on the host (this is also the timed CPU baseline); the
GPU's step-0 status/value columns and its value state after step 0 must match bit for bit ("parity" in the JSON
line; any mismatch exits non-zero).

Multi-GPU (`--gpus N`): without WORLD_SIZE in the environment bench.py starts N ranks itself
(torch.distributed.run, one process per GPU, RCCL) before touching any GPU.  Rank r applies its share of ONE global
log: the global resources r, r+N, ... (weak scaling: 100M rows over 65,536 resources per rank per step), rows
carrying the global log indices (copycat_amd.workload.AtomicLongClients, copycat_amd.shard).  After every batch each
rank writes its applied watermark into HBM (cc_applied_index_async) and the watermarks are all-gathered over RCCL
(SURVEY §8(e)); c4/c5 also all-gather (OR) the session-expiry bitmap.  Nothing else crosses GPUs.

roofline: the WHOLE step -- SURVEY §8(d)'s algorithmic bytes per commit (c2 39, c3 34.6, c5 48; c4 64 per group +
8.125 per session) x the commits of one step / the step time, against 8 TB/s; `traffic` = the measured HBM bytes of
the same step from the committed rocprofv3 FETCH_SIZE / WRITE_SIZE passes (profiles/traffic_latest.json).  Sub-fields:
the dominant kernel's own figure (HIP events recorded on the launch stream around every launch of the timed region,
cc_profile_*) and every profiled kernel's time per step.
cpu_baseline: the oracle (C++ restatement of the Java apply path, single thread, as the reference's single
state-machine thread) over step 0's rows (rank 0, N=1 only); cpu_baseline_all_cores: the same rows sharded by
resource over the box's CPU share, one oracle per thread.

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
import socket
import subprocess
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
RESULT_SENTINEL = 0xFF  # result prefill: status 0xFF (tag nibble 15) is never a legal status (copycat_amd.engine)


# the kernels each profiling marker spans (their HBM traffic adds up); the first present partition kernel is the one
# (value-only engines: k_part_v4; engines with maps, coordination or value events: k_part_ext)
MARKER_KERNELS = {"k_part_tile": ("k_part_v4", "k_part_ext"),
                  "k_unpermute": ("k_unpermute_v3", "k_unpermute"),
                  "k_apply_value": ("k_apply_value_v3", "k_apply_value_ws"),
                  "k_events": ("k_ev_count", "k_ev_tiles", "k_ev_chist", "k_ev_cscan", "k_ev_place", "k_ev_tile_out",
                               "k_ev_rows", "k_ev_perm", "k_ev_out"),
                  "k_map_hot": ("k_hot_detect", "k_hot_agg", "k_hot_lists", "k_hot_apply")}
MARKER_SUM = {"k_events", "k_map_hot"}
# the rocprofv3 kernel name(s) behind a profiling marker, per workload (the marker names are the engine's
# profile slots; the partition slot runs k_part_v4 on value-only engines and k_part_ext otherwise)
TRACE_NAMES = {"k_part_tile": {"c2": "k_part_v4<4, 8>", "c3": "k_part_ext", "c5": "k_part_ext"},
               "k_apply_value": {"c2": "k_apply_value_v3<256>"}, "k_apply_map": {"c3": "k_apply_map<false>"},
               "k_unpermute": {"c2": "k_unpermute_v3<512, 8192>", "c3": "k_unpermute<1024, 16384>", "c5": "k_unpermute<1024, 16384>"},
               "k_map_hot": {"c3": "k_hot_detect + k_hot_lists + k_hot_agg + k_hot_apply"},
               "k_events": {"c5": "k_ev_count + k_ev_tiles + k_ev_chist + k_ev_cscan + k_ev_place + k_ev_tile_out"}}


WINDOW_MARKERS = False  # --window-markers


def window_marker():
    """The timed window in a rocprofv3 kernel trace (--window-markers): one tiny `spin_kernel` (torch.cuda._sleep)
    launched right before a timed region's first step and right after its closing synchronize; scripts/gpu_prof.sh
    charges to the timed steps exactly the kernels that start between the two (no set-up launch is counted)."""
    if WINDOW_MARKERS:
        torch.cuda._sleep(1)


def trace_name(marker, workload):
    return TRACE_NAMES.get(marker, {}).get(workload, marker)


def pmc_traffic(kernel, workload):
    """HBM-side bytes per launch of `kernel` from the committed rocprofv3 FETCH_SIZE/WRITE_SIZE passes of the same
    bench command (scripts/pmc_traffic.py -> profiles/traffic_latest.json; counters cannot be read in-process)."""
    p = os.path.join(ROOT, "profiles", "traffic_latest.json")
    try:
        with open(p) as f:
            d = json.load(f)
        if "workloads" in d:
            if workload not in d["workloads"]:
                return None
            ks = d["workloads"][workload]["kernels"]
        else:
            if d.get("workload", "c2") != workload:
                return None
            ks = d["kernels"]
        names = [n for n in MARKER_KERNELS.get(kernel, (kernel,)) if n in ks]
        if not names:
            return None
        if kernel in MARKER_SUM:
            return round(sum(ks[n]["bytes_per_launch"] for n in names) / 1e9, 4)
        return round(ks[names[0]]["bytes_per_launch"] / 1e9, 4)
    except (OSError, KeyError, ValueError):
        return None


def pmc_step_traffic(workload):
    """Measured HBM-side bytes per commit of the WHOLE step: every engine kernel's (2 x FETCH_SIZE + WRITE_SIZE) per
    launch x its launches, over the commits the profiled bench command applied (scripts/pmc_traffic.py with the
    command's commit count -> profiles/traffic_latest.json "bytes_per_commit_total")."""
    p = os.path.join(ROOT, "profiles", "traffic_latest.json")
    try:
        with open(p) as f:
            return json.load(f)["workloads"][workload]["bytes_per_commit_total"]
    except (OSError, KeyError, ValueError, TypeError):
        return None


def roofline_step(prof, workload, n, steps, ms_per_step, b_op, extra=None):
    """The roofline of the whole step (round-4 verdict: `frac` is the step's, not one kernel's): SURVEY §8(d)'s
    algorithmic bytes per commit x the commits of one step / the step time, against the 8 TB/s HBM peak.  `traffic`
    is the measured HBM bytes of the same step from the committed PMC passes (null without them).  The dominant
    kernel's own figure (HIP events around every launch of the timed region, on the launch stream) and every profiled
    kernel's time per step are kept as sub-fields."""
    achieved = b_op * n / (ms_per_step * 1e-3) / 1e9
    tr = pmc_step_traffic(workload)
    out = {"bound": "hbm", "scope": "whole step (every kernel and launch gap of cc_apply_batch over one step's batch)",
           "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
           "traffic": round(tr * n / 1e9, 3) if tr else None,
           "traffic_unit": "GB per step (HBM-side, 2 x FETCH_SIZE + WRITE_SIZE summed over every kernel, "
                           "profiles/traffic_latest.json)",
           "traffic_bytes_per_commit": round(tr, 1) if tr else None, "alg_bytes_per_commit": b_op,
           "alg_gb_per_step": round(b_op * n / 1e9, 4)}
    if prof:
        dom = max(prof, key=lambda k: prof[k][0])
        ms_tot, launches = prof[dom]
        commits_per_launch = n * steps / max(launches, 1)
        avg_ms = ms_tot / max(launches, 1)
        k_ach = b_op * commits_per_launch / (avg_ms * 1e-3) / 1e9
        out["dominant_kernel"] = {
            "kernel": dom, "trace_name": trace_name(dom, workload), "avg_launch_ms": round(avg_ms, 4),
            "launches": launches, "commits_per_launch": round(commits_per_launch),
            "achieved": round(k_ach, 1), "frac": round(k_ach / HBM_PEAK_GBPS, 4),
            "traffic": pmc_traffic(dom, workload), "traffic_unit": "GB per launch",
            "note": "all of the step's algorithmic bytes charged to this kernel's launch time (an upper bound on its "
                    "own fraction; the whole-step figure above is the honest one)"}
        out["per_kernel_ms_per_step"] = {k: round(v[0] / steps, 4) for k, v in prof.items()}
    if extra:
        out.update(extra)
    return out


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def c3_whole_map_rows(part, lo, cv_rate, clear_rate, seed, null_rate=0.0, delete_rate=0.0):
    """The whole-map variant of c3: in a generated block, a share cv_rate of the rows become
    MapState.containsValue rows whose operand is the value a put of the block stored a little earlier (same map: the
    row takes that put's instance; many answers are true), and a share clear_rate become MapState.clear rows.  The
    barrier variant adds null-valued puts (null_rate of the rows: a containsValue row on a map that
    may hold a null is a barrier, answered in HashMap order, MapState.java:49-60) and ResourceStateMachine.Delete rows
    (delete_rate: MapState.delete :264-274, a barrier).  Deterministic per (seed, block start): the parity gate
    regenerates the same rows."""
    from copycat_amd import abi

    if not cv_rate and not clear_rate and not null_rate and not delete_rate:
        return
    rng = np.random.default_rng([seed, lo])
    n = len(part)
    if null_rate:  # puts that store a null (value tag NULL)
        nr = np.nonzero(rng.random(n) < null_rate)[0]
        nr = nr[part.op[nr] == abi.CC_OP_MAP_PUT]
        part.flags[nr] = part.flags[nr] & np.uint8(0xF8)
    if cv_rate:
        rows = np.nonzero(rng.random(n) < cv_rate)[0]
        puts = np.nonzero(part.op == abi.CC_OP_MAP_PUT)[0]
        back = np.searchsorted(puts, rows) - 1 - rng.integers(0, 64, len(rows))
        rows = rows[back >= 0]
        src = puts[back[back >= 0]]
        inst, a, tag = part.inst[src].copy(), part.a[src].copy(), (part.flags[src] & np.uint8(7)).copy()
        part.op[rows] = abi.CC_OP_MAP_CONTAINSVALUE
        part.inst[rows] = inst
        part.a[rows] = a
        part.flags[rows] = tag
    if clear_rate:
        cl = np.nonzero(rng.random(n) < clear_rate)[0]
        cl = cl[part.op[cl] != abi.CC_OP_MAP_CONTAINSVALUE]
        part.op[cl] = abi.CC_OP_MAP_CLEAR
    if delete_rate:
        dl = np.nonzero(rng.random(n) < delete_rate)[0]
        dl = dl[part.op[dl] != abi.CC_OP_MAP_CONTAINSVALUE]
        part.op[dl] = abi.CC_OP_DELETE


def upload_c3(n, maps, pairs, zipf, rank, dev, keep_host, block=1 << 26, cv_rate=0.0, clear_rate=0.0, null_rate=0.0,
              delete_rate=0.0):
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
        c3_whole_map_rows(part, lo, cv_rate, clear_rate, SEED_C3 + rank, null_rate, delete_rate)
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
    # resident input sets used in turn, so each step reads inputs the previous steps have pushed out of the 256 MiB
    # Infinity Cache (one set is 72 MB at 1M groups + 1M sessions: re-read every step it would be served on-die)
    nsets = max(1, args.c4_sets)

    def dev_u64(a):
        return torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)

    sets = []
    for j in range(nsets):
        match, ts, ci = quorum_groups(G, replicas=5, seed=0xA700000 + 4 + rank + 1000 * j)
        last, now, timeout = expiry_sessions(S, seed=0xA700000 + 5 + rank + 1000 * j)
        sets.append((dev_u64(match), dev_u64(ts), dev_u64(ci), dev_u64(last)))
    match, ts, ci = quorum_groups(G, replicas=5, seed=0xA700000 + 4 + rank)  # set 0 on the host: the CPU baseline
    last, now, timeout = expiry_sessions(S, seed=0xA700000 + 5 + rank)
    d_out = torch.zeros(G, dtype=torch.int64, device=dev)
    d_bm = torch.zeros((S + 63) // 64, dtype=torch.int64, device=dev)
    # rank r sweeps the global sessions [r*S, (r+1)*S): the all-gather concatenates the global expired bitmap
    bm_all = torch.zeros(world * d_bm.numel(), dtype=torch.int64, device=dev)
    d_cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
           torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]

    calls = [0]

    def step(k=None):
        d_match, d_ts, d_ci, d_last = sets[calls[0] % nsets]
        calls[0] += 1
        if k is not None:
            ev[k][0].record(stream)
        quorum_commit(d_match, d_ts, d_ci, d_out, stream=stream)
        if k is not None:
            ev[k][1].record(stream)
        d_cnt.zero_()
        expire_sweep(d_last, now, timeout, d_bm, d_cnt, stream=stream)
        if k is not None:
            ev[k][2].record(stream)
        if dist is not None:  # the expired-session bitmap exchange (RCCL all-gather over xGMI)
            dist.all_gather_into_tensor(bm_all, d_bm)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    parity = None
    if not args.no_parity:  # set 0 through both kernels (untimed) against the oracle: every group and every bit
        from oracle.oracle_py import expire_sweep as ox
        from oracle.oracle_py import quorum_commit as oq

        d_match, d_ts, d_ci, d_last = sets[0]
        d_out.fill_(-1)
        d_bm.fill_(-1)
        d_cnt.zero_()
        quorum_commit(d_match, d_ts, d_ci, d_out, stream=stream)
        expire_sweep(d_last, now, timeout, d_bm, d_cnt, stream=stream)
        torch.cuda.synchronize(dev)
        q_ref = oq(match, ts, ci)
        b_ref, c_ref = ox(last, now, timeout)
        q_gpu = d_out.cpu().numpy().view(np.uint64)
        b_gpu = d_bm.cpu().numpy().view(np.uint64)
        parity = {"groups": G, "group_mismatches": int(np.count_nonzero(q_gpu != q_ref)), "sessions": S,
                  "bitmap_word_mismatches": int(np.count_nonzero(b_gpu != b_ref)),
                  "expired": int(d_cnt.item()), "expired_ref": c_ref,
                  "checked": "input set 0: new commit index of every group (output prefilled with -1) and every word of "
                             "the expired-session bitmap (prefilled with all ones), GPU vs oracle/oracle.cpp"}
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    window_marker()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(k)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    window_marker()
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # Per-kernel launch durations: each kernel alone, back to back over the resident input sets, between one event
    # pair (an event pair around every ~15 us launch adds its own few us).  k_quorum moves 88% of the algorithmic
    # bytes (64 B/group vs 8.125 B/session): it is the roofline kernel; k_expire is launch-latency bound (8.5 MB).
    reps = 64
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    e0.record(stream)
    for k in range(reps):
        d_match, d_ts, d_ci, d_last = sets[k % nsets]
        quorum_commit(d_match, d_ts, d_ci, d_out, stream=stream)
    e1.record(stream)
    for k in range(reps):
        d_match, d_ts, d_ci, d_last = sets[k % nsets]
        expire_sweep(d_last, now, timeout, d_bm, d_cnt, stream=stream)
    e2.record(stream)
    torch.cuda.synchronize(dev)
    q_ms, x_ms = e0.elapsed_time(e1) / reps, e1.elapsed_time(e2) / reps
    step_q_ms = sum(e[0].elapsed_time(e[1]) for e in ev) / args.steps
    step_x_ms = sum(e[1].elapsed_time(e[2]) for e in ev) / args.steps
    q_gbps = 64 * G / (q_ms * 1e-3) / 1e9
    x_gbps = 8.125 * S / (x_ms * 1e-3) / 1e9
    dom = "k_quorum"
    ach = q_gbps
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
        step_gbps = (64 * G + 8.125 * S) / (ms * 1e-3) / 1e9
        qt, xt = pmc_traffic("k_quorum", "c4"), pmc_traffic("k_expire", "c4")
        c4_traffic = round(qt + xt, 4) if qt is not None and xt is not None else None
        out = {
            "metric": METRIC, "value": round((G + S) * args.steps * world / elapsed, 1), "unit": "groups+sessions/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic",
            "config": {"workload": f"c4: quorum commit index for {G:,} 5-replica Raft groups + expiry sweep over "
                                   f"{S:,} sessions per GPU", "parallelism": f"shard{world}",
                       "input_sets": nsets, "input_set_mb": round((64 + 8) * G / 1e6, 1),
                       "note": "steps take the resident input sets in turn; with >= 4 sets a step's inputs are not in "
                               "the 256 MiB Infinity Cache"},
            "roofline": {"bound": "hbm", "scope": "whole step (one quorum aggregation + one expiry sweep + the RCCL "
                                                   "exchanges)",
                         "achieved": round(step_gbps, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(step_gbps / HBM_PEAK_GBPS, 4),
                         "traffic": c4_traffic, "traffic_unit": "GB per step (k_quorum + k_expire, 2 x FETCH_SIZE + "
                                                                "WRITE_SIZE, profiles/traffic_latest.json)",
                         "alg_gb_per_step": round((64 * G + 8.125 * S) / 1e9, 4),
                         "bytes_per_unit": {"group": 64, "session": 8.125},
                         "dominant_kernel": {"kernel": dom, "trace_name": "k_quorum<5>", "achieved": round(ach, 1),
                                             "frac": round(ach / HBM_PEAK_GBPS, 4), "avg_launch_ms": round(q_ms, 5),
                                             "traffic": pmc_traffic("k_quorum", "c4"), "traffic_unit": "GB per launch",
                                             "alg_gb_per_launch": round(64 * G / 1e9, 4)},
                         "timing": f"{reps} back-to-back launches of each kernel over the resident input sets, one event pair",
                         "per_kernel_ms": {"k_quorum": round(q_ms, 5), "k_expire": round(x_ms, 5)},
                         "per_step_event_ms": {"k_quorum": round(step_q_ms, 5), "k_expire": round(step_x_ms, 5)},
                         "per_kernel_gbps": {"k_quorum": round(q_gbps, 1), "k_expire": round(x_gbps, 1)}},
            "parity": parity, "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    if parity is not None and (parity["group_mismatches"] or parity["bitmap_word_mismatches"]
                               or parity["expired"] != parity["expired_ref"]):
        sys.stderr.write(f"PARITY FAILURE: {parity}\n")
        sys.exit(3)


def per_target(ev, keys=("pos", "target", "code", "tag", "payload", "src")):
    """The event stream regrouped by target session, each target's events in stream (emission) order: the order a
    client session observes (SURVEY A12 -- only per-target order is defined across sessions)."""
    order = np.argsort(np.asarray(ev["target"]), kind="stable")
    return {k: np.asarray(ev[k])[order] for k in keys}


def run_c5(args, dev, rank, world, dist):
    """Mixed coordination through cc_apply_batch with the event stream; a new batch every step (the
    lock client model continues, copycat_amd.workload.CoordClients); step 0 checked against the oracle in full."""
    from copycat_amd import abi
    from copycat_amd.batch import Batch
    from copycat_amd.engine import DeviceBatch, DeviceEvents, Engine
    from copycat_amd.workload import CoordClients

    n = args.commits or 100_000_000
    R = args.resources or 262_144 // 8  # 262,144 resources sharded res % 8 -> 32,768 per GPU
    kinds = np.array([abi.CC_RES_LOCK, abi.CC_RES_ELECTION, abi.CC_RES_GROUP], np.uint8)
    if args.c5_layout == "grouped":  # slot ranges by type: locks, then elections, then groups
        types = np.repeat(kinds, (R + 2) // 3)[:R]
    else:  # resources created in turn (a lock, an election, a group, ...): instance r's resource has type r % 3
        types = np.resize(kinds, R)
    total_steps = args.warmup + args.steps
    nstreams = max(1, min(total_steps, int(args.hbm_budget_gb * 1e9 // (n * 54))))
    flags = abi.CC_CFG_TIMERS_DEFERRED
    t_gen = time.time()
    # Session expiry: S_glob client sessions; rank r holds the keep-alives of sessions
    # [r*S_local, (r+1)*S_local) and sweeps them; the all-gathered (OR-merged) bitmap is the global expired set, and
    # every rank closes the instances IT hosts of every expired session (cc_sessions_expire, ResourceManager.expire
    # :237-247).  Besides the R client instances (owned by the live sessions 1..world), every rank hosts V more
    # instances that no commit addresses, owned by sessions spread over the whole id range: their sessions expire
    # on whichever rank sweeps them, and only the merged bitmap closes them where they live.
    S_local = max(64, (65536 // world) // 64 * 64)
    S_glob = S_local * world
    now_s, timeout_s = 10_000_000, 5000
    last_glob = np.concatenate([now_s - np.random.default_rng(0xA700000 + 55 + r).integers(0, 2 * timeout_s, S_local)
                                for r in range(world)]).astype(np.int64)
    last_glob[:64] = now_s  # the sessions that own the client instances stay alive
    V = 1024
    victim_res = (np.arange(V, dtype=np.int64) * (R // V)) % R
    victim_sess = (np.arange(V, dtype=np.int64) * 2654435761 + rank * 40503) % (S_glob - 64) + 64
    expired_glob = (now_s - last_glob) > timeout_s
    victims_expiring = int(expired_glob[victim_sess].sum())
    clients = CoordClients(types, K=1, max_inst=R + V, seed=0xA700000 + 5 + rank)
    host = Batch(n)
    streams, parity_ref, cpu, cpu_all = [], None, None, None
    for k in range(nstreams):
        clients.next(n, out=host)
        if k == 0 and rank == 0 and not args.no_parity:
            from oracle.oracle_py import Oracle

            O = Oracle(R, R + V, flags)
            for r in range(R):
                O.resource_create(r, int(types[r]))
                O.instance_open(r, r, 1000 + r, 1 + rank)
            for j in range(V):
                O.instance_open(R + j, int(victim_res[j]), 10_000_000 + j, int(victim_sess[j]))
            tc = time.perf_counter()
            s_ref, v_ref = O.apply(host)
            tc = time.perf_counter() - tc
            oe = O.take_events()
            apos, amem = O.take_aux()
            parity_ref = (s_ref, v_ref, per_target(oe), (apos, amem))
            if world == 1 and not args.no_cpu_baseline:
                cpu = {"value": round(n / tc, 1), "unit": "ops/s", "cores": 1, "kind": "port",
                       "sample": f"step 0's {n:,} commits of the same c5 stream (events included; the parity reference), "
                                 f"C++ restatement of the Java apply path (oracle/oracle.cpp), 1 thread, {cpu_model()}"}
            del O, oe
            if world == 1 and not args.no_cpu_baseline:
                v_all, thr = cpu_all_cores(host, R, types, cpu_threads(), flags)
                cpu_all = {"value": round(v_all, 1), "unit": "ops/s", "cores": thr, "kind": "port",
                           "sample": f"the same {n:,} commits (events included) sharded by resource (slot % {thr}) over "
                                     f"{thr} threads, one oracle each, {cpu_model()}"}
        streams.append(DeviceBatch.upload(host, device=dev))
    del host
    t_gen = time.time() - t_gen
    status = torch.full((n,), RESULT_SENTINEL, dtype=torch.uint8, device=dev)  # sentinel: unwritten rows show
    value = torch.full((n,), -1, dtype=torch.int64, device=dev)
    evs = DeviceEvents(2 * n, device=dev)
    # slot capacity with one spare super-bucket: each type's last 64-slot group is partly filled (32,768 / 3 is no
    # multiple of 64), and without spare groups the allocator would have to mix types in a group (a divergent walk)
    E = Engine(R + 256, R + V, n, device=dev.index, sub_batch=args.sub_batch, flags=flags, max_events=2 * n)
    if args.c5_layout == "manager":  # through the product's ResourceManager (cc_create_resource): the allocator
        for r in range(R):           # places each type in 64-slot groups of its own; instance r = the r-th create
            st, iid, islot = E.create_resource(r + 1, int(types[r]), 1 + rank, 1000 + r)
            assert abi.status_code(st) == abi.CC_ST_OK and iid == 1000 + r and islot == r, (st, iid, islot)
    else:  # raw slots: resource r in slot r
        for r in range(R):
            E.resource_create(r, int(types[r]))
        E.instance_open_range(0, R, 0, 1000, 1 + rank)
    for j in range(V):  # (manager layout: resource r has id = its CreateResource commit's index 1000 + r)
        rslot = E.resource_slot(1000 + int(victim_res[j])) if args.c5_layout == "manager" else int(victim_res[j])
        assert rslot >= 0
        E.instance_open(R + j, rslot, 10_000_000 + j, int(victim_sess[j]))
    stream = torch.cuda.current_stream(dev)
    wm_all = torch.zeros(world, dtype=torch.int64, device=dev)
    wm_local = torch.zeros(1, dtype=torch.int64, device=dev)
    from copycat_amd.engine import expire_sweep

    d_last = torch.from_numpy(np.ascontiguousarray(last_glob[rank * S_local:(rank + 1) * S_local])).to(dev)
    d_bm = torch.zeros(S_local // 64, dtype=torch.int64, device=dev)
    d_cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    bm_all = torch.zeros(world * (S_local // 64), dtype=torch.int64, device=dev)
    close_evs = DeviceEvents(1 << 16, device=dev)
    closed_total = [0]

    def step(k):
        E.apply_events(streams[k % nstreams], status, value, evs, stream=stream)
        E.applied_index_async(wm_local, stream=stream)
        expire_sweep(d_last, now_s, timeout_s, d_bm, d_cnt, stream=stream)
        if dist is not None:  # watermark, then expired-session bitmap (RCCL all-gathers over xGMI)
            dist.all_gather_into_tensor(wm_all, wm_local)
            dist.all_gather_into_tensor(bm_all, d_bm)
        # the expired sessions' instances on this rank leave (synchronous control plane, like the reference's expire)
        closed, _ = E.sessions_expire(bm_all if dist is not None else d_bm, S_glob, events=close_evs)
        closed_total[0] += closed

    parity = None
    for k in range(args.warmup):
        step(k)
        if k == 0 and parity_ref is not None:
            E.sync()
            parity = c5_parity(parity_ref, status, value, evs, abi)
    torch.cuda.synchronize(dev)
    if not args.no_profile:
        E.profile(True)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    window_marker()
    t0 = time.perf_counter()
    for k in range(args.warmup, total_steps):
        step(k)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    window_marker()
    E.sync()
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if parity is None and parity_ref is not None and args.warmup == 0 and nstreams >= total_steps and total_steps == 1:
        parity = c5_parity(parity_ref, status, value, evs, abi)
    prof = E.profile_read() if not args.no_profile else {}
    n_events = int(evs.count.item())
    ms_per_step = elapsed * 1e3 / args.steps
    roofline = roofline_step(prof, "c5", n, args.steps, ms_per_step, B_OP_C5)
    if rank == 0:
        out = {
            "metric": METRIC, "value": round(n * args.steps * world / elapsed, 1), "unit": "ops/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "int64", "data": "synthetic",
            "config": {"workload": f"c5: mixed coordination (lock / election / group, a third each, {args.c5_layout} slots) over {R:,} resources, "
                                   f"{n:,} committed entries per GPU per step with the ordered event stream, a new "
                                   f"client-model batch every step",
                       "commits_per_step_per_gpu": n, "resources_per_gpu": R, "parallelism": f"shard{world}",
                       "resident_streams": nstreams, "events_last_step": n_events, "gen_s": round(t_gen, 2),
                       "watermarks": wm_all.cpu().tolist() if dist is not None else [int(wm_local.item())],
                       "expired_sessions_per_step": int(np.unpackbits(
                           (bm_all if dist is not None else d_bm).cpu().numpy().view(np.uint8)).sum()),
                       "expiry": {"sessions": S_glob, "expired": int(expired_glob.sum()), "instances_closed": closed_total[0],
                                  "instances_expected": victims_expiring,
                                  "path": "per-rank cc_expire_sweep -> RCCL all-gather of the bitmaps -> "
                                          "cc_sessions_expire on every rank, every step"}},
            "parity": parity, "roofline": roofline, "cpu_baseline": cpu, "cpu_baseline_all_cores": cpu_all,
        }
        print(json.dumps(out), flush=True)
    bad = parity is not None and (parity["mismatches"] or parity["unwritten"] or not parity["events_equal"])
    if closed_total[0] != victims_expiring:
        sys.stderr.write(f"EXPIRY FAILURE: closed {closed_total[0]} instances, expected {victims_expiring}\n")
        bad = True
    if dist is not None:
        dist.destroy_process_group()
    if bad:
        sys.stderr.write(f"PARITY FAILURE: {parity}\n")
        sys.exit(3)


def c5_parity(ref, status, value, evs, abi):
    s_ref, v_ref, ev_ref, (apos, amem) = ref
    s = status.cpu().numpy()
    v = value.cpu().numpy().view(np.uint64)
    ev = evs.host()
    member = ev["code"] == abi.CC_EV_MEMBER
    got = per_target({k: ev[k][~member] for k in ("pos", "target", "code", "tag", "payload", "src")})
    n_ev = len(got["pos"])
    same_len = n_ev == len(ev_ref["pos"])
    ev_bad = 0 if same_len else -1
    if same_len:
        d = np.zeros(n_ev, bool)
        for k in got:
            d |= got[k] != ev_ref[k]
        ev_bad = int(np.count_nonzero(d))
    mem_ok = np.array_equal(ev["pos"][member], apos) and np.array_equal(ev["payload"][member], amem)
    return {"rows": len(s), "mismatches": int(np.count_nonzero((s != s_ref) | (v != v_ref))),
            "unwritten": int(np.count_nonzero(s == RESULT_SENTINEL)),
            "events": n_ev, "events_ref": len(ev_ref["pos"]), "event_mismatches": ev_bad,
            "events_equal": bool(same_len and ev_bad == 0 and mem_ok),
            "checked": "step 0: per-commit status+value (results prefilled with the 0xFF sentinel status); every event "
                       "per target session in emission order (row, target, code, tag, payload, src; SURVEY A12); "
                       "join member sets in stream order; GPU vs oracle/oracle.cpp"}


def cpu_threads():
    """The box's CPU share for host work (the GPU box exposes far more CPUs than one GPU's share of 16)."""
    return max(1, min(16, os.cpu_count() or 1))


def cpu_all_cores(batch, R, rtype, threads, flags=None):
    """The same rows sharded by resource over `threads` threads, one oracle (C++ restatement) per thread; ctypes
    releases the GIL inside each apply.  Returns (ops/s, threads)."""
    from concurrent.futures import ThreadPoolExecutor

    from copycat_amd import abi
    from oracle.oracle_py import Oracle

    own = (batch.inst % threads).astype(np.uint8)
    order = np.argsort(own, kind="stable")
    cuts = np.searchsorted(own[order], np.arange(threads + 1))
    parts = []
    for t in range(threads):
        rows = order[cuts[t]:cuts[t + 1]]
        sub = type(batch)(0)
        for name in type(batch).__slots__:
            setattr(sub, name, np.ascontiguousarray(getattr(batch, name)[rows]))
        parts.append(sub)
    oracles = []
    for t in range(threads):
        O = Oracle(R, R) if flags is None else Oracle(R, R, flags)
        for r in range(t, R, threads):
            O.resource_create(r, int(rtype[r]) if hasattr(rtype, "__len__") else rtype)
            O.instance_open(r, r, 1000 + r, 1)
        oracles.append(O)
    with ThreadPoolExecutor(threads) as ex:
        tc = time.perf_counter()
        list(ex.map(lambda t: oracles[t].apply(parts[t]), range(threads)))
        tc = time.perf_counter() - tc
    return len(batch) / tc, threads


def c3_full_gate(n, R, args, rank, status0, value0, gpu_tab, block=1 << 26):
    """c3 step 0 in full: the same stream regenerated block by block and applied by one oracle (oracle/oracle.cpp) per
    host thread, sharded by map (map r on oracle r % threads: one map's rows stay in log order on one oracle); every
    row's status + value against the GPU's step-0 results, then every map's entries after step 0 against the GPU
    table read right after step 0.  The oracles' apply time over the whole step is the all-cores CPU baseline."""
    from concurrent.futures import ThreadPoolExecutor

    from copycat_amd import abi
    from copycat_amd.batch import Batch
    from copycat_amd.workload import SEED_C3, map_zipf_rows
    from oracle.oracle_py import Oracle

    threads = cpu_threads()
    oracles = []
    for t in range(threads):
        O = Oracle(R, R)
        for r in range(t, R, threads):  # (the engine's registry: instance r = map r, id 1 + rank + r)
            O.resource_create(r, abi.CC_RES_MAP)
            O.instance_open(r, r, 1 + rank + r, 1 + rank)
        oracles.append(O)
    mism = unwritten = 0
    t_apply = 0.0
    host = Batch(min(n, block))
    with ThreadPoolExecutor(threads) as ex:
        for lo in range(0, n, block):
            m = min(block, n - lo)
            b = host if m == len(host) else Batch(m)
            map_zipf_rows(lo, m, maps=R, pairs=args.pairs, s=args.zipf, seed=SEED_C3 + rank, threads=threads, out=b)
            c3_whole_map_rows(b, lo, args.cv_rate, args.clear_rate, SEED_C3 + rank, args.null_rate, args.delete_rate)
            own = (b.inst % threads).astype(np.uint16)
            order = np.argsort(own, kind="stable")
            cuts = np.searchsorted(own[order], np.arange(threads + 1))
            subs = []
            for t in range(threads):
                rows = order[cuts[t]:cuts[t + 1]]
                part = Batch(0)
                for name in Batch.__slots__:
                    setattr(part, name, np.ascontiguousarray(getattr(b, name)[rows]))
                subs.append(part)
            tc = time.perf_counter()
            res = list(ex.map(lambda t: oracles[t].apply(subs[t]), range(threads)))
            t_apply += time.perf_counter() - tc
            s_ref = np.empty(m, np.uint8)
            v_ref = np.empty(m, np.uint64)
            for t in range(threads):
                rows = order[cuts[t]:cuts[t + 1]]
                s_ref[rows] = res[t][0]
                v_ref[rows] = res[t][1]
            s_gpu = status0[lo:lo + m].cpu().numpy()
            v_gpu = value0[lo:lo + m].cpu().numpy().view(np.uint64)
            bad_rows = np.flatnonzero((s_gpu != s_ref) | (v_gpu != v_ref))
            mism += len(bad_rows)
            unwritten += int(np.count_nonzero(s_gpu == RESULT_SENTINEL))
            for r in bad_rows[:8]:  # (a failing gate names its first rows)
                sys.stderr.write(f"c3 mismatch row {lo + r}: inst {b.inst[r]} op {b.op[r]} key {b.key[r]} gpu "
                                 f"({s_gpu[r]}, {v_gpu[r]}) ref ({s_ref[r]}, {v_ref[r]})\n")
            del subs, res
    sl, kt, k, vt, v, ci = gpu_tab
    bounds = np.searchsorted(sl, np.arange(R + 1))
    maps_bad, entries = 0, 0
    for r in range(R):
        a, z = bounds[r], bounds[r + 1]
        want = oracles[r % threads].map_entries(r)
        got = (kt[a:z], k[a:z], vt[a:z], v[a:z], ci[a:z])
        entries += int(z - a)
        maps_bad += 0 if all(np.array_equal(x, y) for x, y in zip(got, want)) else 1
    parity = {"rows": n, "mismatches": mism, "unwritten": unwritten, "maps": R, "map_entries": entries,
              "maps_mismatched": maps_bad,
              "checked": f"step 0 in full: per-commit status+value of all {n:,} rows (results prefilled with the 0xFF "
                         f"sentinel status) and every map's entries (key, value, commit index) after step 0, GPU vs "
                         f"{threads} oracle/oracle.cpp instances sharded by map"}
    cpu_all = {"value": round(n / t_apply, 1), "unit": "ops/s", "cores": threads, "kind": "port",
               "sample": f"the whole step-0 stream ({n:,} commits) sharded by map (slot % {threads}) over {threads} "
                         f"threads, one oracle each (apply time only; Zipf-hot maps load their shard), {cpu_model()}"}
    return parity, cpu_all


def run_c2(args, dev, rank, world, dist):
    """Config 2 (the headline): per-step client-model streams, full-size parity on step 0, CAS success shares."""
    from copycat_amd import abi
    from copycat_amd.batch import Batch
    from copycat_amd.engine import DeviceBatch, Engine
    from copycat_amd.workload import SEED_C2, AtomicLongClients

    n = args.commits or 100_000_000
    R = args.resources or 65536
    cols = ("index", "inst", "op", "flags", "a", "b")
    total_steps = args.warmup + args.steps
    per_stream = n * (30 + 9)  # device bytes per step: columns + results
    nstreams = max(1, min(total_steps, int(args.hbm_budget_gb * 1e9 // per_stream)))
    t_gen = time.time()
    clients = AtomicLongClients(resources=R, seed=SEED_C2, rank=rank, world=world, threads=cpu_threads())
    host = Batch(n)
    streams, results = [], []
    parity_ref = None
    cpu = cpu_all = None
    E = Engine(R, R, n, device=dev.index, sub_batch=args.sub_batch,
               flags=abi.CC_CFG_TIMERS_DEFERRED | (abi.CC_CFG_VALUE_RETAINED if args.retained else 0))
    E.resource_create_range(0, R, abi.CC_RES_VALUE)
    # local slot k = global resource rank + world*k; its instance id = that global id + 1
    E.instance_open_range(0, R, 0, 1 + rank, 1 + rank)
    for k in range(nstreams):
        clients.next(n, out=host)
        if k == 0 and rank == 0 and not args.no_parity:
            from oracle.oracle_py import Oracle

            O = Oracle(R, R)
            for r in range(R):
                O.resource_create(r, abi.CC_RES_VALUE)
                O.instance_open(r, r, 1 + r, 1)
            tc = time.perf_counter()
            s_ref, v_ref = O.apply(host)  # step 0's rows from the fresh state: the parity reference
            tc = time.perf_counter() - tc
            parity_ref = (s_ref, v_ref, O.value_state())
            if world == 1 and not args.no_cpu_baseline:
                cpu = {"value": round(n / tc, 1), "unit": "ops/s", "cores": 1, "kind": "port",
                       "sample": f"step 0's {n:,} commits of the same c2 stream (the parity reference), C++ restatement "
                                 f"of the Java apply path (oracle/oracle.cpp), 1 thread, {cpu_model()}"}
                v_all, thr = cpu_all_cores(host, R, abi.CC_RES_VALUE, cpu_threads())
                cpu_all = {"value": round(v_all, 1), "unit": "ops/s", "cores": thr, "kind": "port",
                           "sample": f"the same {n:,} commits sharded by resource (slot % {thr}) over {thr} threads, "
                                     f"one oracle each, {cpu_model()}"}
            del O
        streams.append(DeviceBatch.upload(host, device=dev, columns=cols))
        # sentinel prefill (status 0xFF is no legal status): a row the kernels never write fails the step-0 parity
        results.append((torch.full((n,), RESULT_SENTINEL, dtype=torch.uint8, device=dev),
                        torch.full((n,), -1, dtype=torch.int64, device=dev)))
    del host
    t_gen = time.time() - t_gen
    stream = torch.cuda.current_stream(dev)
    wm_local = torch.zeros(1, dtype=torch.int64, device=dev)
    wm_all = torch.zeros(world, dtype=torch.int64, device=dev)

    def step(k):
        st, va = results[k % nstreams]
        E.apply(streams[k % nstreams], st, va, stream=stream)
        E.applied_index_async(wm_local, stream=stream)
        if dist is not None:  # applied-index watermark exchange (RCCL all-gather over xGMI)
            dist.all_gather_into_tensor(wm_all, wm_local)

    state0 = None
    for k in range(args.warmup):
        step(k)
        if k == 0:
            torch.cuda.synchronize(dev)
            state0 = E.value_state()  # the GPU's state after step 0 (parity vs the oracle's)
    torch.cuda.synchronize(dev)
    if not args.no_profile:
        E.profile(True)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    window_marker()
    t0 = time.perf_counter()
    for k in range(args.warmup, total_steps):
        step(k)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    window_marker()
    E.sync()  # surfaces device-side errors
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    prof = E.profile_read() if not args.no_profile else {}

    # watermarks: every rank's last applied global log index, as all-gathered after the last step; stream k of rank r
    # holds the global indices k*n*world + 1 + r + i*world
    watermarks = wm_all.cpu().tolist() if dist is not None else [int(wm_local.item())]
    k_last = (total_steps - 1) % nstreams
    wm_expect = [k_last * n * world + 1 + (n - 1) * world + r for r in range(world)]
    if watermarks != wm_expect:
        sys.stderr.write(f"watermark mismatch: all-gathered {watermarks}, expected {wm_expect}\n")
        sys.exit(4)
    # CAS success share of every timed step (the stated ~0.9 of the client model)
    shares = []
    for k in range(args.warmup, total_steps):
        db, (st, va) = streams[k % nstreams], results[k % nstreams]
        cas = db.cols["op"] == abi.CC_OP_VALUE_CAS
        shares.append(float(((va == 1) & cas).sum().item()) / max(1, int(cas.sum().item())))
    parity = None
    if parity_ref is not None:
        s_ref, v_ref, st_ref = parity_ref
        st0, va0 = results[0]
        s_gpu = st0.cpu().numpy()
        v_gpu = va0.cpu().numpy().view(np.uint64)
        mism = int(np.count_nonzero((s_gpu != s_ref) | (v_gpu != v_ref)))
        smism = None
        if state0 is not None:
            smism = int(sum(np.count_nonzero(a != b) for a, b in zip(state0, st_ref)))
        parity = {"rows": n, "mismatches": mism, "unwritten": int(np.count_nonzero(s_gpu == RESULT_SENTINEL)),
                  "state_slots": R, "state_mismatches": smism,
                  "checked": "step 0: per-commit status+value (results prefilled with the 0xFF sentinel status) and the "
                             "value state after it, GPU vs oracle/oracle.cpp"}
    ms_per_step = elapsed * 1e3 / args.steps
    roofline = roofline_split(prof, n, args.steps, ms_per_step)
    if rank == 0:
        out = {
            "metric": METRIC, "value": round(n * args.steps * world / elapsed, 1), "unit": "ops/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "int64", "data": "synthetic",
            "config": {"workload": ("c2: DistributedAtomicLong Get/CompareAndSet client-model stream, "
                                    f"{n:,} committed entries per step over {R:,} AtomicValueState resources per GPU, "
                                    "a new client-model batch every step"),
                       "commits_per_step_per_gpu": n, "resources_per_gpu": R, "parallelism": f"shard{world}",
                       "sub_batch": args.sub_batch or "default(24Mi)", "resident_streams": nstreams,
                       "cas_success_share": {"min": round(min(shares), 4), "mean": round(sum(shares) / len(shares), 4)},
                       "watermarks": watermarks, "gen_s": round(t_gen, 2)},
            "parity": parity, "roofline": roofline, "cpu_baseline": cpu, "cpu_baseline_all_cores": cpu_all,
        }
        if not args.no_split and world == 1:  # one global log reaching 8 engines, split on this host
            out["global_log_split"] = global_log_split(n, 8, cpu_threads())
        if not args.no_e2e:  # the PCIe-inclusive figure beside the device-resident one (never `value`)
            out["end_to_end"] = end_to_end_c2(E, clients, n, dev)
            out["end_to_end_pipelined"] = end_to_end_c2_pipelined(E, clients, n, dev)
    bad = parity is not None and (parity["mismatches"] or parity["unwritten"] or parity["state_mismatches"])
    c3_bad = False
    if rank == 0 and world == 1 and not args.no_c3:
        # the c3 line inside the default run (an extra key, never `value`): the c2 batches leave HBM first
        del streams, results, E
        torch.cuda.synchronize(dev)
        torch.cuda.empty_cache()
        out["c3"], c3_bad = c3_subrecord(args, dev)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    if bad:
        sys.stderr.write(f"PARITY FAILURE: {parity}\n")
        sys.exit(3)
    if c3_bad:
        sys.stderr.write(f"c3 PARITY FAILURE: {out['c3']['parity']}\n")
        sys.exit(3)


def c3_subrecord(args, dev):
    """BASELINE configs[2] (c3) measured inside the default c2 run, so the driver's own run records it: one 1e9-row
    DistributedMap Zipf(0.99) step over 4,096 maps and 1,048,576 pairs, 1 warm-up + 3 timed steps, step 0 checked in
    full against 16 oracles sharded by map (every row's status and value, every map's entries), its whole-step
    roofline and CPU baselines (measure_c3).  Returns (the c3 JSON object, parity failed)."""
    import argparse as _ap

    a = _ap.Namespace(**vars(args))
    a.cv_rate = a.clear_rate = a.null_rate = a.delete_rate = 0.0
    a.pairs, a.zipf, a.sub_batch, a.cpu_sample = 1 << 20, 0.99, 0, 20_000_000
    t = time.time()
    out, bad = measure_c3(a, dev, 0, 1, None, 1_000_000_000, 3, 1, 4096)
    out["wall_s"] = round(time.time() - t, 1)
    out["note"] = ("BASELINE configs[2] inside the default run (bench.py c3_subrecord); the line's own `value` stays "
                   "c2's, the configuration BASELINE places on one MI355X")
    return out, bad


def global_log_split(n, world, threads, reps=3):
    """The host half of the multi-GPU drop-in: one global c2 log of n rows over world x 65,536 resources
    (ResourceManager multiplexes every resource in one log, ResourceManager.java:37-39) split by owner into `world`
    per-rank batches (cc_split_batch, every column, log order kept per rank), and the per-rank results merged back
    (cc_merge_results).  Staging buffers allocated once and reused; best of `reps` after a warm-up call."""
    import ctypes as C

    from copycat_amd import abi, shard
    from copycat_amd.batch import Batch
    from copycat_amd.engine import _check, _np, lib
    from copycat_amd.workload import atomic_long_stream

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
    ts = []
    for it in range(reps + 1):
        t0 = time.perf_counter()
        _check(lib().cc_split_batch(C.byref(cols), n, _np(tab), R, world, threads, outs, _np(cap), _np(counts), None))
        ts.append(time.perf_counter() - t0)
    pr = (abi.cc_results * world)()
    keep = [(np.full(int(c), r, np.uint8), subs[r].index) for r, c in enumerate(counts)]
    for r, (st, va) in enumerate(keep):
        pr[r].status, pr[r].value = _np(st), _np(va)
    st, va = np.empty(n, np.uint8), np.empty(n, np.uint64)
    out = abi.cc_results(_np(st), _np(va))
    tm = []
    for it in range(reps + 1):
        t0 = time.perf_counter()
        _check(lib().cc_merge_results(_np(b.inst), n, _np(tab), R, world, threads, pr, C.byref(out)))
        tm.append(time.perf_counter() - t0)
    ok = bool(np.array_equal(va, b.index) and np.array_equal(st, tab[b.inst]))
    s, m = min(ts[1:]), min(tm[1:])
    return {"split_rows_per_s": round(n / s, 1), "split_ms": round(s * 1e3, 2), "merge_rows_per_s": round(n / m, 1),
            "merge_ms": round(m * 1e3, 2), "rows": n, "ranks": world, "threads": threads, "cpu": cpu_model(),
            "round_trip_ok": ok, "bytes_per_row": 54,
            "path": "one global c2 log over 8 x 65,536 resources -> cc_split_batch (every column, stable per rank) -> "
                    "cc_merge_results of per-rank status/value back to log order; host memory, best of 3 after a warm-up"}


def end_to_end_c2(E, clients, n, dev):
    """One more client-model step through the PCIe: pinned host columns -> H2D -> apply -> D2H results, synced."""
    from copycat_amd.batch import Batch
    from copycat_amd.engine import DeviceBatch

    host = clients.next(n, out=Batch(n))
    names = ("index", "inst", "op", "flags", "a", "b")
    tdt = {"index": torch.int64, "inst": torch.int32, "op": torch.uint8, "flags": torch.uint8, "a": torch.int64,
           "b": torch.int64}
    pinned = {k: torch.from_numpy(getattr(host, k).view(np.dtype(str(tdt[k]).replace("torch.", "")))).pin_memory()
              for k in names}
    dcols = {k: torch.empty(n, dtype=tdt[k], device=dev) for k in names}
    st, va = torch.empty(n, dtype=torch.uint8, device=dev), torch.empty(n, dtype=torch.int64, device=dev)
    hs, hv = torch.empty(n, dtype=torch.uint8).pin_memory(), torch.empty(n, dtype=torch.int64).pin_memory()
    torch.cuda.synchronize(dev)
    cs = torch.cuda.current_stream(dev)
    t = [time.perf_counter()]
    for k in names:
        dcols[k].copy_(pinned[k], non_blocking=True)
    torch.cuda.synchronize(dev)
    t.append(time.perf_counter())
    E.apply(DeviceBatch(dcols, n), st, va, stream=cs)
    torch.cuda.synchronize(dev)
    t.append(time.perf_counter())
    hs.copy_(st, non_blocking=True)
    hv.copy_(va, non_blocking=True)
    torch.cuda.synchronize(dev)
    t.append(time.perf_counter())
    dt = t[3] - t[0]
    h2d, app, d2h = ((t[i + 1] - t[i]) * 1e3 for i in range(3))
    return {"value": round(n / dt, 1), "unit": "ops/s", "ms": round(dt * 1e3, 3),
            "ms_h2d": round(h2d, 3), "ms_apply": round(app, 3), "ms_d2h": round(d2h, 3),
            "pcie_gbps": round((30 + 9) * n / ((h2d + d2h) * 1e-3) / 1e9, 1),
            "path": "pinned host columns (30 B/commit) H2D + cc_apply_batch + D2H of status/value (9 B/commit), "
                    "one synced step, PCIe-inclusive"}


def end_to_end_c2_pipelined(E, clients, n, dev, chunk=1 << 24):
    """The PCIe-inclusive step as a pipeline: the batch in chunks (one cc_apply_batch each, in log order); chunk i+1's
    H2D (copy stream), chunk i's apply (compute stream) and chunk i-1's D2H (second copy stream) overlap, ordered by
    events.  Bound by the slowest of the three totals (the 30 B/commit H2D) instead of their sum."""
    from copycat_amd.batch import Batch
    from copycat_amd.engine import DeviceBatch

    host = clients.next(n, out=Batch(n))
    names = ("index", "inst", "op", "flags", "a", "b")
    tdt = {"index": torch.int64, "inst": torch.int32, "op": torch.uint8, "flags": torch.uint8, "a": torch.int64,
           "b": torch.int64}
    pinned = {k: torch.from_numpy(getattr(host, k).view(np.dtype(str(tdt[k]).replace("torch.", "")))).pin_memory()
              for k in names}
    dcols = {k: torch.empty(n, dtype=tdt[k], device=dev) for k in names}
    st, va = torch.empty(n, dtype=torch.uint8, device=dev), torch.empty(n, dtype=torch.int64, device=dev)
    hs, hv = torch.empty(n, dtype=torch.uint8).pin_memory(), torch.empty(n, dtype=torch.int64).pin_memory()
    s_in, s_cmp, s_out = torch.cuda.Stream(dev), torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for lo in range(0, n, chunk):
        hi = min(n, lo + chunk)
        e_in, e_cmp = torch.cuda.Event(), torch.cuda.Event()
        with torch.cuda.stream(s_in):
            for k in names:
                dcols[k][lo:hi].copy_(pinned[k][lo:hi], non_blocking=True)
            e_in.record(s_in)
        s_cmp.wait_event(e_in)
        E.apply(DeviceBatch({k: dcols[k][lo:hi] for k in names}, hi - lo), st[lo:hi], va[lo:hi], stream=s_cmp)
        e_cmp.record(s_cmp)
        s_out.wait_event(e_cmp)
        with torch.cuda.stream(s_out):
            hs[lo:hi].copy_(st[lo:hi], non_blocking=True)
            hv[lo:hi].copy_(va[lo:hi], non_blocking=True)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    return {"value": round(n / dt, 1), "unit": "ops/s", "ms": round(dt * 1e3, 3), "chunk": chunk,
            "path": "pinned host columns H2D (copy stream) -> cc_apply_batch per chunk (compute stream) -> D2H of "
                    "status/value (second copy stream), chunks overlapped, PCIe-inclusive, synced at the end"}


def roofline_split(prof, n, steps, ms_per_step):
    """c2 roofline: the whole step's (roofline_step), plus the split of the 39 algorithmic bytes over the kernels that
    move them at the interface (30 input bytes read by the partition, 9 result bytes written by the kernel that stores
    the results) with each one's rate over its own launch time."""
    extra = None
    if prof:
        writer = "k_unpermute" if prof.get("k_unpermute", (0, 0))[1] else "k_apply_value"
        share = {"k_part_tile": 30.0, writer: 9.0}
        per_kernel = {k: round(share[k] * n * steps / (ms * 1e-3) / 1e9, 1) for k, (ms, nl) in prof.items()
                      if nl and k in share}
        extra = {"interface_split": share, "per_kernel_alg_gbps": per_kernel}
    return roofline_step(prof, "c2", n, steps, ms_per_step, B_OP_C2, extra)


def run_c3(args, dev, rank, world, dist):
    """Config 3: DistributedMap Zipf stream (1e9 rows, generated block by block and uploaded once)."""
    out, bad = measure_c3(args, dev, rank, world, dist, args.commits or 1_000_000_000, args.steps, args.warmup,
                          args.resources or 4096)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    if bad:
        sys.stderr.write(f"PARITY FAILURE: {out['parity']}\n")
        sys.exit(3)


def measure_c3(args, dev, rank, world, dist, n, steps, warmup, R):
    """c3 measured: `steps` timed steps after `warmup` untimed ones, step 0 checked in full against the oracle
    (c3_full_gate), the CPU baselines.  Returns (the JSON object, parity failed)."""
    from copycat_amd import abi
    from copycat_amd.engine import Engine

    cpu_sample = args.cpu_sample or 20_000_000
    t_gen = time.time()
    batch, db = upload_c3(n, R, args.pairs, args.zipf, rank, dev, keep_host=min(n, cpu_sample), cv_rate=args.cv_rate,
                          clear_rate=args.clear_rate, null_rate=args.null_rate, delete_rate=args.delete_rate)
    t_gen = time.time() - t_gen
    status = torch.full((n,), RESULT_SENTINEL, dtype=torch.uint8, device=dev)  # sentinel: unwritten rows show
    value = torch.full((n,), -1, dtype=torch.int64, device=dev)
    E = Engine(R, R, n, device=dev.index, sub_batch=args.sub_batch, map_capacity=args.pairs)
    E.resource_create_range(0, R, abi.CC_RES_MAP)
    E.instance_open_range(0, R, 0, 1 + rank, 1 + rank)
    stream = torch.cuda.current_stream(dev)
    wm_local = torch.zeros(1, dtype=torch.int64, device=dev)
    wm_all = torch.zeros(world, dtype=torch.int64, device=dev)

    def step():
        E.apply(db, status, value, stream=stream)
        E.applied_index_async(wm_local, stream=stream)
        if dist is not None:
            dist.all_gather_into_tensor(wm_all, wm_local)

    m = min(n, cpu_sample)
    gpu0 = None  # step 0's results (applied from the fresh state) and the map table right after it: the parity gate

    def capture0():
        torch.cuda.synchronize(dev)
        return status.clone(), value.clone(), E.map_table()

    gate = rank == 0 and not args.no_parity
    for k in range(warmup):
        step()
        if k == 0 and gate:
            gpu0 = capture0()
    torch.cuda.synchronize(dev)
    if not args.no_profile:
        E.profile(True)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    window_marker()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    window_marker()
    E.sync()
    if gpu0 is None and gate and warmup == 0 and steps == 1:  # the one timed step is step 0
        gpu0 = capture0()
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    prof = E.profile_read() if not args.no_profile else {}
    ms_per_step = elapsed * 1e3 / steps
    variant = "b" if args.null_rate or args.delete_rate else ("w" if args.cv_rate or args.clear_rate else "")
    roofline = roofline_step(prof, "c3" + variant, n, steps, ms_per_step, B_OP_C3)
    cpu = parity = cpu_all = None
    if rank == 0 and (not args.no_parity or (world == 1 and not args.no_cpu_baseline)):
        from oracle.oracle_py import Oracle

        O = Oracle(R, R)
        for r in range(R):  # the engine's registry (instance_open_range above)
            O.resource_create(r, abi.CC_RES_MAP)
            O.instance_open(r, r, 1 + rank + r, 1 + rank)
        tc = time.perf_counter()
        O.apply(batch.slice(0, m))
        tc = time.perf_counter() - tc
        if world == 1 and not args.no_cpu_baseline:
            cpu = {"value": round(m / tc, 1), "unit": "ops/s", "cores": 1, "kind": "port",
                   "sample": f"first {m:,} commits of the same c3 stream, C++ restatement of the Java apply path "
                             f"(oracle/oracle.cpp), 1 thread, {cpu_model()}"}
        del O
        if not args.no_parity and gpu0 is not None:
            parity, cpu_all = c3_full_gate(n, R, args, rank, *gpu0)
            if world > 1 or args.no_cpu_baseline:
                cpu_all = None
        gpu0 = None
    out = None
    if rank == 0:
        out = {
            "metric": METRIC, "value": round(n * steps * world / elapsed, 1), "unit": "ops/s", "n_gpus": world,
            "steps": steps, "warmup": warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "int64", "data": "synthetic",
            "config": {"workload": (f"c3: DistributedMap put/get/remove 45/45/10, Zipf({args.zipf}) over {args.pairs:,} "
                                    f"(map, key) pairs in {R:,} MapState resources, {n:,} committed entries per GPU"
                                    + (f"; whole-map variant: {args.cv_rate:.2%} containsValue (operands stored shortly "
                                       f"before), {args.clear_rate:.3%} clear"
                                       if args.cv_rate or args.clear_rate else "")
                                    + (f"; barrier variant: {args.null_rate:.2%} null-valued puts, {args.delete_rate:.4%} "
                                       f"Delete" if args.null_rate or args.delete_rate else "")),
                       "whole_map": ({"containsValue_rate": args.cv_rate, "clear_rate": args.clear_rate,
                                      "null_put_rate": args.null_rate, "delete_rate": args.delete_rate,
                                      "engine_counters": dict(zip(("barrier_rows", "in_stream_containsValue",
                                                                   "sub_batches", "map_events", "big_models"),
                                                                  E.counters()))}
                                     if args.cv_rate or args.clear_rate or args.null_rate or args.delete_rate else None),
                       "map_big_models": E.counters()[4],  # maps followed past 64 for a tree bin (map_big.hip)
                       "commits_per_step_per_gpu": n, "resources_per_gpu": R, "parallelism": f"shard{world}",
                       "sub_batch": args.sub_batch or "default(16M)", "gen_s": round(t_gen, 2),
                       "watermarks": wm_all.cpu().tolist() if dist is not None else [int(wm_local.item())]},
            "parity": parity, "roofline": roofline, "cpu_baseline": cpu, "cpu_baseline_all_cores": cpu_all,
        }
    del E, db, status, value
    bad = parity is not None and bool(parity["mismatches"] or parity["unwritten"] or parity.get("maps_mismatched"))
    return out, bad


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def count_gpus():
    """GPUs this process may use, without any HIP / amdsmi call: the KFD topology nodes that have SIMDs
    (/sys/class/kfd/kfd/topology/nodes/*/properties), narrowed by the *_VISIBLE_DEVICES lists the ROCm runtime honours."""
    root = "/sys/class/kfd/kfd/topology/nodes"
    n = 0
    try:
        for node in os.listdir(root):
            try:
                with open(os.path.join(root, node, "properties")) as f:
                    props = dict(line.split(None, 1) for line in f if len(line.split(None, 1)) == 2)
            except OSError:
                continue
            if int(props.get("simd_count", "0").strip() or 0) > 0:
                n += 1
    except OSError:
        return 0
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        if var in os.environ:
            v = os.environ[var].strip()
            n = min(n, len([x for x in v.split(",") if x.strip()]) if v else 0)
    return n


def launch_ranks(args):
    """`--gpus N` (N > 1) without WORLD_SIZE: start N ranks (torch.distributed.run, one process per GPU) as a child
    process, before anything touches a GPU, and return its exit code; None when this process is already a rank or
    runs alone."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    visible = count_gpus()  # no HIP call in the parent: the ranks are the first processes to touch a GPU
    if visible < args.gpus:
        sys.stderr.write(f"bench.py --gpus {args.gpus}: only {visible} GPU(s) visible on this node; "
                         f"one rank per GPU is required\n")
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=("c2", "c3", "c4", "c5"), default="c2")
    ap.add_argument("--commits", type=int, default=0, help="default: 100M (c2, c5), 1e9 (c3)")
    ap.add_argument("--resources", type=int, default=0, help="default: 65536 resources (c2), 4096 maps (c3)")
    ap.add_argument("--pairs", type=int, default=1 << 20, help="c3: distinct (map, key) pairs")
    ap.add_argument("--zipf", type=float, default=0.99, help="c3: Zipf exponent of the pair rank (0 = uniform)")
    ap.add_argument("--cv-rate", type=float, default=0.0, help="c3 whole-map variant: share of containsValue rows")
    ap.add_argument("--clear-rate", type=float, default=0.0, help="c3 whole-map variant: share of clear rows")
    ap.add_argument("--null-rate", type=float, default=0.0, help="c3 barrier variant: share of null-valued put rows")
    ap.add_argument("--delete-rate", type=float, default=0.0, help="c3 barrier variant: share of Delete rows")
    ap.add_argument("--sub-batch", type=int, default=0)
    ap.add_argument("--cpu-sample", type=int, default=0, help="c3: 20M, c5: 10M (c2 uses step 0's rows)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true",
                    help="skip the oracle parity check of step 0 (c2, c5: all rows; c3: the first --cpu-sample rows; "
                         "c4: input set 0)")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--no-split", action="store_true",
                    help="c2: skip the single-global-log split leg (cc_split_batch / cc_merge_results on the host cores)")
    ap.add_argument("--no-e2e", action="store_true",
                    help="c2: skip the PCIe-inclusive step (pinned H2D + apply + D2H) timed after the timed region")
    ap.add_argument("--hbm-budget-gb", type=float, default=200.0,
                    help="c2: HBM for resident per-step batches (more steps than fit replay the resident ones)")
    ap.add_argument("--c4-sets", type=int, default=6, help="c4: resident input sets used in turn (Infinity Cache)")
    ap.add_argument("--c5-layout", choices=("manager", "interleaved", "grouped"), default="manager",
                    help="c5: resource types by slot: r %% 3 (created in turn) or in thirds")
    ap.add_argument("--retained", action="store_true", help="c2: also keep the retained value commit per slot (CC_CFG_VALUE_RETAINED)")
    ap.add_argument("--no-c3", action="store_true", help="c2: skip the c3 sub-record (a 1e9-row c3 step with its gate)")
    ap.add_argument("--window-markers", action="store_true",
                    help="mark the timed window in a kernel trace with two spin_kernel launches (scripts/gpu_prof.sh)")
    args = ap.parse_args()
    global WINDOW_MARKERS
    WINDOW_MARKERS = args.window_markers

    rc = launch_ranks(args)
    if rc is not None:
        sys.exit(rc)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.stderr.write(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}\n")
        sys.exit(2)
    if not torch.cuda.is_available():
        sys.stderr.write("bench.py: no GPU visible (the engine runs on MI355X only)\n")
        sys.exit(2)
    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local if world > 1 else 0)
    run = {"c2": run_c2, "c3": run_c3, "c4": run_c4, "c5": run_c5}[args.workload]
    return run(args, dev, rank, world, dist)


if __name__ == "__main__":
    main()
