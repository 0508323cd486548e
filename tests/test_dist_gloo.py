"""N>1 path on CPU: world_size-2 gloo processes shard a committed batch by resource, apply their shards
(CPU oracle as the per-rank state machine here; the engine on the GPU box), exchange watermarks and
expiry bitmaps with all-gathers, and the merged result must equal one replica applying the whole batch."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from copycat_amd import abi, shard
from copycat_amd.workload import value_random_stream


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


R, N = 512, 40_000


def _worker(rank, world, port, outdir):
    import torch.distributed as dist

    from oracle.oracle_py import Oracle, expire_sweep

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b = value_random_stream(N, R, R + 8, seed=77, hot=8, p_hot=0.2)
    inst_res = np.arange(R)
    own = shard.inst_owner_table(inst_res, world)
    rows, part = shard.split_batch(b, own, world)[rank]
    O = Oracle(R, R + 8)
    for r in range(R):  # every rank hosts the slots it owns (others stay unused)
        if shard.owner_of(r, world) == rank:
            O.resource_create(r, abi.CC_RES_VALUE)
            O.instance_open(r, r, 1000 + r, 7)
    st, va = O.apply(part)
    # unknown instances (slot >= R) were routed to rank 0, whose registry reports UNKNOWN_SESSION
    wm = shard.allgather_watermark(int(part.index[-1]) if len(part) else int(b.index[-1]))
    last = np.full(1000, 9_000, np.uint64)
    last[rank::world] = 1  # each rank owns every world-th session; expired iff now - last > timeout
    bm, _ = expire_sweep(last, now=10_000, timeout=5_000)
    mine = np.zeros_like(bm)
    for s in range(rank, 1000, world):
        mine[s // 64] |= bm[s // 64] & np.uint64(1 << (s % 64))
    merged = shard.allgather_expired(mine)
    tag, val, cur = O.value_state()
    np.savez(os.path.join(outdir, f"r{rank}.npz"), rows=rows, st=st, va=va, wm=np.array(wm), bm=merged,
             tag=tag, val=val, cur=cur)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(240)
def test_two_rank_shard_matches_single_replica(tmp_path, oracle_lib):
    world, port = 2, _free_port()
    mp.spawn(_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    from oracle.oracle_py import Oracle

    b = value_random_stream(N, R, R + 8, seed=77, hot=8, p_hot=0.2)
    O = Oracle(R, R + 8)
    for r in range(R):
        O.resource_create(r, abi.CC_RES_VALUE)
        O.instance_open(r, r, 1000 + r, 7)
    st1, va1 = O.apply(b)
    parts, tags = [], []
    for rank in range(world):
        z = np.load(tmp_path / f"r{rank}.npz")
        parts.append((z["rows"], z["st"], z["va"]))
        tags.append(z)
    st, va = shard.merge_results(len(b), parts)
    assert np.array_equal(st, st1) and np.array_equal(va, va1)
    # final state: each slot from its owner
    tag1, val1, cur1 = O.value_state()
    for r in range(R):
        z = tags[shard.owner_of(r, world)]
        assert (z["tag"][r], z["val"][r], z["cur"][r]) == (tag1[r], val1[r], cur1[r])
    # watermark exchange: every rank saw both watermarks; the global one is the batch end here
    assert tags[0]["wm"].tolist() == tags[1]["wm"].tolist()
    assert shard.global_watermark(tags[0]["wm"]) <= int(b.index[-1])
    # expiry bitmap: OR over ranks = the full sweep
    assert np.array_equal(tags[0]["bm"], tags[1]["bm"])
    full = np.zeros_like(tags[0]["bm"])
    for s in range(1000):
        full[s // 64] |= np.uint64(1 << (s % 64))
    assert np.array_equal(tags[0]["bm"], full)


# ---- bench.py's multi-GPU c2 layout: each rank generates its share of ONE global log ------------------------------
R2, N2 = 1024, 30_000


def _c2_worker(rank, world, port, outdir):
    import torch
    import torch.distributed as dist

    from copycat_amd.workload import AtomicLongClients
    from oracle.oracle_py import Oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    clients = AtomicLongClients(resources=R2, rank=rank, world=world, threads=2)
    O = Oracle(R2, R2)
    for k in range(R2):  # local slot k = global resource rank + world*k
        O.resource_create(k, abi.CC_RES_VALUE)
        O.instance_open(k, k, 1 + rank + world * k, 1 + rank)
    outs = []
    for step in range(2):
        b = clients.next(N2)
        st, va = O.apply(b)
        wm = torch.tensor([O.applied_index()], dtype=torch.int64)
        allw = torch.zeros(world, dtype=torch.int64)
        dist.all_gather_into_tensor(allw, wm)
        outs.append((b, st, va, allw.tolist()))
    np.savez(os.path.join(outdir, f"c2_r{rank}.npz"),
             **{f"{c}{s}": getattr(outs[s][0], c) for s in range(2) for c in ("index", "inst", "op", "flags", "a", "b")},
             **{f"st{s}": outs[s][1] for s in range(2)}, **{f"va{s}": outs[s][2] for s in range(2)},
             **{f"wm{s}": np.array(outs[s][3]) for s in range(2)})
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(240)
def test_two_rank_c2_is_a_split_of_one_global_log(tmp_path, oracle_lib):
    """The per-rank c2 streams of bench.py --gpus N merge (by log index) into one gap-free global log over
    world * R resources; shard.split_batch of that log by resource owner gives back each rank's stream; one replica
    applying the global log returns exactly the merged per-rank results; all-gathered watermarks are the global log
    positions each rank reached."""
    from copycat_amd.batch import Batch
    from oracle.oracle_py import Oracle

    world, port = 2, _free_port()
    mp.spawn(_c2_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    z = [np.load(tmp_path / f"c2_r{r}.npz") for r in range(world)]
    G = Oracle(world * R2, world * R2)
    for g in range(world * R2):
        G.resource_create(g, abi.CC_RES_VALUE)
        G.instance_open(g, g, 1 + g, 1 + g % world)
    for s in range(2):
        # merge: global row = local row i of rank r at log index s*N2*world + 1 + r + i*world; global slot = r + world*k
        glog = Batch(world * N2)
        for r in range(world):
            idx = z[r][f"index{s}"]
            assert np.array_equal(idx, s * N2 * world + 1 + r + np.arange(N2, dtype=np.uint64) * world)
            pos = (idx - 1 - s * N2 * world).astype(np.int64)
            glog.index[pos] = idx
            glog.inst[pos] = r + world * z[r][f"inst{s}"]
            for c in ("op", "flags", "a", "b"):
                getattr(glog, c)[pos] = z[r][f"{c}{s}"]
        assert np.array_equal(glog.index, s * N2 * world + 1 + np.arange(world * N2, dtype=np.uint64))
        parts = shard.split_batch(glog, shard.inst_owner_table(np.arange(world * R2), world), world)
        for r, (rows, part) in enumerate(parts):
            assert np.array_equal(part.index, z[r][f"index{s}"])
            assert np.array_equal(part.inst // world, z[r][f"inst{s}"])
        st, va = G.apply(glog)
        mst, mva = shard.merge_results(len(glog), [(rows, z[r][f"st{s}"], z[r][f"va{s}"]) for r, (rows, _) in enumerate(parts)])
        assert np.array_equal(st, mst) and np.array_equal(va, mva)
        assert z[0][f"wm{s}"].tolist() == z[1][f"wm{s}"].tolist() == [(s + 1) * N2 * world - 1 + r for r in range(world)]
        cas = glog.op == abi.CC_OP_VALUE_CAS
        assert 0.85 < float((va[cas] == 1).mean()) < 0.95  # the stated stale-CAS mix in every step


def test_bench_gpus_flag_fails_fast_without_gpus():
    """bench.py --gpus N launches N ranks itself; on a box with fewer GPUs it stops before any GPU work."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=120, env=dict(os.environ, CUDA_VISIBLE_DEVICES=""))
    assert r.returncode == 2 and "GPU(s) visible" in r.stderr, (r.returncode, r.stderr[-400:])


# ---- cross-shard session expiry: one client session owns instances on every rank ----------------------------------
RX, KX, SX, NX = 96, 4, 40, 20_000  # coordination resources, instances per resource, client sessions, commits
TYPES_X = np.resize(np.array([abi.CC_RES_LOCK, abi.CC_RES_ELECTION, abi.CC_RES_GROUP], np.uint8), RX)


def _client_of(slot):
    """Owner session of instance slot r*KX + k: the KX instances of a resource belong to KX distinct sessions (a
    client reaches a resource through one instance, ResourceManager.getResource :125-141), spread so that every
    session owns instances on every rank."""
    r, k = divmod(int(slot), KX)
    return (r * 7 + k * 11) % SX


def _expiry_last():
    last = np.full(SX, 9_000, np.uint64)
    last[np.arange(SX) % 3 == 1] = 1  # every third session is expired at now = 10_000, timeout = 5_000
    return last


def _open_x(O, rank=None, world=1):
    for r in range(RX):
        if rank is not None and shard.owner_of(r, world) != rank:
            continue
        O.resource_create(r, int(TYPES_X[r]))
        for k in range(KX):
            s = r * KX + k
            O.instance_open(s, r, 1000 + s, _client_of(s))


def _expire_worker(rank, world, port, outdir):
    import torch.distributed as dist

    from copycat_amd.workload import coord_random_stream
    from oracle.oracle_py import Oracle, expire_sweep

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b = coord_random_stream(NX, TYPES_X, KX, RX * KX, seed=91)
    own = shard.inst_owner_table(np.arange(RX * KX) // KX, world)
    rows, part = shard.split_batch(b, own, world)[rank]
    O = Oracle(RX, RX * KX)
    _open_x(O, rank, world)
    st, va = O.apply(part)
    O.take_events()
    O.take_aux()
    # rank r sweeps the sessions s with s % world == r (the session's owner: it holds its keep-alives) ...
    bm, _ = expire_sweep(_expiry_last(), now=10_000, timeout=5_000)
    mine = np.zeros_like(bm)
    for s in range(rank, SX, world):
        mine[s // 64] |= bm[s // 64] & np.uint64(1 << (s % 64))
    # ... and every rank closes the instances IT hosts of every expired session: the merged bitmap drives the fan-out
    merged = shard.allgather_expired(mine)
    expired = shard.expired_sessions(merged, SX)
    for s in expired:
        O.session_expire(s)
    ev = O.take_events()
    state = {}
    for r in range(RX):
        if shard.owner_of(r, world) == rank:
            t = TYPES_X[r]
            state[r] = (O.lock_state(r) if t == abi.CC_RES_LOCK else
                        O.election_state(r) if t == abi.CC_RES_ELECTION else O.group_members(r))
    np.savez(os.path.join(outdir, f"x_r{rank}.npz"), rows=rows, st=st, va=va, expired=np.array(expired),
             state=np.array(repr(state)), **{f"ev_{k}": v for k, v in ev.items()})
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(240)
def test_two_rank_session_expiry_fans_out_like_one_replica(tmp_path, oracle_lib):
    """ResourceManager.expire (ResourceManager.java:237-247, close :250-264) for a client session that owns instances
    on both ranks: the expired set is swept by the session's owner rank, OR-merged over the all-gather, and every rank
    closes the instances it hosts.  The merged close events, regrouped per target session in emission order (A12),
    and every resource's final state equal one replica expiring the same sessions."""
    from copycat_amd.workload import coord_random_stream
    from oracle.oracle_py import Oracle, expire_sweep

    world, port = 2, _free_port()
    mp.spawn(_expire_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    b = coord_random_stream(NX, TYPES_X, KX, RX * KX, seed=91)
    O = Oracle(RX, RX * KX)
    _open_x(O)
    st1, va1 = O.apply(b)
    O.take_events()
    O.take_aux()
    bm, _ = expire_sweep(_expiry_last(), now=10_000, timeout=5_000)
    expired = shard.expired_sessions(bm, SX)
    assert len(expired) == len(range(1, SX, 3))
    for s in expired:
        O.session_expire(s)
    ev1 = O.take_events()
    z = [np.load(tmp_path / f"x_r{r}.npz") for r in range(world)]
    st, va = shard.merge_results(len(b), [(q["rows"], q["st"], q["va"]) for q in z])
    assert np.array_equal(st, st1) and np.array_equal(va, va1)
    for q in z:
        assert q["expired"].tolist() == expired
    keys = ("pos", "target", "code", "tag", "payload", "src")
    merged = {k: np.concatenate([q[f"ev_{k}"] for q in z]) for k in keys}
    assert len(merged["pos"]) == len(ev1["pos"]) > 0
    assert np.all(merged["src"] == abi.CC_EVSRC_CLOSE)

    def per_target(e):
        o = np.argsort(e["target"], kind="stable")
        return [np.asarray(e[k])[o] for k in keys]

    for g, w in zip(per_target(merged), per_target(ev1)):
        assert np.array_equal(g, w)
    import ast

    state = {}
    for q in z:
        state.update(ast.literal_eval(str(q["state"])))
    for r in range(RX):
        t = TYPES_X[r]
        want = (O.lock_state(r) if t == abi.CC_RES_LOCK else
                O.election_state(r) if t == abi.CC_RES_ELECTION else O.group_members(r))
        assert state[r] == want, r
