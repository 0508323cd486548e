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
