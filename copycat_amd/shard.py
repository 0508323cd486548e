"""Multi-GPU routing of the commit-apply path (host side): one engine per GPU, resources sharded by id.

SURVEY §8(e): resources are independent state machines multiplexed in one log (ResourceManager.java:37-39),
so a committed batch splits by resource owner with no cross-shard order dependence; only the order of
commits WITHIN a resource matters, and a stable split keeps it.  The only exchanges are:
  * the applied-index watermark (global applied = min over ranks), and
  * the session-expiry result (OR of per-rank bitmaps),
both tiny and all-gathered over RCCL (torch.distributed "nccl" on ROCm) once per batch.
"""
import ctypes as C
import os

import numpy as np

from . import abi
from .batch import Batch

NO_OWNER = -1


def owner_of(resource_slot, world):
    """Resource -> rank (round-robin by global resource slot)."""
    return resource_slot % world


def inst_owner_table(inst_res, world):
    """inst_res[inst] = global resource slot (or -1 for a closed instance) -> owning rank per instance."""
    inst_res = np.asarray(inst_res, dtype=np.int64)
    own = np.where(inst_res >= 0, inst_res % world, 0)  # unknown instances: rank 0 reports UNKNOWN_SESSION
    return own.astype(np.int32)


def _threads(threads):
    if threads:
        return int(threads)
    n = os.cpu_count() or 1
    return max(1, min(n, int(os.environ.get("OMP_NUM_THREADS", n))))


def _rank_table(inst_owner, world):
    t = np.ascontiguousarray(inst_owner)
    if world > 256:
        raise ValueError("world must be <= 256")
    if t.dtype != np.uint8:
        if len(t) and (t.min() < 0 or t.max() >= world):
            raise ValueError("inst_owner names a rank outside [0, world)")
        t = t.astype(np.uint8)
    return t


def split_counts(b: Batch, inst_owner, world, threads=0):
    """Rows per rank of a stable split (cc_split_batch with no outputs)."""
    from .engine import _check, _np, lib

    tab = _rank_table(inst_owner, world)
    counts = np.zeros(world, np.uint64)
    cols = abi.cc_batch(**{name: _np(getattr(b, name)) for name in Batch.__slots__})
    _check(lib().cc_split_batch(C.byref(cols), len(b), _np(tab), len(tab), world, _threads(threads), None, None,
                                _np(counts), None))
    return counts


def split_batch(b: Batch, inst_owner, world, threads=0, rows=True):
    """Stable split of one global log's batch into per-rank batches (native, multi-threaded: cc_split_batch).

    Returns [(rows, Batch)] indexed by rank; rows[r] are the rank's rows of `b` in log order (None if rows=False:
    merge_by_owner does not need them).  Rows whose instance slot is beyond the owner table go to rank 0."""
    from .engine import _check, _np, lib

    tab = _rank_table(inst_owner, world)
    counts = split_counts(b, tab, world, threads)
    parts = []
    outs = (abi.cc_batch_out * world)()
    rowp = (C.c_void_p * world)()
    for r in range(world):
        sub = Batch(int(counts[r]))
        ridx = np.empty(int(counts[r]), np.uint64) if rows else None
        for name in Batch.__slots__:
            setattr(outs[r], name, _np(getattr(sub, name)))
        rowp[r] = _np(ridx) if rows else None
        parts.append((ridx, sub))
    cap = counts.copy()
    cols = abi.cc_batch(**{name: _np(getattr(b, name)) for name in Batch.__slots__})
    _check(lib().cc_split_batch(C.byref(cols), len(b), _np(tab), len(tab), world, _threads(threads), outs, _np(cap),
                                _np(counts), rowp if rows else None))
    return parts


def merge_by_owner(inst, inst_owner, world, parts, threads=0):
    """parts[r] = (status, value) of rank r, in its split order -> (status[n], value[n]) in log order
    (cc_merge_results: the split's owner walk backwards, no row ids needed)."""
    from .engine import _check, _np, lib

    tab = _rank_table(inst_owner, world)
    inst = np.ascontiguousarray(inst, np.uint32)
    n = len(inst)
    status = np.empty(n, np.uint8)
    value = np.empty(n, np.uint64)
    pr = (abi.cc_results * world)()
    keep = []
    for r, (s, v) in enumerate(parts):
        s, v = np.ascontiguousarray(s, np.uint8), np.ascontiguousarray(v, np.uint64)
        keep.append((s, v))
        pr[r].status, pr[r].value = _np(s), _np(v)
    out = abi.cc_results(_np(status), _np(value))
    _check(lib().cc_merge_results(_np(inst), n, _np(tab), len(tab), world, _threads(threads), pr, C.byref(out)))
    return status, value


def merge_results(n, parts):
    """parts: [(rows, status, value)] -> (status[n], value[n]) in log order."""
    status = np.zeros(n, np.uint8)
    value = np.zeros(n, np.uint64)
    for rows, s, v in parts:
        status[rows] = s
        value[rows] = v
    return status, value


def global_watermark(local_applied):
    """All ranks have applied every entry up to min(local watermarks) (a rank with no work reports the batch end)."""
    return int(min(local_applied))


def allgather_watermark(local, device=None, group=None):
    """RCCL/gloo all-gather of one u64 watermark per rank -> list of ints."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    t = torch.tensor([int(local)], dtype=torch.int64, device=device)
    out = torch.zeros(world, dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(out, t, group=group)
    return out.cpu().tolist()


def allgather_expired(bitmap, device=None, group=None):
    """OR-merge of per-rank expired-session bitmaps (u64 words) over all ranks."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    t = torch.as_tensor(np.ascontiguousarray(bitmap).view(np.int64), device=device)
    out = torch.zeros(world * t.numel(), dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(out, t, group=group)
    words = out.view(world, -1).cpu().numpy().view(np.uint64)
    return np.bitwise_or.reduce(words, axis=0)


def expired_sessions(bitmap, sessions):
    """Session ids whose bit is set in an expired-session bitmap (u64 words, LSB first), ascending -- the order
    cc_sessions_expire closes them in."""
    words = np.ascontiguousarray(bitmap, np.uint64)
    bits = np.unpackbits(words.view(np.uint8), bitorder="little")[:sessions]
    return np.nonzero(bits)[0].tolist()
