"""Multi-GPU routing of the commit-apply path (host side): one engine per GPU, resources sharded by id.

SURVEY §8(e): resources are independent state machines multiplexed in one log (ResourceManager.java:37-39),
so a committed batch splits by resource owner with no cross-shard order dependence; only the order of
commits WITHIN a resource matters, and a stable split keeps it.  The only exchanges are:
  * the applied-index watermark (global applied = min over ranks), and
  * the session-expiry result (OR of per-rank bitmaps),
both tiny and all-gathered over RCCL (torch.distributed "nccl" on ROCm) once per batch.
"""
import numpy as np

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


def split_batch(b: Batch, inst_owner, world):
    """Stable split of a batch into per-rank batches.  Returns [(rows, Batch)] indexed by rank."""
    inst = b.inst.astype(np.int64)
    own = np.where(inst < len(inst_owner), np.asarray(inst_owner)[np.minimum(inst, len(inst_owner) - 1)], 0)
    parts = []
    for r in range(world):
        rows = np.nonzero(own == r)[0]
        sub = Batch(0)
        for name in Batch.__slots__:
            setattr(sub, name, np.ascontiguousarray(getattr(b, name)[rows]))
        parts.append((rows, sub))
    return parts


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
