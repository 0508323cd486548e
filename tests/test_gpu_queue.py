"""GPU parity: QueueState (DistributedQueue) on the MI355X vs the CPU oracle.

A queue is an ArrayDeque of commits (QueueState.java:33): here a FIFO ring of CC_QUEUE_CAP (value tag, payload)
entries in the coordination block of its slot, applied in log order by the slot's owner thread
(apply_coord.hip).  Bar: bit-exact per-commit status/value (NoSuchElementException and the NPE of a stored
null's equals included) and the applied index; the final contents are checked through size/peek/poll rows."""
import collections

import numpy as np
import pytest

from copycat_amd import abi
from copycat_amd.batch import Batch

pytestmark = pytest.mark.gpu

OPS = np.array([abi.CC_OP_QUEUE_CONTAINS, abi.CC_OP_QUEUE_ADD, abi.CC_OP_QUEUE_OFFER, abi.CC_OP_QUEUE_PEEK,
                abi.CC_OP_QUEUE_POLL, abi.CC_OP_QUEUE_ELEMENT, abi.CC_OP_QUEUE_REMOVE, abi.CC_OP_QUEUE_SIZE,
                abi.CC_OP_QUEUE_ISEMPTY, abi.CC_OP_QUEUE_CLEAR, abi.CC_OP_DELETE, abi.CC_OP_LOCK_LOCK], np.uint8)
P = np.array([10, 16, 16, 8, 14, 6, 14, 6, 5, 1, 0.5, 0.5])


def _stream(n, Q, max_inst, seed):
    """Random queue ops; a host model of each queue's length turns adds into polls near the capacity."""
    rng = np.random.default_rng(seed)
    op = rng.choice(OPS, size=n, p=P / P.sum())
    q = rng.integers(0, Q, n)
    tag = rng.choice([abi.CC_TAG_NULL, abi.CC_TAG_LONG, abi.CC_TAG_INT], size=n, p=[0.08, 0.72, 0.2]).astype(np.uint8)
    val = rng.integers(0, 6, n).astype(np.uint64)
    inst = q.astype(np.uint32)
    inst[rng.random(n) < 0.003] = max_inst + 5  # unknown instance
    model = [collections.deque() for _ in range(Q)]
    for i in range(n):
        d, o = model[q[i]], int(op[i])
        if o in (abi.CC_OP_QUEUE_ADD, abi.CC_OP_QUEUE_OFFER) and len(d) >= abi.CC_QUEUE_CAP - 4:
            op[i] = o = abi.CC_OP_QUEUE_POLL
        if inst[i] >= max_inst:
            continue
        if o in (abi.CC_OP_QUEUE_ADD, abi.CC_OP_QUEUE_OFFER):
            d.append((int(tag[i]), int(val[i]) if tag[i] else 0))
        elif o == abi.CC_OP_QUEUE_POLL or (o == abi.CC_OP_QUEUE_REMOVE and tag[i] == abi.CC_TAG_NULL):
            if d:
                d.popleft()
        elif o == abi.CC_OP_QUEUE_REMOVE:
            for k, e in enumerate(d):
                if e[0] == abi.CC_TAG_NULL:
                    break
                if e == (int(tag[i]), int(val[i])):
                    del d[k]
                    break
        elif o in (abi.CC_OP_QUEUE_CLEAR, abi.CC_OP_DELETE):
            d.clear()
    return Batch.from_columns(index=np.arange(1, n + 1, dtype=np.uint64), time=np.arange(n, dtype=np.uint64) // 16,
                              inst=inst, op=op, flags=tag, a=val)


@pytest.mark.parametrize("n,Q,seed,sub_batch", [(1, 2, 1, 0), (5_000, 3, 2, 0), (120_000, 300, 3, 16384)])
def test_queue_random_parity(n, Q, seed, sub_batch):
    from copycat_amd.engine import Engine
    from oracle.oracle_py import Oracle

    max_inst = Q + 8
    E = Engine(Q, max_inst, max(n, 4 * abi.CC_QUEUE_CAP * Q), sub_batch=sub_batch, max_events=1 << 20)
    O = Oracle(Q, max_inst)
    E.resource_create_range(0, Q, abi.CC_RES_QUEUE)
    E.instance_open_range(0, Q, 0, 1000, 7)
    for r in range(Q):
        O.resource_create(r, abi.CC_RES_QUEUE)
        O.instance_open(r, r, 1000 + r, 7)
    b = _stream(n, Q, max_inst, seed)
    cuts = [0, n // 2, n] if n > 1 else [0, n]
    for lo, hi in zip(cuts[:-1], cuts[1:]):
        part = b.slice(lo, hi)
        s, v, _ = E.apply_host_events(part)
        s2, v2 = O.apply(part)
        bad = np.nonzero((s != s2) | (v != v2))[0]
        assert len(bad) == 0, (f"{len(bad)} rows differ; first {bad[:5]}: ops {part.op[bad[:5]]} gpu {s[bad[:5]]},"
                               f"{v[bad[:5]]} oracle {s2[bad[:5]]},{v2[bad[:5]]}")
        O.take_events()
    # drain every queue: its contents, in order, must agree
    m = 4 * abi.CC_QUEUE_CAP * Q
    d = Batch.from_columns(index=np.arange(n + 1, n + 1 + m, dtype=np.uint64), time=np.full(m, n, np.uint64),
                           inst=np.tile(np.arange(Q, dtype=np.uint32), 4 * abi.CC_QUEUE_CAP),
                           op=np.full(m, abi.CC_OP_QUEUE_POLL, np.uint8))
    s, v, _ = E.apply_host_events(d)
    s2, v2 = O.apply(d)
    assert np.array_equal(s, s2) and np.array_equal(v, v2)
    assert E.applied_index() == O.applied_index()


def test_queue_capacity_fails_loudly():
    from copycat_amd.engine import Engine, EngineError

    E = Engine(1, 4, 1024, max_events=1024)
    E.resource_create(0, abi.CC_RES_QUEUE)
    E.instance_open(0, 0, 1000, 7)
    n = abi.CC_QUEUE_CAP + 1
    b = Batch.from_columns(index=np.arange(1, n + 1, dtype=np.uint64), inst=np.zeros(n, np.uint32),
                           op=np.full(n, abi.CC_OP_QUEUE_ADD, np.uint8), flags=np.full(n, abi.CC_TAG_LONG, np.uint8))
    with pytest.raises(EngineError) as ei:
        E.apply_host_events(b)
    assert ei.value.rc == abi.CC_ERR_CAPACITY
