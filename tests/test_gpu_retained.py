"""GPU parity: the retained AtomicValue commit per slot (the compaction side of Commit.clean(),
AtomicValueState.java:88-157) vs the oracle's `current`, through cc_read_value_retained.

Bar: bit-exact log indices (integer path).  The random stream holds set / CAS / getAndSet / get / Delete,
unknown sessions and wrong-type ops; split batches check that the retained commit carries across batches."""
import numpy as np
import pytest

from copycat_amd import abi
from copycat_amd.batch import Batch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,resources,seed,hot,p_hot,parts,events", [
    (1, 64, 11, 0, 0.0, 1, False),
    (10_000, 64, 12, 0, 0.0, 3, False),
    (300_001, 4096, 13, 16, 0.2, 4, False),
    (200_000, 65536, 14, 0, 0.0, 2, False),
    (50_000, 1000, 15, 4, 0.5, 2, True),   # value events on: values run on the coordination kernel
])
def test_value_retained_parity(n, resources, seed, hot, p_hot, parts, events):
    from copycat_amd.engine import Engine
    from copycat_amd.workload import value_random_stream
    from oracle.oracle_py import Oracle

    max_inst = resources + 8
    b = value_random_stream(n, resources, max_inst, seed=seed, hot=hot, p_hot=p_hot)
    flags = abi.CC_CFG_TIMERS_DEFERRED | abi.CC_CFG_VALUE_RETAINED | (abi.CC_CFG_VALUE_EVENTS if events else 0)
    E = Engine(resources, max_inst, n, flags=flags, max_events=(4 * n if events else 0))
    O = Oracle(resources, max_inst)
    E.resource_create_range(0, resources, abi.CC_RES_VALUE)
    E.instance_open_range(0, resources, 0, 1000, 7)
    for r in range(resources):
        O.resource_create(r, abi.CC_RES_VALUE)
        O.instance_open(r, r, 1000 + r, 7)
    cuts = np.linspace(0, n, parts + 1).astype(int)
    for lo, hi in zip(cuts[:-1], cuts[1:]):
        if hi <= lo:
            continue
        part = b.slice(lo, hi)
        s, v = E.apply_host_events(part)[:2] if events else E.apply_host(part)
        s2, v2 = O.apply(part)
        assert np.array_equal(s, s2) and np.array_equal(v, v2)
        got, want = E.value_retained(), O.value_retained()
        bad = np.nonzero(got != want)[0]
        assert len(bad) == 0, f"{len(bad)} slots differ; first {bad[:5]}: gpu {got[bad[:5]]} oracle {want[bad[:5]]}"
    assert (O.value_retained() != 0).any() or n < 100


def test_value_retained_resource_delete():
    from copycat_amd.engine import Engine
    from copycat_amd.workload import value_random_stream

    R = 256
    b = value_random_stream(5000, R, R + 8, seed=21)
    E = Engine(R, R + 8, len(b), flags=abi.CC_CFG_TIMERS_DEFERRED | abi.CC_CFG_VALUE_RETAINED)
    E.resource_create_range(0, R, abi.CC_RES_VALUE)
    E.instance_open_range(0, R, 0, 1000, 7)
    E.apply_host(b)
    live = E.value_retained()
    slot = int(np.nonzero(live)[0][0])
    E.resource_delete(slot)
    assert E.value_retained()[slot] == 0


def _value_engine(R, flags, n=1 << 16):
    from copycat_amd.engine import Engine

    E = Engine(R, R + 8, n, flags=flags)
    E.resource_create_range(0, R, abi.CC_RES_VALUE)
    E.instance_open_range(0, R, 0, 1000, 7)
    return E


def test_retained_batch_without_index_is_rejected_before_any_work():
    """CC_CFG_VALUE_RETAINED needs the index column: the call fails before any kernel runs, so device state, the
    applied watermark and the retained commits are untouched and a retry with the column applies the batch once."""
    import torch

    from copycat_amd.engine import DeviceBatch, EngineError
    from copycat_amd.workload import value_random_stream
    from oracle.oracle_py import Oracle

    R = 128
    E = _value_engine(R, abi.CC_CFG_TIMERS_DEFERRED | abi.CC_CFG_VALUE_RETAINED)
    b = value_random_stream(4000, R, R + 8, seed=31)
    db = DeviceBatch.upload(b, device="cuda", columns=("inst", "op", "flags", "a", "b"))
    st = torch.zeros(len(b), dtype=torch.uint8, device="cuda")
    va = torch.zeros(len(b), dtype=torch.int64, device="cuda")
    with pytest.raises(EngineError) as ei:
        E.apply(db, st, va)
    assert ei.value.rc == abi.CC_ERR_INVALID
    tag, val, cur = E.value_state()
    assert not tag.any() and not cur.any() and not E.value_retained().any() and E.applied_index() == 0
    O = Oracle(R, R + 8)
    for r in range(R):
        O.resource_create(r, abi.CC_RES_VALUE)
        O.instance_open(r, r, 1000 + r, 7)
    s, v = E.apply_host(b)
    s2, v2 = O.apply(b)
    assert np.array_equal(s, s2) and np.array_equal(v, v2)
    assert np.array_equal(E.value_retained(), O.value_retained())


def test_retained_snapshot_roundtrip_and_config_check():
    """The retained-commit section travels in the snapshot (SnapHdr flag), and a snapshot restores only into an engine
    with the same CC_CFG_VALUE_RETAINED setting, rejected before anything is copied."""
    from copycat_amd.engine import EngineError
    from copycat_amd.workload import value_random_stream
    from oracle.oracle_py import Oracle

    R = 256
    flags = abi.CC_CFG_TIMERS_DEFERRED | abi.CC_CFG_VALUE_RETAINED
    b = value_random_stream(20_000, R, R + 8, seed=33)
    E = _value_engine(R, flags)
    O = Oracle(R, R + 8)
    for r in range(R):
        O.resource_create(r, abi.CC_RES_VALUE)
        O.instance_open(r, r, 1000 + r, 7)
    E.apply_host(b.slice(0, 10_000))
    O.apply(b.slice(0, 10_000))
    snap = E.snapshot()
    F = _value_engine(R, flags)
    F.restore(snap)
    assert np.array_equal(F.value_retained(), O.value_retained())
    s, v = F.apply_host(b.slice(10_000, 20_000))
    s2, v2 = O.apply(b.slice(10_000, 20_000))
    assert np.array_equal(s, s2) and np.array_equal(v, v2)
    assert np.array_equal(F.value_retained(), O.value_retained())
    plain = _value_engine(R, abi.CC_CFG_TIMERS_DEFERRED)
    before = plain.value_state()
    with pytest.raises(EngineError) as ei:
        plain.restore(snap)
    assert ei.value.rc == abi.CC_ERR_INVALID
    for x, y in zip(before, plain.value_state()):
        assert np.array_equal(x, y)
    with pytest.raises(EngineError):
        _value_engine(R, flags).restore(plain.snapshot())


# ---- every state machine: cc_read_retained vs the oracle's retained() ---------------------------------------------
def _retained_all(E, O, slots):
    for r in slots:
        got, want = E.retained(int(r)), O.retained(int(r))
        assert got == want, (int(r), len(got), len(want), sorted(set(got) ^ set(want))[:8])


def _with_schedules(b, types, K, max_inst, rng, count):
    """MembershipGroup.schedule rows on group instances (retained until their timer fires, :86-103)."""
    G = abi.CC_RES_GROUP
    res_of = np.where(b.inst < max_inst, b.inst // K, 0)
    grp = np.nonzero((types[np.minimum(res_of, len(types) - 1)] == G) & (b.inst < len(types) * K))[0]
    rows = rng.choice(grp, size=min(count, len(grp)), replace=False)
    b.op[rows] = abi.CC_OP_GROUP_SCHEDULE
    b.key[rows] = (1000 + res_of[rows] * K + rng.integers(0, K, len(rows))).astype(np.uint64)
    b.flags[rows] = abi.cc_flags(abi.CC_TAG_HANDLE, 0, 0)
    b.a[rows] = rng.integers(0, 1 << 20, len(rows)).astype(np.uint64)
    b.aux[rows] = rng.integers(1, 400, len(rows)).astype(np.uint64)
    return b


@pytest.mark.parametrize("n,R,K,seed", [(2_000, 16, 3, 31), (120_000, 512, 5, 32)])
def test_retained_coordination_parity(n, R, K, seed):
    """Locks (holder until delete() cleans it, waiters), elections (leader, listeners), groups (members, pending
    schedule commits, members dropped by close: leaked for good), values with listeners (current + listeners +
    re-listen leaks): every slot's retained set after each batch, after session closes, across a snapshot round
    trip and after the schedule timers fire."""
    from copycat_amd.engine import Engine
    from copycat_amd.workload import coord_random_stream
    from tests.test_gpu_coord import FLAGS, _check_batch, _setup

    L, E_, G, V = abi.CC_RES_LOCK, abi.CC_RES_ELECTION, abi.CC_RES_GROUP, abi.CC_RES_VALUE
    types = np.array([L, E_, G, V] * ((R + 3) // 4), np.uint8)[:R]
    flags = FLAGS | abi.CC_CFG_VALUE_RETAINED
    E, O, max_inst = _setup(types, K, flags)
    rng = np.random.default_rng(seed)
    b = _with_schedules(coord_random_stream(n, types, K, max_inst, seed=seed), types, K, max_inst, rng, 40)
    cuts = [0, n // 3, n // 3 + 1, n]
    for lo, hi in zip(cuts[:-1], cuts[1:]):
        _check_batch(E, O, b.slice(lo, hi))
        _retained_all(E, O, range(R))
    assert sum(len(O.retained(r)) for r in range(R)) > R // 2
    vals = np.nonzero(types == V)[0]
    if n >= 100_000:  # re-listen leaks: more retained value commits than current + one listener per instance
        assert sum(len(O.retained(int(r))) for r in vals) > (K + 1) * len(vals)
    # a close drops group members without clean() (leaked) and value listeners / election listeners (cleaned)
    for client in (7, 8):
        E.sessions_close([client], capacity=1 << 18)
        O.session_close(client)
        O.take_events()
    _retained_all(E, O, range(R))
    grps = np.nonzero(types == G)[0]
    if n >= 100_000:  # members dropped by close stay retained (MembershipGroupState.close :36-42)
        assert sum(len(O.retained(int(r))) - len(O.group_members(int(r))) for r in grps) > 0
    # snapshot round trip: the leak lists and pending schedule commits travel with the state
    E2 = Engine(R, max_inst, 1 << 20, flags=flags, max_events=1 << 22)
    E2.restore(E.snapshot())
    _retained_all(E2, O, range(R))
    # the schedule timers fire: their commits are released
    now = int(b.time[-1]) + 1000
    E.advance_time_events(now, capacity=1 << 16)
    O.advance_time(now)
    O.take_events()
    _retained_all(E, O, range(R))


def test_retained_queue_parity():
    """QueueState: every element's commit, less heads element() cleaned (QueueState.java:111-124); poll/remove/clear
    release theirs."""
    from copycat_amd.engine import Engine
    from oracle.oracle_py import Oracle
    from tests.test_gpu_queue import _stream

    Q, n = 64, 40_000
    E = Engine(Q, Q + 8, n, flags=abi.CC_CFG_TIMERS_DEFERRED, max_events=1 << 16)
    O = Oracle(Q, Q + 8)
    E.resource_create_range(0, Q, abi.CC_RES_QUEUE)
    E.instance_open_range(0, Q, 0, 1000, 7)
    for q in range(Q):
        O.resource_create(q, abi.CC_RES_QUEUE)
        O.instance_open(q, q, 1000 + q, 7)
    b = _stream(n, Q, Q + 8, 41)
    for lo, hi in ((0, n // 2), (n // 2, n)):
        s, v = E.apply_host(b.slice(lo, hi))
        s2, v2 = O.apply(b.slice(lo, hi))
        assert np.array_equal(s, s2) and np.array_equal(v, v2)
        _retained_all(E, O, range(Q))
    # clear, add, add, element (cleans the head it leaves queued), poll (removes it), element, add
    ops = [abi.CC_OP_QUEUE_CLEAR, abi.CC_OP_QUEUE_ADD, abi.CC_OP_QUEUE_ADD, abi.CC_OP_QUEUE_ELEMENT, abi.CC_OP_QUEUE_POLL,
           abi.CC_OP_QUEUE_ELEMENT, abi.CC_OP_QUEUE_ADD]
    idx0 = n + 1
    k = Batch.from_columns(index=np.arange(idx0, idx0 + len(ops), dtype=np.uint64),
                           time=np.full(len(ops), int(b.time[-1]), np.uint64), inst=np.zeros(len(ops), np.uint32),
                           op=np.array(ops, np.uint8), flags=np.full(len(ops), abi.CC_TAG_LONG, np.uint8),
                           a=np.arange(len(ops), dtype=np.uint64))
    E.apply_host(k)
    O.apply(k)
    got = E.retained(0)
    assert got == O.retained(0) == [idx0 + 6]  # the two heads element() touched are no longer retained


def test_retained_map_parity():
    """MapState: each live entry's commit (replaced / removed / expired entries are cleaned)."""
    from copycat_amd.workload import map_random_stream
    from tests.test_gpu_map import _engines

    maps, n = 128, 60_000
    E, O = _engines(maps, maps + 8, n, 1 << 16)
    b = map_random_stream(n, maps, maps + 8, keys=32, seed=51)
    for lo, hi in ((0, n // 2), (n // 2, n)):
        s, v = E.apply_host(b.slice(lo, hi))
        s2, v2 = O.apply(b.slice(lo, hi))
        assert np.array_equal(s, s2) and np.array_equal(v, v2)
        _retained_all(E, O, range(maps))


def test_leak_log_drained_across_batches_without_multimaps():
    """AtomicValueState.listen (AtomicValueState.java:41-49) replaces a session's listener with listeners.put and
    never clean()s the replaced commit: it stays in the log for good (the engine's leak log, drained into the per-slot
    retained lists).  More re-listens than the device log holds between drains (1,048,576) over several batches, on an
    engine with value events and no multimaps, all apply, and every slot's retained commits equal the oracle's."""
    from copycat_amd.engine import Engine
    from oracle.oracle_py import Oracle

    R, n, batches = 1024, 450_000, 3
    flags = abi.CC_CFG_TIMERS_DEFERRED | abi.CC_CFG_VALUE_EVENTS
    E = Engine(R, R, n, flags=flags | abi.CC_CFG_VALUE_RETAINED, max_events=4 * n)
    O = Oracle(R, R, flags)
    E.resource_create_range(0, R, abi.CC_RES_VALUE)
    E.instance_open_range(0, R, 0, 1000, 7)
    for r in range(R):
        O.resource_create(r, abi.CC_RES_VALUE)
        O.instance_open(r, r, 1000 + r, 7)
    for k in range(batches):
        idx = np.arange(k * n + 1, (k + 1) * n + 1, dtype=np.uint64)
        b = Batch.from_columns(index=idx, time=idx, inst=(idx % R).astype(np.uint32),
                               op=np.full(n, abi.CC_OP_VALUE_LISTEN, np.uint8))
        s, v, _ = E.apply_host_events(b)
        s2, v2 = O.apply(b)
        assert np.array_equal(s, s2) and np.array_equal(v, v2), k
    assert batches * n - R > 1 << 20
    for slot in list(range(0, R, 97)) + [R - 1]:
        got, want = E.retained(slot), O.retained(slot, cap=1 << 12)
        assert got == want and len(got) >= batches * n // R, slot


# ---- the bulk compaction feed: cc_retained_bitmap == the union of every slot's cc_read_retained -----------------
def _bitmap_indices(bm, first, count):
    words = bm.cpu().numpy().view(np.uint64)[: (count + 63) // 64]
    bits = np.unpackbits(words.view(np.uint8), bitorder="little")[:count]
    return (np.nonzero(bits)[0].astype(np.uint64) + np.uint64(first)).tolist()


def _oracle_union(O, slots):
    out = set()
    for r in slots:
        got = O.retained(int(r), cap=1 << 16)
        if got is not None:
            out.update(got)
    return out


def test_retained_bitmap_coordination_32k_resources():
    """Locks, elections, groups, values with listeners and queues over 32,768+ resources: after every batch, after a
    session close and after the group timers fire, the device bitmap over the whole log range equals the union of the
    oracle's per-slot retained sets (ResourceManagerCommit.clean :79-81 sites of every state machine); a sub-range and
    the count agree too, and bits only clear between calls when a clean() released them."""
    from copycat_amd.workload import coord_random_stream
    from tests.test_gpu_coord import FLAGS, _check_batch, _setup

    L_, E2, G, V, Q = abi.CC_RES_LOCK, abi.CC_RES_ELECTION, abi.CC_RES_GROUP, abi.CC_RES_VALUE, abi.CC_RES_QUEUE
    R, K, n = 32_768 + 256, 2, 600_000
    types = np.resize(np.array([L_, E2, G, V], np.uint8), R)
    flags = FLAGS | abi.CC_CFG_VALUE_RETAINED
    E, O, max_inst = _setup(types, K, flags, max_batch=n, max_events=1 << 23)
    rng = np.random.default_rng(61)
    b = _with_schedules(coord_random_stream(n, types, K, max_inst, seed=61), types, K, max_inst, rng, 200)
    span = n + 1
    prev = None
    for lo, hi in ((0, n // 2), (n // 2, n)):
        _check_batch(E, O, b.slice(lo, hi), capacity=8 * (hi - lo))
        bm, cnt = E.retained_bitmap(1, span)
        got = _bitmap_indices(bm, 1, span)
        want = sorted(_oracle_union(O, range(R)))
        assert cnt == len(got) and got == want, (cnt, len(got), len(want), sorted(set(got) ^ set(want))[:8])
        assert len(want) > R // 2
        if prev is not None:  # a commit of the first batch that is no longer retained was clean()ed in between
            assert set(prev) - set(got) and not (set(got) - set(prev)) & set(range(1, n // 2 + 1))
        prev = got
    sub_first, sub_count = n // 3, 12_345
    bm, cnt = E.retained_bitmap(sub_first, sub_count)
    assert _bitmap_indices(bm, sub_first, sub_count) == [i for i in prev if sub_first <= i < sub_first + sub_count]
    E.sessions_close([7], capacity=1 << 20)
    O.session_close(7)
    O.take_events()
    bm, _ = E.retained_bitmap(1, span)
    assert _bitmap_indices(bm, 1, span) == sorted(_oracle_union(O, range(R)))
    now = int(b.time[-1]) + 1000
    E.advance_time_events(now, capacity=1 << 16)
    O.advance_time(now)
    O.take_events()
    bm, _ = E.retained_bitmap(1, span)
    assert _bitmap_indices(bm, 1, span) == sorted(_oracle_union(O, range(R)))


def test_retained_bitmap_maps_sets_multimaps_queues():
    """Map and set entries (replace / remove / TTL expiry clean them), multimap puts (never cleaned, A18) and queue
    elements in one engine: after each batch the bitmap equals the union of the oracle's per-slot retained sets."""
    from copycat_amd.engine import Engine
    from oracle.oracle_py import Oracle
    from tests.test_gpu_multimap import _stream as keyed_stream
    from tests.test_gpu_queue import _stream as queue_stream

    M = 256
    types = np.array([abi.CC_RES_MAP, abi.CC_RES_MULTIMAP, abi.CC_RES_SET] * M, np.uint8)
    R = len(types) + M  # + M queues after the keyed resources
    n = 60_000
    E = Engine(R, R + 8, n, flags=abi.CC_CFG_TIMERS_DEFERRED, map_capacity=1 << 16, max_events=1 << 18)
    O = Oracle(R, R + 8)
    for r in range(R):
        t = int(types[r]) if r < len(types) else abi.CC_RES_QUEUE
        E.resource_create(r, t)
        E.instance_open(r, r, 1000 + r, 7)
        O.resource_create(r, t)
        O.instance_open(r, r, 1000 + r, 7)
    a = keyed_stream(n, types, 24, seed=71)
    q = queue_stream(n, M, M + 8, 72)
    q.inst[:] = np.where(q.inst < M, q.inst + len(types), R + 5)
    q.index[:] = np.arange(n + 1, 2 * n + 1, dtype=np.uint64)
    q.time[:] = int(a.time[-1]) + np.arange(n, dtype=np.uint64) // 8
    for part in (a, q):
        s, v = E.apply_host(part)
        s2, v2 = O.apply(part)
        assert np.array_equal(s, s2) and np.array_equal(v, v2)
        bm, cnt = E.retained_bitmap(1, 2 * n)
        got = _bitmap_indices(bm, 1, 2 * n)
        want = sorted(_oracle_union(O, range(R)))
        assert got == want and cnt == len(want) > M, (len(got), len(want), sorted(set(got) ^ set(want))[:8])
