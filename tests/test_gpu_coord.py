"""GPU parity: LockState / LeaderElectionState / MembershipGroupState and AtomicValue listeners on the MI355X vs
the CPU oracle, through the C-ABI device path with an event stream.

Bar: bit-exact per-commit status/value; the published events (pos, src, target, code, tag, payload) as the
same multiset per commit (each commit publishes at most one event per target, so this also fixes per-target
order); join's member sets; final lock holders/queues, election leaders/listeners, group members and value
state; the applied index."""
import numpy as np
import pytest

from copycat_amd import abi
from copycat_amd.batch import Batch

pytestmark = pytest.mark.gpu

L, E_, G, V = abi.CC_RES_LOCK, abi.CC_RES_ELECTION, abi.CC_RES_GROUP, abi.CC_RES_VALUE


def _setup(types, K, flags, sub_batch=0, max_batch=1 << 20, max_events=1 << 22, coord_cap=0):
    from copycat_amd.engine import Engine
    from oracle.oracle_py import Oracle

    R = len(types)
    max_inst = R * K + 8
    E = Engine(R, max_inst, max_batch, flags=flags, sub_batch=sub_batch, max_events=max_events, coord_cap=coord_cap)
    O = Oracle(R, max_inst, flags & abi.CC_CFG_TIMERS_DEFERRED)
    for r, t in enumerate(types):
        E.resource_create(r, int(t))
        O.resource_create(r, int(t))
        for k in range(K):
            E.instance_open(r * K + k, r, 1000 + r * K + k, 7 + k)
            O.instance_open(r * K + k, r, 1000 + r * K + k, 7 + k)
    return E, O, max_inst


def _oracle_events(O):
    e = O.take_events()
    pos, mem = O.take_aux()
    return e, pos, mem


def _canon(pos, src, target, code, tag, payload):
    rows = list(zip(pos.tolist(), src.tolist(), target.tolist(), code.tolist(), tag.tolist(), payload.tolist()))
    return sorted(rows)


def _check_batch(E, O, b, capacity=0):
    s, v, ev = E.apply_host_events(b, capacity=capacity or max(8 * len(b), 1024))
    s2, v2 = O.apply(b)
    bad = np.nonzero((s != s2) | (v != v2))[0]
    assert len(bad) == 0, (f"{len(bad)} rows differ; first {bad[:5]}: ops {b.op[bad[:5]]} gpu {s[bad[:5]]},{v[bad[:5]]} "
                           f"oracle {s2[bad[:5]]},{v2[bad[:5]]}")
    oe, apos, amem = _oracle_events(O)
    member = ev["code"] == abi.CC_EV_MEMBER
    got = _canon(*(ev[k][~member] for k in ("pos", "src", "target", "code", "tag", "payload")))
    want = _canon(oe["pos"], oe["src"], oe["target"], oe["code"], oe["tag"], oe["payload"])
    assert len(got) == len(want), f"{len(got)} events vs oracle {len(want)}"
    assert got == want, next(((i, g, w) for i, (g, w) in enumerate(zip(got, want)) if g != w), None)
    # join results: the member rows, per join, ascending ids (== the oracle's aux stream)
    gm = list(zip(ev["pos"][member].tolist(), ev["payload"][member].tolist()))
    assert gm == list(zip(apos.tolist(), amem.tolist()))
    # the stream is ordered by log row
    assert np.all(np.diff(ev["pos"].astype(np.int64)) >= 0)
    return s, v, ev


def _check_state(E, O, types):
    for r, t in enumerate(types):
        if t == L:
            h, hi, hc, q = E.lock_state(r)
            oh, ohi, ohc, oq = O.lock_state(r)
            assert (h, hc, q) == (oh, ohc, oq), (r, (h, hc, q), (oh, ohc, oq))
            if h >= 0:
                assert hi == ohi
        elif t == E_:
            assert E.election_state(r) == O.election_state(r), r
        elif t == G:
            assert E.group_members(r) == O.group_members(r), r
    vals = [r for r, t in enumerate(types) if t == V]
    for r in vals:
        assert tuple(int(x[0]) for x in E.value_state(r, 1)) == tuple(int(x[0]) for x in O.value_state(r, 1)), r
    assert E.applied_index() == O.applied_index()


FLAGS = abi.CC_CFG_TIMERS_DEFERRED | abi.CC_CFG_VALUE_EVENTS


def test_coord_event_fanout_burst():
    """Groups and elections of 300 members in one partition tile: join / leave and leadership changes fan out to
    every member, hundreds of thousands of events in the tile (k_ev_tile_out writes such a tile's events straight
    to their rows instead of re-reading its list per 2,048-event window).  Events per commit vs the oracle."""
    from copycat_amd.workload import coord_random_stream

    types = np.array([G, G, E_, V], np.uint8)
    K = 300
    E, O, max_inst = _setup(types, K, FLAGS, coord_cap=512, max_events=1 << 23)
    b = coord_random_stream(8000, types, K, max_inst, seed=17)
    s, v, ev = _check_batch(E, O, b, capacity=1 << 23)
    assert len(ev["pos"]) > 16 * 2048  # past the windowed path's limit in that tile
    _check_state(E, O, types)


@pytest.mark.parametrize("n,R,K,seed,flags", [
    (1, 4, 2, 1, FLAGS),
    (500, 8, 3, 2, FLAGS),
    (20_000, 16, 6, 3, FLAGS),                                  # long per-resource chains
    (20_000, 16, 6, 4, abi.CC_CFG_VALUE_EVENTS),                # module-mode timer order (A8)
    (300_000, 1024, 4, 5, FLAGS),                               # many super-buckets; ragged tail
    (200_000, 600, 8, 6, FLAGS),
])
def test_coord_random_parity(n, R, K, seed, flags):
    from copycat_amd.workload import coord_random_stream

    types = np.array([L, E_, G, V] * ((R + 3) // 4), np.uint8)[:R]
    E, O, max_inst = _setup(types, K, flags)
    b = coord_random_stream(n, types, K, max_inst, seed=seed)
    _check_batch(E, O, b)
    _check_state(E, O, types)


def test_coord_sub_batches_batches_and_clock():
    """State and the log clock carried across sub-batches and calls; advance_time expires lock waiters."""
    from copycat_amd.workload import coord_random_stream

    types = np.array([L, L, E_, G, V, L] * 20, np.uint8)
    K = 5
    E, O, max_inst = _setup(types, K, FLAGS, sub_batch=16384)
    b = coord_random_stream(90_000, types, K, max_inst, seed=9)
    for lo, hi in [(0, 1), (1, 30_000), (30_000, 30_000), (30_000, 90_000)]:
        _check_batch(E, O, b.slice(lo, hi))
    _check_state(E, O, types)
    E.advance_time(int(b.time[-1]) + 1000)
    O.advance_time(int(b.time[-1]) + 1000)
    O.take_events()
    _check_state(E, O, types)


def _one(op, inst, aux=0, time=1, index=1, key=0, a=0, flags=0):
    from copycat_amd.batch import Batch

    return Batch.from_columns(index=[index], time=[time], inst=[inst], op=np.array([op], np.uint8),
                              flags=np.array([flags], np.uint8), key=[key], a=[a], aux=[aux])


def test_lock_queue_capacity_fails_loudly():
    from copycat_amd.batch import Batch
    from copycat_amd.engine import EngineError

    K = abi.CC_LOCK_QUEUE + 2
    E, O, max_inst = _setup(np.array([L], np.uint8), K, FLAGS)
    n = K
    b = Batch.from_columns(index=np.arange(1, n + 1), time=np.ones(n), inst=np.arange(n),
                           op=np.full(n, abi.CC_OP_LOCK_LOCK, np.uint8), aux=np.full(n, 2**64 - 1, np.uint64))
    with pytest.raises(EngineError) as ei:
        E.apply_host_events(b)
    assert ei.value.rc == abi.CC_ERR_CAPACITY


@pytest.mark.parametrize("cap,K,n", [(256, 200, 30_000), (1024, 700, 20_000)])
def test_large_coordination_blocks(cap, K, n):
    """cc_config.coord_cap: locks with hundreds of waiters, elections with hundreds of listeners, groups with hundreds
    of members (entries past the walkers' 8 LDS-cached ones live in global memory), bit-exact vs the oracle; the
    capacity error moves with the configured cap."""
    from copycat_amd.batch import Batch
    from copycat_amd.engine import EngineError
    from copycat_amd.workload import coord_random_stream

    types = np.array([L, E_, G, L, E_, G, V], np.uint8)
    E, O, max_inst = _setup(types, K, FLAGS, coord_cap=cap, max_events=1 << 25)
    b = coord_random_stream(n, types, K, max_inst, seed=11 + cap)
    _check_batch(E, O, b, capacity=1 << 25)
    _check_state(E, O, types)
    # a queue of waiters past the cap fails loudly
    E2, O2, _ = _setup(np.array([L], np.uint8), cap + 2, FLAGS, coord_cap=cap)
    m = cap + 2
    b2 = Batch.from_columns(index=np.arange(1, m + 1), time=np.ones(m), inst=np.arange(m),
                            op=np.full(m, abi.CC_OP_LOCK_LOCK, np.uint8), aux=np.full(m, 2**64 - 1, np.uint64))
    with pytest.raises(EngineError) as ei:
        E2.apply_host_events(b2)
    assert ei.value.rc == abi.CC_ERR_CAPACITY


def test_coord_cap_must_be_power_of_two():
    from copycat_amd.engine import Engine, EngineError

    for bad in (32, 100, 1 << 17):
        with pytest.raises(EngineError) as ei:
            Engine(8, 8, 1024, coord_cap=bad)
        assert ei.value.rc == abi.CC_ERR_INVALID


def test_events_without_stream_fail_loudly():
    from copycat_amd.engine import EngineError

    E, O, _ = _setup(np.array([L, G], np.uint8), 2, FLAGS)
    with pytest.raises(EngineError) as ei:  # the lock event has nowhere to go
        E.apply_host(_one(abi.CC_OP_LOCK_LOCK, 0))
    assert ei.value.rc == abi.CC_ERR_UNSUPPORTED


def test_time_must_not_decrease():
    from copycat_amd.batch import Batch
    from copycat_amd.engine import EngineError

    E, O, _ = _setup(np.array([L], np.uint8), 2, FLAGS)
    b = Batch.from_columns(index=[1, 2], time=[10, 5], inst=[0, 1], op=np.array([115, 115], np.uint8),
                           aux=[5, 5])
    with pytest.raises(EngineError) as ei:
        E.apply_host_events(b)
    assert ei.value.rc == abi.CC_ERR_INVALID


def test_event_stream_capacity():
    from copycat_amd.engine import EngineError
    from copycat_amd.workload import coord_random_stream

    types = np.array([G] * 8, np.uint8)
    E, O, max_inst = _setup(types, 8, FLAGS)
    b = coord_random_stream(5000, types, 8, max_inst, seed=12)
    with pytest.raises(EngineError) as ei:
        E.apply_host_events(b, capacity=100)
    assert ei.value.rc == abi.CC_ERR_CAPACITY


@pytest.mark.parametrize("flags", [FLAGS, abi.CC_CFG_VALUE_EVENTS], ids=["manager", "module"])
def test_group_schedule_timers(flags):
    """MembershipGroup.schedule (MembershipGroupState.java:86-103) as batch barriers: unknown member ->
    IllegalArgumentException; otherwise a timer that publishes "execute"(callback) to the member, if it is still
    in the group, at the commit where the reference's fire_due runs (A8: after the commit that advanced the clock
    in manager mode, before it in module mode); timers carried across batches and fired by advance_time."""
    from copycat_amd.workload import coord_random_stream

    types = np.array([L, E_, G, V, G, G] * 8, np.uint8)
    K = 5
    E, O, max_inst = _setup(types, K, flags)
    b = coord_random_stream(60_000, types, K, max_inst, seed=17)
    rng = np.random.default_rng(17)
    res_of = np.where(b.inst < max_inst, b.inst // K, 0)
    grp = np.nonzero((types[np.minimum(res_of, len(types) - 1)] == G) & (b.inst < len(types) * K))[0]
    rows = rng.choice(grp, size=300, replace=False)
    b.op[rows] = abi.CC_OP_GROUP_SCHEDULE
    g = res_of[rows]
    member = 1000 + g * K + rng.integers(0, K + 2, len(rows))  # some ids are not instances of this group
    b.key[rows] = member.astype(np.uint64)
    b.flags[rows] = abi.cc_flags(abi.CC_TAG_HANDLE, 0, 0)
    b.a[rows] = rng.integers(0, 1 << 20, len(rows)).astype(np.uint64)
    b.aux[rows] = rng.integers(-5, 400, len(rows)).astype(np.int64).view(np.uint64)
    for lo, hi in [(0, 20_000), (20_000, 20_001), (20_001, 60_000)]:
        _check_batch(E, O, b.slice(lo, hi))
    _check_state(E, O, types)
    now = int(b.time[-1]) + 500
    ev = E.advance_time_events(now, capacity=4096)
    O.advance_time(now)
    oe = O.take_events()
    got = sorted(zip(ev["target"].tolist(), ev["code"].tolist(), ev["tag"].tolist(), ev["payload"].tolist()))
    want = sorted(zip(oe["target"].tolist(), oe["code"].tolist(), oe["tag"].tolist(), oe["payload"].tolist()))
    assert got == want
    assert (ev["src"] == abi.CC_EVSRC_TIMER).all() and (ev["pos"] == 0xFFFFFFFF).all()


def test_coordination_on_a_full_partition_fails_at_creation():
    """A 2M-entry map engine over 100,000 resources fills k_part_ext's LDS counters without the coordination
    instance-id plane (8 more bytes per chunk commit).  Creating a lock there must fail with CC_ERR_CAPACITY at
    cc_resource_create (and leave the engine usable for its maps), not make every later cc_apply_batch fail; an engine
    asking for value events at creation is refused the same way."""
    from copycat_amd.engine import Engine, EngineError
    from oracle.oracle_py import Oracle

    R = 100_000
    E = Engine(R, 64, 4096, map_capacity=2 * 1024 * 1024)
    E.resource_create(0, abi.CC_RES_MAP)
    with pytest.raises(EngineError) as ei:
        E.resource_create(1, abi.CC_RES_LOCK)
    assert ei.value.rc == abi.CC_ERR_CAPACITY
    E.instance_open(0, 0, 100, 7)
    O = Oracle(R, 64)
    O.resource_create(0, abi.CC_RES_MAP)
    O.instance_open(0, 0, 100, 7)
    n = 64
    b = Batch.from_columns(index=np.arange(1, n + 1, dtype=np.uint64), time=np.arange(1, n + 1, dtype=np.uint64),
                           inst=np.zeros(n, np.uint32),
                           op=np.where(np.arange(n) % 2 == 0, abi.CC_OP_MAP_PUT, abi.CC_OP_MAP_GET).astype(np.uint8),
                           flags=np.full(n, abi.cc_flags(abi.CC_TAG_LONG, 0, 0), np.uint8),
                           key=(np.arange(n, dtype=np.uint64) // 4), a=np.arange(n, dtype=np.uint64) * 3)
    s, v = E.apply_host(b)
    s2, v2 = O.apply(b)
    assert np.array_equal(s, s2) and np.array_equal(v, v2)
    with pytest.raises(EngineError) as ei:
        Engine(R, 64, 4096, map_capacity=2 * 1024 * 1024, flags=abi.CC_CFG_VALUE_EVENTS)
    assert ei.value.rc == abi.CC_ERR_CAPACITY


def _barrier_event_batch(locks=256, K=4, maps=2, n=150_000):
    """Lock traffic (coord_random_stream, kept whole) with 70,000 map rows (puts, then containsValue) between its rows."""
    from copycat_amd.workload import coord_random_stream

    max_inst = (locks + maps) * K + 8
    # the lock stream stays whole (its client model keeps every queue within coord_cap); the map rows go between
    rng = np.random.default_rng(811)
    nm = 70_000
    lk = coord_random_stream(n - nm, np.full(locks, L, np.uint8), K, max_inst, seed=811, p_delete=0.0)
    rows = np.sort(rng.choice(n, nm, replace=False))
    at = np.ones(n, bool)
    at[rows] = False
    cols = {}
    for name, _ in abi.BATCH_COLUMNS:
        src = getattr(lk, name)
        col = np.zeros(n, src.dtype)
        col[at] = src
        cols[name] = col
    cols["index"] = np.arange(1, n + 1, dtype=np.uint64)
    cols["time"] = np.maximum.accumulate(cols["time"])  # (a map row takes the clock of the lock row before it)
    mrow = rows[: nm // 10]  # some puts first, so the containsValue answers vary
    cols["op"][rows] = abi.CC_OP_MAP_CONTAINSVALUE
    cols["op"][mrow] = abi.CC_OP_MAP_PUT
    cols["inst"][rows] = (locks + rng.integers(0, maps, nm)) * K + rng.integers(0, K, nm)
    cols["key"][rows] = rng.integers(0, 64, nm).astype(np.uint64)
    cols["a"][rows] = rng.integers(0, 4, nm).astype(np.uint64)
    nul = rng.random(nm) < 0.05
    cols["flags"][rows] = np.where(nul, abi.cc_flags(abi.CC_TAG_NULL, 0, 0), abi.cc_flags(abi.CC_TAG_LONG, 0, 0))
    cols["aux"][rows] = 0
    b = Batch.from_columns(**cols)
    return b


def test_more_barrier_rows_than_one_listing_with_events():
    """A batch with more whole-map rows than one barrier listing holds (kBarCap = 65,536) on an engine with an event
    stream runs as two consecutive calls: the second call's events follow the first's, their rows moved by the
    first half's length.  Lock traffic (events on almost every row) interleaved with 70,000 containsValue rows on two
    maps: every row and every event (row, target, code, payload) as the oracle publishes them."""
    from copycat_amd.engine import Engine
    from oracle.oracle_py import Oracle

    locks, K, maps, n = 256, 4, 2, 150_000  # (256 locks: every queue stays well within coord_cap)
    R = locks + maps
    max_inst = R * K + 8
    E = Engine(R, max_inst, n, flags=abi.CC_CFG_TIMERS_DEFERRED, max_events=1 << 20, map_capacity=4096)
    O = Oracle(R, max_inst, abi.CC_CFG_TIMERS_DEFERRED)
    for r in range(R):
        t = L if r < locks else abi.CC_RES_MAP
        E.resource_create(r, t)
        O.resource_create(r, t)
        for k in range(K):
            E.instance_open(r * K + k, r, 1000 + r * K + k, 7 + k)
            O.instance_open(r * K + k, r, 1000 + r * K + k, 7 + k)
    b = _barrier_event_batch(locks, K, maps, n)
    s, v, ev = _check_batch(E, O, b, capacity=4 * n)
    assert ev["pos"].max() >= n // 2  # events of the second call, at their own rows
    _check_state(E, O, [L] * locks)


def test_prefix_apply_stops_before_a_full_lock_queue_and_resumes():
    """cc_apply_batch_host_prefix (ABI 5): a lock queue of coord_cap (64) waiters; the 65th waiter's row is not applied
    -- the call returns CC_ERR_CAPACITY with applied = that row and the engine in exactly the oracle's state after the
    rows before it (results, events, lock queues) -- and the host resumes after it (here: the commit failed) to
    oracle-equal state.  Other locks' traffic runs through the same batch."""
    from copycat_amd.engine import Engine
    from oracle.oracle_py import Oracle

    R, K = 4, 80  # lock 0 gets 66 lockers; locks 1..3 random traffic
    max_inst = R * K + 8
    E = Engine(R, max_inst, 1 << 16, flags=abi.CC_CFG_TIMERS_DEFERRED, max_events=1 << 16)
    O = Oracle(R, max_inst, abi.CC_CFG_TIMERS_DEFERRED)
    for r in range(R):
        E.resource_create(r, L)
        O.resource_create(r, L)
        for k in range(K):
            E.instance_open(r * K + k, r, 1000 + r * K + k, 7 + r * K + k)
            O.instance_open(r * K + k, r, 1000 + r * K + k, 7 + r * K + k)
    rng = np.random.default_rng(5)
    rows = [(0, abi.CC_OP_LOCK_LOCK, -1)] + [(k, abi.CC_OP_LOCK_LOCK, -1) for k in range(1, 66)]
    rows += [(0, abi.CC_OP_LOCK_UNLOCK, 0), (66, abi.CC_OP_LOCK_LOCK, -1), (1, abi.CC_OP_LOCK_UNLOCK, 0)]
    mixed = []
    for _ in range(400):  # other locks, interleaved
        r = int(rng.integers(1, R))
        k = int(rng.integers(0, 20))
        mixed.append((r * K + k, abi.CC_OP_LOCK_LOCK if rng.random() < 0.5 else abi.CC_OP_LOCK_UNLOCK,
                      int(rng.choice([-1, 0, 50]))))
    allrows = []
    for i, x in enumerate(rows):
        allrows.append(x)
        allrows.extend(mixed[i * 5:(i + 1) * 5])
    n = len(allrows)
    b = Batch(n)
    b.index[:] = np.arange(1, n + 1, dtype=np.uint64)
    b.time[:] = np.arange(n, dtype=np.uint64)
    b.inst[:] = [x[0] for x in allrows]
    b.op[:] = [x[1] for x in allrows]
    b.aux[:] = np.array([x[2] for x in allrows], np.int64).view(np.uint64)
    stop = allrows.index((65, abi.CC_OP_LOCK_LOCK, -1))
    applied, s, v, ev = E.apply_host_prefix(b)
    assert applied == stop
    s2, v2 = O.apply(b.slice(0, stop))
    assert np.array_equal(s[:stop], s2) and np.array_equal(v[:stop], v2)
    assert np.all(s[stop:] == 0xFF)  # not applied: the rows keep the caller's prefill
    oe, _, _ = _oracle_events(O)
    got = _canon(*(ev[k] for k in ("pos", "src", "target", "code", "tag", "payload")))
    assert got == _canon(oe["pos"], oe["src"], oe["target"], oe["code"], oe["tag"], oe["payload"])
    _check_state(E, O, [L] * R)
    assert E.applied_index() == O.applied_index() == stop
    # resume after the commit the engine could not hold (the host failed it)
    rest = b.slice(stop + 1, n)
    applied2, s3, v3, ev3 = E.apply_host_prefix(rest)
    assert applied2 == len(rest)
    s4, v4 = O.apply(rest)
    assert np.array_equal(s3, s4) and np.array_equal(v3, v4)
    oe = O.take_events()
    got = _canon(*(ev3[k] for k in ("pos", "src", "target", "code", "tag", "payload")))
    assert got == _canon(oe["pos"], oe["src"], oe["target"], oe["code"], oe["tag"], oe["payload"])
    _check_state(E, O, [L] * R)


def test_prefix_apply_churned_near_full_lock_queue_scans_once():
    """cc_apply_batch_host_prefix (ABI 5) on a lock queue that stays at coord_cap under churn: the holder unlocks (its
    first waiter takes the lock, LockState.java:73-85) and a new client queues, 1,500 times, while 255 other locks take
    random traffic.  Every add on the hot lock meets the upper bound, so the call re-reads that lock's count at each one
    and goes on (one scan of the batch, one header read per stop: ADVICE r5); nothing overflows, every row applies, and
    results, events and lock queues equal the oracle's.  The run time is bounded (the round-5 form rescanned the rest of
    the batch and read one header per addressed lock at every stop)."""
    import time as _time

    from copycat_amd.engine import Engine
    from oracle.oracle_py import Oracle

    R, churn = 256, 1500
    hot = 65 + churn           # clients of lock 0: the holder, 64 waiters, then one new client per churn step
    K = 8                      # clients of every other lock
    max_inst = hot + (R - 1) * K + 8
    E = Engine(R, max_inst, 1 << 16, flags=abi.CC_CFG_TIMERS_DEFERRED, max_events=1 << 18)
    O = Oracle(R, max_inst, abi.CC_CFG_TIMERS_DEFERRED)
    for r in range(R):
        E.resource_create(r, L)
        O.resource_create(r, L)
    inst_of = []
    for k in range(hot):
        inst_of.append((k, 0))
    for r in range(1, R):
        for k in range(K):
            inst_of.append((hot + (r - 1) * K + k, r))
    for i, r in inst_of:
        E.instance_open(i, r, 1000 + i, 7 + i)
        O.instance_open(i, r, 1000 + i, 7 + i)
    rng = np.random.default_rng(17)
    rows = [(k, abi.CC_OP_LOCK_LOCK, -1) for k in range(65)]  # holder 0 + 64 waiters: the queue is full
    for j in range(churn):
        rows.append((j, abi.CC_OP_LOCK_UNLOCK, 0))              # the holder leaves, waiter j + 1 holds
        rows.append((65 + j, abi.CC_OP_LOCK_LOCK, -1))          # a new waiter: back at coord_cap
        for _ in range(2):                                      # other locks' traffic (adds among it)
            r = int(rng.integers(1, R))
            k = int(rng.integers(0, K))
            rows.append((hot + (r - 1) * K + k, abi.CC_OP_LOCK_LOCK if rng.random() < 0.5 else abi.CC_OP_LOCK_UNLOCK,
                         int(rng.choice([-1, 0, 50]))))
    n = len(rows)
    b = Batch(n)
    b.index[:] = np.arange(1, n + 1, dtype=np.uint64)
    b.time[:] = np.arange(n, dtype=np.uint64)
    b.inst[:] = [x[0] for x in rows]
    b.op[:] = [x[1] for x in rows]
    b.aux[:] = np.array([x[2] for x in rows], np.int64).view(np.uint64)
    t0 = _time.perf_counter()
    applied, s, v, ev = E.apply_host_prefix(b)
    dt = _time.perf_counter() - t0
    assert applied == n
    s2, v2 = O.apply(b)
    assert np.array_equal(s, s2) and np.array_equal(v, v2)
    oe, _, _ = _oracle_events(O)
    got = _canon(*(ev[k] for k in ("pos", "src", "target", "code", "tag", "payload")))
    assert got == _canon(oe["pos"], oe["src"], oe["target"], oe["code"], oe["tag"], oe["payload"])
    _check_state(E, O, [L] * R)
    assert dt < 30.0, f"{dt:.1f} s for {churn} stops"
