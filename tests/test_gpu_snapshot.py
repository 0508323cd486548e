"""GPU snapshot / restore: a fresh engine restored from a snapshot taken mid-stream
continues bit-exact against the CPU oracle that never stopped — AtomicValue, Map (TTL timers, whole-map ops)
and coordination state (lock queues with timeouts, election listeners, group members, events)."""
import numpy as np
import pytest

from copycat_amd import abi

pytestmark = pytest.mark.gpu


def _rows_equal(a, b):
    for x, y in zip(a, b):
        bad = np.nonzero(x != y)[0]
        assert len(bad) == 0, f"{len(bad)} rows differ, first {bad[:5]}"


def test_snapshot_restore_values_and_maps():
    from copycat_amd.engine import Engine
    from copycat_amd.workload import map_random_stream, value_random_stream
    from oracle.oracle_py import Oracle
    from tests.test_gpu_map import _no_null_values, _with_barriers, _with_ttl

    V, M = 256, 32
    slots, max_inst = V + M, V + M + 8
    bv = value_random_stream(60_000, V, max_inst, seed=101, hot=4, p_hot=0.2)
    bm = map_random_stream(60_000, M, max_inst, keys=64, first_inst=V, seed=102)
    _no_null_values(bm)
    _with_ttl(bm, 103)
    _with_barriers(bm, 0.002, 104, ops=np.array([abi.CC_OP_MAP_SIZE, abi.CC_OP_MAP_CONTAINSVALUE], np.uint8))
    order = np.random.default_rng(7).permutation(len(bv) + len(bm))
    from copycat_amd.batch import Batch
    cols = {name: np.concatenate([getattr(bv, name), getattr(bm, name)])[order] for name, _ in abi.BATCH_COLUMNS}
    cols["index"] = np.arange(1, len(order) + 1, dtype=np.uint64)
    cols["time"] = np.sort(cols["time"])
    b = Batch.from_columns(**cols)

    def engine():
        E = Engine(slots, max_inst, len(b), map_capacity=16384)
        E.resource_create_range(0, V, abi.CC_RES_VALUE)
        E.resource_create_range(V, M, abi.CC_RES_MAP)
        E.instance_open_range(0, slots, 0, 1000, 7)
        return E

    from tests.handles import register_key_strings

    E = engine()
    O = Oracle(slots, max_inst)
    for r in range(slots):
        O.resource_create(r, abi.CC_RES_VALUE if r < V else abi.CC_RES_MAP)
        O.instance_open(r, r, 1000 + r, 7)
    register_key_strings(E, O)  # (the restored engine gets them from the snapshot)
    cut = len(b) // 2
    first = b.slice(0, cut)
    _rows_equal(E.apply_host(first), O.apply(first))
    snap = E.snapshot()
    del E
    E2 = Engine(slots, max_inst, len(b), map_capacity=16384)  # empty registry: everything comes from the snapshot
    E2.restore(snap)
    rest = b.slice(cut, len(b))
    _rows_equal(E2.apply_host(rest), O.apply(rest))
    for x, y in zip(E2.value_state(0, V), O.value_state(0, V)):
        assert np.array_equal(x, y)
    for m in range(V, slots):
        for x, y in zip(E2.map_entries(m), O.map_entries(m)):
            assert np.array_equal(x, y)
    assert E2.applied_index() == O.applied_index()


def test_snapshot_restore_coordination():
    from copycat_amd.engine import Engine
    from copycat_amd.workload import coord_random_stream
    from tests.test_gpu_coord import E_, FLAGS, G, L, V, _check_batch, _check_state, _setup

    types = np.array([L, E_, G, V] * 24, np.uint8)
    K = 5
    E, O, max_inst = _setup(types, K, FLAGS)
    b = coord_random_stream(60_000, types, K, max_inst, seed=21)
    _check_batch(E, O, b.slice(0, 30_000))
    snap = E.snapshot()
    del E
    E2 = Engine(len(types), max_inst, 1 << 20, flags=FLAGS, max_events=1 << 22)
    E2.restore(snap)
    _check_state(E2, O, types)
    _check_batch(E2, O, b.slice(30_000, 60_000))
    _check_state(E2, O, types)


def test_snapshot_rejects_other_configuration():
    from copycat_amd.engine import Engine, EngineError

    E = Engine(64, 64, 16)
    snap = E.snapshot()
    with pytest.raises(EngineError) as ei:
        Engine(128, 64, 16).restore(snap)
    assert ei.value.rc == abi.CC_ERR_INVALID
    with pytest.raises(EngineError):
        Engine(64, 64, 16).restore(snap[:100])


def test_snapshot_corrupt_counts_rejected_before_any_state_changes():
    """A snapshot whose trailing counts (group timers, resource sessions, leak lists) are corrupt -- huge values whose
    byte size would wrap a pointer check -- or that is truncated anywhere is rejected with CC_ERR_INVALID, and the
    engine keeps the state it had (the whole buffer is validated before anything is written)."""
    import struct

    from copycat_amd.engine import Engine, EngineError
    from copycat_amd.workload import value_random_stream
    from oracle.oracle_py import Oracle

    R = 64
    b = value_random_stream(3000, R, R + 8, seed=5)
    E = Engine(R, R + 8, len(b))
    E.resource_create_range(0, R, abi.CC_RES_VALUE)
    E.instance_open_range(0, R, 0, 1000, 7)
    E.apply_host(b)
    snap = bytearray(E.snapshot())
    before = [x.copy() for x in E.value_state()]
    # the trailer: ... ng(8) seq(8) [timers] ns(8) [24 B each] nl(8) [16 B each]; with no timers / sessions / leaks
    # the last 32 bytes are ng, seq, ns, nl
    F = Engine(R, R + 8, len(b))
    F.resource_create_range(0, R, abi.CC_RES_VALUE)
    F.instance_open_range(0, R, 0, 1000, 7)
    F.apply_host(b.slice(0, 1000))
    f_before = [x.copy() for x in F.value_state()]
    for off in (32, 16, 8):  # ng, ns, nl
        bad = bytearray(snap)
        struct.pack_into("<Q", bad, len(bad) - off, (1 << 64) - 3)
        with pytest.raises(EngineError) as ei:
            F.restore(bytes(bad))
        assert ei.value.rc == abi.CC_ERR_INVALID
        for x, y in zip(F.value_state(), f_before):
            assert np.array_equal(x, y)
    for cut in (len(snap) - 1, len(snap) // 2, 200):
        with pytest.raises(EngineError):
            F.restore(bytes(snap[:cut]))
        for x, y in zip(F.value_state(), f_before):
            assert np.array_equal(x, y)
    F.restore(bytes(snap))  # the intact snapshot still restores
    for x, y in zip(F.value_state(), before):
        assert np.array_equal(x, y)
    O = Oracle(R, R + 8)
    for r in range(R):
        O.resource_create(r, abi.CC_RES_VALUE)
        O.instance_open(r, r, 1000 + r, 7)
    O.apply(b)
    for x, y in zip(F.value_state(), O.value_state()):
        assert np.array_equal(x, y)


def test_snapshot_after_overlapped_small_map_replay():
    """Outside TTL mode the small maps' HashMap replay of a sub-batch runs on a side stream while the next sub-batch
    runs (map_small.hip); a snapshot taken right after the batch, barrier rows in the batch (order-dependent
    containsValue on maps holding nulls), in-stream containsValue / clear / size rows and hot keys: the restored engine
    continues bit-exact against the oracle that never stopped, order-dependent answers included."""
    from copycat_amd.engine import Engine
    from copycat_amd.workload import map_random_stream
    from oracle.oracle_py import Oracle
    from tests.handles import register_key_strings
    from tests.test_gpu_map import _cv_rows, _with_barriers

    M, n = 12, 160_000
    slots, max_inst = M, M + 8
    b = map_random_stream(n, M, max_inst, keys=20, seed=111, hot=2, p_hot=0.4)  # small tables (<= 20 keys)
    _cv_rows(b, 0.004, 111, clear_rate=0.0005)
    _with_barriers(b, 0.0015, 112, ops=np.array([abi.CC_OP_MAP_CONTAINSVALUE, abi.CC_OP_MAP_SIZE], np.uint8), p=[0.7, 0.3])

    def engine():
        E = Engine(slots, max_inst, n, map_capacity=16384, sub_batch=16384)
        return E

    E = engine()
    E.resource_create_range(0, M, abi.CC_RES_MAP)
    E.instance_open_range(0, M, 0, 1000, 7)
    O = Oracle(slots, max_inst)
    for r in range(M):
        O.resource_create(r, abi.CC_RES_MAP)
        O.instance_open(r, r, 1000 + r, 7)
    register_key_strings(E, O)
    cut = n // 2
    _rows_equal(E.apply_host(b.slice(0, cut)), O.apply(b.slice(0, cut)))
    assert E.counters()[3] > 0  # the small maps' events were replayed
    snap = E.snapshot()
    del E
    E2 = engine()
    E2.restore(snap)
    _rows_equal(E2.apply_host(b.slice(cut, n)), O.apply(b.slice(cut, n)))
    for m in range(M):
        for x, y in zip(E2.map_entries(m), O.map_entries(m)):
            assert np.array_equal(x, y)
    assert E2.applied_index() == O.applied_index()
