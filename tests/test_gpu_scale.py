"""GPU parity at (near) bench scale — the c2 / c3 / c5 streams at sizes where the bench's kernels run their full grids.

c2 (100M rows) is checked in full by bench.py itself on every run (the "parity" field: step 0's 100M rows against
the oracle, bit for bit); here:
  * c3: 20M rows of the Zipf(0.99) DistributedMap stream over 4,096 maps and 1,048,576 (map, key) pairs — every
    row's status/value, the applied index, and the final entries of a sample of maps (incl. the hottest);
  * c5: 10M rows of the mixed coordination stream over 32,768 resources (a third each LockState,
    LeaderElectionState, MembershipGroupState — the per-GPU share of SURVEY §8(d) c5) — every row's status/value,
    every event (compared as sorted (row, target, code, tag, payload) arrays), join member sets, final lock /
    election / group state of a sample of resources;
  * c2 over several continued steps (AtomicLongClients): 3 x 20M rows, results and value state after each step.
Bar: bit-exact (integer path)."""
import numpy as np
import pytest

from copycat_amd import abi

pytestmark = pytest.mark.gpu


def _sorted_rows(*cols):
    cols = [np.asarray(c).astype(np.uint64) for c in cols]
    order = np.lexsort(cols[::-1])
    return [c[order] for c in cols]


def test_c3_zipf_20m_rows():
    from tests.test_gpu_map import _apply_both, _assert_maps, _assert_rows, _engines
    from copycat_amd.workload import map_zipf_rows

    n, maps, pairs = 20_000_000, 4096, 1 << 20
    b = map_zipf_rows(0, n, maps=maps, pairs=pairs, threads=8)
    E, O = _engines(maps, maps, n, pairs)
    _assert_rows(*_apply_both(E, O, [b]))
    hot = np.bincount(b.inst.astype(np.int64), minlength=maps).argsort()[-4:]
    _assert_maps(E, O, sorted(set(range(0, maps, 257)) | set(int(h) for h in hot)))


def test_c3_zipf_with_1pct_size_rows_20m():
    """MapState.size / isEmpty (:233-250) as ordinary rows: 1% of a 20M-row Zipf map stream (200,000 of them, three
    times the whole-map barrier list's 65,536) are size / isEmpty.  They are answered in the stream from the exact size
    tracking -- no barrier, no host sync per row, no CC_ERR_CAPACITY -- bit-exact against the oracle, across
    sub-batches (16,384 x 128 rows each)."""
    from tests.test_gpu_map import _apply_both, _assert_maps, _assert_rows, _engines
    from copycat_amd.workload import map_zipf_rows

    n, maps, pairs = 20_000_000, 4096, 1 << 20
    b = map_zipf_rows(0, n, maps=maps, pairs=pairs, threads=8)
    rng = np.random.default_rng(77)
    rows = np.nonzero(rng.random(n) < 0.01)[0]
    b.op[rows] = rng.choice(np.array([abi.CC_OP_MAP_SIZE, abi.CC_OP_MAP_ISEMPTY], np.uint8), size=len(rows))
    E, O = _engines(maps, maps, n, pairs, sub_batch=16384 * 128)
    gs, gv, os_, ov = _apply_both(E, O, [b.slice(0, n // 2), b.slice(n // 2, n)])
    _assert_rows(gs, gv, os_, ov)
    sz = rows[b.op[rows] == abi.CC_OP_MAP_SIZE]
    assert len(rows) > 3 * 65536 and len(np.unique(gv[sz])) > 100  # the sizes grow through the stream
    _assert_maps(E, O, sorted(set(range(0, maps, 257))))


def test_c5_mixed_coordination_10m_rows():
    from copycat_amd.engine import Engine
    from copycat_amd.workload import coord_random_stream
    from oracle.oracle_py import Oracle

    n, R = 10_000_000, 32_768
    third = (R + 2) // 3
    types = np.repeat(np.array([abi.CC_RES_LOCK, abi.CC_RES_ELECTION, abi.CC_RES_GROUP], np.uint8), third)[:R]
    b = coord_random_stream(n, types, 1, R, seed=0xA700000 + 5)
    flags = abi.CC_CFG_TIMERS_DEFERRED
    E = Engine(R, R, n, flags=flags, max_events=2 * n)
    O = Oracle(R, R, flags)
    for k, t in enumerate((abi.CC_RES_LOCK, abi.CC_RES_ELECTION, abi.CC_RES_GROUP)):
        E.resource_create_range(k * third, min(third, R - k * third), int(t))
    E.instance_open_range(0, R, 0, 1000, 1)
    for r in range(R):
        O.resource_create(r, int(types[r]))
        O.instance_open(r, r, 1000 + r, 1)
    s, v, ev = E.apply_host_events(b, capacity=2 * n)
    s2, v2 = O.apply(b)
    bad = np.nonzero((s != s2) | (v != v2))[0]
    assert len(bad) == 0, (len(bad), bad[:5])
    oe = O.take_events()
    apos, amem = O.take_aux()
    member = ev["code"] == abi.CC_EV_MEMBER
    got = _sorted_rows(*(ev[k][~member] for k in ("pos", "target", "code", "tag", "payload", "src")))
    want = _sorted_rows(*(oe[k] for k in ("pos", "target", "code", "tag", "payload", "src")))
    assert len(got[0]) == len(want[0]) and len(got[0]) > n // 10
    for g, w in zip(got, want):
        assert np.array_equal(g, w)
    assert np.array_equal(ev["pos"][member], apos) and np.array_equal(ev["payload"][member], amem)
    assert np.all(np.diff(ev["pos"].astype(np.int64)) >= 0)
    for r in range(0, R, 331):
        t = types[r]
        if t == abi.CC_RES_LOCK:
            h, hi, hc, q = E.lock_state(r)
            oh, ohi, ohc, oq = O.lock_state(r)
            assert (h, hc, q) == (oh, ohc, oq) and (h < 0 or hi == ohi), r
        elif t == abi.CC_RES_ELECTION:
            assert E.election_state(r) == O.election_state(r), r
        else:
            assert E.group_members(r) == O.group_members(r), r
    assert E.applied_index() == O.applied_index()


def test_c2_continued_steps():
    from copycat_amd.engine import Engine
    from copycat_amd.workload import AtomicLongClients
    from oracle.oracle_py import Oracle

    n, R = 20_000_000, 65536
    E = Engine(R, R, n)
    E.resource_create_range(0, R, abi.CC_RES_VALUE)
    E.instance_open_range(0, R, 0, 1, 1)
    O = Oracle(R, R)
    for r in range(R):
        O.resource_create(r, abi.CC_RES_VALUE)
        O.instance_open(r, r, 1 + r, 1)
    clients = AtomicLongClients(R, threads=8)
    for step in range(3):
        b = clients.next(n)
        s, v = E.apply_host(b)
        s2, v2 = O.apply(b)
        assert np.array_equal(s, s2) and np.array_equal(v, v2), step
        cas = b.op == abi.CC_OP_VALUE_CAS
        assert 0.88 < float((v[cas] == 1).mean()) < 0.93
        for x, y in zip(E.value_state(), O.value_state()):
            assert np.array_equal(x, y)
    assert E.applied_index() == O.applied_index() == 3 * n


def test_c2_two_sub_batches_at_the_24mi_default():
    """A value-only batch longer than the default sub-batch (24 Mi = 3,072 tiles of 8,192, the apply's LDS run-table
    limit): the first sub-batch uses every tile slot, the second is ragged; every row and the final state against the
    oracle, then a second batch continues the state."""
    from copycat_amd.engine import Engine
    from copycat_amd.workload import AtomicLongClients
    from oracle.oracle_py import Oracle

    n, R = 24 * (1 << 20) + 3_000_001, 65536
    E = Engine(R, R, n)
    E.resource_create_range(0, R, abi.CC_RES_VALUE)
    E.instance_open_range(0, R, 0, 1, 1)
    O = Oracle(R, R)
    for r in range(R):
        O.resource_create(r, abi.CC_RES_VALUE)
        O.instance_open(r, r, 1 + r, 1)
    clients = AtomicLongClients(R, threads=8)
    subs0 = E.counters()[2]  # (barrier rows, in-stream containsValue rows, sub-batches, map events, big models)
    for step in range(2):
        b = clients.next(n if step == 0 else 5_000_000)
        s, v = E.apply_host(b)
        s2, v2 = O.apply(b)
        assert np.array_equal(s, s2) and np.array_equal(v, v2), step
        for x, y in zip(E.value_state(), O.value_state()):
            assert np.array_equal(x, y)
    assert E.counters()[2] - subs0 == 3  # (2 for the first batch, 1 for the second)
    assert E.applied_index() == O.applied_index() == n + 5_000_000
