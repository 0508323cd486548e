"""GPU: cc_apply_batch_host_prefix (ABI 5) on the fixed capacities beyond coordination collections.

A full map table region or a full event stream fails one commit, not the batch: the call stops before the row that
does not fit, with the engine state, results and events exactly those after the rows before it (a device checkpoint
and a bisection over the part, copycat_amd/csrc/host_path.hip), and the host resumes from there.  In the reference an
exception fails one commit only (ResourceManager.operateResource, manager/src/main/java/io/atomix/manager/
ResourceManager.java:56-72).  Bar: bit-exact against the oracle (oracle/oracle.cpp) on the rows that were applied."""
import numpy as np
import pytest

from copycat_amd import abi
from copycat_amd.batch import Batch
from tests.test_gpu_coord import L, _canon, _check_state, _oracle_events
from tests.test_gpu_map import _assert_maps, _engines

pytestmark = pytest.mark.gpu


def _map_rows(keys, ops, index0=1):
    n = len(keys)
    return Batch.from_columns(index=np.arange(index0, index0 + n, dtype=np.uint64), inst=np.zeros(n, np.uint32),
                              op=np.asarray(ops, np.uint8),
                              flags=np.full(n, abi.cc_flags(abi.CC_TAG_LONG, 0, 0), np.uint8),
                              key=np.asarray(keys, np.uint64), a=np.asarray(keys, np.uint64) * np.uint64(3) + np.uint64(1))


def test_prefix_apply_map_region_full_fails_one_commit():
    """One map in two 2,048-entry table regions (map_capacity 1,024): 4,300 distinct keys are put (gets between), so
    puts into a full region cannot be held; then half the keys are removed (the next launches compact the regions)
    and more keys are put.  The host calls the prefix apply again after each row it reports (failing that commit), and
    every applied row, the map's entries and the applied index equal the oracle applying the same rows."""
    from oracle.oracle_py import Oracle  # noqa: F401  (the _engines oracle)

    E, O = _engines(1, 4, 16384, 1024)
    rng = np.random.default_rng(41)
    k1 = rng.permutation(4300).astype(np.uint64) * np.uint64(7919) + np.uint64(3)
    keys, ops = [], []
    for i, k in enumerate(k1):
        keys.append(k)
        ops.append(abi.CC_OP_MAP_PUT)
        if i % 5 == 0:
            keys.append(k1[int(rng.integers(0, i + 1))])
            ops.append(abi.CC_OP_MAP_GET)
    for k in k1[:2150]:
        keys.append(k)
        ops.append(abi.CC_OP_MAP_REMOVE)
    k2 = np.arange(600, dtype=np.uint64) * np.uint64(104729) + np.uint64(1 << 40)
    for k in k2:
        keys.append(k)
        ops.append(abi.CC_OP_MAP_PUT)
    b = _map_rows(keys, ops)
    n = len(b)
    pos, failed, calls = 0, [], 0
    gs = np.zeros(n, np.uint8)
    gv = np.zeros(n, np.uint64)
    while pos < n:
        calls += 1
        assert calls < 400
        rest = b.slice(pos, n)
        applied, s, v, _ = E.apply_host_prefix(rest)
        gs[pos:pos + applied] = s[:applied]
        gv[pos:pos + applied] = v[:applied]
        assert np.all(s[applied:] == 0xFF)  # rows not applied keep the caller's prefill
        if applied == len(rest):
            break
        failed.append(pos + applied)
        pos += applied + 1
    assert failed, "no region filled"
    keep = np.ones(n, bool)
    keep[failed] = False
    cuts = [0] + [f for f in failed] + [n]
    for a, z in zip(cuts[:-1], cuts[1:]):
        lo = a + 1 if a in failed else a
        if z > lo:
            s2, v2 = O.apply(b.slice(lo, z))
            assert np.array_equal(gs[lo:z], s2) and np.array_equal(gv[lo:z], v2), (lo, z)
    _assert_maps(E, O, [0])


def test_prefix_apply_event_stream_full_resumes():
    """Lock traffic on 64 locks whose events (LockState.lock / unlock publish to the waiter, LockState.java:41-85)
    outnumber a host event stream of 300: each prefix call stops before the first row whose events do not fit, with
    that stream holding exactly the events of the rows before it; the host drains it and calls again from that row.
    Every result and every event (row, target, code, payload) equals the oracle applying the whole batch."""
    from copycat_amd.engine import Engine
    from copycat_amd.workload import coord_random_stream
    from oracle.oracle_py import Oracle

    R, K = 64, 4
    max_inst = R * K + 8
    E = Engine(R, max_inst, 1 << 16, flags=abi.CC_CFG_TIMERS_DEFERRED, max_events=1 << 16)
    O = Oracle(R, max_inst, abi.CC_CFG_TIMERS_DEFERRED)
    for r in range(R):
        E.resource_create(r, L)
        O.resource_create(r, L)
        for k in range(K):
            E.instance_open(r * K + k, r, 1000 + r * K + k, 7 + k)
            O.instance_open(r * K + k, r, 1000 + r * K + k, 7 + k)
    b = coord_random_stream(6000, np.full(R, L, np.uint8), K, max_inst, seed=77, p_delete=0.0)
    n = len(b)
    gs = np.zeros(n, np.uint8)
    gv = np.zeros(n, np.uint64)
    evs = {k: [] for k in ("pos", "src", "target", "code", "tag", "payload")}
    pos, calls = 0, 0
    while pos < n:
        calls += 1
        assert calls < 200
        rest = b.slice(pos, n)
        applied, s, v, ev = E.apply_host_prefix(rest, capacity=300)
        assert applied > 0 or len(rest) == 0
        gs[pos:pos + applied] = s[:applied]
        gv[pos:pos + applied] = v[:applied]
        assert len(ev["pos"]) <= 300 and (len(ev["pos"]) == 0 or ev["pos"].max() < applied)
        for k in evs:
            evs[k].append(ev[k] + (pos if k == "pos" else 0))
        pos += applied
    assert calls > 3  # the stream filled several times
    s2, v2 = O.apply(b)
    assert np.array_equal(gs, s2) and np.array_equal(gv, v2)
    oe, _, _ = _oracle_events(O)
    got = _canon(*(np.concatenate(evs[k]) for k in ("pos", "src", "target", "code", "tag", "payload")))
    assert got == _canon(oe["pos"], oe["src"], oe["target"], oe["code"], oe["tag"], oe["payload"])
    _check_state(E, O, [L] * R)
