"""GPU parity: the retained AtomicValue commit per slot (the compaction side of Commit.clean(),
AtomicValueState.java:88-157) vs the oracle's `current`, through cc_read_value_retained.

Bar: bit-exact log indices (integer path).  The random stream holds set / CAS / getAndSet / get / Delete,
unknown sessions and wrong-type ops; split batches check that the retained commit carries across batches."""
import numpy as np
import pytest

from copycat_amd import abi

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
