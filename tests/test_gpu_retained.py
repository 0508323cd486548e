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
