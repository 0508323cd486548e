"""GPU parity: SetState (DistributedSet) on the MI355X vs the CPU oracle.

Set elements live in the map table as keys holding Boolean TRUE: contains/add/remove run as
containsKey/putIfAbsent/remove in the region kernels (results rewritten to SetState's, SetState.java:38-87),
size/isEmpty/clear/Delete as whole-map barriers, add's ttl as a map TTL timer.  Bar: bit-exact per-commit
status/value, final elements (read back through cc_read_map_entries) and the applied index."""
import numpy as np
import pytest

from copycat_amd import abi
from copycat_amd.batch import Batch

pytestmark = pytest.mark.gpu

_AS_SET = {abi.CC_OP_MAP_PUT: abi.CC_OP_SET_ADD, abi.CC_OP_MAP_PUTIFABSENT: abi.CC_OP_SET_ADD,
           abi.CC_OP_MAP_REPLACE: abi.CC_OP_SET_ADD, abi.CC_OP_MAP_REPLACEIFPRESENT: abi.CC_OP_SET_ADD,
           abi.CC_OP_MAP_GET: abi.CC_OP_SET_CONTAINS, abi.CC_OP_MAP_GETORDEFAULT: abi.CC_OP_SET_CONTAINS,
           abi.CC_OP_MAP_CONTAINSKEY: abi.CC_OP_SET_CONTAINS, abi.CC_OP_MAP_REMOVE: abi.CC_OP_SET_REMOVE,
           abi.CC_OP_MAP_REMOVEIFPRESENT: abi.CC_OP_SET_REMOVE}
_SET_WIDE = np.array([abi.CC_OP_SET_SIZE, abi.CC_OP_SET_ISEMPTY, abi.CC_OP_SET_CLEAR, abi.CC_OP_DELETE], np.uint8)


def _set_stream(n, sets, max_inst, first_inst, seed, ttl=False, hot=0, p_hot=0.0):
    from copycat_amd.workload import map_random_stream
    from tests.test_gpu_map import _with_barriers, _with_ttl

    b = map_random_stream(n, sets, max_inst, keys=64, first_inst=first_inst, seed=seed, hot=hot, p_hot=p_hot)
    op = b.op.copy()
    for m, s in _AS_SET.items():
        b.op[op == m] = s
    if ttl:
        _with_ttl(b, seed + 1)
    _with_barriers(b, 0.002, seed + 2, ops=_SET_WIDE)
    return b


def _mixed(flags, ttl, n=80_000, seed=61, sub_batch=0):
    from copycat_amd.engine import Engine
    from copycat_amd.workload import map_random_stream
    from oracle.oracle_py import Oracle
    from tests.test_gpu_map import _no_null_values, _with_ttl

    M, S = 16, 16
    slots, max_inst = M + S, M + S + 8
    bm = map_random_stream(n, M, max_inst, keys=64, seed=seed)
    _no_null_values(bm)
    if ttl:
        _with_ttl(bm, seed + 5)
    bs = _set_stream(n, S, max_inst, M, seed + 10, ttl=ttl, hot=2, p_hot=0.2)
    order = np.random.default_rng(seed).permutation(2 * n)
    cols = {name: np.concatenate([getattr(bm, name), getattr(bs, name)])[order] for name, _ in abi.BATCH_COLUMNS}
    cols["index"] = np.arange(1, 2 * n + 1, dtype=np.uint64)
    cols["time"] = np.sort(cols["time"])
    b = Batch.from_columns(**cols)
    E = Engine(slots, max_inst, len(b), map_capacity=65536, flags=flags, sub_batch=sub_batch)
    O = Oracle(slots, max_inst, flags & abi.CC_CFG_TIMERS_DEFERRED)
    E.resource_create_range(0, M, abi.CC_RES_MAP)
    E.resource_create_range(M, S, abi.CC_RES_SET)
    E.instance_open_range(0, slots, 0, 1000, 7)
    for r in range(slots):
        O.resource_create(r, abi.CC_RES_MAP if r < M else abi.CC_RES_SET)
        O.instance_open(r, r, 1000 + r, 7)
    from tests.handles import register_key_strings

    register_key_strings(E, O)
    return E, O, b, slots


def _check(E, O, parts, slots):
    for p in parts:
        s, v = E.apply_host(p)
        s2, v2 = O.apply(p)
        bad = np.nonzero((s != s2) | (v != v2))[0]
        assert len(bad) == 0, (f"{len(bad)} rows differ; first {bad[:5]}: ops {p.op[bad[:5]]} gpu {s[bad[:5]]},"
                               f"{v[bad[:5]]} oracle {s2[bad[:5]]},{v2[bad[:5]]}")
    for r in range(slots):
        for x, y in zip(E.map_entries(r), O.map_entries(r)):
            assert np.array_equal(x, y), r
    assert E.applied_index() == O.applied_index()


def test_sets_and_maps_in_one_table():
    E, O, b, slots = _mixed(abi.CC_CFG_TIMERS_DEFERRED, ttl=False)
    _check(E, O, [b.slice(0, 50_000), b.slice(50_000, len(b))], slots)


@pytest.mark.parametrize("flags", [abi.CC_CFG_TIMERS_DEFERRED, 0], ids=["manager", "module"])
def test_sets_with_ttl(flags):
    E, O, b, slots = _mixed(flags, ttl=True, sub_batch=32768)
    _check(E, O, [b.slice(0, 70_000), b.slice(70_000, len(b))], slots)


def test_set_results_and_unknown_ops():
    """add answers false even when it adds, remove answers whether the element was there; a map op on a set is
    an unknown operation (ResourceStateMachineExecutor.java:78)."""
    from tests.test_gpu_map import _puts

    E, O, b, slots = _mixed(abi.CC_CFG_TIMERS_DEFERRED, ttl=False, n=10)
    M = 16
    p = _puts([5, 5, 6, 5, 5, 5], M, index0=100)
    p.op[:] = [abi.CC_OP_SET_ADD, abi.CC_OP_SET_ADD, abi.CC_OP_MAP_PUT, abi.CC_OP_SET_REMOVE, abi.CC_OP_SET_REMOVE,
               abi.CC_OP_SET_CONTAINS]
    s, v = E.apply_host(p)
    s2, v2 = O.apply(p)
    assert np.array_equal(s, s2) and np.array_equal(v, v2)
    BOOL = abi.cc_status(abi.CC_ST_OK, abi.CC_TAG_BOOL)
    assert list(s) == [BOOL, BOOL, abi.cc_status(abi.CC_ST_UNKNOWN_OP, abi.CC_TAG_NULL), BOOL, BOOL, BOOL]
    assert list(v) == [0, 0, 0, 1, 0, 0]
