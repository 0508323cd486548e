"""GPU parity: MultiMapState (DistributedMultiMap) on the MI355X vs the CPU oracle.

MultiMapState.put registers the key's value map but never stores the value (MultiMapState.java:70-82, A18), so the
state is the set of keys put and not removed since: multimap keys live in the shared map table (a key holding
Boolean TRUE), their ops run as map key ops rewritten in the partition, removeValue / isEmpty / clear / Delete are
batch barriers (map_wide.hip) and k_keyed_results writes put / get / remove / size answers.  Every Put commit stays
retained (never cleaned): checked through cc_read_retained.  No reference test covers MultiMap (there is no
DistributedMultiMapTest): parity is pinned to the restatement of MultiMapState.java:37-222 and the A18 KAT.

Bar: bit-exact per-commit status/value, the key sets, the retained Put commits and the applied index, with maps,
sets and multimaps interleaved in one table."""
import numpy as np
import pytest

from copycat_amd import abi
from copycat_amd.batch import Batch

pytestmark = pytest.mark.gpu

MM_OPS = np.array([abi.CC_OP_MMAP_CONTAINSKEY, abi.CC_OP_MMAP_CONTAINSENTRY, abi.CC_OP_MMAP_CONTAINSVALUE,
                   abi.CC_OP_MMAP_PUT, abi.CC_OP_MMAP_GET, abi.CC_OP_MMAP_REMOVE, abi.CC_OP_MMAP_REMOVEVALUE,
                   abi.CC_OP_MMAP_ISEMPTY, abi.CC_OP_MMAP_SIZE, abi.CC_OP_MMAP_CLEAR, abi.CC_OP_DELETE,
                   abi.CC_OP_MAP_PUT], np.uint8)
MM_P = np.array([14, 1, 1, 30, 8, 18, 0.3, 3, 5, 0.2, 0.1, 0.5])
MAP_OPS = np.array([abi.CC_OP_MAP_PUT, abi.CC_OP_MAP_GET, abi.CC_OP_MAP_REMOVE, abi.CC_OP_MAP_CONTAINSKEY,
                    abi.CC_OP_MAP_PUTIFABSENT, abi.CC_OP_MAP_SIZE], np.uint8)
SET_OPS = np.array([abi.CC_OP_SET_ADD, abi.CC_OP_SET_CONTAINS, abi.CC_OP_SET_REMOVE, abi.CC_OP_SET_SIZE], np.uint8)


def _stream(n, types, keys, seed, index0=1, t0=0):
    """Random rows over resources r (instance slot r) of the given types; keys in [0, keys) with LONG / INT tags."""
    rng = np.random.default_rng(seed)
    R = len(types)
    r = rng.integers(0, R, n)
    op = np.empty(n, np.uint8)
    ty = types[r]
    for t, ops, p in ((abi.CC_RES_MULTIMAP, MM_OPS, MM_P / MM_P.sum()), (abi.CC_RES_MAP, MAP_OPS, None),
                      (abi.CC_RES_SET, SET_OPS, None)):
        m = ty == t
        op[m] = rng.choice(ops, size=int(m.sum()), p=p)
    ktag = rng.choice([0, 1], size=n, p=[0.8, 0.2]).astype(np.uint8)  # LONG / INT keys
    atag = rng.choice([abi.CC_TAG_NULL, abi.CC_TAG_LONG, abi.CC_TAG_HANDLE], size=n, p=[0.3, 0.5, 0.2]).astype(np.uint8)
    flags = (atag | (ktag << 6)).astype(np.uint8)
    aux = np.where(rng.random(n) < 0.05, rng.integers(1, 50, n), 0).astype(np.uint64)  # some TTLs
    inst = r.astype(np.uint32)
    inst[rng.random(n) < 0.002] = R + 3  # unknown instance
    return Batch.from_columns(index=np.arange(index0, index0 + n, dtype=np.uint64),
                              time=(t0 + np.arange(n, dtype=np.uint64) // 8), inst=inst, op=op, flags=flags,
                              key=rng.integers(0, keys, n).astype(np.uint64), a=rng.integers(0, 4, n).astype(np.uint64),
                              aux=aux)


def _engines(types, flags=abi.CC_CFG_TIMERS_DEFERRED, sub_batch=0, map_capacity=1 << 16):
    from copycat_amd.engine import Engine
    from oracle.oracle_py import Oracle

    R = len(types)
    E = Engine(R, R + 8, 1 << 20, map_capacity=map_capacity, flags=flags, sub_batch=sub_batch)
    O = Oracle(R, R + 8, flags & abi.CC_CFG_TIMERS_DEFERRED)
    for s, t in enumerate(types):
        E.resource_create(s, int(t))
        O.resource_create(s, int(t))
        E.instance_open(s, s, 1000 + s, 7)
        O.instance_open(s, s, 1000 + s, 7)
    return E, O


def _check(E, O, b, types):
    s, v = E.apply_host(b)
    s2, v2 = O.apply(b)
    bad = np.nonzero((s != s2) | (v != v2))[0]
    assert len(bad) == 0, (f"{len(bad)} rows differ; first {bad[:5]}: ops {b.op[bad[:5]]} gpu {s[bad[:5]]},{v[bad[:5]]} "
                           f"oracle {s2[bad[:5]]},{v2[bad[:5]]}")
    for r, t in enumerate(types):
        if t == abi.CC_RES_MULTIMAP:
            for x, y in zip(E.map_entries(r), O.map_entries(r)):
                assert np.array_equal(x, y), r
            assert E.retained(r) == O.retained(r), r
    assert E.applied_index() == O.applied_index()
    return s, v


@pytest.mark.parametrize("n,R,keys,seed,sub_batch", [(1, 4, 8, 1, 0), (3_000, 8, 16, 2, 0), (200_000, 96, 64, 3, 16384)])
def test_multimap_random_parity(n, R, keys, seed, sub_batch):
    types = np.array([abi.CC_RES_MULTIMAP, abi.CC_RES_MAP, abi.CC_RES_MULTIMAP, abi.CC_RES_SET] * R, np.uint8)[:R]
    E, O = _engines(types, sub_batch=sub_batch)
    b = _stream(n, types, keys, seed)
    cuts = [0, n // 2, n]
    for lo, hi in zip(cuts[:-1], cuts[1:]):
        if hi > lo:
            s, _ = _check(E, O, b.slice(lo, hi), types)
    mm = types[np.minimum(b.inst, len(types) - 1)] == abi.CC_RES_MULTIMAP
    if n > 1000:  # the rewritten answers all occur: empty collections, size 0, put's true
        lo = cuts[-2]
        tags = {(int(o), int(abi.status_tag(x))) for o, x in zip(b.op[lo:][mm[lo:]], s[mm[lo:]])}
        assert {(abi.CC_OP_MMAP_GET, abi.CC_TAG_LIST), (abi.CC_OP_MMAP_SIZE, abi.CC_TAG_INT),
                (abi.CC_OP_MMAP_PUT, abi.CC_TAG_BOOL)} <= tags
        assert sum(len(O.retained(r)) for r in range(R) if types[r] == abi.CC_RES_MULTIMAP) > 100


def test_multimap_delete_and_reuse():
    """cc_resource_delete drops a multimap's keys and its retained Put commits; the slot can hold a map next."""
    types = np.array([abi.CC_RES_MULTIMAP, abi.CC_RES_MULTIMAP], np.uint8)
    E, O = _engines(types)
    b = _stream(2_000, types, 8, 9)
    _check(E, O, b, types)
    assert E.retained(0)
    E.resource_delete(0)
    O.resource_delete(0)
    E.resource_create(0, abi.CC_RES_MAP)
    O.resource_create(0, abi.CC_RES_MAP)
    E.instance_open(0, 0, 5000, 7)
    O.instance_open(0, 0, 5000, 7)
    assert E.retained(0) == O.retained(0) == []
    b2 = _stream(2_000, np.array([abi.CC_RES_MAP, abi.CC_RES_MULTIMAP], np.uint8), 8, 10, index0=2_001,
                 t0=int(b.time[-1]))
    _check(E, O, b2, np.array([abi.CC_RES_MAP, abi.CC_RES_MULTIMAP], np.uint8))


def test_multimap_puts_beyond_leak_log_chunk():
    """More Put commits than one leak-log allocation holds across batches: the log is drained and regrown."""
    types = np.array([abi.CC_RES_MULTIMAP] * 4, np.uint8)
    E, O = _engines(types, map_capacity=1 << 12)
    n = 1_200_000
    b = Batch.from_columns(index=np.arange(1, n + 1, dtype=np.uint64), time=np.zeros(n, np.uint64),
                           inst=(np.arange(n) % 4).astype(np.uint32), op=np.full(n, abi.CC_OP_MMAP_PUT, np.uint8),
                           flags=np.full(n, abi.CC_TAG_LONG, np.uint8), key=(np.arange(n) % 64).astype(np.uint64),
                           a=np.arange(n, dtype=np.uint64))
    for lo, hi in ((0, 600_000), (600_000, n)):
        s, v = E.apply_host(b.slice(lo, hi))
        assert (v == 1).all() and (abi.status_tag(s) == abi.CC_TAG_BOOL).all()
    got = E.retained(1)
    assert len(got) == n // 4 and got == list(range(2, n + 1, 4))
