"""GPU parity: AtomicValueState apply on the MI355X vs the CPU oracle, through the C-ABI.

Bar: bit-exact per-commit status/value, final state and applied index (integer path, no tolerance)."""
import numpy as np
import pytest

from copycat_amd import abi
from copycat_amd.batch import Batch

pytestmark = pytest.mark.gpu


def _setup(E, O, resources, first_inst=0):
    E.resource_create_range(0, resources, abi.CC_RES_VALUE)
    E.instance_open_range(first_inst, resources, 0, 1000, 7)
    for r in range(resources):
        O.resource_create(r, abi.CC_RES_VALUE)
        O.instance_open(first_inst + r, r, 1000 + r, 7)


def _run_both(b: Batch, resources, max_inst, sub_batch=0, split=None, map_capacity=0):
    from copycat_amd.engine import Engine
    from oracle.oracle_py import Oracle

    E = Engine(resources, max_inst, max(len(b), 1), sub_batch=sub_batch, map_capacity=map_capacity)
    O = Oracle(resources, max_inst)
    _setup(E, O, resources)
    parts = [b] if split is None else [b.slice(lo, hi) for lo, hi in split]
    gs, gv, os_, ov = [], [], [], []
    for part in parts:
        s, v = E.apply_host(part)
        s2, v2 = O.apply(part)
        gs.append(s); gv.append(v); os_.append(s2); ov.append(v2)
    gs, gv, os_, ov = (np.concatenate(x) if x else np.zeros(0) for x in (gs, gv, os_, ov))
    return E, O, gs, gv, os_, ov


def _assert_same(E, O, gs, gv, os_, ov, resources):
    bad = np.nonzero((gs != os_) | (gv != ov))[0]
    assert len(bad) == 0, f"{len(bad)} rows differ; first {bad[:5]}: gpu {gs[bad[:5]]},{gv[bad[:5]]} oracle {os_[bad[:5]]},{ov[bad[:5]]}"
    for x, y in zip(E.value_state(0, resources), O.value_state(0, resources)):
        assert np.array_equal(x, y)
    assert E.applied_index() == O.applied_index()


@pytest.mark.parametrize("n,resources,seed,hot,p_hot", [
    (1, 64, 1, 0, 0.0),
    (63, 64, 2, 0, 0.0),
    (65, 128, 3, 0, 0.0),
    (10_000, 64, 4, 0, 0.0),          # ~156 commits per slot: long same-slot chains in every step
    (50_000, 1000, 5, 4, 0.5),        # half the rows on 4 hot slots; ragged bucket (1000 % 64 != 0)
    (200_000, 65536, 6, 0, 0.0),
    (300_001, 4096, 7, 16, 0.2),
    (1_000_003, 256, 8, 1, 0.9),      # one slot takes 90% of the rows: 1800-long chains per chunk
    (700_000, 131072, 9, 0, 0.0),     # max_resources: 512 super-buckets
])
def test_value_random_parity(n, resources, seed, hot, p_hot):
    from copycat_amd.workload import value_random_stream

    max_inst = resources + 8
    b = value_random_stream(n, resources, max_inst, seed=seed, hot=hot, p_hot=p_hot)
    _assert_same(*_run_both(b, resources, max_inst), resources)


def test_value_multi_subbatch_and_batches():
    """Sub-batches inside one call (state carried across partitions) and across calls."""
    from copycat_amd.workload import value_random_stream

    resources, max_inst = 3000, 3100
    b = value_random_stream(100_000, resources, max_inst, seed=11, hot=8, p_hot=0.3)
    E, O, gs, gv, os_, ov = _run_both(b, resources, max_inst, sub_batch=16384 * 2,
                                      split=[(0, 1), (1, 40_000), (40_000, 40_000), (40_000, 100_000)])
    _assert_same(E, O, gs, gv, os_, ov, resources)


def test_atomic_long_stream_parity():
    """Config-2 client-model stream (Get + CompareAndSet) at 2M rows over 64K resources."""
    from copycat_amd.workload import atomic_long_stream

    R = 65536
    b = atomic_long_stream(2_000_000, resources=R)
    E, O, gs, gv, os_, ov = _run_both(b, R, R)
    _assert_same(E, O, gs, gv, os_, ov, R)
    cas = b.op == abi.CC_OP_VALUE_CAS
    ok = gv[cas] == 1
    assert 0.85 < ok.mean() < 0.95  # ~10% stale CAS fail (stream model)


def test_device_resident_apply_matches_host_path():
    import torch

    from copycat_amd.engine import DeviceBatch, Engine
    from copycat_amd.workload import value_random_stream

    R = 4096
    b = value_random_stream(123_457, R, R, seed=21, hot=3, p_hot=0.1)
    E1 = Engine(R, R, len(b))
    E1.resource_create_range(0, R, abi.CC_RES_VALUE)
    E1.instance_open_range(0, R, 0, 1000, 7)
    E2 = Engine(R, R, len(b), sub_batch=20000)
    E2.resource_create_range(0, R, abi.CC_RES_VALUE)
    E2.instance_open_range(0, R, 0, 1000, 7)
    s1, v1 = E1.apply_host(b)
    db = DeviceBatch.upload(b)
    st = torch.zeros(len(b), dtype=torch.uint8, device="cuda")
    va = torch.zeros(len(b), dtype=torch.int64, device="cuda")
    E2.apply(db, st, va)
    E2.sync()
    assert np.array_equal(st.cpu().numpy(), s1)
    assert np.array_equal(va.view(torch.int64).cpu().numpy().view(np.uint64), v1)
    for x, y in zip(E1.value_state(), E2.value_state()):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("map_capacity", [0, 1024])
def test_cas_update_deltas_at_the_record_boundary(map_capacity):
    """Chains of CASes that always succeed (AtomicValueState.compareAndSet :123-133), with differences of every size
    (0, +-1, both sides of 2^32, the i64 wrap), tag changes (Long -> Integer -> null) and expected NULLs, are bit-exact
    against the oracle -- on the value-only pipeline (k_part_v4 -> k_apply_value_v3, whose 8-byte records escape to
    the batch columns for every difference past 14 bits) and, with map_capacity > 0, on the extended one (k_part_ext
    -> k_apply_value_ws, which carries whole operands)."""
    R, steps = 512, 48
    deltas = [0, 1, -1, (1 << 32) - 1, -(1 << 32), 1 << 32, -(1 << 32) - 1, (1 << 32) + 1, -(1 << 32) + 1,
              (1 << 31), -(1 << 31) - 1, (1 << 63), (1 << 64) - 1, 12345678901234, -(1 << 62), (1 << 46) + 3]
    rng = np.random.default_rng(3)
    cur = np.zeros(R, np.uint64)
    ctag = np.zeros(R, np.uint8)
    rows = []
    for k in range(steps):
        for r in rng.permutation(R):
            d = deltas[(k + r) % len(deltas)] if k % 7 else int(rng.integers(0, 1 << 63))
            ntag = abi.CC_TAG_LONG if (k + r) % 11 else (abi.CC_TAG_INT if (k + r) % 2 else abi.CC_TAG_NULL)
            upd = (int(cur[r]) + d) % (1 << 64) if ntag != abi.CC_TAG_NULL else 0
            if ntag == abi.CC_TAG_INT:
                upd = upd & 0x7FFFFFFF
            rows.append((r, abi.CC_OP_VALUE_CAS, int(ctag[r]) | (ntag << 3), int(cur[r]), upd))
            cur[r], ctag[r] = upd, ntag
            if (k + r) % 13 == 0:
                rows.append((r, abi.CC_OP_VALUE_GET, 0, 0, 0))
    n = len(rows)
    arr = np.array(rows, dtype=object)
    b = Batch.from_columns(index=np.arange(1, n + 1, dtype=np.uint64), time=np.arange(1, n + 1, dtype=np.uint64),
                           inst=np.array(arr[:, 0], np.uint32), op=np.array(arr[:, 1], np.uint8),
                           flags=np.array(arr[:, 2], np.uint8), a=np.array([int(x) for x in arr[:, 3]], np.uint64),
                           b=np.array([int(x) for x in arr[:, 4]], np.uint64))
    # both sides of the boundary occur among the Long -> Long CASes
    ll = (b.op == abi.CC_OP_VALUE_CAS) & (b.flags == (abi.CC_TAG_LONG | (abi.CC_TAG_LONG << 3)))
    dd = (b.b[ll] - b.a[ll]).view(np.int64)
    for d in ((1 << 32) - 1, -(1 << 32), 1 << 32, -(1 << 32) - 1):
        assert np.any(dd == d), d
    E, O, gs, gv, os_, ov = _run_both(b, R, R, sub_batch=16384 * 2, map_capacity=map_capacity)
    _assert_same(E, O, gs, gv, os_, ov, R)
    cas = b.op == abi.CC_OP_VALUE_CAS
    assert np.all(gv[cas] == 1)  # every CAS expected the value it found


@pytest.mark.parametrize("n,sub", [(8191, 0), (8193, 0), (16384 * 3 + 8191, 16384), (100_001, 16384 * 2)])
def test_value_ragged_tiles_and_sub_batches(n, sub):
    """Batches that end inside an 8192-commit tile, and sub-batches of whole 16384-commit multiples."""
    from copycat_amd.workload import atomic_long_stream

    R = 4096
    b = atomic_long_stream(n, resources=R)
    _assert_same(*_run_both(b, R, R + 8, sub_batch=sub), R)


@pytest.mark.parametrize("offset", [1, 2, 4])
def test_value_partition_byte_columns_at_any_alignment(offset):
    """k_part_v4 loads a full tile's op / flags columns as 4-row words when both column pointers are 4-byte aligned,
    and byte by byte otherwise (and for a partial tile): the same results from op / flags columns that start 1, 2
    or 4 bytes into their buffers, against the host path on aligned columns (itself checked against the oracle)."""
    import torch

    from copycat_amd.engine import DeviceBatch, Engine
    from copycat_amd.workload import atomic_long_stream

    R = 65536
    b = atomic_long_stream(100_003, resources=R, seed=17)  # 12 full 8192-row tiles and a partial one
    E1 = Engine(R, R, len(b))
    E1.resource_create_range(0, R, abi.CC_RES_VALUE)
    E1.instance_open_range(0, R, 0, 1000, 7)
    s1, v1 = E1.apply_host(b)
    E2 = Engine(R, R, len(b))
    E2.resource_create_range(0, R, abi.CC_RES_VALUE)
    E2.instance_open_range(0, R, 0, 1000, 7)
    db = DeviceBatch.upload(b)
    for name in ("op", "flags"):
        buf = torch.zeros(len(b) + offset, dtype=torch.uint8, device="cuda")
        buf[offset:] = db.cols[name]
        db.cols[name] = buf[offset:]
        assert db.cols[name].data_ptr() % 4 == offset % 4
    st = torch.full((len(b),), 0xFF, dtype=torch.uint8, device="cuda")
    va = torch.zeros(len(b), dtype=torch.int64, device="cuda")
    E2.apply(db, st, va)
    E2.sync()
    assert np.array_equal(st.cpu().numpy(), s1)
    assert np.array_equal(va.cpu().numpy().view(np.uint64), v1)
    for x, y in zip(E1.value_state(), E2.value_state()):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("map_capacity", [0, 1024])
def test_value_record_operand_boundaries(map_capacity):
    """value_path.hip's 8-byte record packs a CAS's expected value as a 32-bit and its update as a 14-bit two's
    complement difference, and a set / getAndSet value as a 46-bit number; a commit whose operands do not fit escapes
    (its tile row is kept and the apply reads the a / b columns).  Values and differences on both sides of each
    boundary (2^31 - 1 / -2^31 fit, 2^31 / -2^31 - 1 escape; 8191 / -8192 fit, 8192 / -8193 escape; 2^45 - 1 / -2^45
    fit, 2^45 / -2^45 - 1 escape), with Long / Integer / null tags, and failing CASes on each side, are bit-exact
    against the oracle; so are results on both sides of the packed result word's 56-bit payload (get / getAndSet of
    2^55 - 1 / -2^55, packed, and 2^55 / -2^55 - 1, escaped to the value array) (AtomicValueState.java get :77-83, set :114-118, compareAndSet :123-133, getAndSet :138-144)."""
    R = 256
    M = 1 << 64
    exps = [0, 1, -1, (1 << 31) - 1, -(1 << 31), 1 << 31, -(1 << 31) - 1, (1 << 32), 1 << 62, -(1 << 63)]
    dels = [0, 1, -1, 8191, -8192, 8192, -8193, 1 << 20, -(1 << 40)]
    sets = [0, 5, -5, (1 << 45) - 1, -(1 << 45), 1 << 45, -(1 << 45) - 1, (1 << 63) - 1, -(1 << 63),
            (1 << 55) - 1, -(1 << 55), 1 << 55, -(1 << 55) - 1]
    rng = np.random.default_rng(11)
    L, I, N = abi.CC_TAG_LONG, abi.CC_TAG_INT, abi.CC_TAG_NULL
    rows = []
    for k in range(40):
        for r in range(R):
            e = exps[(k * 7 + r) % len(exps)]
            d = dels[(k * 3 + r) % len(dels)]
            sv = sets[(k + r * 5) % len(sets)]
            et = L if (k + r) % 9 else I
            if et == I:
                e &= 0x7FFFFFFF
            # set the expected value, then a CAS from it (succeeds), a CAS from a stale value (fails), a get,
            # a getAndSet to a set value, and a set to null every so often
            rows.append((r, abi.CC_OP_VALUE_SET, et, e % M, 0))
            rows.append((r, abi.CC_OP_VALUE_CAS, et | (L << 3), e % M, (e + d) % M))
            rows.append((r, abi.CC_OP_VALUE_CAS, L | (L << 3), (e + d + 1) % M, (e + 2 * d + 3) % M))
            rows.append((r, abi.CC_OP_VALUE_GET, 0, 0, 0))
            rows.append((r, abi.CC_OP_VALUE_GETANDSET, L, sv % M, 0))
            if (k + r) % 5 == 0:
                rows.append((r, abi.CC_OP_VALUE_SET, N, int(rng.integers(0, 1 << 62)), 0))
                rows.append((r, abi.CC_OP_VALUE_CAS, N | (L << 3), int(rng.integers(0, 1 << 62)), d % M))
    perm = np.arange(len(rows))
    n = len(rows)
    arr = np.array(rows, dtype=object)[perm]
    b = Batch.from_columns(index=np.arange(1, n + 1, dtype=np.uint64), time=np.arange(1, n + 1, dtype=np.uint64),
                           inst=np.array(arr[:, 0], np.uint32), op=np.array(arr[:, 1], np.uint8),
                           flags=np.array(arr[:, 2], np.uint8), a=np.array([int(x) for x in arr[:, 3]], np.uint64),
                           b=np.array([int(x) for x in arr[:, 4]], np.uint64))
    E, O, gs, gv, os_, ov = _run_both(b, R, R, sub_batch=16384 * 2, map_capacity=map_capacity)
    _assert_same(E, O, gs, gv, os_, ov, R)
    cas = b.op == abi.CC_OP_VALUE_CAS
    assert 0 < int(np.sum(gv[cas] == 1)) < int(np.sum(cas))  # both outcomes occur
