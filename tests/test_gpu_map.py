"""GPU parity: MapState key operations on the MI355X vs the CPU oracle, through the C-ABI.

Bar: bit-exact per-commit status/value, every map's final entries (key tag, key, value tag, value, commit
index) and the applied index (integer path, no tolerance)."""
import numpy as np
import pytest

from copycat_amd import abi
from copycat_amd.batch import Batch

pytestmark = pytest.mark.gpu


def _engines(maps, max_inst, max_batch, map_capacity, sub_batch=0, first_slot=0, flags=abi.CC_CFG_TIMERS_DEFERRED):
    from copycat_amd.engine import Engine
    from oracle.oracle_py import Oracle

    slots = first_slot + maps
    E = Engine(slots, max_inst, max_batch, map_capacity=map_capacity, sub_batch=sub_batch, flags=flags)
    O = Oracle(slots, max_inst, flags & abi.CC_CFG_TIMERS_DEFERRED)
    E.resource_create_range(first_slot, maps, abi.CC_RES_MAP)
    E.instance_open_range(first_slot, maps, first_slot, 1000, 7)
    for m in range(first_slot, slots):
        O.resource_create(m, abi.CC_RES_MAP)
        O.instance_open(m, m, 1000 + m, 7)
    from tests.handles import register_key_strings

    register_key_strings(E, O)  # String keys: java.util.HashMap places them by String.hashCode
    return E, O


def _apply_both(E, O, parts):
    out = []
    for part in parts:
        s, v = E.apply_host(part)
        s2, v2 = O.apply(part)
        out.append((s, v, s2, v2))
    return [np.concatenate([o[i] for o in out]) for i in range(4)]


def _assert_rows(gs, gv, os_, ov):
    bad = np.nonzero((gs != os_) | (gv != ov))[0]
    assert len(bad) == 0, (f"{len(bad)} rows differ; first {bad[:5]}: gpu {gs[bad[:5]]},{gv[bad[:5]]} "
                           f"oracle {os_[bad[:5]]},{ov[bad[:5]]}")


def _assert_maps(E, O, slots):
    for m in slots:
        g, o = E.map_entries(m), O.map_entries(m)
        for x, y, what in zip(g, o, ("key tag", "key", "value tag", "value", "commit index")):
            assert np.array_equal(x, y), f"map {m}: {what} differs ({len(g[0])} vs {len(o[0])} entries)"
    assert E.applied_index() == O.applied_index()


@pytest.mark.parametrize("n,maps,keys,seed,hot,p_hot,cap", [
    (1, 1, 4, 1, 0, 0.0, 1024),
    (100, 3, 8, 2, 0, 0.0, 1024),
    (10_000, 16, 64, 3, 0, 0.0, 8192),        # ~600 commits per map over ~150 keys: long same-key chains
    (200_000, 64, 256, 4, 2, 0.3, 65536),     # 30% of rows on 2 keys of 2 maps
    (500_001, 1000, 256, 5, 0, 0.0, 1 << 20),  # ragged sub-batch tail; 1024 regions
    (300_000, 7, 4, 6, 1, 0.9, 1024),         # one key takes 90% of the rows
])
def test_map_random_parity(n, maps, keys, seed, hot, p_hot, cap):
    from copycat_amd.workload import map_random_stream

    max_inst = maps + 8
    b = map_random_stream(n, maps, max_inst, keys=keys, seed=seed, hot=hot, p_hot=p_hot)
    E, O = _engines(maps, max_inst, n, cap)
    _assert_rows(*_apply_both(E, O, [b]))
    _assert_maps(E, O, range(maps))


def test_map_table_bulk_readback():
    """cc_read_map_table (every map's entries in one table pass, sorted by slot, key tag, key) equals the per-map
    readback and the oracle's maps."""
    from copycat_amd.workload import map_random_stream

    maps = 37
    b = map_random_stream(60_000, maps, maps + 8, keys=64, seed=81, hot=2, p_hot=0.3)
    E, O = _engines(maps, maps + 8, len(b), 65536)
    _assert_rows(*_apply_both(E, O, [b]))
    sl, kt, k, vt, v, ci = E.map_table()
    assert np.all(np.diff(sl.astype(np.int64)) >= 0)
    bounds = np.searchsorted(sl, np.arange(maps + 1))
    for m in range(maps):
        a, z = bounds[m], bounds[m + 1]
        one = E.map_entries(m)
        for x, y in zip((kt[a:z], k[a:z], vt[a:z], v[a:z], ci[a:z]), one):
            assert np.array_equal(x, y), m
        for x, y in zip(one, O.map_entries(m)):
            assert np.array_equal(x, y), m


@pytest.mark.parametrize("n,sub_batch,hot,p_hot,seed", [
    (400_000, 65536, 8, 0.6, 41),    # 7 sub-batches; each hot key ~5K commits per sub-batch: 2 scan pieces
    (2_000_000, 0, 8, 0.6, 42),      # one sub-batch: ~37 pieces per hot key (carry across many pieces)
    (6_000_000, 0, 1, 0.9, 43),      # one key takes 90%: ~5,300 pieces in one sub-batch (k_hot_carry's long scan)
    (300_000, 0, 1, 0.97, 43),       # one key takes 97%: ~71 pieces
])
def test_map_hot_key_scan_parity(n, sub_batch, hot, p_hot, seed):
    """Hot keys (detected per sub-batch) applied by the multi-workgroup scan: every key op except the
    value-comparing ones, which force the sequential path (covered by test_map_random_parity)."""
    from copycat_amd.workload import map_random_stream

    maps, max_inst = 16, 24
    b = map_random_stream(n, maps, max_inst, keys=64, seed=seed, hot=hot, p_hot=p_hot, value_compare_ops=False)
    E, O = _engines(maps, max_inst, n, 8192, sub_batch=sub_batch)
    _assert_rows(*_apply_both(E, O, [b]))
    _assert_maps(E, O, range(maps))


def test_map_multi_subbatch_and_batches():
    """Table state carried across sub-batches inside one call and across calls."""
    from copycat_amd.workload import map_random_stream

    maps, max_inst, n = 40, 48, 150_000
    b = map_random_stream(n, maps, max_inst, keys=128, seed=11, hot=4, p_hot=0.2)
    E, O = _engines(maps, max_inst, n, 32768, sub_batch=16384 * 2)
    parts = [b.slice(lo, hi) for lo, hi in [(0, 1), (1, 50_000), (50_000, 50_000), (50_000, n)]]
    _assert_rows(*_apply_both(E, O, parts))
    _assert_maps(E, O, range(maps))


def test_maps_and_values_in_one_engine():
    """AtomicValue and Map resources side by side: each commit goes to its own kernel, results interleave."""
    from copycat_amd.engine import Engine
    from copycat_amd.workload import map_random_stream, value_random_stream
    from oracle.oracle_py import Oracle

    V, M = 192, 64  # value slots [0, 192), map slots [192, 256)
    slots, max_inst = V + M, V + M + 8
    bv = value_random_stream(120_000, V, max_inst, seed=31, hot=4, p_hot=0.2)
    bm = map_random_stream(100_000, M, max_inst, keys=64, first_inst=V, seed=32, hot=2, p_hot=0.2)
    rng = np.random.default_rng(5)
    order = rng.permutation(len(bv) + len(bm))
    cols = {}
    for name, _ in abi.BATCH_COLUMNS:
        cols[name] = np.concatenate([getattr(bv, name), getattr(bm, name)])[order]
    cols["index"] = np.arange(1, len(order) + 1, dtype=np.uint64)
    b = Batch.from_columns(**cols)
    E = Engine(slots, max_inst, len(b), map_capacity=65536)
    O = Oracle(slots, max_inst)
    E.resource_create_range(0, V, abi.CC_RES_VALUE)
    E.resource_create_range(V, M, abi.CC_RES_MAP)
    E.instance_open_range(0, slots, 0, 1000, 7)
    for r in range(slots):
        O.resource_create(r, abi.CC_RES_VALUE if r < V else abi.CC_RES_MAP)
        O.instance_open(r, r, 1000 + r, 7)
    from tests.handles import register_key_strings

    register_key_strings(E, O)
    _assert_rows(*_apply_both(E, O, [b]))
    for x, y in zip(E.value_state(0, V), O.value_state(0, V)):
        assert np.array_equal(x, y)
    _assert_maps(E, O, range(V, slots))


def _puts(keys, slot_inst, op=abi.CC_OP_MAP_PUT, index0=1):
    n = len(keys)
    return Batch.from_columns(index=np.arange(index0, index0 + n, dtype=np.uint64), inst=np.full(n, slot_inst),
                              op=np.full(n, op, np.uint8),
                              flags=np.full(n, abi.cc_flags(abi.CC_TAG_LONG, 0, 0), np.uint8),
                              key=np.asarray(keys, np.uint64), a=np.asarray(keys, np.uint64) * np.uint64(3))


def test_map_region_compaction():
    """Removed keys keep their entries until a launch finds the region > 3/4 bound and compacts it: without
    compaction the third batch would overflow the two 2048-entry regions."""
    E, O = _engines(1, 4, 4000, 2048)
    old = np.arange(3400, dtype=np.uint64) * np.uint64(7919) + np.uint64(11)
    new = old + np.uint64(1 << 40)
    b1 = _puts(old, 0)
    b2 = _puts(old, 0, op=abi.CC_OP_MAP_REMOVE, index0=3401)
    b3 = _puts(new, 0, index0=6801)
    _assert_rows(*_apply_both(E, O, [b1, b2, b3]))
    b4 = _puts(np.concatenate([old[:100], new[:100]]), 0, op=abi.CC_OP_MAP_GET, index0=10201)
    _assert_rows(*_apply_both(E, O, [b4]))
    _assert_maps(E, O, [0])


def test_map_capacity_error():
    from copycat_amd.engine import EngineError

    E, _ = _engines(1, 4, 8192, 1024)  # 2 regions of 2048 entries
    with pytest.raises(EngineError) as ei:
        E.apply_host(_puts(np.arange(6000, dtype=np.uint64), 0))
    assert ei.value.rc == abi.CC_ERR_CAPACITY


@pytest.mark.parametrize("sub_batch", [0, 32768])
def test_map_event_positions_across_index_gaps(sub_batch):
    """A small map's insertions (and size / containsValue rows' maps') are followed as events keyed by their log index
    within the sub-batch, 32 bits (common.h kEvPosBits).  A batch whose index column jumps by 2^33 several times (inside
    sub-batches, and across the batch) is cut by the host before each row 2^32 past its sub-batch's first
    (k_span_cut: round 5 failed such a call with CC_ERR_STATE); every row, every map and the applied index equal the
    oracle's, with random key ops, stored nulls, size / isEmpty and containsValue rows on small maps."""
    from copycat_amd.workload import map_random_stream

    n, maps = 120_000, 6
    b = map_random_stream(n, maps, maps, keys=40, seed=29)
    rng = np.random.default_rng(29)
    rows = rng.choice(n, 900, replace=False)
    b.op[rows[:300]] = abi.CC_OP_MAP_SIZE
    b.op[rows[300:600]] = abi.CC_OP_MAP_ISEMPTY
    b.op[rows[600:]] = abi.CC_OP_MAP_CONTAINSVALUE
    b.aux[rows] = 0
    for at in sorted(rng.choice(np.arange(1, n), 7, replace=False)):
        b.index[at:] += np.uint64(1 << 33)
    E, O = _engines(maps, maps, n, 4096, sub_batch=sub_batch)
    _assert_rows(*_apply_both(E, O, [b]))
    _assert_maps(E, O, range(maps))


def test_map_get_with_positive_aux_is_applied():
    """ttl is read by put/putIfAbsent/replace/replaceIfPresent only: a get row whose aux column holds a
    positive number is an ordinary get (MapCommands.java: Get carries no ttl)."""
    E, O = _engines(1, 4, 16, 1024)
    b = _puts([1, 2, 3], 0)
    b.op[2] = abi.CC_OP_MAP_GET
    b.key[2] = 1
    b.aux[2] = 99
    _assert_rows(*_apply_both(E, O, [b]))


def test_map_resource_delete_drops_entries():
    """ResourceManager.deleteResource -> MapState.delete (MapState.java:264-274): a map re-created in the
    same slot starts empty; other maps keep their entries."""
    E, O = _engines(2, 4, 64, 1024)
    b = _puts(np.arange(20, dtype=np.uint64), 0)
    b2 = _puts(np.arange(20, dtype=np.uint64), 1, index0=21)
    _apply_both(E, O, [b, b2])
    E.resource_delete(0)
    E.resource_create(0, abi.CC_RES_MAP)
    E.instance_open(0, 0, 5000, 7)
    assert len(E.map_entries(0)[0]) == 0
    g = _puts(np.arange(20, dtype=np.uint64), 0, op=abi.CC_OP_MAP_GET, index0=41)
    s, v = E.apply_host(g)
    assert (s == abi.cc_status(abi.CC_ST_OK, abi.CC_TAG_NULL)).all() and (v == 0).all()
    g2 = _puts(np.arange(20, dtype=np.uint64), 1, op=abi.CC_OP_MAP_GET, index0=61)
    s, v = E.apply_host(g2)
    assert (s == abi.cc_status(abi.CC_ST_OK, abi.CC_TAG_LONG)).all() and (v == np.arange(20) * 3).all()


def test_map_capacity_2m_live_entries():
    """map_capacity 2M (2048 table regions: the extended partition stages 1024-commit chunks so its per-bucket
    counters fit the LDS): 1.5M distinct keys put over 512 maps, then a random key-op stream over them."""
    from copycat_amd.workload import map_random_stream

    maps, max_inst, n0 = 512, 520, 1_500_000
    i = np.arange(n0, dtype=np.uint64)
    b0 = Batch.from_columns(index=i + np.uint64(1), inst=(i % np.uint64(maps)).astype(np.uint32),
                            op=np.full(n0, abi.CC_OP_MAP_PUT, np.uint8),
                            flags=np.full(n0, abi.cc_flags(abi.CC_TAG_LONG, 0, 0), np.uint8),
                            key=i // np.uint64(maps), a=i * np.uint64(7))
    b1 = map_random_stream(400_000, maps, max_inst, keys=4096, seed=404, index0=n0 + 1)
    E, O = _engines(maps, max_inst, n0, 2 << 20)
    _assert_rows(*_apply_both(E, O, [b0, b1]))
    _assert_maps(E, O, range(0, maps, 37))
    assert sum(len(E.map_entries(m)[0]) for m in range(0, maps, 64)) > 1_500_000 // 64  # well past 1M live in all


def test_map_zipf_stream_parity():
    """Config-3 stream (Zipf 0.99 put/get/remove over 1M (map, key) pairs, 4096 maps) at 2M rows."""
    from copycat_amd.workload import map_zipf_rows

    n, maps = 2_000_000, 4096
    b = map_zipf_rows(0, n, maps=maps)
    E, O = _engines(maps, maps, n, 1 << 20)
    _assert_rows(*_apply_both(E, O, [b]))
    _assert_maps(E, O, range(0, maps, 97))


@pytest.mark.parametrize("sub_batch", [16384, 65536])
def test_small_maps_leave_window_beside_hot_keys(sub_batch):
    """Maps that start empty and pass 64 entries one sub-batch after another, hot keys among them.  Each sub-batch's
    small-map replay runs on the side stream and clears a map's small flag while the next sub-batch's hot-key and
    region kernels decide whether its commits are map events (a flag they must read once per workgroup item and
    per position: DESIGN.md, round 5).  Short sub-batches make every replay overlap the next sub-batch."""
    from copycat_amd.workload import map_zipf_rows

    n, maps = 1_500_000, 256
    b = map_zipf_rows(0, n, maps=maps, pairs=1 << 16, s=0.99, seed=777)
    E, O = _engines(maps, maps, n, 1 << 18, sub_batch=sub_batch)
    parts = [b.slice(0, n // 3), b.slice(n // 3, n)]
    _assert_rows(*_apply_both(E, O, parts))
    _assert_maps(E, O, range(maps))
    assert E.counters()[3] > 0  # the small maps' events were followed


# ---- whole-map ops: containsValue / size / isEmpty / clear / Delete (MapState.java:49-60, 233-274) ----------

_WIDE = np.array([abi.CC_OP_MAP_SIZE, abi.CC_OP_MAP_ISEMPTY, abi.CC_OP_MAP_CONTAINSVALUE, abi.CC_OP_MAP_CLEAR,
                  abi.CC_OP_DELETE], np.uint8)


def _with_barriers(b, rate, seed, ops=_WIDE, p=None):
    """Turn a share of a key-op stream's rows into whole-map ops (operand a of containsValue: a small Long)."""
    rng = np.random.default_rng(seed)
    rows = np.nonzero(rng.random(len(b)) < rate)[0]
    b.op[rows] = rng.choice(ops, size=len(rows), p=p)
    cv = rows[b.op[rows] == abi.CC_OP_MAP_CONTAINSVALUE]
    b.a[cv] = rng.integers(0, 3, len(cv)).astype(np.uint64)
    b.flags[cv] = (b.flags[cv] & np.uint8(0xF8)) | np.uint8(abi.CC_TAG_LONG)
    return rows


def _no_null_values(b):
    """Key ops store non-null values only: containsValue is then independent of HashMap iteration order."""
    f = b.flags
    ta, tb = f & 7, (f >> 3) & 7
    f[ta == abi.CC_TAG_NULL] |= np.uint8(abi.CC_TAG_LONG)
    f[tb == abi.CC_TAG_NULL] |= np.uint8(abi.CC_TAG_LONG << 3)


@pytest.mark.parametrize("n,maps,keys,rate,sub_batch,hot,p_hot,seed", [
    (2_000, 2, 16, 0.02, 0, 0, 0.0, 71),
    (50_000, 8, 64, 0.002, 0, 0, 0.0, 72),
    (200_000, 64, 256, 0.0005, 32768, 2, 0.3, 73),   # barriers inside and across sub-batches, hot keys
])
def test_map_wide_ops_parity(n, maps, keys, rate, sub_batch, hot, p_hot, seed):
    """size/isEmpty/containsValue/clear/Delete rows split the batch into segments; each is applied against the
    table exactly as it stands at its log position."""
    from copycat_amd.workload import map_random_stream

    max_inst = maps + 8
    b = map_random_stream(n, maps, max_inst, keys=keys, seed=seed, hot=hot, p_hot=p_hot)
    _no_null_values(b)
    rows = _with_barriers(b, rate, seed)
    assert len(rows) > 0
    E, O = _engines(maps, max_inst, n, 65536, sub_batch=sub_batch)
    gs, gv, os_, ov = _apply_both(E, O, [b])
    _assert_rows(gs, gv, os_, ov)
    _assert_maps(E, O, range(maps))
    wide = gs[rows]
    assert (wide == abi.cc_status(abi.CC_ST_OK, abi.CC_TAG_INT)).any()  # some size rows landed on live maps


def _cv_rows(b, rate, seed, clear_rate=0.0):
    """Turn a share of a stream's rows into containsValue rows whose operand is the value an earlier put of the same
    map stored (so many answers are true), and another share into clears."""
    rng = np.random.default_rng(seed)
    n = len(b)
    rows = np.nonzero(rng.random(n) < rate)[0]
    puts = np.nonzero(b.op == abi.CC_OP_MAP_PUT)[0]
    back = np.searchsorted(puts, rows) - 1 - rng.integers(0, 40, len(rows))
    src = puts[np.clip(back, 0, len(puts) - 1)]
    inst, a, tag = b.inst[src].copy(), b.a[src].copy(), (b.flags[src] & np.uint8(7)).copy()
    b.op[rows] = abi.CC_OP_MAP_CONTAINSVALUE
    b.inst[rows] = inst
    b.a[rows] = a
    b.flags[rows] = tag
    if clear_rate:
        cl = np.nonzero(rng.random(n) < clear_rate)[0]
        cl = cl[b.op[cl] != abi.CC_OP_MAP_CONTAINSVALUE]
        b.op[cl] = abi.CC_OP_MAP_CLEAR
    return rows


@pytest.mark.parametrize("n,maps,keys,sub_batch,hot,p_hot,seed", [
    (3_000, 2, 16, 0, 0, 0.0, 301),
    (100_000, 16, 64, 8192, 2, 0.3, 302),
    (400_000, 64, 256, 32768, 4, 0.4, 303),
])
def test_map_contains_value_in_stream_parity(n, maps, keys, sub_batch, hot, p_hot, seed):
    """containsValue answered in the stream (map_cv.hip): maps with even slots store no null, so their containsValue
    rows need no barrier; odd maps keep their nulls (their rows stay barriers, answered in HashMap order), and one even
    map stores a null mid-batch (its rows after that become barriers).  Operands are values the stream stored; clears,
    hot keys and several sub-batches run through the same batch.  Every row and every map as the oracle has them."""
    from copycat_amd.workload import map_random_stream

    max_inst = maps + 8
    b = map_random_stream(n, maps, max_inst, keys=keys, seed=seed, hot=hot, p_hot=p_hot)
    even = (b.inst % 2) == 0
    f = b.flags
    ta, tb = f & 7, (f >> 3) & 7
    f[even & (ta == abi.CC_TAG_NULL)] |= np.uint8(abi.CC_TAG_LONG)
    f[even & (tb == abi.CC_TAG_NULL)] |= np.uint8(abi.CC_TAG_LONG << 3)
    rows = _cv_rows(b, 0.02, seed, clear_rate=0.0005)
    mid = n // 2
    b.op[mid], b.inst[mid], b.flags[mid] = abi.CC_OP_MAP_PUT, 0, np.uint8(abi.CC_TAG_NULL)  # a null into map 0
    E, O = _engines(maps, max_inst, n, 65536, sub_batch=sub_batch)
    c0 = E.counters()
    gs, gv, os_, ov = _apply_both(E, O, [b])
    _assert_rows(gs, gv, os_, ov)
    _assert_maps(E, O, range(maps))
    c1 = E.counters()
    assert c1[1] > c0[1]  # rows answered in the stream
    assert c1[0] > c0[0]  # and barrier rows (odd maps, map 0 after its null, clears)
    ok_bool = gs[rows] == abi.cc_status(abi.CC_ST_OK, abi.CC_TAG_BOOL)
    assert (gv[rows][ok_bool] == 1).any() and (gv[rows][ok_bool] == 0).any()


def test_map_contains_value_in_stream_zipf():
    """The c3 stream (Zipf 0.99 over 1M (map, key) pairs, 4096 maps, hot keys) with 0.1 % containsValue rows (operands:
    values stored shortly before, 64-bit: fingerprinted operands) and 0.01 % clears: every containsValue row is
    answered in the stream, every row as the oracle has it."""
    from copycat_amd.workload import map_zipf_rows

    n, maps = 2_000_000, 4096
    b = map_zipf_rows(0, n, maps=maps)
    rows = _cv_rows(b, 0.001, 911, clear_rate=0.0001)
    E, O = _engines(maps, maps, n, 1 << 20)
    c0 = E.counters()
    gs, gv, os_, ov = _apply_both(E, O, [b])
    _assert_rows(gs, gv, os_, ov)
    _assert_maps(E, O, range(0, maps, 97))
    c1 = E.counters()
    assert c1[1] - c0[1] == len(rows)
    assert (gv[rows] == 1).any() and (gv[rows] == 0).any()


def _cv_fingerprint(m, tag, v):
    """common.h cv_key for an operand past 43 bits: the 63-bit hashed fingerprint (restated for the collision test)."""
    M = (1 << 64) - 1
    h = ((v ^ ((((m & 0x1FFFF) << 3) | (tag & 7)) * 0xC2B2AE3D27D4EB4F & M)) * 0x9E3779B97F4A7C15) & M
    h ^= h >> 31
    h = (h * 0xBF58476D1CE4E5B9) & M & ~(1 << 63)
    return h or 1


def _cv_colliding_value(m, tag, v1):
    """A second operand of map m (same tag) whose fingerprint equals v1's: invert the hash chain from v1's pre-mask
    value with bit 63 flipped (both mask to the same 63 bits)."""
    M = (1 << 64) - 1
    s = ((((m & 0x1FFFF) << 3) | (tag & 7)) * 0xC2B2AE3D27D4EB4F) & M
    x = ((v1 ^ s) * 0x9E3779B97F4A7C15) & M
    x ^= x >> 31
    z = (x * 0xBF58476D1CE4E5B9) & M
    z ^= 1 << 63
    u = (z * pow(0xBF58476D1CE4E5B9, -1, 1 << 64)) & M
    u ^= (u >> 31) ^ (u >> 62)  # the inverse of x ^= x >> 31
    w = (u * pow(0x9E3779B97F4A7C15, -1, 1 << 64)) & M
    v2 = w ^ s
    assert v2 != v1 and _cv_fingerprint(m, tag, v2) == _cv_fingerprint(m, tag, v1)
    return v2


def test_map_contains_value_fingerprint_collision_in_stream():
    """Two containsValue operands of one map whose 63-bit fingerprints are equal (constructed by inverting the hash):
    round 5 failed the call (kErrCvKey); now each gets its own set position (map_cv.hip k_cv_verify -> k_cv_fix) and
    every answer follows its own operand (MapState.containsValue :49-60): puts and removes of either value, queries of
    both, interleaved, several pairs and maps, against the oracle."""
    rng = np.random.default_rng(77)
    maps, n = 3, 6000
    pairs = []
    for m in range(maps):
        for _ in range(3):
            v1 = int(rng.integers(1 << 50, 1 << 62))
            pairs.append((m, v1, _cv_colliding_value(m, abi.CC_TAG_LONG, v1)))
    cols = {k: np.zeros(n, np.uint64) for k in ("index", "key", "a", "b", "aux", "time")}
    inst = np.zeros(n, np.uint32)
    op = np.zeros(n, np.uint8)
    fl = np.full(n, abi.cc_flags(abi.CC_TAG_LONG, 0, 0), np.uint8)
    for i in range(n):
        m, v1, v2 = pairs[int(rng.integers(0, len(pairs)))]
        inst[i] = m
        x = rng.random()
        cols["key"][i] = int(rng.integers(0, 8))
        if x < 0.45:
            op[i] = abi.CC_OP_MAP_PUT
            cols["a"][i] = v1 if rng.random() < 0.5 else v2
        elif x < 0.6:
            op[i] = abi.CC_OP_MAP_REMOVE
        else:
            op[i] = abi.CC_OP_MAP_CONTAINSVALUE
            cols["a"][i] = v1 if rng.random() < 0.5 else v2
    cols["index"][:] = np.arange(1, n + 1, dtype=np.uint64)
    b = Batch.from_columns(index=cols["index"], inst=inst, op=op, flags=fl, key=cols["key"], a=cols["a"])
    E, O = _engines(maps, maps, n, 4096)
    c0 = E.counters()
    gs, gv, os_, ov = _apply_both(E, O, [b])
    _assert_rows(gs, gv, os_, ov)
    _assert_maps(E, O, range(maps))
    cvr = op == abi.CC_OP_MAP_CONTAINSVALUE
    assert E.counters()[1] - c0[1] == int(cvr.sum())  # every one answered in the stream
    assert (gv[cvr] == 1).any() and (gv[cvr] == 0).any()


@pytest.mark.parametrize("n,maps,keys,clear_rate,sub_batch,hot,p_hot,seed", [
    (4_000, 2, 16, 0.02, 0, 0, 0.0, 501),            # small maps (the HashMap model) cleared in the stream
    (60_000, 4, 16, 0.05, 0, 0, 0.0, 502),           # > 127 clears of one map in one sub-batch: the host cuts it
    (200_000, 16, 1024, 0.003, 16384, 2, 0.3, 503),  # large maps, several sub-batches, hot keys of other maps
])
def test_map_clear_in_stream_parity(n, maps, keys, clear_rate, sub_batch, hot, p_hot, seed):
    """MapState.clear applied in the stream (map_clear.hip): a clear is an epoch; later commits see the map empty,
    sizes restart at 0, the HashMap keeps its capacity.  Mixed into the same batch: size / isEmpty rows (answered by
    the cleared maps' replay), containsValue rows on maps that store nulls (barriers, answered in HashMap order: the
    capacity and the small maps' models went through the clears), and stored values.  Every row and map as the oracle
    has them; no clear row is a barrier."""
    from copycat_amd.workload import map_random_stream

    max_inst = maps + 8
    b = map_random_stream(n, maps, max_inst, keys=keys, seed=seed, hot=hot, p_hot=p_hot)
    rng = np.random.default_rng(seed)
    rows = np.nonzero(rng.random(n) < clear_rate)[0]
    b.op[rows] = abi.CC_OP_MAP_CLEAR
    q = np.nonzero(rng.random(n) < 0.01)[0]
    q = q[b.op[q] != abi.CC_OP_MAP_CLEAR]
    b.op[q] = rng.choice(np.array([abi.CC_OP_MAP_SIZE, abi.CC_OP_MAP_ISEMPTY, abi.CC_OP_MAP_CONTAINSVALUE], np.uint8), len(q))
    cv = q[b.op[q] == abi.CC_OP_MAP_CONTAINSVALUE]
    b.a[cv] = rng.integers(0, 3, len(cv)).astype(np.uint64)
    b.flags[cv] = (b.flags[cv] & np.uint8(0xF8)) | np.uint8(abi.CC_TAG_LONG)
    E, O = _engines(maps, max_inst, n, 65536, sub_batch=sub_batch)
    c0 = E.counters()
    gs, gv, os_, ov = _apply_both(E, O, [b])
    _assert_rows(gs, gv, os_, ov)
    _assert_maps(E, O, range(maps))
    c1 = E.counters()
    live = (b.inst[rows] < maps)
    assert c1[0] - c0[0] <= len(q)  # barriers: containsValue rows only, never a clear
    assert live.sum() > 0


def test_map_contains_value_iteration_order():
    """A map holding both null values and matches: containsValue NPEs iff a null comes first in
    java.util.HashMap iteration order (A5, MapState.java:52).  Puts only, so the peak size (and with it the
    table capacity) is exact."""
    rng = np.random.default_rng(81)
    E, O = _engines(3, 8, 4096, 8192)
    idx = 1
    seen_npe = seen_true = 0
    for step in range(6):
        k = rng.integers(0, 1 << 40, 150).astype(np.uint64)
        b = _puts(k, int(step % 3), index0=idx)
        tags = rng.choice([abi.CC_TAG_NULL, abi.CC_TAG_LONG, abi.CC_TAG_INT], size=len(k), p=[0.1, 0.6, 0.3])
        b.flags[:] = tags.astype(np.uint8)
        b.a[:] = rng.integers(0, 40, len(k)).astype(np.uint64)
        b.key[::7] = (b.key[::7] & np.uint64(0x7FFFFFFF))  # Integer-sized keys in some rows
        b.flags[::7] |= np.uint8(1 << 6)                  # ... with the Integer key tag
        cv = np.arange(5, len(k), 5)
        b.op[cv] = abi.CC_OP_MAP_CONTAINSVALUE
        b.a[cv] = rng.integers(0, 40, len(cv)).astype(np.uint64)
        gs, gv, os_, ov = _apply_both(E, O, [b])
        _assert_rows(gs, gv, os_, ov)
        seen_npe += int((gs[cv] == abi.cc_status(abi.CC_ST_NULL_POINTER, abi.CC_TAG_NULL)).sum())
        seen_true += int(((gs[cv] == abi.cc_status(abi.CC_ST_OK, abi.CC_TAG_BOOL)) & (gv[cv] == 1)).sum())
        idx += len(k)
    assert seen_npe > 0 and seen_true > 0
    _assert_maps(E, O, range(3))


def _peak_stream(with_size, ttl_row=False):
    """Peak 30 (capacity 64) that no barrier observes, then 25 removes and 10 puts: the live size (15) and the
    bound entries (40) straddle a resize, and the map holds both nulls and matches of the final query."""
    keys = np.arange(30, dtype=np.uint64) * np.uint64(1 << 20) + np.uint64(5)
    b1 = _puts(keys, 0)
    b1.flags[::3] = np.uint8(abi.CC_TAG_NULL)  # some stored nulls
    b1.a[:] = 7
    if ttl_row:
        b1.time[:] = 1
        b1.aux[0] = 1 << 40  # a timer that never fires in the test: the engine enters TTL mode
    parts = [b1]
    if with_size:
        parts.append(_puts([0], 0, op=abi.CC_OP_MAP_SIZE, index0=31))
    parts.append(_puts(keys[:25], 0, op=abi.CC_OP_MAP_REMOVE, index0=40))
    b3 = _puts(np.arange(10, dtype=np.uint64) + np.uint64(1 << 50), 0, index0=70)
    b3.a[:] = 7
    parts.append(b3)
    q = _puts([0], 0, op=abi.CC_OP_MAP_CONTAINSVALUE, index0=90)
    q.a[:] = 7
    parts.append(q)
    if ttl_row:
        for p in parts[1:]:
            p.time[:] = 2
    return parts


def test_map_contains_value_exact_capacity():
    """The engine tracks every map's size and HashMap capacity exactly (launch_map_size): an order-dependent
    containsValue after an unobserved peak is answered as the reference answers it, with or without a size
    barrier at the peak, in one batch or over several (MapState.java:49-60)."""
    for with_size in (False, True):
        E, O = _engines(1, 4, 64, 1024)
        _assert_rows(*_apply_both(E, O, _peak_stream(with_size)))
        _assert_maps(E, O, [0])
        parts = _peak_stream(with_size)
        one = Batch.from_columns(**{name: np.concatenate([getattr(x, name) for x in parts]) for name, _ in abi.BATCH_COLUMNS})
        E, O = _engines(1, 4, 128, 1024)
        _assert_rows(*_apply_both(E, O, [one]))


def test_map_contains_value_ttl_mode_exact():
    """In TTL mode (entries also leave when timers fire) sizes and capacities stay exact: commits and expiries are
    replayed as events in log order (map_small.hip, common.h TtlEmit), so the order-dependent containsValue after an
    unobserved peak is answered as the reference answers it, with or without a size barrier at the peak."""
    for with_size in (False, True):
        E, O = _engines(1, 4, 64, 1024)
        _assert_rows(*_apply_both(E, O, _peak_stream(with_size, ttl_row=True)))
        _assert_maps(E, O, [0])


@pytest.mark.parametrize("flags", [abi.CC_CFG_TIMERS_DEFERRED, 0], ids=["manager", "module"])
@pytest.mark.parametrize("n,maps,keys,sub_batch,seed,clustered", [
    (40_000, 3, 40, 0, 401, False),             # sizes oscillate around the 24 / 48 thresholds; timers fire mid-batch
    (200_000, 12, 48, 16384 * 2, 402, True),    # several sub-batches; clustered keys: treeifyBin's early resizes
])
def test_map_contains_value_ttl_churn_parity(flags, n, maps, keys, sub_batch, seed, clustered):
    """TTL mode with stored nulls: put / remove churn where a share of the stores arm timers that fire inside the
    batch (module and manager order, A8), containsValue / size barriers, two batches, cc_advance_time, then a third
    batch of containsValue rows.  Every answer -- the order-dependent containsValue included -- matches the oracle
    (no CC_ERR_STATE), and every barrier checks the tracked size against the table."""
    from copycat_amd.workload import map_random_stream

    max_inst = maps + 8
    b = map_random_stream(n, maps, max_inst, keys=keys, seed=seed)
    if clustered:
        lk = (b.flags >> 6) == 0  # Long keys
        c = (b.inst.astype(np.uint64) % np.uint64(3)) + np.uint64(5)
        b.key[lk] = ((b.key[lk] & np.uint64(15)) << np.uint64(20)) + c[lk]
    _with_ttl(b, seed, p_ttl=0.3, max_ttl=120, step=4)
    rows = _with_barriers(b, 0.002, seed, ops=np.array([abi.CC_OP_MAP_CONTAINSVALUE, abi.CC_OP_MAP_SIZE], np.uint8),
                          p=[0.8, 0.2])
    E, O = _engines(maps, max_inst, n, 65536, sub_batch=sub_batch, flags=flags)
    cut = n // 2
    gs, gv, os_, ov = _apply_both(E, O, [b.slice(0, cut), b.slice(cut, n)])
    _assert_rows(gs, gv, os_, ov)
    _assert_maps(E, O, range(maps))
    cv = rows[b.op[rows] == abi.CC_OP_MAP_CONTAINSVALUE]
    npe = int((gs[cv] == abi.cc_status(abi.CC_ST_NULL_POINTER, abi.CC_TAG_NULL)).sum())
    assert 0 < npe < len(cv)  # both outcomes occur
    now = int(b.time[-1]) + 60  # some timers fire without a commit
    E.advance_time(now)
    O.advance_time(now)
    _assert_maps(E, O, range(maps))
    q = _puts(np.zeros(maps * 4, np.uint64), 0, op=abi.CC_OP_MAP_CONTAINSVALUE, index0=int(b.index[-1]) + 1)
    q.inst[:] = np.repeat(np.arange(maps, dtype=np.uint32), 4)
    q.a[:] = np.tile(np.arange(4, dtype=np.uint64), maps)
    q.time[:] = now + 1
    _assert_rows(*_apply_both(E, O, [q]))


@pytest.mark.parametrize("clustered", [False, True], ids=["spread", "clustered"])
@pytest.mark.parametrize("n,maps,keys,sub_batch,hot,p_hot,seed", [
    (60_000, 3, 40, 0, 0, 0.0, 301),             # sizes oscillate around the 24 / 48 thresholds inside tiles
    (400_000, 16, 48, 16384 * 3, 2, 0.3, 302),   # several sub-batches, hot keys (k_hot_apply deltas)
    (300_000, 200, 30, 0, 0, 0.0, 303),          # many maps, few commits per map per tile
])
def test_map_contains_value_churn_parity(n, maps, keys, sub_batch, hot, p_hot, seed, clustered):
    """Put / remove churn with stored nulls and containsValue / size barriers: every containsValue whose answer
    depends on HashMap iteration order uses the exact tracked capacity; every size barrier checks the tracked size
    against the table (the engine fails the batch on a difference).  Clustered: the Long keys are i * 2^20 + c
    (i < 16), so all 16 of a map's Long keys share a bin of 16 and 8 a bin of 32 -- with the Integer keys that
    join them treeifyBin resizes the table early (java.util.HashMap, MapState.java:33,49-60) -- while a bin of 64
    holds 4 of them (no tree bin)."""
    from copycat_amd.workload import map_random_stream

    max_inst = maps + 8
    b = map_random_stream(n, maps, max_inst, keys=keys, seed=seed, hot=hot, p_hot=p_hot)
    if clustered:
        lk = (b.flags >> 6) == 0  # Long keys
        c = (b.inst.astype(np.uint64) % np.uint64(3)) + np.uint64(5)
        b.key[lk] = ((b.key[lk] & np.uint64(15)) << np.uint64(20)) + c[lk]
    rows = _with_barriers(b, 0.0015, seed, ops=np.array([abi.CC_OP_MAP_CONTAINSVALUE, abi.CC_OP_MAP_SIZE], np.uint8),
                          p=[0.8, 0.2])
    cut = n // 2
    E, O = _engines(maps, max_inst, n, 65536, sub_batch=sub_batch)
    gs, gv, os_, ov = _apply_both(E, O, [b.slice(0, cut), b.slice(cut, n)])
    _assert_rows(gs, gv, os_, ov)
    _assert_maps(E, O, range(maps))
    cv = rows[b.op[rows] == abi.CC_OP_MAP_CONTAINSVALUE]
    npe = int((gs[cv] == abi.cc_status(abi.CC_ST_NULL_POINTER, abi.CC_TAG_NULL)).sum())
    assert 0 < npe < len(cv)  # both outcomes occur


def test_map_hot_placeholders_after_clear_then_ttl():
    """Hot-key candidates are counted once per batch and bound before every sub-batch, so after a clear / Delete
    barrier a sub-batch binds entries for keys its map no longer holds.  Those are placeholders (kMwUnseen): no key
    the map ever held, left out of the bound-key counts behind the tree-bin test.  Clears and containsValue rows
    mid-batch with hot keys over several sub-batches, then a batch that switches to TTL mode with more containsValue
    rows: every answer and every map's entries match the oracle."""
    from copycat_amd.workload import map_random_stream

    maps, n = 4, 120_000
    max_inst = maps + 8
    b = map_random_stream(n, maps, max_inst, keys=64, seed=71, hot=2, p_hot=0.5)
    _with_barriers(b, 0.0015, 71, ops=np.array([abi.CC_OP_MAP_CLEAR, abi.CC_OP_MAP_CONTAINSVALUE], np.uint8), p=[0.3, 0.7])
    E, O = _engines(maps, max_inst, n, 65536, sub_batch=16384 * 2)
    _assert_rows(*_apply_both(E, O, [b]))
    _assert_maps(E, O, range(maps))
    b2 = map_random_stream(40_000, maps, max_inst, keys=64, seed=72, hot=2, p_hot=0.5, index0=int(b.index[-1]) + 1)
    _with_ttl(b2, 72, p_ttl=0.2, max_ttl=200, step=4)
    b2.time[:] += np.uint64(int(b.time.max()))
    _with_barriers(b2, 0.002, 72, ops=np.array([abi.CC_OP_MAP_CONTAINSVALUE, abi.CC_OP_MAP_SIZE], np.uint8), p=[0.8, 0.2])
    _assert_rows(*_apply_both(E, O, [b2]))
    _assert_maps(E, O, range(maps))


def test_map_more_barrier_rows_than_one_listing():
    """More containsValue / clear rows in one batch than one barrier listing holds (kBarCap = 65,536): the engine
    applies the batch as consecutive halves (no CC_ERR_CAPACITY), every row as the oracle answers it."""
    from copycat_amd.workload import map_random_stream

    maps, n = 2, 150_000
    b = map_random_stream(n, maps, maps + 8, keys=16, seed=91)
    rng = np.random.default_rng(91)
    rows = np.sort(rng.choice(n, 70_000, replace=False))
    b.op[rows] = np.where(rng.random(len(rows)) < 0.98, abi.CC_OP_MAP_CONTAINSVALUE, abi.CC_OP_MAP_CLEAR).astype(np.uint8)
    b.a[rows] = rng.integers(0, 3, len(rows)).astype(np.uint64)
    b.flags[rows] = np.uint8(abi.cc_flags(abi.CC_TAG_LONG, 0, 0))
    E, O = _engines(maps, maps + 8, n, 4096)
    _assert_rows(*_apply_both(E, O, [b]))
    _assert_maps(E, O, range(maps))


def test_map_clear_then_reuse_keys():
    """clear / Delete drop every entry of one map (other maps keep theirs); the same keys are then re-put
    as new HashMap nodes; size and isEmpty follow."""
    E, O = _engines(2, 4, 256, 1024)
    k = np.arange(40, dtype=np.uint64)
    parts = [_puts(k, 0), _puts(k, 1, index0=41)]
    for i, op in enumerate([abi.CC_OP_MAP_SIZE, abi.CC_OP_MAP_CLEAR, abi.CC_OP_MAP_ISEMPTY, abi.CC_OP_MAP_SIZE]):
        parts.append(_puts([0], 0, op=op, index0=100 + i))
    parts.append(_puts(k[:10], 0, index0=200))
    parts.append(_puts([0, 0], 0, op=abi.CC_OP_MAP_SIZE, index0=300))
    parts.append(_puts([0], 1, op=abi.CC_OP_DELETE, index0=400))
    parts.append(_puts([0, 0], 1, op=abi.CC_OP_MAP_ISEMPTY, index0=500))
    one = Batch.from_columns(**{name: np.concatenate([getattr(x, name) for x in parts]) for name, _ in abi.BATCH_COLUMNS})
    _assert_rows(*_apply_both(E, O, [one]))
    _assert_maps(E, O, [0, 1])


# ---- TTL timers: put/putIfAbsent/replace/replaceIfPresent with ttl > 0 (MapState.java:91-93,119-121,189-192,218-220)

def _with_ttl(b, seed, p_ttl=0.4, max_ttl=300, step=8):
    """Log time advances by one every `step` rows; a share of the ttl-reading rows arm timers of 1..max_ttl."""
    rng = np.random.default_rng(seed)
    n = len(b)
    b.time[:] = np.arange(n, dtype=np.uint64) // np.uint64(step) + np.uint64(1000)
    arm = rng.random(n) < p_ttl
    b.aux[:] = np.where(arm, rng.integers(1, max_ttl, n), rng.choice([0, -5], n)).astype(np.int64).view(np.uint64)


@pytest.mark.parametrize("flags", [abi.CC_CFG_TIMERS_DEFERRED, 0], ids=["manager", "module"])
@pytest.mark.parametrize("n,maps,keys,sub_batch,seed", [
    (3_000, 2, 16, 0, 91),
    (120_000, 32, 128, 16384 * 2, 92),
])
def test_map_ttl_parity(flags, n, maps, keys, sub_batch, seed):
    """Entries expire when the reference's timer fires (before the commit in module mode, after the commit that
    advanced the clock in manager mode, A8); a later store re-arms or cancels; size sees only live entries;
    state read back between batches and after advance_time excludes expired keys."""
    from copycat_amd.workload import map_random_stream

    max_inst = maps + 8
    b = map_random_stream(n, maps, max_inst, keys=keys, seed=seed)
    _no_null_values(b)
    _with_ttl(b, seed)
    _with_barriers(b, 0.002, seed, ops=np.array([abi.CC_OP_MAP_SIZE, abi.CC_OP_MAP_CONTAINSVALUE, abi.CC_OP_MAP_ISEMPTY], np.uint8))
    E, O = _engines(maps, max_inst, n, 65536, sub_batch=sub_batch, flags=flags)
    cut = n // 3
    _assert_rows(*_apply_both(E, O, [b.slice(0, cut)]))
    _assert_maps(E, O, range(maps))
    _assert_rows(*_apply_both(E, O, [b.slice(cut, n)]))
    _assert_maps(E, O, range(maps))
    now = int(b.time[-1]) + 150
    E.advance_time(now)
    O.advance_time(now)
    _assert_maps(E, O, range(maps))


def test_map_ttl_expiry_boundary():
    """A put with ttl 10 at time 100 expires at 110: in manager mode a get at time 110 still sees it (the timer
    fires after that commit), in module mode it does not."""
    for flags, expect in ((abi.CC_CFG_TIMERS_DEFERRED, abi.CC_TAG_LONG), (0, abi.CC_TAG_NULL)):
        E, O = _engines(1, 4, 16, 1024, flags=flags)
        b = _puts([7, 7, 7], 0)
        b.op[1:] = abi.CC_OP_MAP_GET
        b.time[:] = [100, 109, 110]
        b.aux[0] = 10
        gs, gv, os_, ov = _apply_both(E, O, [b])
        _assert_rows(gs, gv, os_, ov)
        assert gs[1] == abi.cc_status(abi.CC_ST_OK, abi.CC_TAG_LONG)
        assert gs[2] == abi.cc_status(abi.CC_ST_OK, expect)


@pytest.mark.parametrize("seed", [901, 902])
def test_map_contains_value_compacting_churn_parity(seed):
    """The tree-bin test on churned maps whose regions compact (round-4 verdict): 3 maps of ~600 live keys each
    (table capacity 1024) churn through 1,200 keys apiece in a 2-region table, so removed keys are compacted away
    again and again; stored nulls; order-dependent containsValue rows decided inside one bin (keys come in pairs
    that share a bin at capacity 1024).  Every answer matches the oracle, and none fails with CC_ERR_STATE: a key
    counts toward the test only in the bins it shared before the table grew past them, and a compacted key counts
    once however often it comes back."""
    rng = np.random.default_rng(seed)
    maps = 3
    bases = [rng.choice(1024, 600, replace=False) for _ in range(maps)]
    univ = [np.concatenate([b, b + 1024]).astype(np.uint64) for b in bases]  # Long keys < 2^16: bin = key & (cap - 1)
    E, O = _engines(maps, maps + 8, 60_000, 2048)

    def rows(n, index0, fill=False):
        m = rng.integers(0, maps, n).astype(np.uint32)
        k = np.array([univ[x][i] for x, i in zip(m, rng.integers(0, 1200, n))], np.uint64)
        if fill:
            op = np.full(n, abi.CC_OP_MAP_PUT, np.uint8)
        else:
            op = rng.choice(np.array([abi.CC_OP_MAP_PUT, abi.CC_OP_MAP_REMOVE, abi.CC_OP_MAP_GET,
                                      abi.CC_OP_MAP_CONTAINSVALUE], np.uint8), n, p=[0.40, 0.40, 0.195, 0.005])
        nul = rng.random(n) < 0.3
        a = rng.integers(0, 4, n).astype(np.uint64)
        ta = np.where(nul & (op == abi.CC_OP_MAP_PUT), abi.CC_TAG_NULL, abi.CC_TAG_LONG).astype(np.uint8)
        return Batch.from_columns(index=np.arange(index0, index0 + n, dtype=np.uint64), inst=m, op=op,
                                  flags=(ta | (0 << 6)).astype(np.uint8), key=k, a=np.where(ta == 0, 0, a).astype(np.uint64))

    parts = [rows(2_100, 1, fill=True)]  # the tables grow 16 -> 1024 inside one batch (one sub-batch)
    for q in range(4):
        parts.append(rows(50_000, int(parts[-1].index[-1]) + 1))
    gs, gv, os_, ov = _apply_both(E, O, parts)
    _assert_rows(gs, gv, os_, ov)
    _assert_maps(E, O, range(maps))
    allop = np.concatenate([p.op for p in parts])
    cv = np.nonzero(allop == abi.CC_OP_MAP_CONTAINSVALUE)[0]
    npe = int((gs[cv] == abi.cc_status(abi.CC_ST_NULL_POINTER, abi.CC_TAG_NULL)).sum())
    true = int((gs[cv] == abi.cc_status(abi.CC_ST_OK, abi.CC_TAG_BOOL)).sum() and (gv[cv] == 1).sum())
    assert npe > 0 and true > 0  # both outcomes
    # and many of them decided inside one bin (a light model of the live keys: the lowest bin holding a null or a
    # match holds both; every table is at capacity 1024 after the fill)
    live = [dict() for _ in range(maps)]
    same = 0
    for p in parts:
        for i in range(len(p)):
            m, k, o = int(p.inst[i]), int(p.key[i]), int(p.op[i])
            if o == abi.CC_OP_MAP_PUT:
                live[m][k] = None if (p.flags[i] & 7) == abi.CC_TAG_NULL else int(p.a[i])
            elif o == abi.CC_OP_MAP_REMOVE:
                live[m].pop(k, None)
            elif o == abi.CC_OP_MAP_CONTAINSVALUE:
                v = int(p.a[i])
                nb = [kk & 1023 for kk, vv in live[m].items() if vv is None]
                mb = [kk & 1023 for kk, vv in live[m].items() if vv == v]
                same += bool(nb and mb and min(nb) == min(mb))
    assert same >= 20, same


@pytest.mark.parametrize("seed,nbin", [(601, 11), (602, 11), (603, 9)])
def test_small_map_alternating_chains_tree_bin(seed, nbin):
    """A small map (capacity <= 64) whose bin 5 holds nbin Long keys i * 2^22 + 5: 11 make it a red-black tree bin;
    9 leave a list chain of 9 at capacity 32 (treeifyBin's resize keeps it whole), where a put after a removal calls
    treeifyBin again (resize to 64, then a tree bin).  Long alternating remove / put chains of one key of that bin and
    of one key in a list bin, stored nulls, and containsValue rows whose answer is decided inside a bin
    (map_small.hip: chains compacted away in short list bins, applied one by one otherwise; the small model gives
    the bin's order).  Several sub-batches, hot keys."""
    rng = np.random.default_rng(seed)
    tree = [(i << 22) + 5 for i in range(nbin)]
    lst = [7, 8, 9, 40]
    L, N = abi.CC_TAG_LONG, abi.CC_TAG_NULL
    rows = [(abi.CC_OP_MAP_PUT, k, L, 1 + k % 3) for k in tree + lst]
    hot = [tree[3], lst[0]]
    while len(rows) < 60_000:
        u = rng.random()
        if u < 0.75:
            h = hot[int(rng.integers(2))]
            for _ in range(int(rng.integers(1, 14))):
                rows.append((abi.CC_OP_MAP_REMOVE, h, N, 0))
                rows.append((abi.CC_OP_MAP_PUT, h, L, int(rng.integers(1, 4))))
        elif u < 0.87:
            k = tree[int(rng.integers(len(tree)))]
            rows.append((abi.CC_OP_MAP_PUT, k, N if rng.random() < 0.3 else L, int(rng.integers(1, 4))))
        elif u < 0.93:
            k = (tree + lst)[int(rng.integers(len(tree) + len(lst)))]
            rows.append((abi.CC_OP_MAP_REMOVE, k, N, 0))
            if rng.random() < 0.7:
                rows.append((abi.CC_OP_MAP_PUT, k, L, int(rng.integers(1, 4))))
        else:
            rows.append((abi.CC_OP_MAP_CONTAINSVALUE, 0, L, int(rng.integers(1, 4))))
    op, key, tag, val = (np.array(c) for c in zip(*rows))
    n = len(op)
    b = Batch.from_columns(index=np.arange(1, n + 1, dtype=np.uint64), inst=np.zeros(n, np.uint32),
                           op=op.astype(np.uint8), flags=np.array([abi.cc_flags(int(t), 0, 0) for t in tag], np.uint8),
                           key=key.astype(np.uint64), a=val.astype(np.uint64))
    E, O = _engines(1, 4, n, 4096, sub_batch=16384)
    gs, gv, os_, ov = _apply_both(E, O, [b.slice(0, n // 3), b.slice(n // 3, n)])
    _assert_rows(gs, gv, os_, ov)
    _assert_maps(E, O, [0])
    cv = np.nonzero(op == abi.CC_OP_MAP_CONTAINSVALUE)[0]
    npe = int((gs[cv] == abi.cc_status(abi.CC_ST_NULL_POINTER, abi.CC_TAG_NULL)).sum())
    assert 0 < npe < len(cv)  # both outcomes occur


@pytest.mark.parametrize("flags", [abi.CC_CFG_TIMERS_DEFERRED, 0], ids=["manager", "module"])
@pytest.mark.parametrize("n,maps,keys,sub_batch,rate,seed", [
    (20_000, 3, 24, 0, 0.01, 701),               # sizes around the thresholds, timers firing between the rows
    (200_000, 40, 64, 16384 * 2, 0.003, 702),    # several sub-batches (boundaries owned by the next sub-batch)
])
def test_map_ttl_size_rows_in_stream(flags, n, maps, keys, sub_batch, rate, seed):
    """TTL mode: MapState.size / isEmpty rows are answered in the stream (k_ttl_replay: each query sits at its row's
    position among the commits and the expiries that fire at the boundaries before it), not as barriers; every answer,
    every map's entries and the applied index match the oracle, in both timer orders (A8)."""
    from copycat_amd.workload import map_random_stream

    max_inst = maps + 8
    b = map_random_stream(n, maps, max_inst, keys=keys, seed=seed)
    _with_ttl(b, seed, p_ttl=0.3, max_ttl=150, step=4)
    rows = _with_barriers(b, rate, seed, ops=np.array([abi.CC_OP_MAP_SIZE, abi.CC_OP_MAP_ISEMPTY], np.uint8))
    E, O = _engines(maps, max_inst, n, 65536, sub_batch=sub_batch, flags=flags)
    cut = n // 3
    gs0, gv0, os0, ov0 = _apply_both(E, O, [b.slice(0, cut)])  # (this batch turns TTL mode on)
    _assert_rows(gs0, gv0, os0, ov0)
    c0 = E.counters()
    gs, gv, os_, ov = _apply_both(E, O, [b.slice(cut, n)])
    _assert_rows(gs, gv, os_, ov)
    _assert_maps(E, O, range(maps))
    assert E.counters()[0] == c0[0]  # no barrier row in the TTL-mode batch
    later = rows[rows >= cut] - cut
    assert len(later) > 0
    sizes = gv[later][b.op[later + cut] == abi.CC_OP_MAP_SIZE]
    assert len(np.unique(sizes)) > 2  # the sizes move
