"""GPU parity: containsValue on maps whose table grew past 64 with a red-black tree bin (map_big.hip, big_jhm.h).

MapState.containsValue (collections/src/main/java/io/atomix/collections/state/MapState.java:49-60) answers by the
first stored null or match in java.util.HashMap iteration order.  A bin that was a tree bin keeps a tree-derived chain
order through every resize (TreeNode.split: halves of <= 6 nodes untreeified, larger ones re-treeified), so after the
table grows past 64 the answer inside such a bin is neither creation order nor hash order.  The engine hands such a
map to a big model when its table passes 64 and follows it node for node from there.

Bar: bit-exact per-commit status / value against the oracle (oracle/oracle.cpp, whose JHM is cross-checked against
tests/java_hashmap.py by tests/test_oracle_hashmap.py), every map's final entries, and no CC_ERR_STATE refusal."""
import numpy as np
import pytest

from copycat_amd import abi
from copycat_amd.batch import Batch
from tests.java_hashmap import MapStateModel
from tests.test_gpu_map import _apply_both, _assert_maps, _assert_rows, _engines

pytestmark = pytest.mark.gpu

L, N = abi.CC_TAG_LONG, abi.CC_TAG_NULL


def _batch(rows, index0, inst=None):
    op, key, tag, val = (np.array(c) for c in zip(*rows))
    n = len(op)
    return Batch.from_columns(index=np.arange(index0, index0 + n, dtype=np.uint64),
                              inst=np.zeros(n, np.uint32) if inst is None else np.asarray(inst, np.uint32),
                              op=op.astype(np.uint8), flags=np.array([abi.cc_flags(int(t), 0, 0) for t in tag], np.uint8),
                              key=key.astype(np.uint64), a=val.astype(np.uint64))


def _decided_in_tree_family(model, v):
    """containsValue(v) on the model: the first null and the first match share one bin whose index is 5 mod 64 (the
    bin that was a tree bin at capacity 64, and the bins it split into)."""
    tab = model.hm.table
    if tab is None:
        return False
    first = {}
    for b, e in enumerate(tab):
        while e is not None:
            s = model.vals[e.key]
            kind = "null" if s is None else ("match" if s == v else None)
            if kind and kind not in first:
                first[kind] = b
            e = e.next
    return len(first) == 2 and first["null"] == first["match"] and first["null"] % 64 == 5


def _tree_rows(rng, n_tree, n_other, churn, clear_rate=0.0, shift=22):
    """Fill: n_tree Long keys i * 2^shift + 5 (shift 22: one bin at every capacity <= 64, a tree bin at 64; shift 26:
    one bin at every capacity <= 1,024) holding null or 1..3,
    and n_other keys in other bins holding values no query asks; the table grows to 16 << k past 64.  Churn: puts
    (null or 1..3) and removals of the tree keys (trees split, untreeify and re-treeify), puts / removals of the
    others (the size stays above the fill's threshold), containsValue(1..3)."""
    tree = [(i << shift) + 5 for i in range(n_tree)]
    other = [k for k in range(1000, 1000 + 2 * n_other) if k % 64 != 5][:n_other]
    rows = []
    for i, k in enumerate(tree):
        rows.append((abi.CC_OP_MAP_PUT, k, N if i % 3 == 0 else L, 1 + i % 3))
    for j, k in enumerate(other):
        rows.append((abi.CC_OP_MAP_PUT, k, L, 100 + j))
        if j % 97 == 0:
            rows.append((abi.CC_OP_MAP_CONTAINSVALUE, 0, L, 1 + j % 3))
    while len(rows) < churn:
        u = rng.random()
        if u < 0.35:
            k = tree[int(rng.integers(n_tree))]
            rows.append((abi.CC_OP_MAP_PUT, k, N if rng.random() < 0.3 else L, int(rng.integers(1, 4))))
        elif u < 0.6:
            rows.append((abi.CC_OP_MAP_REMOVE, tree[int(rng.integers(n_tree))], N, 0))
        elif u < 0.8:
            k = other[int(rng.integers(n_other))]
            rows.append((abi.CC_OP_MAP_PUT if rng.random() < 0.55 else abi.CC_OP_MAP_REMOVE, k, L, 100))
        elif u < 0.8 + clear_rate:
            rows.append((abi.CC_OP_MAP_CLEAR, 0, N, 0))
        else:
            rows.append((abi.CC_OP_MAP_CONTAINSVALUE, 0, L, int(rng.integers(1, 4))))
    return rows


def _count_tree_decided(rows):
    m = MapStateModel()
    n = 0
    cap = 0
    for op, k, t, v in rows:
        if op == abi.CC_OP_MAP_PUT:
            m.put((1, k), None if t == N else v)
        elif op == abi.CC_OP_MAP_REMOVE:
            m.remove((1, k))
        elif op == abi.CC_OP_MAP_CLEAR:
            m.clear()
        elif op == abi.CC_OP_MAP_CONTAINSVALUE:
            n += _decided_in_tree_family(m, v)
        cap = max(cap, m.hm.capacity())
    return n, cap


@pytest.mark.parametrize("seed,n_tree,n_other,sub_batch", [
    (1101, 40, 560, 0),         # 1,024 buckets; the tree halves stay trees at 128 and 256
    (1102, 24, 560, 4096),      # several sub-batches: the model handed over mid-batch, then followed
    (1103, 60, 420, 16384),     # bigger tree family (re-treeified halves), 1,024 buckets
])
def test_tree_bin_grows_past_64_under_churn(seed, n_tree, n_other, sub_batch):
    """A map whose bin 5 becomes a red-black tree bin at capacity 64 grows to 1,024 buckets and churns: every
    containsValue (many decided inside the bins the tree split into) matches the oracle, none is refused."""
    rng = np.random.default_rng(seed)
    rows = _tree_rows(rng, n_tree, n_other, 40_000)
    inside, cap = _count_tree_decided(rows)
    assert cap == 1024 and inside >= 200, (cap, inside)
    b = _batch(rows, 1)
    E, O = _engines(1, 4, len(b), 4096, sub_batch=sub_batch)
    n = len(b)
    gs, gv, os_, ov = _apply_both(E, O, [b.slice(0, n // 4), b.slice(n // 4, n // 2), b.slice(n // 2, n)])
    _assert_rows(gs, gv, os_, ov)
    _assert_maps(E, O, [0])
    cv = np.nonzero(b.op == abi.CC_OP_MAP_CONTAINSVALUE)[0]
    npe = int((gs[cv] == abi.cc_status(abi.CC_ST_NULL_POINTER, abi.CC_TAG_NULL)).sum())
    assert 0 < npe < len(cv)
    assert E.counters()[4] == 1  # the map is followed by a big model


def test_tree_bin_past_64_with_clears():
    """The same map with MapState.clear rows in the churn (barriers when a null is stored, else in the stream): the
    big model empties with the table's capacity kept, and bins become trees again at capacity >= 64 (treeifyBin
    without a resize)."""
    rng = np.random.default_rng(1104)
    rows = _tree_rows(rng, 40, 560, 30_000, clear_rate=0.002)
    b = _batch(rows, 1)
    E, O = _engines(1, 4, len(b), 4096, sub_batch=8192)
    gs, gv, os_, ov = _apply_both(E, O, [b])
    _assert_rows(gs, gv, os_, ov)
    _assert_maps(E, O, [0])


def test_tree_bin_maps_many_and_delete():
    """Six maps with tree bins past 64 side by side in one stream (a big model each); then a Delete of two of them
    (MapState.delete: every key leaves, the table keeps its capacity) and keys that form a tree bin in those tables
    at capacity 1,024 directly (treeifyBin without a resize), followed by the same models."""
    rng = np.random.default_rng(1105)
    maps = 6
    per = [_tree_rows(rng, 30, 300, 6_000) for _ in range(maps)]
    rows, inst = [], []
    pos = [0] * maps
    while any(p < len(r) for p, r in zip(pos, per)):
        m = int(rng.integers(maps))
        if pos[m] < len(per[m]):
            rows.append(per[m][pos[m]])
            inst.append(m)
            pos[m] += 1
    b = _batch(rows, 1, inst)
    E, O = _engines(maps, maps + 8, len(b), 1 << 14, sub_batch=8192)
    gs, gv, os_, ov = _apply_both(E, O, [b])
    _assert_rows(gs, gv, os_, ov)
    _assert_maps(E, O, range(maps))
    assert E.counters()[4] == maps
    d = _batch([(abi.CC_OP_DELETE, 0, N, 0)] * 2, len(b) + 1, [1, 4])
    r2 = _tree_rows(rng, 30, 300, 6_000, shift=26)
    b2 = _batch(r2 + r2, len(b) + 3, [1] * len(r2) + [4] * len(r2))
    gs, gv, os_, ov = _apply_both(E, O, [d, b2])
    _assert_rows(gs, gv, os_, ov)
    _assert_maps(E, O, range(maps))
