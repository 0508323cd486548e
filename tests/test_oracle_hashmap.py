"""The oracle's java.util.HashMap model (oracle/oracle.cpp JHM) against an independent Python restatement of JDK 8's
HashMap (tests/java_hashmap.py), on streams built to exercise every structural path: treeifyBin's early resizes below
capacity 64, tree bins (treeify, putTreeVal linking new nodes after their tree parent, moveRootToFront, the red-black
delete, untreeify when a tree gets too small, split / re-treeify on resize), mixed key classes with equal hashes
(tieBreakOrder by class name), String keys hashed by String.hashCode with equal-hash strings ordered by compareTo,
and MapState.delete's iterator removals.  Every containsValue answer (MapState.java:49-60: true, false or the NPE of a
stored null met first) and the final key sets must agree.  CPU only (the oracle is test infrastructure)."""
import numpy as np
import pytest

from copycat_amd import abi
from copycat_amd.batch import Batch
from tests.java_hashmap import BOOL, INT, LONG, STR, MapStateModel

KT = {LONG: 0, INT: 1, BOOL: 2, STR: 3}
TAG = {LONG: abi.CC_TAG_LONG, INT: abi.CC_TAG_INT, BOOL: abi.CC_TAG_BOOL, STR: abi.CC_TAG_HANDLE}


def _key_family(rng, kind, n):
    if kind == "long_cluster":  # equal low bits at every capacity: one bin, early resizes, then a tree
        s = int(rng.choice([20, 22, 24]))
        c = int(rng.integers(0, 16))
        return [(LONG, i * (1 << s) + c) for i in range(n)]
    if kind == "long_mixed":  # a few clusters + random keys
        out = [(LONG, i * (1 << 22) + 5) for i in range(n // 2)]
        out += [(LONG, int(x)) for x in rng.integers(-(1 << 40), 1 << 40, n - n // 2)]
        return out
    if kind == "tree_split":  # a 16-key bin at capacity 64 that splits (bit 6) as random keys grow the table
        out = [(LONG, i * 64 + 5) for i in range(24)]
        out += [(LONG, int(x)) for x in rng.integers(1 << 20, 1 << 40, n)]
        return out
    if kind == "classes":  # Long / Integer / Boolean keys with equal hashCodes: tieBreakOrder by class name
        out = []
        for i in range(n):
            v = i * 64 + 7
            out.append((LONG, v) if i % 3 == 0 else (INT, v) if i % 3 == 1 else (LONG, v + (1 << 32) * 3))
        out += [(BOOL, 0), (BOOL, 1), (INT, 1231), (LONG, 1237)]
        return out
    if kind == "strings":  # equal String.hashCode ("Aa" == "BB") families, ordered by compareTo inside a tree bin
        base = ["Aa", "BB"]
        out = []
        for a in base:
            for b in base:
                for c in base:
                    out.append((STR, a + b + c))
        out += [(STR, f"key{i}") for i in range(n)]
        out += [(STR, "été"), (STR, "\U0001F600")]  # non-ASCII: UTF-16 units (a surrogate pair)
        return out
    raise ValueError(kind)


def _run(seed, kind, n_ops, nkeys):
    from oracle.oracle_py import Oracle

    rng = np.random.default_rng(seed)
    keys = _key_family(rng, kind, nkeys)
    handles = {}
    O = Oracle(1, 1)
    O.resource_create(0, abi.CC_RES_MAP)
    O.instance_open(0, 0, 100, 1)
    for k in keys:
        if k[0] == STR and k[1] not in handles:
            handles[k[1]] = 1000 + len(handles)
            O.handle_string(handles[k[1]], k[1])
    M = MapStateModel()
    vals = [None, 1, 2, 3]
    rows, want = [], []
    for i in range(n_ops):
        r = rng.random()
        k = keys[int(rng.integers(0, len(keys)))]
        kp = handles[k[1]] if k[0] == STR else (k[1] & 0xFFFFFFFFFFFFFFFF)
        if r < 0.55:
            v = vals[int(rng.integers(0, 4))]
            rows.append((abi.CC_OP_MAP_PUT, KT[k[0]], kp, v))
            M.put(k, v)
            want.append(None)
        elif r < 0.8:
            rows.append((abi.CC_OP_MAP_REMOVE, KT[k[0]], kp, None))
            M.remove(k)
            want.append(None)
        elif r < 0.997:
            v = vals[1 + int(rng.integers(0, 3))]
            rows.append((abi.CC_OP_MAP_CONTAINSVALUE, 0, 0, v))
            want.append(M.contains_value(v))
        else:
            rows.append((abi.CC_OP_MAP_CLEAR, 0, 0, None))
            M.clear()
            want.append(None)
    n = len(rows)
    b = Batch(n)
    b.index[:] = np.arange(1, n + 1)
    b.time[:] = np.arange(1, n + 1)
    b.inst[:] = 0
    for i, (op, kt, kp, v) in enumerate(rows):
        b.op[i] = op
        ta = abi.CC_TAG_NULL if v is None else abi.CC_TAG_LONG
        b.flags[i] = abi.cc_flags(ta, 0, kt)
        b.key[i] = kp
        b.a[i] = 0 if v is None else v
    st, va = O.apply(b)
    checked = kinds = 0
    for i, w in enumerate(want):
        if w is None:
            continue
        code = abi.status_code(st[i])
        got = "NPE" if code == abi.CC_ST_NULL_POINTER else bool(va[i])
        assert code in (abi.CC_ST_OK, abi.CC_ST_NULL_POINTER)
        assert got == w, f"{kind} seed {seed}: row {i} containsValue {got} != JDK 8 model {w}"
        checked += 1
        kinds += w == "NPE"
    n_live = O.map_size(0) if hasattr(O, "map_size") else None
    if n_live is not None:
        assert n_live == len(M.vals)
    return checked, kinds, M


@pytest.mark.parametrize("kind,nkeys,n_ops", [("long_cluster", 40, 6000), ("long_mixed", 200, 8000),
                                              ("classes", 60, 6000), ("strings", 120, 8000),
                                              ("tree_split", 60, 8000)])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_oracle_hashmap_matches_jdk8_model(kind, nkeys, n_ops, seed):
    checked, npes, M = _run(seed * 7919 + len(kind), kind, n_ops, nkeys)
    assert checked > 10 and 0 < npes < checked  # both orders occur


def test_jdk8_model_reaches_every_structural_path():
    """The Python model itself passes through early resizes, tree bins, splits and untreeify on these streams."""
    from tests import java_hashmap as J

    seen = set()
    orig_treeify, orig_untreeify, orig_split = J.HashMap.treeify, J.HashMap.untreeify, J.HashMap.split

    def tr(self, hd, tab):
        seen.add("treeify")
        return orig_treeify(self, hd, tab)

    def un(hd):
        seen.add("untreeify")
        return orig_untreeify(hd)

    def sp(self, *a):
        seen.add("split")
        return orig_split(self, *a)

    J.HashMap.treeify, J.HashMap.untreeify, J.HashMap.split = tr, staticmethod(un), sp
    try:
        m = J.HashMap()
        for i in range(9):  # 9 keys in bin 5 at capacity 16: treeifyBin resizes to 32 (capacity < 64)
            m.put((LONG, i * (1 << 20) + 5))
        assert m.capacity() == 32 and m.size == 9
        _run(5, "long_cluster", 4000, 40)
        _run(6, "strings", 4000, 120)
        _run(7, "tree_split", 6000, 60)
    finally:
        J.HashMap.treeify, J.HashMap.untreeify, J.HashMap.split = orig_treeify, orig_untreeify, orig_split
    assert {"treeify", "untreeify", "split"} <= seen, seen
