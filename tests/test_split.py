"""cc_split_batch / cc_merge_results (copycat_amd/csrc/split.cpp): one global log split by owning rank, on CPU.

The reference multiplexes every resource in one log (ResourceManager.java:37-39,56-72); with one engine per GPU the
host splits each committed batch by owner (stable: log order within every rank) and merges the results back.  Checked
against a numpy restatement (np.nonzero per rank) on ragged sizes, every thread count, unknown instances, missing
columns, and the error cases."""
import ctypes as C

import numpy as np
import pytest

from copycat_amd import abi, shard
from copycat_amd.batch import Batch
from copycat_amd.engine import EngineError, _np, lib


def _batch(n, n_inst, seed, unknown=0.0):
    rng = np.random.default_rng(seed)
    b = Batch(n)
    for name in Batch.__slots__:
        a = getattr(b, name)
        a[:] = rng.integers(0, np.iinfo(a.dtype).max, n, dtype=a.dtype, endpoint=True)
    b.inst[:] = rng.integers(0, n_inst, n, dtype=np.uint32)
    if unknown:
        m = rng.random(n) < unknown
        b.inst[m] = n_inst + rng.integers(0, 1000, int(m.sum()), dtype=np.uint32)
    b.index[:] = np.arange(n, dtype=np.uint64) + 1
    return b


def _ref_owner(b, tab):
    inst = b.inst.astype(np.int64)
    return np.where(inst < len(tab), tab[np.minimum(inst, len(tab) - 1)], 0)


@pytest.mark.parametrize("n,world,threads", [(0, 1, 1), (1, 1, 1), (5, 3, 4), (8191, 2, 1), (8192, 8, 2),
                                             (8193, 8, 3), (100_003, 13, 8), (300_000, 8, 0), (70_001, 1, 5),
                                             (200_000, 256, 7)])
def test_split_merge_matches_numpy(n, world, threads):
    n_inst = 5000
    b = _batch(n, n_inst, seed=n * 31 + world, unknown=0.01)
    tab = np.random.default_rng(world).integers(0, world, n_inst).astype(np.uint8)
    parts = shard.split_batch(b, tab, world, threads=threads)
    own = _ref_owner(b, tab)
    for r, (rows, sub) in enumerate(parts):
        want = np.nonzero(own == r)[0]
        assert np.array_equal(rows, want.astype(np.uint64)), f"rank {r} rows"
        for name in Batch.__slots__:
            assert np.array_equal(getattr(sub, name), getattr(b, name)[want]), f"rank {r} column {name}"
    # results per rank (status = a byte of the row's a column, value = its index) merged back by owner
    res = [((sub.a & 0xFF).astype(np.uint8), sub.index.copy()) for _, sub in parts]
    st, va = shard.merge_by_owner(b.inst, tab, world, res, threads=threads)
    assert np.array_equal(va, b.index) and np.array_equal(st, (b.a & 0xFF).astype(np.uint8))
    st2, va2 = shard.merge_results(n, [(rows, s, v) for (rows, _), (s, v) in zip(parts, res)])
    assert np.array_equal(st2, st) and np.array_equal(va2, va)


def test_split_missing_columns_and_errors():
    n, world, n_inst = 20_000, 4, 100
    b = _batch(n, n_inst, seed=7)
    tab = (np.arange(n_inst) % world).astype(np.uint8)
    counts = np.zeros(world, np.uint64)
    cols = abi.cc_batch(index=None, time=None, inst=_np(b.inst), op=_np(b.op), flags=None, key=_np(b.key), a=None,
                        b=None, aux=None)
    assert lib().cc_split_batch(C.byref(cols), n, _np(tab), n_inst, world, 3, None, None, _np(counts), None) == 0
    own = _ref_owner(b, tab)
    assert counts.tolist() == [int((own == r).sum()) for r in range(world)]
    subs = [Batch(int(c)) for c in counts]
    outs = (abi.cc_batch_out * world)()
    for r in range(world):  # only the columns the input has
        outs[r].inst, outs[r].op, outs[r].key = _np(subs[r].inst), _np(subs[r].op), _np(subs[r].key)
    cap = counts.copy()
    assert lib().cc_split_batch(C.byref(cols), n, _np(tab), n_inst, world, 3, outs, _np(cap), _np(counts), None) == 0
    for r in range(world):
        m = own == r
        assert np.array_equal(subs[r].op, b.op[m]) and np.array_equal(subs[r].key, b.key[m])
        assert not subs[r].a.any() and not subs[r].index.any()  # absent in the input: untouched
    small = cap.copy()
    small[2] -= 1
    assert lib().cc_split_batch(C.byref(cols), n, _np(tab), n_inst, world, 3, outs, _np(small), _np(counts), None) \
        == abi.CC_ERR_CAPACITY
    bad = tab.copy()
    bad[5] = world  # names no rank
    assert lib().cc_split_batch(C.byref(cols), n, _np(bad), n_inst, world, 3, None, None, _np(counts), None) \
        == abi.CC_ERR_INVALID
    outs[1].op = None  # a present column without an output
    assert lib().cc_split_batch(C.byref(cols), n, _np(tab), n_inst, world, 3, outs, _np(cap), _np(counts), None) \
        == abi.CC_ERR_INVALID
    with pytest.raises(ValueError):
        shard.split_batch(b, np.full(n_inst, 9, np.int32), world)
    with pytest.raises(EngineError):
        shard.split_batch(b, tab, 0)
