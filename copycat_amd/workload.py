"""Synthetic committed-command streams, generated natively and deterministically.

Streams are host numpy columns (Batch); benches upload them once so the timed region starts with the
columns resident in HBM.
"""
import ctypes as C
import os

import numpy as np

from . import abi
from .batch import Batch

_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        from .build import WORKLOAD_SO, build_workload

        if not os.path.exists(WORKLOAD_SO):
            build_workload()
        L = C.CDLL(WORKLOAD_SO)
        P, u32, u64 = C.c_void_p, C.c_uint32, C.c_uint64
        L.wl_atomic_long.restype = u64
        L.wl_atomic_long.argtypes = [u64, u32, u32, u64, u32, u32, u64] + [P] * 7
        L.wl_atomic_long_step.restype = u64
        L.wl_atomic_long_step.argtypes = [u64, u32, u32, u64, u32, u32, u64, u64, P, P, u32] + [P] * 7
        L.wl_value_random.restype = u64
        L.wl_value_random.argtypes = [u64, u32, u32, u32, u64, u32, u32, u64] + [P] * 7
        L.wl_map_random.restype = u64
        L.wl_map_random.argtypes = [u64, u32, u32, u32, u32, u64, u32, u32, u64] + [P] * 9 + [u32]
        L.wl_coord_random.restype = u64
        L.wl_coord_random.argtypes = [u64, u32, u32, P, u32, u64, u32, u64] + [P] * 9
        L.wl_coord_model_new.restype = P
        L.wl_coord_model_new.argtypes = [u32]
        L.wl_coord_model_free.restype = None
        L.wl_coord_model_free.argtypes = [P]
        L.wl_coord_random_model.restype = u64
        L.wl_coord_random_model.argtypes = [P, u64, u32, u32, P, u32, u64, u32, u64] + [P] * 9
        L.wl_map_zipf.restype = u64
        L.wl_map_zipf.argtypes = [u64, u64, u32, u32, C.c_double, u32, u64, u32] + [P] * 8
        _LIB = L
    return _LIB


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


SEED_C2 = 0xA700000 + 2  # seed = 0xA70_0000 + config#


def atomic_long_stream(n, resources=65536, first_inst=0, seed=SEED_C2, p_cold=0.2, p_stale=0.1, index0=1):
    """Config 2: DistributedAtomicLong add/CAS client model over `resources` AtomicValueState instances."""
    b = Batch(n)
    lib().wl_atomic_long(n, resources, first_inst, seed, int(p_cold * 1e6), int(p_stale * 1e6), index0,
                         _p(b.index), _p(b.time), _p(b.inst), _p(b.op), _p(b.flags), _p(b.a), _p(b.b))
    return b


class AtomicLongClients:
    """Config 2 client model carried across bench steps (DistributedAtomicLong.java:117-146): each step's stream
    continues from the values the clients' CASes expect after the previous step, so the ~10% stale-CAS mix holds
    in every step.  Rank `rank` of `world` generates its share of ONE global log: its resources are the global
    resources rank + world*k (local slot k) and its rows carry the global log indices index0 + i*world + rank."""

    def __init__(self, resources=65536, seed=SEED_C2, p_cold=0.2, p_stale=0.1, rank=0, world=1, threads=None):
        self.R = resources
        self.seed = seed
        self.p_cold, self.p_stale = p_cold, p_stale
        self.rank, self.world = rank, world
        self.threads = threads or min(16, os.cpu_count() or 1)
        self.tag = np.zeros(resources, np.uint8)
        self.val = np.zeros(resources, np.int64)
        self.next_global = 1  # global log index of the next step's first row (all ranks agree)
        self.step = 0

    def next(self, n, out=None):
        """The next step's n rows (a Batch; `out` is reused when given)."""
        b = out if out is not None else Batch(n)
        got = lib().wl_atomic_long_step(n, self.R, 0, self.seed + 0x9E37 * self.step, int(self.p_cold * 1e6),
                                        int(self.p_stale * 1e6), self.next_global + self.rank, self.world, _p(self.tag),
                                        _p(self.val), self.threads, _p(b.index), _p(b.time), _p(b.inst), _p(b.op),
                                        _p(b.flags), _p(b.a), _p(b.b))
        assert got == n
        self.next_global += n * self.world
        self.step += 1
        return b


def value_random_stream(n, resources, max_inst, first_inst=0, seed=1, hot=0, p_hot=0.0, index0=1):
    """Adversarial AtomicValue stream for parity tests (all ops/tags, unknown sessions, wrong-type ops)."""
    b = Batch(n)
    lib().wl_value_random(n, resources, first_inst, max_inst, seed, hot, int(p_hot * 1e6), index0,
                          _p(b.index), _p(b.time), _p(b.inst), _p(b.op), _p(b.flags), _p(b.a), _p(b.b))
    return b


def map_random_stream(n, maps, max_inst, keys=64, first_inst=0, seed=1, hot=0, p_hot=0.0, index0=1,
                      value_compare_ops=True):
    """Adversarial MapState stream for parity tests (every key op, all tags, null values, hot keys,
    wrong-type ops, unknown sessions, ttl <= 0).  value_compare_ops=False swaps removeIfPresent /
    replaceIfPresent for remove / replace (the hot-key scan family)."""
    b = Batch(n)
    lib().wl_map_random(n, maps, first_inst, max_inst, keys, seed, hot, int(p_hot * 1e6), index0, _p(b.index),
                        _p(b.time), _p(b.inst), _p(b.op), _p(b.flags), _p(b.key), _p(b.a), _p(b.b), _p(b.aux),
                        1 if value_compare_ops else 0)
    return b


def coord_random_stream(n, types, K, max_inst, seed=1, p_delete=0.0005, index0=1):
    """Coordination parity stream over resources with types[r]; resource r owns instance slots r*K + k."""
    types = np.ascontiguousarray(types, np.uint8)
    b = Batch(n)
    lib().wl_coord_random(n, len(types), K, _p(types), max_inst, seed, int(p_delete * 1e6), index0, _p(b.index),
                          _p(b.time), _p(b.inst), _p(b.op), _p(b.flags), _p(b.key), _p(b.a), _p(b.b), _p(b.aux))
    return b


class CoordClients:
    """The coordination stream of coord_random_stream continued across calls (the lock client model carries over), so
    a bench applies one step's batch after another without replaying a stream on state it no longer matches."""

    def __init__(self, types, K=1, max_inst=None, seed=1, p_delete=0.0005):
        self.types = np.ascontiguousarray(types, np.uint8)
        self.K = K
        self.max_inst = max_inst if max_inst is not None else len(self.types) * K
        self.seed = seed
        self.p_delete = p_delete
        self.index0 = 1
        self.step = 0
        self.h = lib().wl_coord_model_new(len(self.types))

    def __del__(self):
        try:
            lib().wl_coord_model_free(self.h)
        except Exception:
            pass

    def next(self, n, out=None):
        b = out if out is not None else Batch(n)
        got = lib().wl_coord_random_model(self.h, n, len(self.types), self.K, _p(self.types), self.max_inst,
                                          self.seed + 0x51ED * self.step, int(self.p_delete * 1e6), self.index0,
                                          _p(b.index), _p(b.time), _p(b.inst), _p(b.op), _p(b.flags), _p(b.key),
                                          _p(b.a), _p(b.b), _p(b.aux))
        assert got == n
        self.index0 += n
        self.step += 1
        return b


SEED_C3 = 0xA700000 + 3


def map_zipf_rows(row0, n, maps=4096, pairs=1 << 20, s=0.99, first_inst=0, seed=SEED_C3, threads=8, out=None):
    """Config 3: rows [row0, row0+n) of the DistributedMap put/get/remove Zipf stream (see wl_map_zipf)."""
    b = out if out is not None else Batch(n)
    got = lib().wl_map_zipf(row0, n, maps, pairs, s, first_inst, seed, threads, _p(b.index), _p(b.time), _p(b.inst),
                            _p(b.op), _p(b.flags), _p(b.key), _p(b.a), _p(b.b))
    assert got == n
    return b


SEED_C4 = 0xA700000 + 4


def quorum_groups(groups, replicas=5, seed=SEED_C4):
    """Config 4a: per group leader lastIndex L ~ U[1e6, 2e6); follower matchIndex = L - U[0, 64);
    termStart = L - U[0, 128); oldCommit = L - U[0, 96).  Returns (match[replicas, groups], term_start, commit_in)."""
    rng = np.random.default_rng(seed)
    last = rng.integers(1_000_000, 2_000_000, groups, dtype=np.uint64)
    match = np.empty((replicas, groups), np.uint64)
    match[0] = last
    for r in range(1, replicas):
        match[r] = last - rng.integers(0, 64, groups, dtype=np.uint64)
    term_start = last - rng.integers(0, 128, groups, dtype=np.uint64)
    commit_in = last - rng.integers(0, 96, groups, dtype=np.uint64)
    return match, term_start, commit_in


def expiry_sessions(sessions, timeout=5000, now=10_000_000, seed=SEED_C4 + 1):
    """Config 4b: lastKeepAlive = now - U[0, 2*timeout)."""
    rng = np.random.default_rng(seed)
    last = now - rng.integers(0, 2 * timeout, sessions, dtype=np.uint64)
    return last, now, timeout


__all__ = ["atomic_long_stream", "AtomicLongClients", "CoordClients", "value_random_stream", "map_random_stream", "map_zipf_rows", "quorum_groups", "expiry_sessions", "abi"]
