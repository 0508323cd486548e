"""The Java drop-in's view of the engine: host memory only, no torch, no device pointers.

Run by tests/test_gpu_host_boundary.py in a fresh interpreter (so that `torch` provably never loads).  It binds
libcopycat_apply.so with bare ctypes exactly as the Panama FFM / JNI stub of INTEGRATION.md §2 does, and drives a
lock / election / group / value-listener stream through the host-memory entry points:

  cc_apply_batch_host_events   ResourceManager.operateResource (ResourceManager.java:56-72) -> LockState.lock / unlock
                               (LockState.java:41-85), LeaderElectionState.listen / unlisten (:57-91),
                               MembershipGroupState.join / leave / execute / schedule (:47-119), AtomicValueState
                               listen / change (:41-72), each publishing through Session.publish ->
                               InstanceEvent{instance, msg} (ManagedResourceSession.java:64-71, InstanceEvent.java:29-80)
  cc_sessions_close_host       ResourceManager.close (:250-264): election hand-over, group "leave" (A10)
  cc_sessions_expire_host      ResourceManager.expire (:238-247)
  cc_advance_time_events_host  MembershipGroup.schedule timers firing (:86-103)
  cc_retained_bitmap_host      the compaction feed (ResourceManagerCommit.clean :79-81)

Every result row and every event, per target session in publish order, is compared with the oracle
(oracle/oracle.cpp, the CPU restatement: test infrastructure only).  Prints "host boundary ok" on success."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from copycat_amd import abi  # noqa: E402  (ctypes structs only)
from copycat_amd.batch import Batch  # noqa: E402
from copycat_amd.workload import coord_random_stream  # noqa: E402
from oracle.oracle_py import Oracle  # noqa: E402

P, i32, u32, u64 = C.c_void_p, C.c_int, C.c_uint32, C.c_uint64


def bind():
    L = C.CDLL(os.path.join(ROOT, "copycat_amd", "libcopycat_apply.so"))
    sig = {
        "cc_abi_version": (i32, []), "cc_last_error": (C.c_char_p, []),
        "cc_engine_create": (i32, [P, P]), "cc_engine_destroy": (i32, [P]),
        "cc_resource_create": (i32, [P, u32, u32]), "cc_instance_open": (i32, [P, u32, u32, u64, u64]),
        "cc_apply_batch_host_events": (i32, [P, P, u64, P, P]),
        "cc_sessions_close_host": (i32, [P, P, u64, P, P]), "cc_sessions_expire_host": (i32, [P, P, u64, P, P]),
        "cc_advance_time_events_host": (i32, [P, u64, P]), "cc_retained_bitmap_host": (i32, [P, u64, u64, P, P]),
        "cc_device_alloc": (i32, [i32, u64, P]), "cc_device_free": (i32, [P]), "cc_memcpy": (i32, [P, P, u64, i32, P]),
        "cc_quorum_commit": (i32, [P, u32, u64, P, P, P, P]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype, f.argtypes = res, args
    assert L.cc_abi_version() == abi.CC_ABI_VERSION
    return L


def ck(L, rc):
    if rc != 0:
        raise RuntimeError(f"cc error {rc}: {L.cc_last_error().decode()}")


class HostEvents:
    """A host cc_events: numpy columns + a host count (what a JVM would allocate off-heap)."""

    def __init__(self, cap):
        self.cols = dict(pos=np.zeros(cap, np.uint32), target=np.zeros(cap, np.uint32), code=np.zeros(cap, np.uint8),
                         src=np.zeros(cap, np.uint8), tag=np.zeros(cap, np.uint8), payload=np.zeros(cap, np.uint64))
        self.count = np.zeros(1, np.uint64)
        self.s = abi.cc_events(*[self.cols[k].ctypes.data for k in ("pos", "target", "code", "src", "tag", "payload")],
                               cap, self.count.ctypes.data)

    def rows(self):
        n = int(self.count[0])
        return {k: v[:n].copy() for k, v in self.cols.items()}


def per_target(ev, member_out=None):
    out = {}
    for i in range(len(ev["pos"])):
        if int(ev["code"][i]) == abi.CC_EV_MEMBER:
            if member_out is not None:
                member_out.append((int(ev["pos"][i]), int(ev["payload"][i])))
            continue
        out.setdefault(int(ev["target"][i]), []).append(
            (int(ev["pos"][i]), int(ev["src"][i]), int(ev["code"][i]), int(ev["tag"][i]), int(ev["payload"][i])))
    return out


def with_schedules(b, types, K, max_inst, rng, count):
    """MembershipGroup.schedule rows on group instances (MembershipGroupState.java:86-103)."""
    res_of = np.where(b.inst < max_inst, b.inst // K, 0)
    grp = np.nonzero((types[np.minimum(res_of, len(types) - 1)] == abi.CC_RES_GROUP) & (b.inst < len(types) * K))[0]
    rows = rng.choice(grp, size=min(count, len(grp)), replace=False)
    b.op[rows] = abi.CC_OP_GROUP_SCHEDULE
    b.key[rows] = (1000 + res_of[rows] * K + rng.integers(0, K, len(rows))).astype(np.uint64)
    b.flags[rows] = abi.cc_flags(abi.CC_TAG_HANDLE, 0, 0)
    b.a[rows] = rng.integers(0, 1 << 20, len(rows)).astype(np.uint64)
    b.aux[rows] = rng.integers(1, 400, len(rows)).astype(np.uint64)
    b.aux[rows[::3]] = 5_000_000  # still pending at the batch end: fired by cc_advance_time_events_host
    return b


def main():
    L = bind()
    types = np.resize(np.array([abi.CC_RES_LOCK, abi.CC_RES_ELECTION, abi.CC_RES_GROUP, abi.CC_RES_VALUE], np.uint8), 2048)
    R, K, n = len(types), 4, 400_000
    max_inst = R * K + 8
    flags = abi.CC_CFG_TIMERS_DEFERRED | abi.CC_CFG_VALUE_EVENTS | abi.CC_CFG_VALUE_RETAINED
    cfg = abi.cc_config()
    cfg.max_resources, cfg.max_instances, cfg.max_batch, cfg.max_events, cfg.flags = R, max_inst, n, 1 << 22, flags
    h = C.c_void_p()
    ck(L, L.cc_engine_create(C.byref(cfg), C.byref(h)))
    O = Oracle(R, max_inst, flags & abi.CC_CFG_TIMERS_DEFERRED)
    for r, t in enumerate(types):
        ck(L, L.cc_resource_create(h, r, int(t)))
        O.resource_create(r, int(t))
        for k in range(K):  # instance r*K+k, id 1000 + r*K + k, owned by client session 7 + k
            ck(L, L.cc_instance_open(h, r * K + k, r, 1000 + r * K + k, 7 + k))
            O.instance_open(r * K + k, r, 1000 + r * K + k, 7 + k)
    rng = np.random.default_rng(71)
    b = with_schedules(coord_random_stream(n, types, K, max_inst, seed=71), types, K, max_inst, rng, 300)
    total_events = 0
    for lo, hi in ((0, n // 3), (n // 3, n)):
        part = b.slice(lo, hi)
        m = hi - lo
        cols = abi.cc_batch(*[getattr(part, name).ctypes.data for name, _ in abi.BATCH_COLUMNS])
        status, value = np.full(m, 0xFF, np.uint8), np.zeros(m, np.uint64)
        res = abi.cc_results(status.ctypes.data, value.ctypes.data)
        ev = HostEvents(8 * m)
        ck(L, L.cc_apply_batch_host_events(h, C.byref(cols), m, C.byref(res), C.byref(ev.s)))
        s2, v2 = O.apply(part)
        assert np.array_equal(status, s2) and np.array_equal(value, v2), np.nonzero((status != s2) | (value != v2))[0][:5]
        got_mem, want_mem = [], []
        got = per_target(ev.rows(), got_mem)
        oe = O.take_events()
        want = per_target(oe)
        apos, amem = O.take_aux()
        assert got == want, "events differ per target session"
        assert got_mem == list(zip(apos.tolist(), amem.tolist())), "join member sets differ"
        total_events += int(ev.count[0])
    assert total_events > n // 4, total_events
    # too small a host event stream: CC_ERR_CAPACITY with the true count
    small = HostEvents(4)
    part = coord_random_stream(2000, types, K, max_inst, seed=72, index0=n + 1)
    part.op[:] = np.where(part.op == abi.CC_OP_GROUP_SCHEDULE, abi.CC_OP_ELECT_ISLEADER, part.op)
    cols = abi.cc_batch(*[getattr(part, name).ctypes.data for name, _ in abi.BATCH_COLUMNS])
    st2, va2 = np.zeros(2000, np.uint8), np.zeros(2000, np.uint64)
    res2 = abi.cc_results(st2.ctypes.data, va2.ctypes.data)
    rc = L.cc_apply_batch_host_events(h, C.byref(cols), 2000, C.byref(res2), C.byref(small.s))
    assert rc == abi.CC_ERR_CAPACITY and int(small.count[0]) > 4, (rc, int(small.count[0]))
    O.apply(part)  # the engine applied the batch; only the stream overflowed
    O.take_events()
    O.take_aux()
    # session close and expire fan-out
    clients = np.array([8], np.uint64)
    ev = HostEvents(1 << 16)
    closed = C.c_uint64()
    ck(L, L.cc_sessions_close_host(h, clients.ctypes.data, 1, C.byref(ev.s), C.byref(closed)))
    O.session_close(8)
    assert closed.value > 0 and per_target(ev.rows()) == per_target(O.take_events())
    bm = np.zeros(1, np.uint64)
    bm[0] = (1 << 9) | (1 << 10)  # sessions 9 and 10, ascending
    ev = HostEvents(1 << 16)
    ck(L, L.cc_sessions_expire_host(h, bm.ctypes.data, 64, C.byref(ev.s), C.byref(closed)))
    O.session_close(9)
    O.session_close(10)
    assert closed.value > 0 and per_target(ev.rows()) == per_target(O.take_events())
    # schedule timers fire
    now = int(max(b.time[-1], part.time[-1])) + 10_000_000
    ev = HostEvents(1 << 16)
    ck(L, L.cc_advance_time_events_host(h, now, C.byref(ev.s)))
    O.advance_time(now)
    fired, ofired = per_target(ev.rows()), per_target(O.take_events())
    nf = sum(len(v) for v in fired.values())
    assert fired == ofired and nf > 0, (nf, sum(len(v) for v in ofired.values()))
    # compaction feed
    span = n + 2001
    words = np.zeros((span + 63) // 64, np.uint64)
    cnt = C.c_uint64()
    ck(L, L.cc_retained_bitmap_host(h, 1, span, words.ctypes.data, C.byref(cnt)))
    bits = np.unpackbits(words.view(np.uint8), bitorder="little")[:span]
    got = set((np.nonzero(bits)[0] + 1).tolist())
    want = set()
    for r in range(R):
        x = O.retained(r)
        if x is not None:
            want.update(int(i) for i in x)
    assert got == want and cnt.value == len(got), (len(got), len(want))
    # the plain device-memory API drives a stateless device call (leader quorum commit)
    G5 = 1000
    match = np.random.default_rng(3).integers(1, 1 << 40, (5, G5)).astype(np.uint64)
    term, cin, out = np.zeros(G5, np.uint64), np.zeros(G5, np.uint64), np.zeros(G5, np.uint64)
    ptrs = [C.c_void_p() for _ in range(4)]
    for p, nbytes in zip(ptrs, (match.nbytes, 8 * G5, 8 * G5, 8 * G5)):
        ck(L, L.cc_device_alloc(0, nbytes, C.byref(p)))
    ck(L, L.cc_memcpy(ptrs[0], match.ctypes.data, match.nbytes, abi.CC_MEMCPY_H2D, None))
    ck(L, L.cc_memcpy(ptrs[1], term.ctypes.data, 8 * G5, abi.CC_MEMCPY_H2D, None))
    ck(L, L.cc_memcpy(ptrs[2], cin.ctypes.data, 8 * G5, abi.CC_MEMCPY_H2D, None))
    ck(L, L.cc_quorum_commit(ptrs[0], 5, G5, ptrs[1], ptrs[2], ptrs[3], None))
    ck(L, L.cc_memcpy(out.ctypes.data, ptrs[3], 8 * G5, abi.CC_MEMCPY_D2H, None))
    assert np.array_equal(out, np.sort(match, axis=0)[2])  # the quorum-th (3rd) largest of 5, old commit 0
    for p in ptrs:
        ck(L, L.cc_device_free(p))
    ck(L, L.cc_engine_destroy(h))
    assert "torch" not in sys.modules, "the host boundary must not need torch"
    print(f"host boundary ok: {n} commits, {total_events} events, {len(got)} retained")


if __name__ == "__main__":
    main()
