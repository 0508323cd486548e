"""ctypes binding of liboracle.so — the CPU restatement of the reference apply path.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg,
as the checker (or the timed CPU baseline).  The product package copycat_amd never imports this module.
"""
import ctypes as C
import os
import subprocess

import numpy as np

from copycat_amd import abi
from copycat_amd.batch import Batch

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def build(force=False):
    so = os.path.join(_HERE, "liboracle.so")
    src = os.path.join(_HERE, "oracle.cpp")
    if force or not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return so


def lib():
    global _LIB
    if _LIB is None:
        so = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(so):
            build()
        L = C.CDLL(so)
        P, u8, u32, u64, i32, i64 = C.c_void_p, C.c_uint8, C.c_uint32, C.c_uint64, C.c_int, C.c_int64
        sig = {
            "orc_create": (P, [u32, u32, u32]),
            "orc_destroy": (None, [P]),
            "orc_resource_create": (i32, [P, u32, u32]),
            "orc_resource_delete": (i32, [P, u32]),
            "orc_instance_open": (i32, [P, u32, u32, u64, u64]),
            "orc_get_resource": (i32, [P, u64, u32, u64, u64, P, P, P]),
            "orc_create_resource": (i32, [P, u64, u32, u64, u64, P, P, P]),
            "orc_delete_resource": (i32, [P, u64, P]),
            "orc_resource_exists": (i32, [P, u64]),
            "orc_inst_slot_of": (i32, [P, u64]),
            "orc_res_slot_of": (i32, [P, u64]),
            "orc_apply": (i32, [P, P, u64, P, P]),
            "orc_advance_time": (i32, [P, u64]),
            "orc_handle_string": (i32, [P, u64, P, u64]),
            "orc_session_close": (i32, [P, u64]),
            "orc_session_expire": (i32, [P, u64]),
            "orc_applied_index": (u64, [P]),
            "orc_event_count": (u64, [P]),
            "orc_events_read": (None, [P, P, P, P, P, P, P]),
            "orc_events_clear": (None, [P]),
            "orc_aux_count": (u64, [P]),
            "orc_aux_read": (None, [P, P, P]),
            "orc_aux_clear": (None, [P]),
            "orc_read_value_state": (i32, [P, u32, u32, P, P, P]),
            "orc_read_value_retained": (i32, [P, u32, u32, P]),
            "orc_map_size": (i64, [P, u32]),
            "orc_read_retained": (i64, [P, u32, u64, P]),
            "orc_map_entries": (i64, [P, u32, u64, P, P, P, P, P]),
            "orc_lock_state": (i64, [P, u32, P, P, P, u64, P, P]),
            "orc_election_state": (i64, [P, u32, P, P, u64, P, P]),
            "orc_group_members": (i64, [P, u32, u64, P]),
            "orc_pending_timers": (u64, [P]),
            "orc_quorum_commit": (None, [P, u32, u64, P, P, P]),
            "orc_expire_sweep": (None, [P, u64, u64, u64, P, P]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _LIB = L
    return _LIB


def _p(arr):
    return arr.ctypes.data_as(C.c_void_p) if arr is not None else None


def batch_struct(b: Batch):
    s = abi.cc_batch()
    for name, _ in abi.BATCH_COLUMNS:
        setattr(s, name, _p(getattr(b, name)))
    return s


class Oracle:
    """One CPU restatement of a ResourceManager-hosted server (one Raft replica's state machine)."""

    def __init__(self, max_resources, max_instances, flags=abi.CC_CFG_TIMERS_DEFERRED):
        self.L = lib()
        self.h = self.L.orc_create(max_resources, max_instances, flags)
        self.max_resources = max_resources

    def close(self):
        if self.h:
            self.L.orc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # registry
    def resource_create(self, slot, rtype):
        rc = self.L.orc_resource_create(self.h, slot, rtype)
        assert rc == 0, rc

    def resource_delete(self, slot):
        return self.L.orc_resource_delete(self.h, slot)

    def instance_open(self, inst, res, instance_id, client):
        rc = self.L.orc_instance_open(self.h, inst, res, instance_id, client)
        assert rc == 0, rc

    def _ctl(self, fn, key, rtype, client, index):
        iid, islot, st = C.c_uint64(), C.c_uint32(), C.c_uint8()
        rc = fn(self.h, key, rtype, client, index, C.byref(iid), C.byref(islot), C.byref(st))
        assert rc == 0, rc
        return st.value, iid.value, islot.value

    def get_resource(self, key, rtype, client, index):
        return self._ctl(self.L.orc_get_resource, key, rtype, client, index)

    def create_resource(self, key, rtype, client, index):
        return self._ctl(self.L.orc_create_resource, key, rtype, client, index)

    def delete_resource(self, resource_id):
        st = C.c_uint8()
        rc = self.L.orc_delete_resource(self.h, resource_id, C.byref(st))
        assert rc == 0
        return st.value

    def resource_exists(self, key):
        return bool(self.L.orc_resource_exists(self.h, key))

    def inst_slot_of(self, instance_id):
        return self.L.orc_inst_slot_of(self.h, instance_id)

    # apply
    def apply(self, b: Batch):
        n = len(b)
        status = np.zeros(n, np.uint8)
        value = np.zeros(n, np.uint64)
        s = batch_struct(b)
        rc = self.L.orc_apply(self.h, C.byref(s), n, _p(status), _p(value))
        assert rc == 0, rc
        return status, value

    def handle_string(self, handle, s):
        """Register the java.lang.String behind HANDLE `handle` (its hashCode / compareTo order the HashMap bins)."""
        u = np.frombuffer(s.encode("utf-16-le"), dtype=np.uint16).copy()
        assert self.L.orc_handle_string(self.h, handle, _p(u) if len(u) else None, len(u)) == 0

    def advance_time(self, now):
        self.L.orc_advance_time(self.h, now)

    def session_close(self, client):
        self.L.orc_session_close(self.h, client)

    def session_expire(self, client):
        self.L.orc_session_expire(self.h, client)

    def applied_index(self):
        return self.L.orc_applied_index(self.h)

    def take_events(self):
        n = self.L.orc_event_count(self.h)
        cols = dict(pos=np.zeros(n, np.uint32), target=np.zeros(n, np.uint32), code=np.zeros(n, np.uint8),
                    src=np.zeros(n, np.uint8), tag=np.zeros(n, np.uint8), payload=np.zeros(n, np.uint64))
        if n:
            self.L.orc_events_read(self.h, *[_p(cols[k]) for k in ("pos", "target", "code", "src", "tag", "payload")])
        self.L.orc_events_clear(self.h)
        return cols

    def take_aux(self):
        n = self.L.orc_aux_count(self.h)
        pos, mem = np.zeros(n, np.uint32), np.zeros(n, np.uint64)
        if n:
            self.L.orc_aux_read(self.h, _p(pos), _p(mem))
        self.L.orc_aux_clear(self.h)
        return pos, mem

    # state
    def value_state(self, first=0, count=None):
        count = self.max_resources - first if count is None else count
        tag, val, cur = np.zeros(count, np.uint8), np.zeros(count, np.uint64), np.zeros(count, np.uint8)
        rc = self.L.orc_read_value_state(self.h, first, count, _p(tag), _p(val), _p(cur))
        assert rc == 0
        return tag, val, cur

    def value_retained(self, first=0, count=None):
        count = self.max_resources - first if count is None else count
        idx = np.zeros(count, np.uint64)
        assert self.L.orc_read_value_retained(self.h, first, count, _p(idx)) == 0
        return idx

    def retained(self, slot, cap=1 << 16):
        """Ascending log indices of every commit the slot's state machine still holds uncleaned (None: no resource)."""
        out = np.zeros(cap, np.uint64)
        n = self.L.orc_read_retained(self.h, slot, cap, _p(out))
        return None if n < 0 else out[:min(n, cap)].tolist()

    def map_entries(self, res):
        n = self.L.orc_map_size(self.h, res)
        if n < 0:
            return None
        kt, k, vt, v, ci = (np.zeros(n, np.uint8), np.zeros(n, np.uint64), np.zeros(n, np.uint8),
                            np.zeros(n, np.uint64), np.zeros(n, np.uint64))
        self.L.orc_map_entries(self.h, res, n, _p(kt), _p(k), _p(vt), _p(v), _p(ci))
        return kt, k, vt, v, ci

    def lock_state(self, res, cap=1024):
        h, hi, hc = C.c_int64(), C.c_uint64(), C.c_uint8()
        qi, qx = np.zeros(cap, np.uint32), np.zeros(cap, np.uint64)
        n = self.L.orc_lock_state(self.h, res, C.byref(h), C.byref(hi), C.byref(hc), cap, _p(qi), _p(qx))
        if n < 0:
            return None
        return h.value, hi.value, hc.value, list(zip(qi[:n].tolist(), qx[:n].tolist()))

    def election_state(self, res, cap=1024):
        ld, li = C.c_int64(), C.c_uint64()
        qi, qx = np.zeros(cap, np.uint32), np.zeros(cap, np.uint64)
        n = self.L.orc_election_state(self.h, res, C.byref(ld), C.byref(li), cap, _p(qi), _p(qx))
        if n < 0:
            return None
        return ld.value, li.value, list(zip(qi[:n].tolist(), qx[:n].tolist()))

    def group_members(self, res, cap=4096):
        ids = np.zeros(cap, np.uint64)
        n = self.L.orc_group_members(self.h, res, cap, _p(ids))
        return None if n < 0 else ids[:n].tolist()

    def pending_timers(self):
        return self.L.orc_pending_timers(self.h)


def quorum_commit(match, term_start, commit_in):
    """match: (replicas, groups) u64 array."""
    match = np.ascontiguousarray(match, np.uint64)
    replicas, groups = match.shape
    out = np.zeros(groups, np.uint64)
    lib().orc_quorum_commit(_p(match), replicas, groups, _p(np.ascontiguousarray(term_start, np.uint64)),
                            _p(np.ascontiguousarray(commit_in, np.uint64)), _p(out))
    return out


def expire_sweep(last, now, timeout):
    last = np.ascontiguousarray(last, np.uint64)
    words = (len(last) + 63) // 64
    bitmap = np.zeros(words, np.uint64)
    count = np.zeros(1, np.uint64)
    lib().orc_expire_sweep(_p(last), len(last), now, timeout, _p(bitmap), _p(count))
    return bitmap, int(count[0])
