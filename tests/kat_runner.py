"""Runs the KATs of tests/golden/kats.json against a backend (the CPU oracle or the GPU engine).

Consecutive commit steps are applied as ONE batch (so a multi-row batch is what gets checked); control,
clock and close steps flush the pending batch first.  Events are compared per step as sorted multisets of
(target instance slot, code, tag, payload) — per-target order is what the reference fixes.
"""
import json
import os

import numpy as np

from copycat_amd import abi
from copycat_amd.batch import Batch

HERE = os.path.dirname(os.path.abspath(__file__))
KAT_PATH = os.path.join(HERE, "golden", "kats.json")

RES = {"VALUE": abi.CC_RES_VALUE, "MAP": abi.CC_RES_MAP, "LOCK": abi.CC_RES_LOCK, "ELECTION": abi.CC_RES_ELECTION,
       "GROUP": abi.CC_RES_GROUP, "SET": abi.CC_RES_SET, "QUEUE": abi.CC_RES_QUEUE,
       "MULTIMAP": abi.CC_RES_MULTIMAP}
TAG = {"NULL": abi.CC_TAG_NULL, "LONG": abi.CC_TAG_LONG, "INT": abi.CC_TAG_INT, "BOOL": abi.CC_TAG_BOOL,
       "H": abi.CC_TAG_HANDLE, "SET": abi.CC_TAG_SET, "LIST": abi.CC_TAG_LIST}
EV = {"CHANGE": abi.CC_EV_CHANGE, "LOCK": abi.CC_EV_LOCK, "ELECT": abi.CC_EV_ELECT, "JOIN": abi.CC_EV_JOIN,
      "LEAVE": abi.CC_EV_LEAVE, "EXECUTE": abi.CC_EV_EXECUTE}
ST = {"OK": abi.CC_ST_OK, "UNKNOWN_SESSION": abi.CC_ST_UNKNOWN_SESSION, "UNKNOWN_OP": abi.CC_ST_UNKNOWN_OP,
      "ILLEGAL_STATE": abi.CC_ST_ILLEGAL_STATE, "ILLEGAL_ARGUMENT": abi.CC_ST_ILLEGAL_ARGUMENT,
      "NULL_POINTER": abi.CC_ST_NULL_POINTER, "TYPE_MISMATCH": abi.CC_ST_TYPE_MISMATCH,
      "UNKNOWN_RESOURCE": abi.CC_ST_UNKNOWN_RESOURCE, "NO_SUCH_ELEMENT": abi.CC_ST_NO_SUCH_ELEMENT}


def load():
    with open(KAT_PATH) as f:
        return json.load(f)


def enc(v):
    """JSON value -> (tag, payload)."""
    t = TAG[v[0]]
    if t == abi.CC_TAG_NULL:
        return t, 0
    if t == abi.CC_TAG_BOOL:
        return t, int(bool(v[1]))
    if t in (abi.CC_TAG_SET, abi.CC_TAG_LIST):
        return t, len(v[1])
    return t, int(v[1]) & 0xFFFFFFFFFFFFFFFF


def op_code(name):
    return getattr(abi, f"CC_OP_{name}")


GPU_VALUE_OPS = {"VALUE_GET", "VALUE_SET", "VALUE_CAS", "VALUE_GETANDSET", "VALUE_LISTEN", "VALUE_UNLISTEN"}
GPU_COORD_OPS = {"LOCK_LOCK", "LOCK_UNLOCK", "ELECT_LISTEN", "ELECT_UNLISTEN", "ELECT_ISLEADER", "GROUP_JOIN",
                 "GROUP_LEAVE", "GROUP_EXECUTE", "GROUP_SCHEDULE"}
GPU_MAP_OPS = {"MAP_CONTAINSKEY", "MAP_PUT", "MAP_PUTIFABSENT", "MAP_GET", "MAP_GETORDEFAULT", "MAP_REMOVE",
               "MAP_REMOVEIFPRESENT", "MAP_REPLACE", "MAP_REPLACEIFPRESENT", "MAP_CONTAINSVALUE", "MAP_SIZE",
               "MAP_ISEMPTY", "MAP_CLEAR"}
GPU_SET_OPS = {"SET_CONTAINS", "SET_ADD", "SET_REMOVE", "SET_SIZE", "SET_ISEMPTY", "SET_CLEAR"}
GPU_QUEUE_OPS = {"QUEUE_CONTAINS", "QUEUE_ADD", "QUEUE_OFFER", "QUEUE_PEEK", "QUEUE_POLL", "QUEUE_ELEMENT", "QUEUE_REMOVE",
                 "QUEUE_SIZE", "QUEUE_ISEMPTY", "QUEUE_CLEAR"}
GPU_MMAP_OPS = {"MMAP_CONTAINSKEY", "MMAP_CONTAINSENTRY", "MMAP_CONTAINSVALUE", "MMAP_PUT", "MMAP_GET", "MMAP_REMOVE",
                "MMAP_REMOVEVALUE", "MMAP_ISEMPTY", "MMAP_SIZE", "MMAP_CLEAR"}


def gpu_eligible(kat):
    """KATs whose every step this build runs through the engine: every op of every covered state machine, Delete,
    clock advances, session closes (the GPU close fan-out) and manager control commands (manager.hip)."""
    if kat.get("gpu") == "refuses":  # the engine fails such a batch loudly (test_gpu_kats.py checks that)
        return False
    types = {r[1] for r in kat["resources"]}
    if not types <= {"VALUE", "MAP", "LOCK", "ELECTION", "GROUP", "SET", "QUEUE", "MULTIMAP"}:
        return False
    for s in kat["steps"]:
        if "commit" in s:
            c = s["commit"]
            if c["op"] != "DELETE" and c["op"] not in GPU_VALUE_OPS | GPU_MAP_OPS | GPU_COORD_OPS | GPU_SET_OPS | GPU_QUEUE_OPS | GPU_MMAP_OPS:
                return False
    return True


class KatRun:
    """Drives one KAT through `backend` and asserts every expectation."""

    def __init__(self, kat, backend):
        self.kat = kat
        self.B = backend
        self.next_index = 1
        self.clock = 0
        self.pending = []  # (step, row fields)
        self.slot_of_id = {}  # instance id -> slot, kept after the instance closes (event targets name it)

    def inst_slot(self, ref):
        if isinstance(ref, int):
            return ref
        if ref.startswith("@"):
            s = self.B.inst_slot_of(int(ref[1:]))
            if s < 0:
                s = self.slot_of_id.get(int(ref[1:]), -1)
            assert s >= 0, f"unknown instance id {ref}"
            return s
        if ref.startswith("#"):
            return int(ref[1:])
        raise ValueError(ref)

    def run(self):
        # the Strings behind HANDLE ids: java.util.HashMap places a String key by String.hashCode
        self.B.handle_strings({h: s for s, h in load()["strings"].items()})
        for r in self.kat["resources"]:
            self.B.resource_create(r[0], RES[r[1]])
        for i in self.kat["instances"]:
            self.B.instance_open(*i)
        for step in self.kat["steps"]:
            if "commit" in step:
                self.pending.append(step)
                continue
            self.flush()
            if "advance" in step:
                self.clock = max(self.clock, step["advance"])
                evs = self.B.advance(step["advance"])
                self.check_events(step, evs)
            elif "close" in step:
                evs = self.B.close(step["close"])
                self.check_events(step, evs)
            elif "control" in step:
                self.control(step)
            elif "state" in step:
                self.check_state(step["state"])
        self.flush()

    def flush(self):
        if not self.pending:
            return
        n = len(self.pending)
        b = Batch(n)
        for i, step in enumerate(self.pending):
            c = step["commit"]
            if "time" in c:
                self.clock = max(self.clock, c["time"])
            b.index[i] = self.next_index
            self.next_index += 1
            b.time[i] = self.clock
            b.inst[i] = self.inst_slot(c["inst"]) if not (isinstance(c["inst"], str) and c["inst"].startswith("@")) \
                else self.inst_slot(c["inst"])
            b.op[i] = op_code(c["op"])
            ta, pa = enc(c["a"]) if "a" in c else (0, 0)
            tb, pb = enc(c["b"]) if "b" in c else (0, 0)
            kt, kp = (0, 0)
            if "key" in c:
                t, kp = enc(c["key"])
                kt = abi.KTAG_OF_TAG[t]
            b.flags[i] = abi.cc_flags(ta, tb, kt)
            b.key[i], b.a[i], b.b[i] = kp, pa, pb
            b.aux[i] = c.get("aux", 0) & 0xFFFFFFFFFFFFFFFF
        status, value, events, aux = self.B.apply(b)
        for i, step in enumerate(self.pending):
            exp = step["expect"]
            name = f"{self.kat['name']} row {i} ({step['commit']['op']})"
            assert abi.status_code(status[i]) == ST[exp["status"]], \
                f"{name}: status {abi.status_code(status[i])} != {exp['status']}"
            if exp["status"] == "OK":
                et, ep = enc(exp["result"])
                assert (abi.status_tag(status[i]), int(value[i])) == (et, ep), \
                    f"{name}: result ({abi.status_tag(status[i])},{int(value[i])}) != {exp['result']}"
                if et == abi.CC_TAG_SET:
                    got = sorted(int(m) for p, m in aux if p == i)
                    assert got == sorted(exp["result"][1]), f"{name}: set {got} != {exp['result'][1]}"
            self.check_events(step, [e for e in events if e[0] == i], name)
        self.pending = []

    def check_events(self, step, evs, name=None):
        name = name or f"{self.kat['name']} {list(step)[0]}"
        want = sorted((self.inst_slot(t), EV[code], *enc(v)) for t, code, v in step.get("events", []))
        got = sorted((int(e[1]), int(e[2]), int(e[3]), int(e[4])) for e in evs)
        assert got == want, f"{name}: events {got} != {want}"

    def control(self, step):
        c = step["control"]
        what = c["what"]
        exp = step["expect"]["status"]
        if what in ("get", "create"):
            key = enc(c["key"])[1]
            self.next_index = max(self.next_index, c["index"] + 1)
            st, iid = self.B.manager(what, key, RES[c["type"]], c["client"], c["index"])
            assert abi.status_code(st) == ST[exp], f"{self.kat['name']} {what}: status {st}"
            if "expect_instance" in c:
                assert iid == c["expect_instance"], f"{self.kat['name']} {what}: instance {iid}"
            if abi.status_code(st) == abi.CC_ST_OK:
                self.slot_of_id[iid] = self.B.inst_slot_of(iid)
        elif what == "delete":
            st = self.B.delete_resource(c["resource"])
            assert abi.status_code(st) == ST[exp], f"{self.kat['name']} delete: status {st}"
        elif what == "exists":
            assert self.B.resource_exists(enc(c["key"])[1]) == c["expect_bool"]
        else:
            raise ValueError(what)

    def check_state(self, s):
        if "value" in s:
            res, v, cur = s["value"]
            tag, val, has = self.B.value_state(res)
            assert (tag, val, bool(has)) == (*enc(v), cur), f"{self.kat['name']} value state {(tag, val, has)}"
        if "lock" in s:
            res, holder, queue = s["lock"]
            h, q = self.B.lock_state(res)
            assert (h, q) == (holder, queue), f"{self.kat['name']} lock state {(h, q)}"
        if "members" in s:
            res, ids = s["members"]
            assert self.B.group_members(res) == ids


class OracleBackend:
    def __init__(self, kat, max_resources=256, max_instances=64):
        from oracle.oracle_py import Oracle

        flags = abi.CC_CFG_TIMERS_DEFERRED if kat.get("timer_mode", "deferred") == "deferred" else 0
        self.O = Oracle(max_resources, max_instances, flags)

    def handle_strings(self, strings):
        for h, x in strings.items():
            self.O.handle_string(h, x)

    def resource_create(self, slot, t):
        self.O.resource_create(slot, t)

    def instance_open(self, inst, res, iid, client):
        self.O.instance_open(inst, res, iid, client)

    def inst_slot_of(self, iid):
        return self.O.inst_slot_of(iid)

    def _events(self):
        e = self.O.take_events()
        return [(int(e["pos"][i]), int(e["target"][i]), int(e["code"][i]), int(e["tag"][i]), int(e["payload"][i]))
                for i in range(len(e["pos"]))]

    def apply(self, b):
        s, v = self.O.apply(b)
        evs = self._events()
        pos, mem = self.O.take_aux()
        return s, v, evs, list(zip(pos.tolist(), mem.tolist()))

    def advance(self, now):
        self.O.advance_time(now)
        return self._events()

    def close(self, client):
        self.O.session_close(client)
        return self._events()

    def manager(self, what, key, t, client, index):
        fn = self.O.get_resource if what == "get" else self.O.create_resource
        st, iid, _ = fn(key, t, client, index)
        return st, iid

    def delete_resource(self, rid):
        return self.O.delete_resource(rid)

    def resource_exists(self, key):
        return self.O.resource_exists(key)

    def value_state(self, res):
        t, v, c = self.O.value_state(res, 1)
        return int(t[0]), int(v[0]), int(c[0])

    def lock_state(self, res):
        h, _, _, q = self.O.lock_state(res)
        return (None if h < 0 else h), [x[0] for x in q]

    def group_members(self, res):
        return self.O.group_members(res)


class EngineBackend:
    """GPU engine backend (the GPU-applied subset of this build: see gpu_eligible).  Batches go through the
    device path with an event stream; join's member-set rows (CC_EV_MEMBER) are the aux results."""

    def __init__(self, kat, max_resources=256, max_instances=64):
        from copycat_amd.engine import Engine

        flags = abi.CC_CFG_VALUE_EVENTS
        if kat.get("timer_mode", "deferred") == "deferred":
            flags |= abi.CC_CFG_TIMERS_DEFERRED
        self.E = Engine(max_resources, max_instances, 4096, map_capacity=4096, flags=flags, max_events=1 << 16)
        self.ids = {}

    def handle_strings(self, strings):
        self.E.handle_strings(strings)

    def resource_create(self, slot, t):
        self.E.resource_create(slot, t)

    def instance_open(self, inst, res, iid, client):
        self.E.instance_open(inst, res, iid, client)
        self.ids[iid] = inst

    def inst_slot_of(self, iid):
        return self.E.instance_slot(iid)

    def apply(self, b):
        s, v, ev = self.E.apply_host_events(b)
        evs, aux = [], []
        for i in range(len(ev["pos"])):
            row = (int(ev["pos"][i]), int(ev["target"][i]), int(ev["code"][i]), int(ev["tag"][i]), int(ev["payload"][i]))
            if row[2] == abi.CC_EV_MEMBER:
                aux.append((row[0], row[4]))
            else:
                evs.append(row)
        return s, v, evs, aux

    @staticmethod
    def _rows(ev):
        return [(int(ev["pos"][i]), int(ev["target"][i]), int(ev["code"][i]), int(ev["tag"][i]), int(ev["payload"][i]))
                for i in range(len(ev["pos"]))]

    def advance(self, now):
        return self._rows(self.E.advance_time_events(now))

    def close(self, client):
        _, ev = self.E.sessions_close([client])
        return self._rows(ev)

    def manager(self, what, key, t, client, index):
        fn = self.E.get_resource if what == "get" else self.E.create_resource
        st, iid, islot = fn(key, t, client, index)
        if abi.status_code(st) == abi.CC_ST_OK:
            self.ids[iid] = islot
        return st, iid

    def delete_resource(self, rid):
        return self.E.delete_resource(rid)

    def resource_exists(self, key):
        return self.E.resource_exists(key)

    def value_state(self, res):
        t, v, c = self.E.value_state(res, 1)
        return int(t[0]), int(v[0]), int(c[0])

    def lock_state(self, res):
        h, _, _, q = self.E.lock_state(res)
        return (None if h < 0 else h), [x[0] for x in q]

    def group_members(self, res):
        return self.E.group_members(res)


def all_kats():
    return load()["kats"]


__all__ = ["KatRun", "OracleBackend", "EngineBackend", "all_kats", "gpu_eligible", "np"]
