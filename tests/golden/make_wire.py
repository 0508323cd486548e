#!/usr/bin/env python3
"""Catalyst wire-format fixtures for the decoder (copycat_amd/csrc/wire.cpp, cc_wire_decode).

An independent Python restatement of how an Atomix 1.x client serializes what it submits, written from the
reference's writeObject methods (cited per op below) — NOT from the decoder's schema table:
  * InstanceCommand / InstanceQuery (@SerializeWith 30 / 31): buffer.writeLong(instance id), then
    serializer.writeObject(operation) (manager/src/main/java/io/atomix/resource/InstanceOperation.java:60-69);
  * serializer.writeObject(obj): null -> one 0x00 byte; a registered type -> an identifier byte giving the id's
    width (1..4 bytes), the id, then the type's payload (Long 8 bytes, Integer 4, Boolean 1, String writeUTF8);
  * manager entries GetResource 35 / CreateResource 36 (KeyOperation writeUTF8(key) + writeInt(len) + the state
    machine class name, GetResource.java:62-65), DeleteResource 37 (writeLong(resource), DeleteResource.java:56),
    ResourceExists 38 (writeUTF8(key)).
Catalyst is not vendored: the identifier bytes, the primitive ids (copycat_apply.h CC_WIRE_ID_*), big-endian
order and writeUTF8's framing (a presence byte, a u16 length) are this repo's restatement — parity unpinned.

Writes tests/golden/wire_fixture.bin (the entries back to back) and wire_fixture.json (offsets, the strings the
test interns first, and the columns each entry must decode to).  Run: python tests/golden/make_wire.py
"""
import json
import os
import struct

ID_BOOLEAN, ID_INTEGER, ID_LONG, ID_STRING = 129, 132, 133, 136

# op codes = @SerializeWith ids (AtomicValueCommands.java:93-261, MapCommands.java:134-451,
# MultiMapCommands.java:205-433, QueueCommands.java:133-236, SetCommands.java:133-238,
# LeaderElectionCommands.java:80-100, LockCommands.java:59-94, MembershipGroupCommands.java:62-141)
OP = dict(VALUE_GET=50, VALUE_SET=51, VALUE_CAS=52, VALUE_GETANDSET=53, VALUE_LISTEN=54, VALUE_UNLISTEN=55,
          MAP_CONTAINSKEY=60, MAP_CONTAINSVALUE=61, MAP_PUT=62, MAP_PUTIFABSENT=63, MAP_GET=64, MAP_GETORDEFAULT=65,
          MAP_REMOVE=66, MAP_REMOVEIFPRESENT=67, MAP_REPLACE=68, MAP_REPLACEIFPRESENT=69, MAP_ISEMPTY=70,
          MAP_SIZE=71, MAP_CLEAR=72, MMAP_CONTAINSKEY=75, MMAP_CONTAINSENTRY=76, MMAP_CONTAINSVALUE=77,
          MMAP_PUT=78, MMAP_GET=79, MMAP_REMOVE=80, MMAP_REMOVEVALUE=81, MMAP_ISEMPTY=82, MMAP_SIZE=83,
          MMAP_CLEAR=84, QUEUE_CONTAINS=90, QUEUE_ADD=91, QUEUE_OFFER=92, QUEUE_PEEK=93, QUEUE_POLL=94,
          QUEUE_ELEMENT=95, QUEUE_REMOVE=96, QUEUE_SIZE=97, QUEUE_ISEMPTY=98, QUEUE_CLEAR=99, SET_CONTAINS=100,
          SET_ADD=101, SET_REMOVE=102, SET_SIZE=103, SET_ISEMPTY=104, SET_CLEAR=105, ELECT_LISTEN=110,
          ELECT_UNLISTEN=111, ELECT_ISLEADER=112, LOCK_LOCK=115, LOCK_UNLOCK=116, GROUP_JOIN=120, GROUP_LEAVE=121,
          GROUP_SCHEDULE=122, GROUP_EXECUTE=123)
TAG = {"NULL": 0, "LONG": 1, "INT": 2, "BOOL": 3, "H": 4}
KTAG = {"LONG": 0, "INT": 1, "BOOL": 2, "H": 3}


def ident(type_id):
    for code, w in ((1, 1), (2, 2), (3, 3), (4, 4)):
        if -(1 << (8 * w - 1)) <= type_id < (1 << (8 * w - 1)):
            return bytes([code]) + (type_id & ((1 << (8 * w)) - 1)).to_bytes(w, "big")
    raise ValueError(type_id)


def utf8(s):
    b = s.encode()
    return b"\x01" + struct.pack(">H", len(b)) + b


def obj(v, strings):
    """serializer.writeObject(v); v = None | ("LONG", n) | ("INT", n) | ("BOOL", b) | ("STR", s)"""
    if v is None:
        return b"\x00"
    t, x = v
    if t == "LONG":
        return ident(ID_LONG) + struct.pack(">q", x)
    if t == "INT":
        return ident(ID_INTEGER) + struct.pack(">i", x)
    if t == "BOOL":
        return ident(ID_BOOLEAN) + bytes([1 if x else 0])
    if t == "STR":
        return ident(ID_STRING) + utf8(x)
    raise ValueError(t)


def col(v, strings):
    """canonical (tag, payload) of a value as the engine sees it"""
    if v is None:
        return "NULL", 0
    t, x = v
    if t == "STR":
        return "H", strings.index(x) + 1
    if t == "BOOL":
        return "BOOL", int(bool(x))
    return t, x & 0xFFFFFFFFFFFFFFFF  # LONG two's complement, INT sign-extended (copycat_apply.h CC_TAG_*)


def instance_op(iid, op, strings, key=None, a=None, b=None, aux=None, member=None, query=False):
    """InstanceCommand / InstanceQuery bytes for `op` with its fields in the reference's writeObject order, and
    the expected decoded row."""
    body = b""
    # field order per op (the reference writeObject chain)
    if op in ("VALUE_SET", "VALUE_GETANDSET"):          # AtomicValueCommands.java:126,228 (no ttl: A2)
        body = obj(a, strings)
    elif op == "VALUE_CAS":                              # :182-184 expect, update
        body = obj(a, strings) + obj(b, strings)
    elif op in ("MAP_CONTAINSKEY", "MAP_GET", "MAP_REMOVE", "MMAP_CONTAINSKEY", "MMAP_GET", "MMAP_SIZE",
                "SET_CONTAINS", "SET_REMOVE"):            # KeyQuery/KeyCommand key; Set ValueCommand value (as key)
        body = obj(key, strings)
    elif op in ("MAP_CONTAINSVALUE", "MMAP_CONTAINSVALUE", "MMAP_REMOVEVALUE", "QUEUE_CONTAINS", "QUEUE_ADD",
                "QUEUE_OFFER", "QUEUE_REMOVE"):          # value only
        body = obj(a, strings)
    elif op in ("MAP_PUT", "MAP_PUTIFABSENT", "MAP_REPLACE", "MMAP_PUT"):  # TtlCommand key, value, ttl
        body = obj(key, strings) + obj(a, strings) + struct.pack(">q", aux or 0)
    elif op == "MAP_REPLACEIFPRESENT":                   # MapCommands.java:421-423 key, value, ttl, replace
        body = obj(key, strings) + obj(a, strings) + struct.pack(">q", aux or 0) + obj(b, strings)
    elif op in ("MAP_GETORDEFAULT", "MAP_REMOVEIFPRESENT", "MMAP_CONTAINSENTRY", "MMAP_REMOVE"):  # key, value
        body = obj(key, strings) + obj(a, strings)
    elif op == "SET_ADD":                                # SetCommands.java:172-174 value, ttl
        body = obj(key, strings) + struct.pack(">q", aux or 0)
    elif op == "LOCK_LOCK":                              # LockCommands.java:80-81 timeout
        body = struct.pack(">q", aux)
    elif op == "GROUP_SCHEDULE":                         # MembershipGroupCommands.java:124-126 member, delay, cb
        body = struct.pack(">qq", member, aux) + obj(a, strings)
    elif op == "GROUP_EXECUTE":                          # :172-174 member, callback
        body = struct.pack(">q", member) + obj(a, strings)
    entry = ident(31 if query else 30) + struct.pack(">Q", iid) + ident(OP[op]) + body
    ta, pa = col(a, strings)
    tb, pb = col(b, strings)
    kt, kv = ("LONG", 0) if key is None else col(key, strings)
    if member is not None:
        kt, kv = "LONG", member & 0xFFFFFFFFFFFFFFFF
    row = {"kind": 0, "iid": iid, "op": OP[op], "flags": TAG[ta] | (TAG[tb] << 3) | (KTAG[kt] << 6), "key": kv,
           "a": pa, "b": pb, "aux": (aux or 0) & 0xFFFFFFFFFFFFFFFF}
    return entry, row


RES_CLASS = {"VALUE": ("io.atomix.atomic.state.AtomicValueState", 1), "MAP": ("io.atomix.collections.state.MapState", 2),
             "LOCK": ("io.atomix.coordination.state.LockState", 3),
             "ELECTION": ("io.atomix.coordination.state.LeaderElectionState", 4),
             "GROUP": ("io.atomix.coordination.state.MembershipGroupState", 5),
             "SET": ("io.atomix.collections.state.SetState", 6), "QUEUE": ("io.atomix.collections.state.QueueState", 7),
             "MULTIMAP": ("io.atomix.collections.state.MultiMapState", 8),
             "TOPIC": ("io.atomix.coordination.state.TopicState", 0)}


def manager_op(kind, strings, key=None, rtype=None, resource=None):
    if kind in (35, 36):
        name = RES_CLASS[rtype][0].encode()
        entry = ident(kind) + utf8(key) + struct.pack(">i", len(name)) + name
        row = {"kind": kind, "key": strings.index(key) + 1, "a": RES_CLASS[rtype][1]}
    elif kind == 38:
        entry = ident(kind) + utf8(key)
        row = {"kind": kind, "key": strings.index(key) + 1, "a": 0}
    else:
        entry = ident(kind) + struct.pack(">Q", resource)
        row = {"kind": kind, "key": 0, "a": 0, "b": resource}
    row.setdefault("b", 0)
    row.update(iid=0, op=0, flags=0, aux=0)
    return entry, row


def fixture():
    strings = ["counter", "Hello world!", "foo", "bar", "k", "élan", ""]
    L, I, B, S = (lambda n: ("LONG", n)), (lambda n: ("INT", n)), (lambda b: ("BOOL", b)), (lambda s: ("STR", s))
    e = []
    e.append(manager_op(35, strings, key="counter", rtype="VALUE"))
    e.append(manager_op(36, strings, key="foo", rtype="MAP"))
    e.append(manager_op(35, strings, key="bar", rtype="TOPIC"))     # not a state machine this engine runs
    e.append(manager_op(38, strings, key="k"))
    e.append(manager_op(37, strings, resource=12))
    e.append(instance_op(1, "VALUE_GET", strings, query=True))
    e.append(instance_op(1, "VALUE_SET", strings, a=S("Hello world!")))
    e.append(instance_op(1, "VALUE_SET", strings, a=None))
    e.append(instance_op(1, "VALUE_CAS", strings, a=L(-1), b=L(1 << 40)))
    e.append(instance_op(1, "VALUE_GETANDSET", strings, a=I(-7)))
    e.append(instance_op(1, "VALUE_LISTEN", strings))
    e.append(instance_op(1, "VALUE_UNLISTEN", strings))
    e.append(instance_op(2, "MAP_PUT", strings, key=S("foo"), a=L(5), aux=100))
    e.append(instance_op(2, "MAP_PUTIFABSENT", strings, key=L(3), a=B(True), aux=0))
    e.append(instance_op(2, "MAP_GET", strings, key=I(4), query=True))
    e.append(instance_op(2, "MAP_GETORDEFAULT", strings, key=B(False), a=S("bar"), query=True))
    e.append(instance_op(2, "MAP_CONTAINSKEY", strings, key=S("élan"), query=True))
    e.append(instance_op(2, "MAP_CONTAINSVALUE", strings, a=None, query=True))
    e.append(instance_op(2, "MAP_REMOVE", strings, key=S("")))
    e.append(instance_op(2, "MAP_REMOVEIFPRESENT", strings, key=L(1), a=L(2)))
    e.append(instance_op(2, "MAP_REPLACE", strings, key=L(1), a=L(3), aux=-5))
    e.append(instance_op(2, "MAP_REPLACEIFPRESENT", strings, key=L(1), a=L(4), b=L(3), aux=7))
    for op in ("MAP_ISEMPTY", "MAP_SIZE"):
        e.append(instance_op(2, op, strings, query=True))
    e.append(instance_op(2, "MAP_CLEAR", strings))
    e.append(instance_op(3, "MMAP_PUT", strings, key=S("k"), a=L(9), aux=50))
    e.append(instance_op(3, "MMAP_CONTAINSENTRY", strings, key=S("k"), a=L(9), query=True))
    e.append(instance_op(3, "MMAP_CONTAINSVALUE", strings, a=L(9), query=True))
    e.append(instance_op(3, "MMAP_CONTAINSKEY", strings, key=S("k"), query=True))
    e.append(instance_op(3, "MMAP_GET", strings, key=S("k"), query=True))
    e.append(instance_op(3, "MMAP_REMOVE", strings, key=S("k"), a=None))
    e.append(instance_op(3, "MMAP_REMOVEVALUE", strings, a=S("foo")))
    e.append(instance_op(3, "MMAP_SIZE", strings, key=None, query=True))   # Size(): null key
    e.append(instance_op(3, "MMAP_SIZE", strings, key=I(2), query=True))
    for op in ("MMAP_ISEMPTY", "MMAP_CLEAR"):
        e.append(instance_op(3, op, strings, query=op.endswith("ISEMPTY")))
    e.append(instance_op(4, "QUEUE_ADD", strings, a=None))
    e.append(instance_op(4, "QUEUE_OFFER", strings, a=I(1)))
    e.append(instance_op(4, "QUEUE_CONTAINS", strings, a=S("foo"), query=True))
    e.append(instance_op(4, "QUEUE_REMOVE", strings, a=None))
    for op in ("QUEUE_PEEK", "QUEUE_POLL", "QUEUE_ELEMENT", "QUEUE_SIZE", "QUEUE_ISEMPTY", "QUEUE_CLEAR"):
        e.append(instance_op(4, op, strings, query=op in ("QUEUE_PEEK", "QUEUE_SIZE", "QUEUE_ISEMPTY")))
    e.append(instance_op(5, "SET_ADD", strings, key=L(77), aux=10))
    e.append(instance_op(5, "SET_CONTAINS", strings, key=L(77), query=True))
    e.append(instance_op(5, "SET_REMOVE", strings, key=S("foo")))
    for op in ("SET_SIZE", "SET_ISEMPTY", "SET_CLEAR"):
        e.append(instance_op(5, op, strings, query=op != "SET_CLEAR"))
    for op in ("ELECT_LISTEN", "ELECT_UNLISTEN"):
        e.append(instance_op(6, op, strings))
    e.append(instance_op(6, "ELECT_ISLEADER", strings, query=True))
    e.append(instance_op(7, "LOCK_LOCK", strings, aux=-1))
    e.append(instance_op(7, "LOCK_LOCK", strings, aux=0))
    e.append(instance_op(7, "LOCK_UNLOCK", strings))
    e.append(instance_op(8, "GROUP_JOIN", strings))
    e.append(instance_op(8, "GROUP_SCHEDULE", strings, member=1008, aux=250, a=S("Hello world!")))
    e.append(instance_op(8, "GROUP_EXECUTE", strings, member=1009, a=None))
    e.append(instance_op(8, "GROUP_LEAVE", strings))
    e.append(instance_op(1 << 40, "VALUE_GET", strings, query=True))   # an instance id no session holds
    return strings, e


def main():
    strings, e = fixture()
    here = os.path.dirname(os.path.abspath(__file__))
    blob = b"".join(x for x, _ in e)
    offs = [0]
    for x, _ in e:
        offs.append(offs[-1] + len(x))
    with open(os.path.join(here, "wire_fixture.bin"), "wb") as f:
        f.write(blob)
    with open(os.path.join(here, "wire_fixture.json"), "w") as f:
        json.dump({"comment": "written by tests/golden/make_wire.py", "strings": strings, "offsets": offs,
                   "rows": [r for _, r in e]}, f, indent=1)
        f.write("\n")
    print(f"wrote {len(e)} entries ({len(blob)} bytes)")


if __name__ == "__main__":
    main()
