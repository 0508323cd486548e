"""The Catalyst wire-format decoder (cc_wire_decode, copycat_amd/csrc/wire.cpp) on CPU, host-only (no engine).

Fixtures: tests/golden/wire_fixture.{bin,json}, written by tests/golden/make_wire.py — an independent Python
restatement of the reference's writeObject field orders (InstanceOperation.java:60-69 and each command class).
Field order per op is pinned to those sources; the Catalyst byte conventions (identifier bytes, primitive ids,
byte order, UTF-8 framing) are not vendored: parity unpinned for the byte layout."""
import json
import os
import struct

import numpy as np
import pytest

from copycat_amd import abi
from copycat_amd.engine import EngineError

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


def _decoder():
    from copycat_amd.wire import Interner, WireDecoder

    return WireDecoder(engine=None, interner=Interner(1))


def _fixture():
    with open(os.path.join(GOLD, "wire_fixture.json")) as f:
        meta = json.load(f)
    blob = np.fromfile(os.path.join(GOLD, "wire_fixture.bin"), np.uint8)
    return meta, blob


def test_fixture_decodes_to_expected_columns():
    meta, blob = _fixture()
    d = _decoder()
    for s in meta["strings"]:  # handles 1.. in fixture order
        d.interner.intern(s)
    b, iid, kind = d.decode(buf=blob, offsets=np.array(meta["offsets"], np.uint64))
    rows = meta["rows"]
    assert len(rows) == len(b) > 50
    for i, r in enumerate(rows):
        got = {"kind": int(kind[i]), "iid": int(iid[i]), "op": int(b.op[i]), "flags": int(b.flags[i]),
               "key": int(b.key[i]), "a": int(b.a[i]), "b": int(b.b[i]), "aux": int(b.aux[i])}
        assert got == r, (i, got, r)
    # every resource operation the engine knows appears in the fixture
    ops = {int(o) for o, k in zip(b.op, kind) if k == 0}
    known = set().union(*(v - {abi.CC_OP_DELETE} for v in abi.TYPE_OPS.values()))
    assert known <= ops | {abi.CC_OP_MMAP_CONTAINSENTRY, abi.CC_OP_MMAP_CONTAINSVALUE}, sorted(known - ops)
    assert d.interner.lookup(6) == "élan" and d.interner.lookup(7) == ""


def test_strings_intern_to_one_handle_per_value():
    from tests.golden.make_wire import instance_op

    d = _decoder()
    strings = ["x", "y"]
    entries = [instance_op(9, "VALUE_SET", strings, a=("STR", s))[0] for s in ("x", "y", "x", "x")]
    b, _, _ = d.decode(entries=entries)
    assert b.a.tolist() == [1, 2, 1, 1] and (abi.flag_tag_a(b.flags) == abi.CC_TAG_HANDLE).all()


@pytest.mark.parametrize("mutate,why", [
    (lambda e: e[:-1], "truncated"),
    (lambda e: e + b"\x00", "trailing"),
    (lambda e: e[:10] + bytes([1, 49]) + e[12:], "no resource operation"),      # unknown inner id 49
    (lambda e: b"\x01\x2a" + e[2:], "not an InstanceCommand"),                   # top-level id 42
])
def test_malformed_entries_fail_loudly_with_their_row(mutate, why):
    from tests.golden.make_wire import instance_op

    good = instance_op(3, "MAP_PUT", [], key=("LONG", 1), a=("LONG", 2), aux=5)[0]
    d = _decoder()
    with pytest.raises(EngineError) as ei:
        d.decode(entries=[good, good, mutate(good)])
    assert ei.value.rc == abi.CC_ERR_INVALID and "wire row 2" in str(ei.value) and why in str(ei.value)


def test_null_key_and_user_objects_are_rejected():
    from tests.golden.make_wire import ident, instance_op

    d = _decoder()
    null_key = instance_op(3, "MAP_GET", [], key=None)[0]
    with pytest.raises(EngineError, match="null key"):
        d.decode(entries=[null_key])
    user_obj = ident(30) + struct.pack(">Q", 3) + ident(abi.CC_OP_VALUE_SET) + ident(300) + b"\x00" * 8
    with pytest.raises(EngineError, match="no canonical tag"):
        d.decode(entries=[user_obj])
    by_class = ident(30) + struct.pack(">Q", 3) + ident(abi.CC_OP_VALUE_SET) + b"\x05"
    with pytest.raises(EngineError, match="unregistered class"):
        d.decode(entries=[by_class])


def test_codec_parameters():
    """Little-endian buffers and other primitive ids decode when the codec says so."""
    from copycat_amd.wire import Interner, WireDecoder, default_codec

    c = default_codec()
    assert (c.big_endian, c.id_long) == (1, abi.CC_WIRE_ID_LONG)
    c.big_endian = 0
    c.id_long = 7
    d = WireDecoder(None, Interner(1), c)
    e = bytes([1, 30]) + struct.pack("<Q", 5) + bytes([1, 51]) + bytes([1, 7]) + struct.pack("<q", -3)
    b, iid, _ = d.decode(entries=[e])
    assert iid[0] == 5 and b.a[0] == (1 << 64) - 3 and abi.flag_tag_a(int(b.flags[0])) == abi.CC_TAG_LONG


def test_random_round_trip():
    """Random operations through the Python restatement, decoded back: every column as encoded."""
    from tests.golden.make_wire import OP, instance_op

    rng = np.random.default_rng(5)
    strings = [f"s{i}" for i in range(20)]
    d = _decoder()
    for s in strings:
        d.interner.intern(s)

    def val(nullable=True):
        k = rng.integers(0, 5 if nullable else 4)
        if k == 0:
            return ("LONG", int(rng.integers(-(1 << 62), 1 << 62)))
        if k == 1:
            return ("INT", int(rng.integers(-(1 << 31), 1 << 31)))
        if k == 2:
            return ("BOOL", bool(rng.integers(0, 2)))
        if k == 3:
            return ("STR", strings[rng.integers(0, len(strings))])
        return None

    entries, rows = [], []
    names = sorted(OP)
    for _ in range(3000):
        op = names[rng.integers(0, len(names))]
        kw = dict(key=val(False), a=val(), b=val(), aux=int(rng.integers(-100, 1000)),
                  member=int(rng.integers(0, 1 << 40)) if op.startswith("GROUP_S") or op.startswith("GROUP_E") else None)
        e, r = instance_op(int(rng.integers(1, 1 << 50)), op, strings, **kw)
        # fields an op does not carry decode as zero / NULL
        from tests.golden.make_wire import TAG
        entries.append(e)
        rows.append((op, r))
    b, iid, kind = d.decode(entries=entries)
    for i, (op, r) in enumerate(rows):
        assert int(iid[i]) == r["iid"] and int(b.op[i]) == r["op"], (i, op)
        carried = _carried(op)
        if "a" in carried:
            assert int(b.a[i]) == r["a"] and abi.flag_tag_a(int(b.flags[i])) == r["flags"] & 7, (i, op)
        if "b" in carried:
            assert int(b.b[i]) == r["b"] and abi.flag_tag_b(int(b.flags[i])) == (r["flags"] >> 3) & 7, (i, op)
        if "key" in carried:
            assert int(b.key[i]) == r["key"] and abi.flag_ktag(int(b.flags[i])) == r["flags"] >> 6, (i, op)
        if "aux" in carried:
            assert int(b.aux[i]) == r["aux"], (i, op)


def _carried(op):
    """the fields each op's writeObject chain carries (make_wire.instance_op's branches)"""
    table = {
        "VALUE_SET": "a", "VALUE_GETANDSET": "a", "VALUE_CAS": "a b",
        "MAP_CONTAINSKEY": "key", "MAP_GET": "key", "MAP_REMOVE": "key", "MMAP_CONTAINSKEY": "key",
        "MMAP_GET": "key", "MMAP_SIZE": "key", "SET_CONTAINS": "key", "SET_REMOVE": "key",
        "MAP_CONTAINSVALUE": "a", "MMAP_CONTAINSVALUE": "a", "MMAP_REMOVEVALUE": "a", "QUEUE_CONTAINS": "a",
        "QUEUE_ADD": "a", "QUEUE_OFFER": "a", "QUEUE_REMOVE": "a",
        "MAP_PUT": "key a aux", "MAP_PUTIFABSENT": "key a aux", "MAP_REPLACE": "key a aux", "MMAP_PUT": "key a aux",
        "MAP_REPLACEIFPRESENT": "key a aux b", "MAP_GETORDEFAULT": "key a", "MAP_REMOVEIFPRESENT": "key a",
        "MMAP_CONTAINSENTRY": "key a", "MMAP_REMOVE": "key a", "SET_ADD": "key aux", "LOCK_LOCK": "aux",
        "GROUP_SCHEDULE": "key aux a", "GROUP_EXECUTE": "key a",
    }
    return set(table.get(op, "").split())


def test_offsets_past_the_buffer_are_rejected():
    """ABI 3: cc_wire_decode takes the buffer length and never reads past it; WireDecoder checks offsets[-1] first."""
    import ctypes as C

    from copycat_amd.engine import lib

    meta, blob = _fixture()
    offs = np.array(meta["offsets"], np.uint64)
    d = _decoder()
    with pytest.raises(ValueError):
        d.decode(buf=blob[:-1], offsets=offs)
    # the C check itself: a buffer length one short of the last entry's end fails with that entry's row
    from copycat_amd.batch import Batch

    n = len(offs) - 1
    b = Batch(n)
    iid = np.zeros(n, np.uint64)
    kind = np.zeros(n, np.uint8)
    p = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    out = abi.cc_wire_out(inst=p(b.inst), iid=p(iid), op=p(b.op), flags=p(b.flags), key=p(b.key), a=p(b.a), b=p(b.b),
                          aux=p(b.aux), kind=p(kind))
    bad = C.c_uint64(0)
    for s in meta["strings"]:
        d.interner.intern(s)
    rc = lib().cc_wire_decode(None, C.byref(d.codec), d.interner.h, p(blob), int(offs[-1]) - 1, p(offs), n,
                              C.byref(out), C.byref(bad))
    assert rc == abi.CC_ERR_INVALID and bad.value == n - 1
