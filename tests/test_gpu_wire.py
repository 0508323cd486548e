"""The reference-pinned KATs through the Catalyst wire path on the GPU: every commit of every KAT is serialized
the way an Atomix client would (tests/golden/make_wire.py, written from the reference's writeObject methods),
decoded by cc_wire_decode against the engine's session registry, and applied; manager get / create steps go
through GetResource / CreateResource entries.  The decoded columns must equal the runner's own columns, and every
KAT expectation must hold (the same expectations tests/test_gpu_kats.py checks on directly built columns)."""
import struct

import numpy as np
import pytest

from copycat_amd import abi
from tests.kat_runner import EngineBackend, KatRun, all_kats, gpu_eligible, load

pytestmark = pytest.mark.gpu

KATS = [k for k in all_kats() if gpu_eligible(k)]
NAME_OF = {h: s for s, h in load()["strings"].items()}
RES_NAME = {abi.CC_RES_VALUE: "VALUE", abi.CC_RES_MAP: "MAP", abi.CC_RES_LOCK: "LOCK", abi.CC_RES_ELECTION: "ELECTION",
            abi.CC_RES_GROUP: "GROUP", abi.CC_RES_SET: "SET", abi.CC_RES_QUEUE: "QUEUE",
            abi.CC_RES_MULTIMAP: "MULTIMAP"}
OP_NAME = {getattr(abi, n): n[len("CC_OP_"):] for n in dir(abi) if n.startswith("CC_OP_") and n != "CC_OP_DELETE"}
MAX_HANDLE = 256


def _name(h):
    return NAME_OF.get(h, f"#handle{h}")


def _value(tag, payload):
    if tag == abi.CC_TAG_NULL:
        return None
    if tag == abi.CC_TAG_LONG:
        return ("LONG", struct.unpack("<q", struct.pack("<Q", int(payload)))[0])
    if tag == abi.CC_TAG_INT:
        return ("INT", struct.unpack("<q", struct.pack("<Q", int(payload)))[0])
    if tag == abi.CC_TAG_BOOL:
        return ("BOOL", bool(payload))
    return ("STR", _name(int(payload)))


class WireBackend(EngineBackend):
    def __init__(self, kat):
        super().__init__(kat)
        from copycat_amd.wire import Interner, WireDecoder

        it = Interner(1)
        for h in range(1, MAX_HANDLE):  # handles coincide with the KAT's interned strings
            assert it.intern(_name(h)) == h
        self.D = WireDecoder(self.E, it)
        self.decoded_rows = 0

    def apply(self, b):
        from tests.golden.make_wire import instance_op

        slot_to_iid = {s: i for i, s in self.ids.items() if self.E.instance_slot(i) == s}  # still registered
        strings = [_name(h) for h in range(1, MAX_HANDLE)]
        entries = []
        for i in range(len(b)):
            op = int(b.op[i])
            if op == abi.CC_OP_DELETE:  # no wire form (ResourceStateMachine's own DeleteCommand): kept as a column row
                entries.append(instance_op(1 << 50, "VALUE_GET", strings)[0])
                continue
            f = int(b.flags[i])
            key = _value([abi.CC_TAG_LONG, abi.CC_TAG_INT, abi.CC_TAG_BOOL, abi.CC_TAG_HANDLE][abi.flag_ktag(f)], b.key[i])
            kw = dict(key=key, a=_value(abi.flag_tag_a(f), b.a[i]), b=_value(abi.flag_tag_b(f), b.b[i]),
                      aux=struct.unpack("<q", struct.pack("<Q", int(b.aux[i])))[0])
            if op in (abi.CC_OP_GROUP_SCHEDULE, abi.CC_OP_GROUP_EXECUTE):
                kw["member"] = kw.pop("key")[1]
            iid = slot_to_iid.get(int(b.inst[i]), 1 << 50)
            entries.append(instance_op(iid, OP_NAME[op], strings, **kw)[0])
        d, iids, kind = self.D.decode(entries=entries)
        assert (kind == 0).all()
        dele = b.op == abi.CC_OP_DELETE
        for name in ("inst", "op", "flags", "key", "a", "b", "aux"):
            getattr(d, name)[dele] = getattr(b, name)[dele]
        known = np.isin(b.inst, list(slot_to_iid)) | dele
        assert np.array_equal(d.inst[known], b.inst[known])
        assert (d.inst[~known] == self.E.max_instances).all()
        assert np.array_equal(d.op, b.op)
        from tests.test_wire import _carried  # fields an op's writeObject does not write decode as 0 (A2: ttl)
        for i in range(len(b)):
            if dele[i]:
                continue
            c = _carried(OP_NAME[int(b.op[i])])
            f, g = int(d.flags[i]), int(b.flags[i])
            for name, df, bf in (("a", abi.flag_tag_a(f), abi.flag_tag_a(g)), ("b", abi.flag_tag_b(f), abi.flag_tag_b(g)),
                                 ("key", abi.flag_ktag(f), abi.flag_ktag(g)), ("aux", 0, 0)):
                if name in c:
                    assert (int(getattr(d, name)[i]), df) == (int(getattr(b, name)[i]), bf), (i, name)
                else:
                    assert int(getattr(d, name)[i]) == 0 and df == 0, (i, name)
        d.index[:] = b.index
        d.time[:] = b.time
        self.decoded_rows += len(b)
        return super().apply(d)

    def manager(self, what, key, t, client, index):
        from tests.golden.make_wire import manager_op

        strings = [_name(h) for h in range(1, MAX_HANDLE)]
        entry, _ = manager_op(35 if what == "get" else 36, strings, key=_name(key), rtype=RES_NAME[t])
        d, _, kind = self.D.decode(entries=[entry])
        assert int(kind[0]) == (35 if what == "get" else 36) and int(d.key[0]) == key and int(d.a[0]) == t
        return super().manager(what, int(d.key[0]), int(d.a[0]), client, index)


@pytest.mark.parametrize("kat", KATS, ids=[k["name"] for k in KATS])
def test_kat_through_wire(kat):
    B = WireBackend(kat)
    KatRun(kat, B).run()
