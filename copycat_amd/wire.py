"""Catalyst wire format -> engine columns (host side of cc_wire_decode, include/copycat_apply.h).

A committed Atomix resource entry is InstanceCommand / InstanceQuery {writeLong(instance id); writeObject(op)}
(manager/src/main/java/io/atomix/resource/InstanceOperation.java:60-69); WireDecoder turns a run of such entries
(plus manager GetResource / CreateResource / DeleteResource / ResourceExists entries) into a Batch the engine
applies, resolving instance ids through the engine's session registry and interning Strings to HANDLE values."""
import ctypes as C

import numpy as np

from . import abi
from .batch import Batch
from .engine import _check, _np, lib

KIND_OP, KIND_GET, KIND_CREATE, KIND_DELETE, KIND_EXISTS = 0, 35, 36, 37, 38


def default_codec():
    c = abi.cc_wire_codec()
    lib().cc_wire_codec_default(C.byref(c))
    return c


class Interner:
    """String <-> CC_TAG_HANDLE handle (cc_wire_interner): equal bytes, equal handle."""

    def __init__(self, first_handle=1):
        self.h = C.c_void_p()
        _check(lib().cc_wire_interner_create(first_handle, C.byref(self.h)))

    def __del__(self):
        try:
            lib().cc_wire_interner_destroy(self.h)
        except Exception:
            pass

    def intern(self, s):
        b = s.encode() if isinstance(s, str) else bytes(s)
        out = C.c_uint64()
        buf = (C.c_uint8 * max(len(b), 1)).from_buffer_copy(b or b"\0")
        _check(lib().cc_wire_intern(self.h, buf, len(b), C.byref(out)))
        return out.value

    def lookup(self, handle):
        n = C.c_uint64()
        _check(lib().cc_wire_lookup(self.h, handle, None, 0, C.byref(n)))
        buf = (C.c_uint8 * max(n.value, 1))()
        _check(lib().cc_wire_lookup(self.h, handle, buf, n.value, C.byref(n)))
        return bytes(buf[:n.value]).decode()


class WireDecoder:
    """Decodes log entries (one bytes object each, or a buffer + offsets) into a Batch and per-row kinds."""

    def __init__(self, engine=None, interner=None, codec=None):
        self.engine = engine
        self.interner = interner or Interner()
        self.codec = codec or default_codec()

    def decode(self, entries=None, buf=None, offsets=None):
        if entries is not None:
            offsets = np.zeros(len(entries) + 1, np.uint64)
            offsets[1:] = np.cumsum([len(e) for e in entries])
            buf = np.frombuffer(b"".join(entries) or b"\0", np.uint8)
        n = len(offsets) - 1
        b = Batch(n)
        iid = np.zeros(n, np.uint64)
        kind = np.zeros(n, np.uint8)
        out = abi.cc_wire_out(inst=_np(b.inst), iid=_np(iid), op=_np(b.op), flags=_np(b.flags), key=_np(b.key),
                              a=_np(b.a), b=_np(b.b), aux=_np(b.aux), kind=_np(kind))
        bad = C.c_uint64(~0 & 0xFFFFFFFFFFFFFFFF)
        eh = self.engine.h if self.engine is not None else None
        buf = np.ascontiguousarray(buf, np.uint8)
        offsets = np.ascontiguousarray(offsets, np.uint64)
        if n and int(offsets[-1]) > buf.size:
            raise ValueError(f"offsets end at {int(offsets[-1])} past the {buf.size}-byte buffer")
        _check(lib().cc_wire_decode(eh, C.byref(self.codec), self.interner.h, _np(buf), buf.size, _np(offsets), n,
                                    C.byref(out), C.byref(bad)))
        return b, iid, kind
