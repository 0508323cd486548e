"""Host-side column encoder: committed commits -> the SoA columns of `cc_batch`.

This is the host half of the drop-in boundary.  In the reference each committed entry is an
InstanceCommand/InstanceQuery {long instance; op} (InstanceOperation.java:59-69) whose inner op carries
its operands (e.g. MapCommands.TtlCommand key/value/ttl, MapCommands.java:215-250).  The encoder turns a
run of such entries into fixed-width columns (one row per entry, log order) that the engine applies in
one call.  Values are canonical tagged values (tag, payload) — see include/copycat_apply.h.
"""
import numpy as np

from . import abi


class Batch:
    """A batch of committed entries as numpy columns (host memory)."""

    __slots__ = tuple(name for name, _ in abi.BATCH_COLUMNS)

    def __init__(self, n):
        for name, dt in abi.BATCH_COLUMNS:
            setattr(self, name, np.zeros(n, dtype=np.dtype(dt)))

    def __len__(self):
        return len(self.op)

    @classmethod
    def from_columns(cls, **cols):
        n = len(cols["op"])
        b = cls(0)
        for name, dt in abi.BATCH_COLUMNS:
            if name in cols and cols[name] is not None:
                arr = np.ascontiguousarray(cols[name], dtype=np.dtype(dt))
                if len(arr) != n:
                    raise ValueError(f"column {name} has {len(arr)} rows, expected {n}")
            else:
                arr = np.zeros(n, dtype=np.dtype(dt))
            setattr(b, name, arr)
        return b

    def slice(self, lo, hi):
        b = Batch(0)
        for name, _ in abi.BATCH_COLUMNS:
            setattr(b, name, getattr(self, name)[lo:hi].copy())  # a copy: callers reuse the source buffer
        return b

    def columns(self):
        return {name: getattr(self, name) for name, _ in abi.BATCH_COLUMNS}


def tagged(v):
    """Python value -> canonical (tag, payload).  None -> NULL; bool -> BOOL; int -> LONG.

    Use `Int(x)` for java.lang.Integer and `Handle(h)` for interned objects (strings, callbacks)."""
    if v is None:
        return abi.CC_TAG_NULL, 0
    if isinstance(v, Int):
        return abi.CC_TAG_INT, v.v & 0xFFFFFFFFFFFFFFFF
    if isinstance(v, Handle):
        return abi.CC_TAG_HANDLE, v.h
    if isinstance(v, bool):
        return abi.CC_TAG_BOOL, int(v)
    if isinstance(v, int):
        return abi.CC_TAG_LONG, v & 0xFFFFFFFFFFFFFFFF
    raise TypeError(f"no canonical encoding for {type(v)}")


def untagged(tag, payload):
    """Inverse of `tagged` (LONG payloads become signed Python ints)."""
    payload = int(payload)
    if tag == abi.CC_TAG_NULL:
        return None
    if tag == abi.CC_TAG_LONG:
        return payload - (1 << 64) if payload >> 63 else payload
    if tag == abi.CC_TAG_INT:
        p = payload & 0xFFFFFFFF
        return Int(p - (1 << 32) if p >> 31 else p)
    if tag == abi.CC_TAG_BOOL:
        return bool(payload)
    if tag == abi.CC_TAG_HANDLE:
        return Handle(payload)
    if tag == abi.CC_TAG_SET:
        return ("set", payload)
    raise ValueError(f"unknown tag {tag}")


class Int:
    """A java.lang.Integer value (Long(1) != Integer(1))."""

    __slots__ = ("v",)

    def __init__(self, v):
        self.v = int(v)

    def __eq__(self, o):
        return isinstance(o, Int) and o.v == self.v

    def __hash__(self):
        return hash(("Int", self.v))

    def __repr__(self):
        return f"Int({self.v})"


class Handle:
    """A host-interned object (String, serialized Runnable, ...): equality is handle equality."""

    __slots__ = ("h",)

    def __init__(self, h):
        self.h = int(h)

    def __eq__(self, o):
        return isinstance(o, Handle) and o.h == self.h

    def __hash__(self):
        return hash(("Handle", self.h))

    def __repr__(self):
        return f"Handle({self.h})"


def java_string_hash(s):
    """java.lang.String.hashCode: s[0]*31^(n-1) + ... + s[n-1] over the UTF-16 code units, as a Java int."""
    b = s.encode("utf-16-le")
    h = 0
    for i in range(0, len(b), 2):
        h = (31 * h + (b[i] | (b[i + 1] << 8))) & 0xFFFFFFFF
    return h - (1 << 32) if h >> 31 else h


class Interner:
    """Interns host objects (e.g. Java Strings) to HANDLE ids so `equals` is id equality."""

    def __init__(self):
        self._ids = {}
        self._objs = []

    def __call__(self, obj):
        if obj not in self._ids:
            self._ids[obj] = len(self._objs) + 1
            self._objs.append(obj)
        return Handle(self._ids[obj])

    def lookup(self, h):
        return self._objs[h.h - 1]


class Encoder:
    """Appends committed entries one at a time (for tests / small host-side batches)."""

    def __init__(self):
        self.rows = []

    def add(self, inst, op, index=0, time=0, key=None, a=None, b=None, aux=0):
        ta, pa = tagged(a)
        tb, pb = tagged(b)
        if key is None:
            kt, kp = 0, 0
        else:
            t, kp = tagged(key)
            if t == abi.CC_TAG_NULL:
                raise ValueError("map keys are never null (MapCommands.java:77)")
            kt = abi.KTAG_OF_TAG[t]
        self.rows.append((index, time, inst, op, abi.cc_flags(ta, tb, kt), kp, pa, pb, aux & 0xFFFFFFFFFFFFFFFF))
        return len(self.rows) - 1

    def batch(self):
        n = len(self.rows)
        b = Batch(n)
        for i, r in enumerate(self.rows):
            (b.index[i], b.time[i], b.inst[i], b.op[i], b.flags[i], b.key[i], b.a[i], b.b[i], b.aux[i]) = r
        return b
