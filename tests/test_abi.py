"""The C-ABI boundary on CPU: header <-> ctypes mirror, exported symbols, host-side encoder logic.

No compute call is made here (no GPU in this container): the library is loaded and its symbol table
checked against include/copycat_apply.h."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from copycat_amd import abi
from copycat_amd.batch import Batch, Encoder, Handle, Int, Interner, tagged, untagged

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "copycat_apply.h")


def header_defines():
    out = {}
    for line in open(HEADER):
        m = re.match(r"#define\s+(CC_[A-Z0-9_]+)\s+(-?\d+)\b", line)
        if m:
            out[m.group(1)] = int(m.group(2))
    return out


def header_functions():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|void\*|const char\*)\s+(cc_[a-z_0-9]+)\s*\(", txt, re.M)))


def test_constants_match_header():
    d = header_defines()
    assert len(d) > 60
    for name, v in d.items():
        assert hasattr(abi, name), f"abi.py lacks {name}"
        assert getattr(abi, name) == v, name


def test_struct_layouts():
    assert C.sizeof(abi.cc_batch) == 9 * 8
    assert C.sizeof(abi.cc_results) == 16
    assert C.sizeof(abi.cc_events) == 8 * 8
    assert C.sizeof(abi.cc_config) == 4 + 4 + 8 + 8 + 8 + 4 + 4 + 8 + 32
    assert abi.cc_config.coord_cap.offset == 48 and abi.cc_config.reserved.offset == 56


def test_config_fields_match_header():
    """cc_config's field names and order in abi.py are the header's."""
    import re

    hdr = open(os.path.join(ROOT, "include", "copycat_apply.h")).read()
    body = hdr[hdr.index("typedef struct cc_config {"):hdr.index("} cc_config;")]
    names = re.findall(r"^\s*(?:u?int\d+_t)\s+(\w+)", body, re.M)
    assert names == [f[0] for f in abi.cc_config._fields_]


def test_engine_library_exports_every_declared_function():
    from copycat_amd import build

    so = build.build_engine()
    funcs = header_functions()
    assert "cc_apply_batch" in funcs and "cc_quorum_commit" in funcs and len(funcs) >= 20
    syms = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (cc_[a-z_0-9]+)$", syms, re.M))
    missing = [f for f in funcs if f not in exported]
    assert not missing, missing
    lib = C.CDLL(so)  # loads (HIP runtime resolved) without touching a device
    for f in funcs:
        getattr(lib, f)
    lib.cc_abi_version.restype = C.c_int
    assert lib.cc_abi_version() == abi.CC_ABI_VERSION


def test_engine_binding_covers_header():
    """Every declared entry point is bound with an explicit signature (ctypes' default restype is c_int and its
    default argtypes None, so only argtypes tells a bound symbol from an unbound one)."""
    import copycat_amd.engine as eng

    L = eng.lib()
    for f in header_functions():
        assert getattr(L, f).argtypes is not None, f"{f} is not bound in copycat_amd/engine.py"


def test_engine_is_gfx950_code_object():
    from copycat_amd import build

    so = build.build_engine()
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", so], capture_output=True, text=True)
    blob = open(so, "rb").read()
    assert b"gfx950" in blob, "engine must be compiled for gfx950"
    del out


def test_oracle_library_exports():
    from oracle import oracle_py

    oracle_py.build()
    L = oracle_py.lib()
    for f in ["orc_create", "orc_apply", "orc_session_close", "orc_quorum_commit", "orc_expire_sweep"]:
        getattr(L, f)


def test_flags_and_status_packing():
    for ta in range(6):
        for tb in range(6):
            for kt in range(4):
                f = abi.cc_flags(ta, tb, kt)
                assert (f & 7, (f >> 3) & 7, (f >> 6) & 3) == (ta, tb, kt)
    s = abi.cc_status(abi.CC_ST_ILLEGAL_STATE, abi.CC_TAG_BOOL)
    assert abi.status_code(s) == abi.CC_ST_ILLEGAL_STATE and abi.status_tag(s) == abi.CC_TAG_BOOL


def test_tagged_values_roundtrip():
    for v in [None, 0, -1, 2**63 - 1, -(2**63), True, False, Int(-5), Int(7), Handle(3)]:
        assert untagged(*tagged(v)) == v
    assert tagged(1) != tagged(Int(1))  # Long(1) != Integer(1) (A15)
    assert tagged(True) != tagged(1)


def test_encoder_and_batch():
    it = Interner()
    e = Encoder()
    e.add(3, abi.CC_OP_MAP_PUT, index=7, time=9, key=it("foo"), a=it("bar"), aux=1000)
    e.add(4, abi.CC_OP_VALUE_CAS, index=8, a=None, b=-5)
    b = e.batch()
    assert len(b) == 2 and b.inst.tolist() == [3, 4] and b.op.tolist() == [62, 52]
    assert b.flags[0] == abi.cc_flags(abi.CC_TAG_HANDLE, 0, 3)
    assert b.b[1] == (2**64 - 5)
    assert it.lookup(Handle(b.key[0])) == "foo"
    s = b.slice(1, 2)
    assert s.index.tolist() == [8]
    with pytest.raises(TypeError):
        Encoder().add(0, abi.CC_OP_MAP_GET, key=object())  # no canonical encoding


def test_batch_from_columns_validates_lengths():
    with pytest.raises(ValueError):
        Batch.from_columns(op=np.zeros(3, np.uint8), inst=np.zeros(2, np.uint32))
    b = Batch.from_columns(op=np.ones(3, np.uint8))
    assert len(b) == 3 and b.a.dtype == np.uint64
