"""ctypes mirror of include/copycat_apply.h (constants and structs).

tests/test_abi.py checks every constant here against the #defines of the header, so the two cannot drift.
"""
import ctypes as C

CC_ABI_VERSION = 5
CC_MEMCPY_H2D, CC_MEMCPY_D2H, CC_MEMCPY_D2D = 1, 2, 3
CC_PROFILE_KERNELS = 7
CC_PHASES = 8  # phase clocks per kernel of the diagnostics build (cc_debug_phases)

CC_OK = 0
CC_ERR_INVALID = -1
CC_ERR_HIP = -2
CC_ERR_CAPACITY = -3
CC_ERR_UNSUPPORTED = -4
CC_ERR_STATE = -5

CC_RES_NONE = 0
CC_RES_VALUE = 1
CC_RES_MAP = 2
CC_RES_LOCK = 3
CC_RES_ELECTION = 4
CC_RES_GROUP = 5
CC_RES_SET = 6
CC_RES_QUEUE = 7
CC_RES_MULTIMAP = 8
CC_QUEUE_CAP = 64

CC_OP_DELETE = 1
CC_OP_VALUE_GET = 50
CC_OP_VALUE_SET = 51
CC_OP_VALUE_CAS = 52
CC_OP_VALUE_GETANDSET = 53
CC_OP_VALUE_LISTEN = 54
CC_OP_VALUE_UNLISTEN = 55
CC_OP_MAP_CONTAINSKEY = 60
CC_OP_MAP_CONTAINSVALUE = 61
CC_OP_MAP_PUT = 62
CC_OP_MAP_PUTIFABSENT = 63
CC_OP_MAP_GET = 64
CC_OP_MAP_GETORDEFAULT = 65
CC_OP_MAP_REMOVE = 66
CC_OP_MAP_REMOVEIFPRESENT = 67
CC_OP_MAP_REPLACE = 68
CC_OP_MAP_REPLACEIFPRESENT = 69
CC_OP_MAP_ISEMPTY = 70
CC_OP_MAP_SIZE = 71
CC_OP_MAP_CLEAR = 72
CC_OP_QUEUE_CONTAINS = 90
CC_OP_QUEUE_ADD = 91
CC_OP_QUEUE_OFFER = 92
CC_OP_QUEUE_PEEK = 93
CC_OP_QUEUE_POLL = 94
CC_OP_QUEUE_ELEMENT = 95
CC_OP_QUEUE_REMOVE = 96
CC_OP_QUEUE_SIZE = 97
CC_OP_QUEUE_ISEMPTY = 98
CC_OP_QUEUE_CLEAR = 99
CC_OP_SET_CONTAINS = 100
CC_OP_SET_ADD = 101
CC_OP_SET_REMOVE = 102
CC_OP_SET_SIZE = 103
CC_OP_SET_ISEMPTY = 104
CC_OP_SET_CLEAR = 105
CC_OP_MMAP_CONTAINSKEY = 75
CC_OP_MMAP_CONTAINSENTRY = 76
CC_OP_MMAP_CONTAINSVALUE = 77
CC_OP_MMAP_PUT = 78
CC_OP_MMAP_GET = 79
CC_OP_MMAP_REMOVE = 80
CC_OP_MMAP_REMOVEVALUE = 81
CC_OP_MMAP_ISEMPTY = 82
CC_OP_MMAP_SIZE = 83
CC_OP_MMAP_CLEAR = 84
CC_OP_ELECT_LISTEN = 110
CC_OP_ELECT_UNLISTEN = 111
CC_OP_ELECT_ISLEADER = 112
CC_OP_LOCK_LOCK = 115
CC_OP_LOCK_UNLOCK = 116
CC_OP_GROUP_JOIN = 120
CC_OP_GROUP_LEAVE = 121
CC_OP_GROUP_SCHEDULE = 122
CC_OP_GROUP_EXECUTE = 123

CC_TAG_NULL = 0
CC_TAG_LONG = 1
CC_TAG_INT = 2
CC_TAG_BOOL = 3
CC_TAG_HANDLE = 4
CC_TAG_SET = 5
CC_TAG_LIST = 6

CC_ST_OK = 0
CC_ST_UNKNOWN_SESSION = 1
CC_ST_UNKNOWN_OP = 2
CC_ST_ILLEGAL_STATE = 3
CC_ST_ILLEGAL_ARGUMENT = 4
CC_ST_NULL_POINTER = 5
CC_ST_TYPE_MISMATCH = 6
CC_ST_UNKNOWN_RESOURCE = 7
CC_ST_NO_SUCH_ELEMENT = 8

CC_EV_CHANGE = 1
CC_EV_LOCK = 2
CC_EV_ELECT = 3
CC_EV_JOIN = 4
CC_EV_LEAVE = 5
CC_EV_EXECUTE = 6
CC_EV_MEMBER = 7

CC_EVSRC_COMMIT = 0
CC_EVSRC_TIMER = 1
CC_EVSRC_CLOSE = 2
CC_EVSRC_RESULT = 3

CC_CFG_TIMERS_DEFERRED = 1
CC_CFG_VALUE_EVENTS = 2
CC_CFG_VALUE_RETAINED = 4
CC_LOCK_QUEUE = 64
CC_ELECTION_LISTENERS = 64
CC_GROUP_MEMBERS = 64
CC_VALUE_LISTENERS = 64

# ops each resource type registers (ResourceStateMachine.init + Copycat reflection `configure`)
TYPE_OPS = {
    CC_RES_VALUE: {CC_OP_DELETE, 50, 51, 52, 53, 54, 55},
    CC_RES_MAP: {CC_OP_DELETE} | set(range(60, 73)),
    CC_RES_LOCK: {CC_OP_DELETE, 115, 116},
    CC_RES_ELECTION: {CC_OP_DELETE, 110, 111, 112},
    CC_RES_GROUP: {CC_OP_DELETE, 120, 121, 122, 123},
    CC_RES_SET: {CC_OP_DELETE} | set(range(100, 106)),
    CC_RES_QUEUE: {CC_OP_DELETE} | set(range(90, 100)),
    CC_RES_MULTIMAP: {CC_OP_DELETE, 75} | set(range(78, 85)),
}
# key tags of the flags column (keys are never null)
KTAG_OF_TAG = {CC_TAG_LONG: 0, CC_TAG_INT: 1, CC_TAG_BOOL: 2, CC_TAG_HANDLE: 3}
TAG_OF_KTAG = {v: k for k, v in KTAG_OF_TAG.items()}


def cc_flags(tag_a=0, tag_b=0, ktag=0):
    return (tag_a & 7) | ((tag_b & 7) << 3) | ((ktag & 3) << 6)


def flag_tag_a(f):
    return f & 7


def flag_tag_b(f):
    return (f >> 3) & 7


def flag_ktag(f):
    return (f >> 6) & 3


def cc_status(code, tag):
    return (code & 15) | ((tag & 15) << 4)


def status_code(s):
    return s & 15


def status_tag(s):
    return (s >> 4) & 15


class cc_config(C.Structure):
    _fields_ = [
        ("max_resources", C.c_uint32),
        ("max_instances", C.c_uint32),
        ("max_batch", C.c_uint64),
        ("max_events", C.c_uint64),
        ("map_capacity", C.c_uint64),
        ("device", C.c_int32),
        ("flags", C.c_uint32),
        ("sub_batch", C.c_uint64),
        ("coord_cap", C.c_uint32),
        ("reserved32", C.c_uint32),
        ("reserved", C.c_uint64 * 3),
    ]


class cc_batch(C.Structure):
    _fields_ = [
        ("index", C.c_void_p),
        ("time", C.c_void_p),
        ("inst", C.c_void_p),
        ("op", C.c_void_p),
        ("flags", C.c_void_p),
        ("key", C.c_void_p),
        ("a", C.c_void_p),
        ("b", C.c_void_p),
        ("aux", C.c_void_p),
    ]


class cc_batch_out(C.Structure):
    _fields_ = cc_batch._fields_


class cc_results(C.Structure):
    _fields_ = [("status", C.c_void_p), ("value", C.c_void_p)]


class cc_events(C.Structure):
    _fields_ = [
        ("pos", C.c_void_p),
        ("target", C.c_void_p),
        ("code", C.c_void_p),
        ("src", C.c_void_p),
        ("tag", C.c_void_p),
        ("payload", C.c_void_p),
        ("capacity", C.c_uint64),
        ("count", C.c_void_p),
    ]


# Catalyst wire format (include/copycat_apply.h "Catalyst wire format"; copycat_amd/csrc/wire.cpp)
CC_WIRE_ID_BOOLEAN = 129
CC_WIRE_ID_INTEGER = 132
CC_WIRE_ID_LONG = 133
CC_WIRE_ID_STRING = 136


class cc_wire_codec(C.Structure):
    _fields_ = [
        ("big_endian", C.c_uint8),
        ("utf8_presence_byte", C.c_uint8),
        ("utf8_len_bytes", C.c_uint8),
        ("reserved8", C.c_uint8),
        ("id_bool", C.c_int32),
        ("id_int", C.c_int32),
        ("id_long", C.c_int32),
        ("id_string", C.c_int32),
        ("reserved", C.c_uint64 * 4),
    ]


class cc_wire_out(C.Structure):
    _fields_ = [(name, C.c_void_p) for name in ("inst", "iid", "op", "flags", "key", "a", "b", "aux", "kind")]


BATCH_COLUMNS = (
    ("index", "u8"),
    ("time", "u8"),
    ("inst", "u4"),
    ("op", "u1"),
    ("flags", "u1"),
    ("key", "u8"),
    ("a", "u8"),
    ("b", "u8"),
    ("aux", "u8"),
)
