"""ctypes binding of libcopycat_apply.so — the host mirror of the reference's state-machine interface.

`Engine` plays the role of the Copycat `StateMachine` the reference's ResourceManager implements
(manager/src/main/java/io/atomix/manager/ResourceManager.java:35-264): resources and instance sessions are
registered (getResource/createResource/deleteResource), then committed entries are applied — here a whole
batch per call instead of one `operateResource` per entry (:56-72).  Per-commit exceptions come back as
status codes (abi.CC_ST_*), never as a failed call.

The HIP library is the only compute path: if it is missing or fails to load, importing this module raises.
Torch is used only as the device allocator / stream provider (it is imported first so that the engine and
torch share one HIP runtime instance).
"""
import ctypes as C
import os

import numpy as np
import torch  # noqa: F401  (shared HIP runtime; device memory and streams)

from . import abi
from .batch import Batch

_HERE = os.path.dirname(os.path.abspath(__file__))
SO_PATH = os.environ.get("CC_ENGINE_SO") or os.path.join(_HERE, "libcopycat_apply.so")  # override: diagnostics builds
_LIB = None


# Result prefill of the test / bench paths: status 0xFF has result tag nibble 15, which no commit can return
# (tags 0..4), so a row the kernels never wrote is told apart from a legal NULL result (status 0, value 0).
RESULT_SENTINEL = 0xFF


class EngineError(RuntimeError):
    def __init__(self, rc, msg):
        super().__init__(f"cc error {rc}: {msg}")
        self.rc = rc


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(SO_PATH):
            raise ImportError(f"{SO_PATH} is missing: build it with `python -m copycat_amd.build` (hipcc, gfx950)")
        L = C.CDLL(SO_PATH)
        P, i32, u32, u64 = C.c_void_p, C.c_int, C.c_uint32, C.c_uint64
        sig = {
            "cc_abi_version": (i32, []),
            "cc_last_error": (C.c_char_p, []),
            "cc_engine_create": (i32, [P, P]),
            "cc_engine_destroy": (i32, [P]),
            "cc_sync": (i32, [P]),
            "cc_engine_stream": (P, [P]),
            "cc_resource_create": (i32, [P, u32, u32]),
            "cc_resource_create_range": (i32, [P, u32, u32, u32]),
            "cc_resource_delete": (i32, [P, u32]),
            "cc_instance_open": (i32, [P, u32, u32, u64, u64]),
            "cc_instance_open_range": (i32, [P, u32, u32, u32, u64, u64]),
            "cc_apply_batch": (i32, [P, P, u64, P, P, P]),
            "cc_apply_batch_host": (i32, [P, P, u64, P]),
            "cc_apply_batch_host_events": (i32, [P, P, u64, P, P]),
            "cc_sessions_close_host": (i32, [P, P, u64, P, P]),
            "cc_sessions_expire_host": (i32, [P, P, u64, P, P]),
            "cc_advance_time_events_host": (i32, [P, u64, P]),
            "cc_retained_bitmap_host": (i32, [P, u64, u64, P, P]),
            "cc_device_alloc": (i32, [i32, u64, P]),
            "cc_device_free": (i32, [P]),
            "cc_memcpy": (i32, [P, P, u64, i32, P]),
            "cc_memset": (i32, [P, i32, u64, P]),
            "cc_applied_index": (i32, [P, P]),
            "cc_engine_counters": (i32, [P, P, u32]),
            "cc_applied_index_async": (i32, [P, P, P]),
            "cc_read_value_state": (i32, [P, u32, u32, P, P, P]),
            "cc_read_value_retained": (i32, [P, u32, u32, P]),
            "cc_read_map_entries": (i32, [P, u32, u64, P, P, P, P, P, P]),
            "cc_read_map_table": (i32, [P, u64, P, P, P, P, P, P, P]),
            "cc_read_lock_state": (i32, [P, u32, P, P, P, u64, P, P, P]),
            "cc_read_election_state": (i32, [P, u32, P, P, u64, P, P, P]),
            "cc_read_group_members": (i32, [P, u32, u64, P, P]),
            "cc_read_retained": (i32, [P, u32, u64, P, P]),
            "cc_retained_bitmap": (i32, [P, u64, u64, P, P]),
            "cc_advance_time": (i32, [P, u64]),
            "cc_advance_time_events": (i32, [P, u64, P]),
            "cc_snapshot_size": (i32, [P, P]),
            "cc_snapshot_save": (i32, [P, P, u64]),
            "cc_snapshot_restore": (i32, [P, P, u64]),
            "cc_quorum_commit": (i32, [P, u32, u64, P, P, P, P]),
            "cc_expire_sweep": (i32, [P, u64, u64, u64, P, P, P]),
            "cc_profile_enable": (i32, [P, i32]),
            "cc_profile_reset": (i32, [P]),
            "cc_profile_read": (i32, [P, i32, P, P, P]),
            "cc_sessions_close": (i32, [P, P, u64, P, P, P]),
            "cc_sessions_expire": (i32, [P, P, u64, P, P, P]),
            "cc_get_resource": (i32, [P, u64, u32, u64, u64, P, P, P]),
            "cc_create_resource": (i32, [P, u64, u32, u64, u64, P, P, P]),
            "cc_resource_exists": (i32, [P, u64, P]),
            "cc_delete_resource": (i32, [P, u64, P]),
            "cc_instance_slot": (i32, [P, u64, P]),
            "cc_resource_slot": (i32, [P, u64, P]),
            "cc_debug_phases": (i32, [P, i32, P]),
            "cc_wire_codec_default": (None, [P]),
            "cc_wire_interner_create": (i32, [u64, P]),
            "cc_wire_interner_destroy": (i32, [P]),
            "cc_wire_intern": (i32, [P, P, u64, P]),
            "cc_wire_lookup": (i32, [P, u64, P, u64, P]),
            "cc_wire_string_hash": (i32, [P, u64, P]),
            "cc_handle_hashes": (i32, [P, P, P, u64]),
            "cc_wire_decode": (i32, [P, P, P, P, u64, P, u64, P, P]),
            "cc_split_batch": (i32, [P, u64, P, u32, u32, u32, P, P, P, P]),
            "cc_apply_batch_host_prefix": (i32, [P, P, u64, P, P, P]),
            "cc_merge_results": (i32, [P, u64, P, u32, u32, u32, P, P]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        if L.cc_abi_version() != abi.CC_ABI_VERSION:
            raise ImportError("libcopycat_apply.so ABI version mismatch")
        _LIB = L
    return _LIB


def _check(rc):
    if rc != abi.CC_OK:
        raise EngineError(rc, lib().cc_last_error().decode(errors="replace"))


def _np(a):
    return a.ctypes.data_as(C.c_void_p)


def _dptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


def _stream_ptr(stream):
    if stream is None:
        return None
    return C.c_void_p(stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream))


class DeviceBatch:
    """Batch columns resident in HBM (torch tensors on a HIP device)."""

    TORCH_DT = {"u8": torch.uint64, "u4": torch.uint32, "u1": torch.uint8}

    def __init__(self, cols, n):
        self.cols = cols
        self.n = n

    @classmethod
    def upload(cls, b: Batch, device="cuda", columns=None):
        cols = {}
        for name, dt in abi.BATCH_COLUMNS:
            if columns is not None and name not in columns:
                continue
            arr = getattr(b, name)
            cols[name] = torch.from_numpy(arr.view({"u8": np.int64, "u4": np.int32, "u1": np.uint8}[dt])).to(
                device, non_blocking=False).view(cls.TORCH_DT[dt])
        return cls(cols, len(b))

    def struct(self):
        s = abi.cc_batch()
        for name, _ in abi.BATCH_COLUMNS:
            t = self.cols.get(name)
            setattr(s, name, t.data_ptr() if t is not None else None)
        return s


class DeviceEvents:
    """An event stream in HBM (cc_events): columns of `capacity` rows + a device row counter."""

    def __init__(self, capacity, device="cuda"):
        self.capacity = capacity
        self.pos = torch.zeros(capacity, dtype=torch.int32, device=device)
        self.target = torch.zeros(capacity, dtype=torch.int32, device=device)
        self.code = torch.zeros(capacity, dtype=torch.uint8, device=device)
        self.src = torch.zeros(capacity, dtype=torch.uint8, device=device)
        self.tag = torch.zeros(capacity, dtype=torch.uint8, device=device)
        self.payload = torch.zeros(capacity, dtype=torch.int64, device=device)
        self.count = torch.zeros(1, dtype=torch.int64, device=device)

    def struct(self):
        return abi.cc_events(self.pos.data_ptr(), self.target.data_ptr(), self.code.data_ptr(), self.src.data_ptr(),
                             self.tag.data_ptr(), self.payload.data_ptr(), self.capacity, self.count.data_ptr())

    def host(self):
        m = min(int(self.count.item()), self.capacity)
        return {"pos": self.pos[:m].cpu().numpy().view(np.uint32), "target": self.target[:m].cpu().numpy().view(np.uint32),
                "code": self.code[:m].cpu().numpy(), "src": self.src[:m].cpu().numpy(), "tag": self.tag[:m].cpu().numpy(),
                "payload": self.payload[:m].cpu().numpy().view(np.uint64), "count": int(self.count.item())}


class Engine:
    def __init__(self, max_resources, max_instances, max_batch, device=0, flags=abi.CC_CFG_TIMERS_DEFERRED,
                 sub_batch=0, max_events=0, map_capacity=0, coord_cap=0):
        L = lib()
        cfg = abi.cc_config()
        cfg.coord_cap = coord_cap  # entries per coordination resource (0 = 64)
        cfg.max_resources = max_resources
        cfg.max_instances = max_instances
        cfg.max_batch = max_batch
        cfg.max_events = max_events
        cfg.map_capacity = map_capacity
        cfg.device = device
        cfg.flags = flags
        cfg.sub_batch = sub_batch
        h = C.c_void_p()
        _check(L.cc_engine_create(C.byref(cfg), C.byref(h)))
        self.h = h
        self.max_resources = max_resources
        self.max_instances = max_instances
        self.device = device
        self.L = L

    def close(self):
        if self.h:
            self.L.cc_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- registry (ResourceManager control commands, host side) --------------------------------------
    def resource_create(self, slot, rtype):
        _check(self.L.cc_resource_create(self.h, slot, rtype))

    def resource_create_range(self, first, count, rtype):
        _check(self.L.cc_resource_create_range(self.h, first, count, rtype))

    def resource_delete(self, slot):
        _check(self.L.cc_resource_delete(self.h, slot))

    def instance_open(self, inst, res, instance_id, client):
        _check(self.L.cc_instance_open(self.h, inst, res, instance_id, client))

    def instance_open_range(self, first, count, res_first, id_first, client):
        _check(self.L.cc_instance_open_range(self.h, first, count, res_first, id_first, client))

    # ---- ResourceManager control commands (ResourceManager.java:77-235; manager.hip) ------------------------
    def _ctl(self, fn, key, rtype, client, index):
        iid, islot, st = C.c_uint64(), C.c_uint32(), C.c_uint8()
        _check(fn(self.h, key, rtype, client, index, C.byref(iid), C.byref(islot), C.byref(st)))
        return st.value, iid.value, islot.value

    def get_resource(self, key, rtype, client, index):
        """GetResource commit -> (status byte, instance id, instance slot)."""
        return self._ctl(self.L.cc_get_resource, key, rtype, client, index)

    def create_resource(self, key, rtype, client, index):
        """CreateResource commit -> (status byte, instance id, instance slot)."""
        return self._ctl(self.L.cc_create_resource, key, rtype, client, index)

    def resource_exists(self, key):
        out = C.c_uint8()
        _check(self.L.cc_resource_exists(self.h, key, C.byref(out)))
        return bool(out.value)

    def delete_resource(self, resource_id):
        """DeleteResource commit (by resource id) -> status byte."""
        st = C.c_uint8()
        _check(self.L.cc_delete_resource(self.h, resource_id, C.byref(st)))
        return st.value

    def instance_slot(self, instance_id):
        out = C.c_int64()
        _check(self.L.cc_instance_slot(self.h, instance_id, C.byref(out)))
        return out.value

    def resource_slot(self, resource_id):
        out = C.c_int64()
        _check(self.L.cc_resource_slot(self.h, resource_id, C.byref(out)))
        return out.value

    # ---- session close / expire fan-out (ResourceManager.java:237-264) -----------------------------------
    def sessions_close(self, clients, capacity=1 << 16, device="cuda"):
        """Close client sessions in order; returns (instances closed, events dict as DeviceEvents.host())."""
        arr = np.ascontiguousarray(np.asarray(clients, dtype=np.uint64).reshape(-1))
        evs = DeviceEvents(capacity, device=device)
        ev = evs.struct()
        closed = C.c_uint64()
        _check(self.L.cc_sessions_close(self.h, _np(arr) if len(arr) else None, len(arr), C.byref(ev), None,
                                        C.byref(closed)))
        return closed.value, evs.host()

    def sessions_expire(self, bitmap, sessions, capacity=1 << 16, device="cuda", events=None):
        """Close every client session whose bit is set in `bitmap` (a device u64 tensor, cc_expire_sweep's output),
        in ascending id order; returns (instances closed, events).  With `events` (a DeviceEvents the caller keeps)
        the close events stay in HBM and the second value is that DeviceEvents (no host copy)."""
        evs = events if events is not None else DeviceEvents(capacity, device=device)
        ev = evs.struct()
        closed = C.c_uint64()
        _check(self.L.cc_sessions_expire(self.h, _dptr(bitmap), sessions, C.byref(ev), None, C.byref(closed)))
        return closed.value, (evs if events is not None else evs.host())

    def handle_strings(self, strings):
        """Register the java.lang.String behind each HANDLE key ({handle: str}): its String.hashCode places the key in
        MapState's java.util.HashMap (containsValue order, treeifyBin resizes; cc_handle_hashes)."""
        from .batch import java_string_hash

        items = sorted(strings.items())
        if not items:
            return
        hk = np.array([h for h, _ in items], np.uint64)
        hv = np.array([java_string_hash(x) for _, x in items], np.int32)
        _check(self.L.cc_handle_hashes(self.h, _np(hk), _np(hv), len(items)))

    # ---- the hot path ----------------------------------------------------------------------------------
    def apply(self, db: DeviceBatch, status, value, stream=None):
        """Apply device-resident columns; `status` (uint8) / `value` (uint64) are device tensors of n rows."""
        s = db.struct()
        r = abi.cc_results(status.data_ptr(), value.data_ptr())
        _check(self.L.cc_apply_batch(self.h, C.byref(s), db.n, C.byref(r), None, _stream_ptr(stream)))

    def apply_events(self, db: DeviceBatch, status, value, events: "DeviceEvents", stream=None):
        """apply() with an event stream (device tensors, see DeviceEvents)."""
        s = db.struct()
        r = abi.cc_results(status.data_ptr(), value.data_ptr())
        ev = events.struct()
        _check(self.L.cc_apply_batch(self.h, C.byref(s), db.n, C.byref(r), C.byref(ev), _stream_ptr(stream)))

    def apply_host_events(self, b: Batch, capacity=None, device="cuda"):
        """Host batch -> (status, value, events) through the device path with an event stream; events is a dict of
        numpy columns (pos, target, code, src, tag, payload) in stream order (log row, then publish order)."""
        n = len(b)
        db = DeviceBatch.upload(b, device=device)
        status = torch.zeros(n, dtype=torch.uint8, device=device)
        value = torch.zeros(n, dtype=torch.int64, device=device)
        status.fill_(RESULT_SENTINEL)  # a row no kernel writes stays 0xFF: never a legal status (see RESULT_SENTINEL)
        value.fill_(-0x5A5A5A5A5A5A5A5B)
        evs = DeviceEvents(capacity if capacity is not None else max(4 * n, 1024), device=device)
        self.apply_events(db, status, value, evs)
        self.sync()
        return status.cpu().numpy(), value.cpu().numpy().view(np.uint64), evs.host()

    def apply_host(self, b: Batch):
        """PCIe-inclusive path: host columns in, host results out (H2D + apply + D2H + sync)."""
        n = len(b)
        status = np.full(n, RESULT_SENTINEL, np.uint8)  # cc_apply_batch_host prefills too; a row never written stays 0xFF
        value = np.zeros(n, np.uint64)
        s = abi.cc_batch()
        for name, _ in abi.BATCH_COLUMNS:
            setattr(s, name, getattr(b, name).ctypes.data)
        r = abi.cc_results(status.ctypes.data, value.ctypes.data)
        _check(self.L.cc_apply_batch_host(self.h, C.byref(s), n, C.byref(r)))
        return status, value

    def apply_host_prefix(self, b: Batch, capacity=None):
        """cc_apply_batch_host_prefix: rows applied up to the first commit a full coordination collection cannot hold.
        Returns (applied, status, value, events): `applied` = rows applied (len(b) on success; the engine state is the
        one after exactly those rows), events as apply_host_events returns them (numpy columns)."""
        n = len(b)
        status = np.full(n, RESULT_SENTINEL, np.uint8)
        value = np.zeros(n, np.uint64)
        s = abi.cc_batch()
        for name, _ in abi.BATCH_COLUMNS:
            setattr(s, name, getattr(b, name).ctypes.data)
        r = abi.cc_results(status.ctypes.data, value.ctypes.data)
        cap = capacity if capacity is not None else max(4 * n, 1024)
        cols = {"pos": np.zeros(cap, np.uint32), "target": np.zeros(cap, np.uint32), "code": np.zeros(cap, np.uint8),
                "src": np.zeros(cap, np.uint8), "tag": np.zeros(cap, np.uint8), "payload": np.zeros(cap, np.uint64)}
        count = np.zeros(1, np.uint64)
        ev = abi.cc_events(*(cols[k].ctypes.data for k in ("pos", "target", "code", "src", "tag", "payload")), cap,
                           count.ctypes.data)
        applied = C.c_uint64()
        rc = self.L.cc_apply_batch_host_prefix(self.h, C.byref(s), n, C.byref(r), C.byref(ev), C.byref(applied))
        if rc not in (abi.CC_OK, abi.CC_ERR_CAPACITY) or (rc == abi.CC_ERR_CAPACITY and applied.value >= n):
            _check(rc)
        m = int(min(count[0], cap))
        return applied.value, status, value, {k: v[:m] for k, v in cols.items()}

    def sync(self):
        _check(self.L.cc_sync(self.h))

    def stream(self):
        return self.L.cc_engine_stream(self.h)

    def counters(self):
        """(barrier rows applied, containsValue rows answered in the stream, sub-batches, map events) since creation,
        and the big HashMap models held now (maps past capacity 64 with a tree bin)."""
        out = np.zeros(5, np.uint64)
        _check(self.L.cc_engine_counters(self.h, out.ctypes.data, 5))
        return tuple(int(x) for x in out)

    def applied_index(self):
        out = C.c_uint64()
        _check(self.L.cc_applied_index(self.h, C.byref(out)))
        return out.value

    def applied_index_async(self, out, stream=None):
        """Write the applied watermark into the device tensor `out` (one int64), stream-ordered, no host sync."""
        _check(self.L.cc_applied_index_async(self.h, C.c_void_p(out.data_ptr()), _stream_ptr(stream)))

    # ---- per-kernel HIP-event timing ------------------------------------------------------------------
    def profile(self, on=True):
        _check(self.L.cc_profile_enable(self.h, 1 if on else 0))
        _check(self.L.cc_profile_reset(self.h))

    def profile_read(self):
        """{kernel name: (total device ms, launches)} since the last profile() call (synchronizes)."""
        out = {}
        for k in range(abi.CC_PROFILE_KERNELS):
            ms, n, name = C.c_double(), C.c_uint64(), C.c_char_p()
            _check(self.L.cc_profile_read(self.h, k, C.byref(ms), C.byref(n), C.byref(name)))
            out[name.value.decode()] = (ms.value, n.value)
        return out

    def value_state(self, first=0, count=None):
        count = self.max_resources - first if count is None else count
        tag, val, cur = np.zeros(count, np.uint8), np.zeros(count, np.uint64), np.zeros(count, np.uint8)
        _check(self.L.cc_read_value_state(self.h, first, count, _np(tag), _np(val), _np(cur)))
        return tag, val, cur

    def value_retained(self, first=0, count=None):
        """Per value slot, the log index of the commit AtomicValueState still retains (0 = none)."""
        count = self.max_resources - first if count is None else count
        idx = np.zeros(count, np.uint64)
        _check(self.L.cc_read_value_retained(self.h, first, count, _np(idx)))
        return idx

    def advance_time(self, now):
        _check(self.L.cc_advance_time(self.h, now))

    def advance_time_events(self, now, capacity=1024, device="cuda"):
        """advance_time publishing the events of group timers that come due (see cc_advance_time_events)."""
        evs = DeviceEvents(capacity, device=device)
        ev = evs.struct()
        _check(self.L.cc_advance_time_events(self.h, now, C.byref(ev)))
        return evs.host()

    def snapshot(self) -> bytes:
        """The engine's whole state (device arrays + host registry mirrors) as bytes (cc_snapshot_save)."""
        n = C.c_uint64()
        _check(self.L.cc_snapshot_size(self.h, C.byref(n)))
        buf = np.zeros(n.value, np.uint8)
        _check(self.L.cc_snapshot_save(self.h, _np(buf), n.value))
        return buf.tobytes()

    def restore(self, snap: bytes):
        """Load a snapshot into this engine (same max_resources / max_instances / map_capacity)."""
        buf = np.frombuffer(snap, np.uint8).copy()
        _check(self.L.cc_snapshot_restore(self.h, _np(buf), len(buf)))

    def lock_state(self, slot, cap=1024):
        """(holder instance slot or -1, holder index, holder cleaned, [(waiter instance slot, index)])"""
        h, hi, hc, n = C.c_int64(), C.c_uint64(), C.c_uint8(), C.c_uint64()
        qi, qx = np.zeros(cap, np.uint32), np.zeros(cap, np.uint64)
        _check(self.L.cc_read_lock_state(self.h, slot, C.byref(h), C.byref(hi), C.byref(hc), cap, C.byref(n), _np(qi),
                                         _np(qx)))
        m = min(n.value, cap)
        return h.value, hi.value, hc.value, list(zip(qi[:m].tolist(), qx[:m].tolist()))

    def election_state(self, slot, cap=1024):
        """(leader instance slot or -1, leader index, [(listener instance slot, index)])"""
        ld, li, n = C.c_int64(), C.c_uint64(), C.c_uint64()
        qi, qx = np.zeros(cap, np.uint32), np.zeros(cap, np.uint64)
        _check(self.L.cc_read_election_state(self.h, slot, C.byref(ld), C.byref(li), cap, C.byref(n), _np(qi), _np(qx)))
        m = min(n.value, cap)
        return ld.value, li.value, list(zip(qi[:m].tolist(), qx[:m].tolist()))

    def group_members(self, slot, cap=4096):
        ids, n = np.zeros(cap, np.uint64), C.c_uint64()
        _check(self.L.cc_read_group_members(self.h, slot, cap, C.byref(n), _np(ids)))
        return ids[:min(n.value, cap)].tolist()

    def retained(self, slot):
        """Ascending log indices of every commit the slot's state machine still holds without having clean()ed it
        (cc_read_retained) — the layout of the oracle's retained()."""
        n = C.c_uint64()
        _check(self.L.cc_read_retained(self.h, slot, 0, C.byref(n), None))
        out = np.zeros(max(n.value, 1), np.uint64)
        _check(self.L.cc_read_retained(self.h, slot, n.value, C.byref(n), _np(out)))
        return out[:n.value].tolist()

    def retained_bitmap(self, first, count, out=None, device="cuda"):
        """cc_retained_bitmap: (device u64 bitmap over log indices [first, first + count), retained count)."""
        words = (count + 63) // 64
        bm = out if out is not None else torch.empty(max(words, 1), dtype=torch.int64, device=device)
        n = C.c_uint64()
        _check(self.L.cc_retained_bitmap(self.h, first, count, _dptr(bm), C.byref(n)))
        return bm, n.value

    def map_entries(self, slot):
        """MapState entries of one map slot sorted by (key tag, key): (key_tag, key, value_tag, value, commit_index)
        — the same layout as the oracle's map_entries."""
        n = C.c_uint64()
        _check(self.L.cc_read_map_entries(self.h, slot, 0, C.byref(n), None, None, None, None, None))
        m = n.value
        kt, k, vt, v, ci = (np.zeros(m, np.uint8), np.zeros(m, np.uint64), np.zeros(m, np.uint8),
                            np.zeros(m, np.uint64), np.zeros(m, np.uint64))
        _check(self.L.cc_read_map_entries(self.h, slot, m, C.byref(n), _np(kt), _np(k), _np(vt), _np(v), _np(ci)))
        return kt, k, vt, v, ci

    def map_table(self):
        """Every map / set slot's entries in one table pass, sorted by (slot, key tag, key):
        (slot, key_tag, key, value_tag, value, commit_index)."""
        n = C.c_uint64()
        _check(self.L.cc_read_map_table(self.h, 0, C.byref(n), None, None, None, None, None, None))
        m = n.value
        sl, kt, k, vt, v, ci = (np.zeros(m, np.uint32), np.zeros(m, np.uint8), np.zeros(m, np.uint64),
                                np.zeros(m, np.uint8), np.zeros(m, np.uint64), np.zeros(m, np.uint64))
        _check(self.L.cc_read_map_table(self.h, m, C.byref(n), _np(sl), _np(kt), _np(k), _np(vt), _np(v), _np(ci)))
        return sl, kt, k, vt, v, ci


def quorum_commit(match, term_start, commit_in, commit_out, stream=None):
    """match: (replicas, groups) uint64 device tensor; others (groups,) uint64 device tensors."""
    replicas, groups = match.shape
    _check(lib().cc_quorum_commit(_dptr(match), replicas, groups, _dptr(term_start), _dptr(commit_in), _dptr(commit_out),
                                  _stream_ptr(stream)))


def expire_sweep(last, now, timeout, bitmap, count, stream=None):
    _check(lib().cc_expire_sweep(_dptr(last), last.numel(), now, timeout, _dptr(bitmap), _dptr(count),
                                 _stream_ptr(stream)))
