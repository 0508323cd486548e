// host_path.hip — the host-memory entry points of the C-ABI (host code only).
//
// A JVM host (Panama FFM / JNI) hands the engine Java heap or off-heap host memory, not HBM
// pointers.  These calls stage host columns into engine-owned device buffers (grown on demand and kept between
// calls: no hipMalloc / hipFree per batch), run the device entry point, and copy results AND events back, so every
// reference path that publishes -- Session.publish -> InstanceEvent{instance, msg}
// (manager/src/main/java/io/atomix/manager/ManagedResourceSession.java:64-71,
//  manager/src/main/java/io/atomix/resource/InstanceEvent.java:29-80) -- has a host-memory route:
//   cc_apply_batch_host / cc_apply_batch_host_events   ResourceManager.operateResource per entry (:56-72)
//   cc_sessions_close_host / cc_sessions_expire_host    ResourceManager.close / expire (:237-264)
//   cc_advance_time_events_host                         timer callbacks (ResourceManagerStateMachineExecutor :104-116)
//   cc_retained_bitmap_host                             the compaction feed (ResourceManagerCommit.clean :79-81)
// plus a plain device-memory API (cc_device_alloc / cc_memcpy ...) for the stateless device calls
// (cc_quorum_commit, cc_expire_sweep) and for hosts that keep columns resident.
#include <algorithm>
#include <cstring>

#include <unordered_map>

#include "engine_state.h"

namespace {

enum HwSlot : int {
  kHwCol = 0,  // 9 input columns
  kHwStatus = 9,
  kHwValue,
  kHwEvPos,
  kHwEvTarget,
  kHwEvCode,
  kHwEvSrc,
  kHwEvTag,
  kHwEvPayload,
  kHwEvCount,
  kHwBitmap,
  kHwNum
};
static_assert(kHwNum <= 24, "cc_engine::hw_buf");

// Device buffer `slot` with room for `bytes` (the previous contents are not kept).  The callers are synchronous, so
// no launch of an earlier call still reads a buffer that is replaced here.
int hw(cc_engine* e, int slot, size_t bytes, void** out) {
  bytes = std::max<size_t>(bytes, 256);
  if (e->hw_cap[slot] < bytes) {
    const size_t cap = std::max(bytes, e->hw_cap[slot] * 3 / 2);  // grow by half: no free + malloc per call
    if (e->hw_buf[slot]) (void)hipFree(e->hw_buf[slot]);
    e->hw_buf[slot] = nullptr;
    e->hw_cap[slot] = 0;
    hipError_t x = hipMalloc(&e->hw_buf[slot], cap);
    if (x != hipSuccess) return set_err(CC_ERR_HIP, "hipMalloc (host-path staging)", x);
    e->hw_cap[slot] = cap;
  }
  *out = e->hw_buf[slot];
  return CC_OK;
}

// Device event columns of `cap` rows mirroring the host cc_events `h` (null: no event stream).
int hw_events(cc_engine* e, const cc_events* h, cc_events* d) {
  std::memset(d, 0, sizeof *d);
  if (!h) return CC_OK;
  if (!h->count || (h->capacity && (!h->pos || !h->target || !h->code || !h->src || !h->tag || !h->payload)))
    return set_err(CC_ERR_INVALID, "host event stream: null column or count");
  const size_t c = std::max<uint64_t>(h->capacity, 1);
  int rc;
  void* p;
  if ((rc = hw(e, kHwEvPos, 4 * c, &p))) return rc;
  d->pos = (uint32_t*)p;
  if ((rc = hw(e, kHwEvTarget, 4 * c, &p))) return rc;
  d->target = (uint32_t*)p;
  if ((rc = hw(e, kHwEvCode, c, &p))) return rc;
  d->code = (uint8_t*)p;
  if ((rc = hw(e, kHwEvSrc, c, &p))) return rc;
  d->src = (uint8_t*)p;
  if ((rc = hw(e, kHwEvTag, c, &p))) return rc;
  d->tag = (uint8_t*)p;
  if ((rc = hw(e, kHwEvPayload, 8 * c, &p))) return rc;
  d->payload = (uint64_t*)p;
  if ((rc = hw(e, kHwEvCount, 8, &p))) return rc;
  d->count = (uint64_t*)p;
  d->capacity = h->capacity;
  HIPCHECK(hipMemsetAsync(d->count, 0, sizeof(uint64_t), e->own_stream));
  return CC_OK;
}

// Events back to the host: *h->count = the events published (may exceed capacity: then the call fails with
// CC_ERR_CAPACITY, and the first `capacity` rows are still copied).
int hw_events_back(cc_engine* e, const cc_events* h, const cc_events* d) {
  if (!h) return CC_OK;
  hipStream_t st = e->own_stream;
  uint64_t cnt = 0;
  HIPCHECK(hipMemcpyAsync(&cnt, d->count, sizeof cnt, hipMemcpyDeviceToHost, st));
  HIPCHECK(hipStreamSynchronize(st));
  *h->count = cnt;
  const uint64_t m = std::min<uint64_t>(cnt, h->capacity);
  if (m) {
    HIPCHECK(hipMemcpyAsync(h->pos, d->pos, 4 * m, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipMemcpyAsync(h->target, d->target, 4 * m, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipMemcpyAsync(h->code, d->code, m, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipMemcpyAsync(h->src, d->src, m, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipMemcpyAsync(h->tag, d->tag, m, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipMemcpyAsync(h->payload, d->payload, 8 * m, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipStreamSynchronize(st));
  }
  if (cnt <= h->capacity) return CC_OK;
  e->last_err_bits |= kErrEvents;  // (cc_apply_batch_host_prefix: a full event stream, like a full max_events arena)
  return set_err(CC_ERR_CAPACITY, "more events than the host event stream holds");
}

int apply_host(cc_engine* e, const cc_batch* h, uint64_t n, const cc_results* hout, const cc_events* hev) {
  if (!e || !h || !hout || (n && (!hout->status || !hout->value))) return set_err(CC_ERR_INVALID, "null argument");
  HIPCHECK(hipSetDevice(e->device));
  e->last_err_bits = 0;
  hipStream_t st = e->own_stream;
  if (st != e->last_stream) HIPCHECK(hipStreamSynchronize(e->last_stream));
  e->last_stream = st;
  cc_events dev{};
  int rc = hw_events(e, hev, &dev);
  if (rc) return rc;
  if (n == 0) {
    if (hev) *hev->count = 0;
    return CC_OK;
  }
  const void* src[9] = {h->index, h->time, h->inst, h->op, h->flags, h->key, h->a, h->b, h->aux};
  const size_t esz[9] = {8, 8, 4, 1, 1, 8, 8, 8, 8};
  void* dcol[9] = {};
  for (int c = 0; c < 9; ++c) {
    if (!src[c]) continue;
    if ((rc = hw(e, kHwCol + c, esz[c] * n, &dcol[c]))) return rc;
    HIPCHECK(hipMemcpyAsync(dcol[c], src[c], esz[c] * n, hipMemcpyHostToDevice, st));
  }
  void *d_status, *d_value;
  if ((rc = hw(e, kHwStatus, n, &d_status)) || (rc = hw(e, kHwValue, 8 * n, &d_value))) return rc;
  // sentinel prefill: status 0xFF is no legal status (tag nibble 15), so a row the kernels never wrote comes back as
  // 0xFF instead of passing for a legal NULL result (status 0, value 0)
  HIPCHECK(hipMemsetAsync(d_status, 0xFF, n, st));
  HIPCHECK(hipMemsetAsync(d_value, 0xA5, 8 * n, st));
  cc_batch d{};
  d.index = (const uint64_t*)dcol[0];
  d.time = (const uint64_t*)dcol[1];
  d.inst = (const uint32_t*)dcol[2];
  d.op = (const uint8_t*)dcol[3];
  d.flags = (const uint8_t*)dcol[4];
  d.key = (const uint64_t*)dcol[5];
  d.a = (const uint64_t*)dcol[6];
  d.b = (const uint64_t*)dcol[7];
  d.aux = (const uint64_t*)dcol[8];
  cc_results r{(uint8_t*)d_status, (uint64_t*)d_value};
  rc = cc_apply_batch(e, &d, n, &r, hev ? &dev : nullptr, st);
  if (rc) {
    (void)hipStreamSynchronize(st);
    return rc;
  }
  HIPCHECK(hipMemcpyAsync(hout->status, d_status, n, hipMemcpyDeviceToHost, st));
  HIPCHECK(hipMemcpyAsync(hout->value, d_value, 8 * n, hipMemcpyDeviceToHost, st));
  const int rs = cc_sync(e);  // device-side checks (capacity, unsupported ops, time order) after the D2H
  const int re = hw_events_back(e, hev, &dev);
  return rs ? rs : re;
}

}  // namespace

extern "C" int cc_apply_batch_host(cc_engine* e, const cc_batch* h_cols, uint64_t n, const cc_results* h_out) {
  return apply_host(e, h_cols, n, h_out, nullptr);
}

extern "C" int cc_apply_batch_host_events(cc_engine* e, const cc_batch* h_cols, uint64_t n, const cc_results* h_out,
                                          const cc_events* h_events) {
  if (!h_events) return set_err(CC_ERR_INVALID, "null event stream (use cc_apply_batch_host)");
  return apply_host(e, h_cols, n, h_out, h_events);
}

// ---- a batch applied up to the first commit the engine cannot hold (ABI 5) ------------------------------------------
// Java's collections are unbounded (LockState's ArrayDeque, LeaderElectionState's LinkedHashMap, MembershipGroupState's
// HashMap, QueueState, AtomicValueState's listeners: LockState.java:35, ...); the engine's coordination blocks hold
// coord_cap entries.  cc_apply_batch fails such a batch after applying it (CC_ERR_CAPACITY).  This call instead applies
// exactly the rows before the first commit that would overflow a collection and reports them: *applied = that row
// (n when every row applied), the state is the one after rows [0, *applied), and the row itself and every row after
// it are not applied (their results are not written), so the host can act (a larger engine from a snapshot, or the
// commit failed) and resume at that row.
//   1. Rows that can add an entry (lock with a timeout != 0, election listen, group join, value listen, queue
//      add / offer) are the only ones that can overflow.  Every resource they address starts with its block's entry
//      count (one strided copy of the block headers), and one pass over the batch keeps an upper bound per resource
//      (+1 per adding row; removals are not counted, so it never falls short).  The rows before the first adding
//      row whose bound would pass coord_cap go as one call.
//   2. At that row the resource's count is read again (after the rows before it: the bound's slack is gone); if the
//      row fits, the pass goes on.  Else the row goes alone: if the device reports a full collection (kErrCoordFull,
//      and nothing else), its resource block, the clock, the applied index and the pending group timers are restored
//      (the engine skips the entry it cannot hold, so nothing else moved) and the call stops there; if it applied
//      (the op did not add after all), the count is read once more and the pass goes on.
// Each row is scanned once, and a stop costs one header read: a queue that stays near coord_cap under churn costs a
// call per stop, not a rescan of the batch.  Other fixed capacities (a full map table region, max_events) still fail
// the call after applying it.
namespace {

bool adds_entry(uint8_t type, uint8_t op, uint64_t aux) {
  switch (type) {
    case CC_RES_LOCK: return op == CC_OP_LOCK_LOCK && aux != 0;  // tryLock() (timeout 0) never queues
    case CC_RES_ELECTION: return op == CC_OP_ELECT_LISTEN;
    case CC_RES_GROUP: return op == CC_OP_GROUP_JOIN;
    case CC_RES_VALUE: return op == CC_OP_VALUE_LISTEN;
    case CC_RES_QUEUE: return op == CC_OP_QUEUE_ADD || op == CC_OP_QUEUE_OFFER;
    default: return false;
  }
}

// apply host rows [lo, hi) appending to the host event stream `hev` (rows shifted to batch positions); *ev_n = events
// so far
int apply_part(cc_engine* e, const cc_batch* h, uint64_t lo, uint64_t hi, const cc_results* hout, const cc_events* hev,
               uint64_t* ev_n) {
  auto sh = [lo](const auto* p) { return p ? p + lo : p; };
  const cc_batch part{sh(h->index), sh(h->time), sh(h->inst), sh(h->op), sh(h->flags), sh(h->key), sh(h->a), sh(h->b),
                      sh(h->aux)};
  const cc_results o{hout->status + lo, hout->value + lo};
  if (!hev) return apply_host(e, &part, hi - lo, &o, nullptr);
  uint64_t cnt = 0;
  cc_events v = *hev;
  const uint64_t k = std::min(*ev_n, hev->capacity);
  v.pos += k, v.target += k, v.code += k, v.src += k, v.tag += k, v.payload += k;
  v.capacity -= k;
  v.count = &cnt;
  const int rc = apply_host(e, &part, hi - lo, &o, &v);
  for (uint64_t i = 0; i < std::min(cnt, v.capacity); ++i) v.pos[i] += (uint32_t)lo;
  *ev_n += cnt;
  return rc;
}

}  // namespace

extern "C" int cc_apply_batch_host_prefix(cc_engine* e, const cc_batch* h, uint64_t n, const cc_results* hout,
                                          const cc_events* hev, uint64_t* h_applied) {
  if (!e || !h || !hout || !h_applied || (n && (!h->inst || !h->op))) return set_err(CC_ERR_INVALID, "null argument");
  if (hev && (!hev->count || (hev->capacity && (!hev->pos || !hev->target || !hev->code || !hev->src || !hev->tag ||
                                                !hev->payload))))
    return set_err(CC_ERR_INVALID, "host event stream: null column or count");
  *h_applied = 0;
  uint64_t ev_n = 0;
  auto finish = [&](int rc) {
    if (hev) *hev->count = ev_n;
    return rc;
  };
  HIPCHECK(hipSetDevice(e->device));
  // Rows [lo, hi) as one part.  On an engine with maps or with an event stream, a part may also fail on a full map
  // table region or a full event stream (kErrCapacity / kErrEvents, and nothing else): the state before the part is a
  // device checkpoint (ckpt_save), and the longest prefix of the part that applies is found by bisection (restore, apply
  // [lo, mid)); the state is then the one after that prefix, its results and events written, the rows after it keep
  // what the caller had there.  *done = the first row not applied (hi on success).
  const bool ck = e->map_bits != 0 || hev != nullptr;
  auto cap_only = [&](int rc) {
    const uint32_t b = e->last_err_bits;
    return rc == CC_ERR_CAPACITY && b && !(b & ~(kErrCapacity | kErrEvents));
  };
  auto attempt = [&](uint64_t lo, uint64_t hi, uint64_t* done) -> int {
    *done = lo;
    if (!ck) {
      const int rc = apply_part(e, h, lo, hi, hout, hev, &ev_n);
      if (!rc) *done = hi;
      return rc;
    }
    std::vector<uint8_t> s0(hout->status + lo, hout->status + hi);  // (the caller's rows, for the rows not applied)
    std::vector<uint64_t> v0(hout->value + lo, hout->value + hi);
    const uint64_t ev0 = ev_n;
    int rc = ckpt_save(e);
    if (rc) return rc;
    rc = apply_part(e, h, lo, hi, hout, hev, &ev_n);
    if (!rc) {
      *done = hi;
      return CC_OK;
    }
    if (!cap_only(rc)) return rc;
    uint64_t good = lo, bad = hi;  // [lo, good) applies, [lo, bad) does not
    bool at_good = false;          // the engine's state is the one after [lo, good)
    while (bad - good > 1) {
      const uint64_t mid = good + (bad - good) / 2;
      if ((rc = ckpt_restore(e))) return rc;
      ev_n = ev0;
      rc = apply_part(e, h, lo, mid, hout, hev, &ev_n);
      if (!rc) {
        good = mid;
        at_good = true;
      } else if (cap_only(rc)) {
        bad = mid;
        at_good = false;
      } else {
        return rc;
      }
    }
    if (!at_good) {
      if ((rc = ckpt_restore(e))) return rc;
      ev_n = ev0;
      if (good > lo && (rc = apply_part(e, h, lo, good, hout, hev, &ev_n))) return rc;
    }
    std::copy(s0.begin() + (good - lo), s0.end(), hout->status + good);
    std::copy(v0.begin() + (good - lo), v0.end(), hout->value + good);
    *done = good;
    return CC_ERR_CAPACITY;
  };
  auto full = [&](uint64_t row) {
    *h_applied = row;
    return finish(set_err(CC_ERR_CAPACITY, "a map table region or the event stream is full: *applied rows were applied"));
  };
  if (!e->coord_on) {  // no coordination collection to overflow: one part
    uint64_t done = 0;
    const int rc = n ? attempt(0, n, &done) : CC_OK;
    if (rc == CC_ERR_CAPACITY && done < n) return full(done);
    if (!rc) *h_applied = n;
    return finish(rc);
  }
  const uint32_t max_inst = e->cfg.max_instances;
  auto res_of = [&](uint64_t i) -> uint32_t {
    const uint32_t in = h->inst[i];
    return in < max_inst ? e->inst_res[in] : kNoRes;
  };
  const uint32_t cap = e->coord_cap;
  const size_t blk = coord_block(cap);
  auto adds = [&](uint64_t i, uint32_t r) {
    return r != kNoRes && r < e->res_type.size() && adds_entry(e->res_type[r], h->op[i], h->aux ? h->aux[i] : 0);
  };
  auto entries = [&](uint32_t r, uint32_t* out) -> int {  // one block's current entry count (CoordHdr.n)
    CoordHdr hd{};
    HIPCHECK(hipMemcpy(&hd, e->d_coord + (uint64_t)r * blk, sizeof hd, hipMemcpyDeviceToHost));
    *out = hd.n;
    return CC_OK;
  };
  // the upper bound of every addressed resource's entry count, from one strided copy of the block headers over the
  // slot range the adding rows address
  std::unordered_map<uint32_t, uint64_t> bound;
  {
    uint32_t rlo = ~0u, rhi = 0;
    for (uint64_t i = 0; i < n; ++i) {
      const uint32_t r = res_of(i);
      if (adds(i, r)) rlo = std::min(rlo, r), rhi = std::max(rhi, r);
    }
    if (rlo <= rhi) {
      std::vector<CoordHdr> hdr(rhi - rlo + 1);
      HIPCHECK(hipMemcpy2D(hdr.data(), sizeof(CoordHdr), e->d_coord + (uint64_t)rlo * blk, blk, sizeof(CoordHdr),
                           hdr.size(), hipMemcpyDeviceToHost));
      for (uint64_t i = 0; i < n; ++i) {
        const uint32_t r = res_of(i);
        if (adds(i, r) && !bound.count(r)) bound[r] = hdr[r - rlo].n;
      }
    }
  }
  uint64_t pos = 0, i = 0;  // rows [0, pos) applied; rows [pos, i) scanned (their adds are in the bounds)
  while (pos < n) {
    uint64_t stop = n;  // the first row whose bound would pass coord_cap
    for (; i < n; ++i) {
      const uint32_t r = res_of(i);
      if (!adds(i, r)) continue;
      uint64_t& b = bound[r];
      if (b + 1 > cap) {
        stop = i;
        break;
      }
      ++b;
    }
    if (stop > pos) {
      uint64_t done = pos;
      const int rc = attempt(pos, stop, &done);
      if (rc == CC_ERR_CAPACITY && done < stop) return full(done);
      if (rc) return finish(rc);
      pos = stop;
      *h_applied = pos;
      if (pos == n) break;
    }
    // row pos (= stop) may overflow: its resource's count now (rows before it applied)
    const uint32_t r = res_of(pos);
    uint32_t cur = 0;
    {
      int rc = entries(r, &cur);
      if (rc) return finish(rc);
    }
    if ((uint64_t)cur + 1 <= cap) {  // it fits: the pass goes on from this row with the exact count
      bound[r] = cur;
      continue;
    }
    // row pos alone: its resource's block, the clock, the applied index and the group timers are saved first
    std::vector<uint8_t> saved(blk);
    uint64_t clock = 0, last = 0;
    HIPCHECK(hipMemcpy(saved.data(), e->d_coord + (uint64_t)r * blk, blk, hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(&clock, e->d_clock, sizeof clock, hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(&last, e->d_last_index, sizeof last, hipMemcpyDeviceToHost));
    const bool pending = e->applied_pending;
    const uint64_t applied0 = e->applied;
    const auto gtimers = e->gtimers;
    const uint64_t ev0 = ev_n;
    const uint8_t st0 = hout->status[pos];
    const uint64_t va0 = hout->value[pos];
    uint64_t done1 = pos;
    const int rc = attempt(pos, pos + 1, &done1);
    if (rc == CC_ERR_CAPACITY && e->last_err_bits != kErrCoordFull) return full(pos);
    // (only a full coordination collection, and nothing else, is rolled back: any other failure is returned as is)
    if (rc == CC_ERR_CAPACITY && e->last_err_bits == kErrCoordFull) {
      hout->status[pos] = st0;  // (the row is not applied: its result row keeps what the caller had there)
      hout->value[pos] = va0;
      HIPCHECK(hipMemcpy(e->d_coord + (uint64_t)r * blk, saved.data(), blk, hipMemcpyHostToDevice));
      HIPCHECK(hipMemcpy(e->d_clock, &clock, sizeof clock, hipMemcpyHostToDevice));
      HIPCHECK(hipMemcpy(e->d_last_index, &last, sizeof last, hipMemcpyHostToDevice));
      e->applied_pending = pending;
      e->applied = applied0;
      e->gtimers = gtimers;
      ev_n = ev0;
      return finish(set_err(CC_ERR_CAPACITY, "a coordination collection is full (coord_cap): *applied rows were applied"));
    }
    if (rc) return finish(rc);
    pos += 1;
    i = pos;
    *h_applied = pos;
    {
      int rc2 = entries(r, &cur);
      if (rc2) return finish(rc2);
    }
    bound[r] = cur;
  }
  return finish(CC_OK);
}

extern "C" int cc_sessions_close_host(cc_engine* e, const uint64_t* h_clients, uint64_t count, const cc_events* h_events,
                                      uint64_t* h_closed) {
  if (!e) return set_err(CC_ERR_INVALID, "null engine");
  HIPCHECK(hipSetDevice(e->device));
  cc_events dev{};
  int rc = hw_events(e, h_events, &dev);
  if (rc) return rc;
  rc = cc_sessions_close(e, h_clients, count, h_events ? &dev : nullptr, e->own_stream, h_closed);
  const int re = hw_events_back(e, h_events, &dev);
  return rc ? rc : re;
}

extern "C" int cc_sessions_expire_host(cc_engine* e, const uint64_t* h_bitmap, uint64_t sessions, const cc_events* h_events,
                                       uint64_t* h_closed) {
  if (!e || (sessions && !h_bitmap)) return set_err(CC_ERR_INVALID, "null argument");
  std::vector<uint64_t> clients;  // ascending client session ids, as cc_sessions_expire orders them
  for (uint64_t wi = 0; wi < (sessions + 63) / 64; ++wi)
    for (uint64_t b = h_bitmap[wi]; b; b &= b - 1) {
      const uint64_t sid = wi * 64 + (uint64_t)__builtin_ctzll(b);
      if (sid < sessions) clients.push_back(sid);
    }
  return cc_sessions_close_host(e, clients.data(), clients.size(), h_events, h_closed);
}

extern "C" int cc_advance_time_events_host(cc_engine* e, uint64_t now, const cc_events* h_events) {
  if (!e) return set_err(CC_ERR_INVALID, "null engine");
  HIPCHECK(hipSetDevice(e->device));
  cc_events dev{};
  int rc = hw_events(e, h_events, &dev);
  if (rc) return rc;
  rc = cc_advance_time_events(e, now, h_events ? &dev : nullptr);
  const int re = hw_events_back(e, h_events, &dev);
  return rc ? rc : re;
}

extern "C" int cc_retained_bitmap_host(cc_engine* e, uint64_t first, uint64_t count, uint64_t* h_bitmap, uint64_t* h_count) {
  if (!e || (count && !h_bitmap)) return set_err(CC_ERR_INVALID, "null argument");
  if (count == 0) {
    if (h_count) *h_count = 0;
    return CC_OK;
  }
  HIPCHECK(hipSetDevice(e->device));
  const uint64_t words = (count + 63) / 64;
  void* d = nullptr;
  int rc = hw(e, kHwBitmap, 8 * words, &d);
  if (rc) return rc;
  if ((rc = cc_retained_bitmap(e, first, count, (uint64_t*)d, h_count))) return rc;
  HIPCHECK(hipMemcpy(h_bitmap, d, 8 * words, hipMemcpyDeviceToHost));
  return CC_OK;
}

// ---- plain device memory (for the stateless device calls and hosts that keep columns resident) ---------------
extern "C" int cc_device_alloc(int device, uint64_t bytes, void** d_out) {
  if (!d_out) return set_err(CC_ERR_INVALID, "null argument");
  *d_out = nullptr;
  HIPCHECK(hipSetDevice(device));
  HIPCHECK(hipMalloc(d_out, std::max<uint64_t>(bytes, 1)));
  return CC_OK;
}

extern "C" int cc_device_free(void* d_ptr) {
  if (d_ptr) HIPCHECK(hipFree(d_ptr));
  return CC_OK;
}

extern "C" int cc_memcpy(void* dst, const void* src, uint64_t bytes, int kind, void* stream) {
  if (bytes == 0) return CC_OK;
  if (!dst || !src) return set_err(CC_ERR_INVALID, "null argument");
  const hipMemcpyKind k = kind == CC_MEMCPY_H2D ? hipMemcpyHostToDevice
                          : kind == CC_MEMCPY_D2H ? hipMemcpyDeviceToHost
                          : kind == CC_MEMCPY_D2D ? hipMemcpyDeviceToDevice
                                                  : hipMemcpyDefault;
  if (kind < CC_MEMCPY_H2D || kind > CC_MEMCPY_D2D) return set_err(CC_ERR_INVALID, "memcpy kind");
  HIPCHECK(hipMemcpyAsync(dst, src, bytes, k, (hipStream_t)stream));
  HIPCHECK(hipStreamSynchronize((hipStream_t)stream));
  return CC_OK;
}

extern "C" int cc_memset(void* d_ptr, int byte, uint64_t bytes, void* stream) {
  if (bytes == 0) return CC_OK;
  if (!d_ptr) return set_err(CC_ERR_INVALID, "null argument");
  HIPCHECK(hipMemsetAsync(d_ptr, byte, bytes, (hipStream_t)stream));
  HIPCHECK(hipStreamSynchronize((hipStream_t)stream));
  return CC_OK;
}
