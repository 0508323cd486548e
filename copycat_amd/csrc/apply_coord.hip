// apply_coord.hip — coordination state machines (LockState, LeaderElectionState, MembershipGroupState) and
// AtomicValue with listeners, with their published events.
//
// Like apply_value.hip, one thread owns one resource slot and applies that slot's commits in log order; here a
// workgroup owns a quarter super-bucket (64 slots, see k_apply_coord).  The super-buckets handled here are those holding a
// coordination resource (or every value super-bucket with CC_CFG_VALUE_EVENTS); k_apply_value skips them.
// State that has variable size in the reference lives in a fixed block per slot (common.h CoordHdr/CoordEnt):
// the lock's waiter FIFO (ArrayDeque, LockState.java:35), the election's listener LinkedHashMap
// (LeaderElectionState.java:33), the group's member HashMap (MembershipGroupState.java:34, kept sorted by
// instance id), the value's listener map (AtomicValueState.java:36).
//
// Events (Session.publish -> InstanceEvent, ManagedResourceSession.java:64-71) go to an LDS buffer per chunk and
// from there to the sub-batch's event arena with one global atomic per chunk; each commit's event count goes
// to ev_cnt[staging position].  events.hip orders them by (log row, emission order) into the caller's stream.
//
// Semantics restated (file:line in the reference):
//   LockState.lock :41-61 (timeout -1 wait, 0 try, > 0 timed wait: the timer silently dequeues, A7),
//   LockState.unlock :66-85, LockState.delete :87-98 (holder cleaned, not nulled);
//   LeaderElectionState.listen :57-66, unlisten :71-91, isLeader :96-98 (epoch not serialized -> 0, A3),
//   delete :100-108;  MembershipGroupState.join :47-64 (Set<Long> result), leave :69-81, execute :108-119,
//   delete :121-125 (schedule :86-103 is a timer with a payload: not applied on the GPU);
//   AtomicValueState.listen :41-49, unlisten :54-63, change :68-72, get/set/compareAndSet/getAndSet :77-144.
// Lock timeouts: a waiter whose deadline (clock at lock + timeout) is <= the clock at which due timers fire
// before a commit (the previous commit's clock in manager mode, this commit's in module mode, A8) is gone
// before that commit is applied; they publish nothing, so applying them lazily per lock is exact.
#include <cstddef>

#include "common.h"
#include "engine_internal.h"

namespace cc {

#ifdef CC_PHASE_TIMING
__device__ unsigned long long g_wg_t[4 * 4096];  // last launch: per workgroup (start, end) wall clock, records, events
int phase_read_coord_wg(uint64_t* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wg_t), sizeof(unsigned long long) * 4 * 4096) == hipSuccess ? CC_OK : CC_ERR_HIP;
}
__device__ unsigned long long g_ph_coord[kPhases];
int phase_read_coord(uint64_t* out) {
  unsigned long long z[kPhases] = {};
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ph_coord), sizeof z) != hipSuccess ||
      hipMemcpyToSymbol(HIP_SYMBOL(g_ph_coord), z, sizeof z) != hipSuccess)
    return CC_ERR_HIP;
  return CC_OK;
}
#endif


typedef __attribute__((address_space(3))) uint64_t LdsU64;
typedef __attribute__((address_space(3))) uint32_t LdsU32;
// The walkers' LDS state (event buffers, cached entries) is laid out lane-minor: word w of item i of lane l sits at
// [(i * words + w) * kLanes + l], so a wave's access to the same item of every lane covers consecutive banks.  (The
// lane-major layout put lanes 192 or 384 bytes apart: 16- to 32-way bank conflicts on every access of the walk.)
constexpr uint32_t kLanes = kWave;
static_assert(sizeof(EvRec) == 24 && offsetof(EvRec, payload) == 8 && offsetof(EvRec, k) == 16 &&
                  offsetof(EvRec, code) == 18 && offsetof(EvRec, tag) == 19 && offsetof(EvRec, src) == 20,
              "Emitter::emit packs EvRec as three u64 words");
// Events of the walking lane: its own region of the LDS buffer (no atomics between lanes), a running count in a
// register; past the region's end straight to the sub-batch arena (one global atomic per event).
struct Emitter {
  LdsU64* buf;       // this lane's column of the event planes: word w of event q at buf[(q * 3 + w) * kLanes]
  uint32_t cap;      // events per lane region
  EvRec* arena;
  unsigned long long* arena_n;
  uint64_t arena_cap;
  LeakRec* leak;     // the engine's leak log (commits dropped without clean())
  unsigned long long* leak_n;
  uint64_t leak_cap;
  __device__ void leaked(uint32_t slot, uint64_t idx, uint32_t& err) const {
    const unsigned long long a = atomicAdd(leak_n, 1ull);
    if (a < leak_cap) {
      leak[a].idx = idx;
      leak[a].slot = slot;
      leak[a].pad = 0;
    } else {
      err |= kErrCapacity;
    }
  }
  __device__ void emit(uint32_t& n, uint32_t g, uint32_t k, uint32_t target, uint32_t code, uint32_t src, uint32_t tag,
                       uint64_t payload) const {
#ifdef CC_DIAG_NO_EMIT  // diagnostics build only: events dropped
    if (code != 0xFF) return;
#endif
    const uint64_t pl = tag == CC_TAG_NULL ? 0 : payload;
    const uint32_t q = n++;
    if (q < cap) {  // the record as three 8-byte LDS stores (EvRec layout: {g, target}, payload, {k, code, tag, src})
      buf[(q * 3 + 0) * kLanes] = (uint64_t)g | ((uint64_t)target << 32);
      buf[(q * 3 + 1) * kLanes] = pl;
      buf[(q * 3 + 2) * kLanes] = (uint64_t)(k & 0xFFFFu) | ((uint64_t)(code & 0xFFu) << 16) |
                                  ((uint64_t)(tag & 0xFFu) << 24) | ((uint64_t)(src & 0xFFu) << 32);
    } else {  // region full: straight to the arena
      EvRec e;
      e.g = g;
      e.target = target;
      e.payload = pl;
      e.k = (uint16_t)k;
      e.code = (uint8_t)code;
      e.tag = (uint8_t)tag;
      e.src = (uint8_t)src;
      e.pad[0] = e.pad[1] = e.pad[2] = 0;
      const unsigned long long a = atomicAdd(arena_n, 1ull);
      if (a < arena_cap) arena[a] = e;
    }
  }
};

__device__ inline CoordEnt* ents(uint8_t* blk) { return reinterpret_cast<CoordEnt*>(blk + sizeof(CoordHdr)); }

// A slot's entries during k_apply_coord: entry 0 lives in the walking lane's registers, entries 1..kECache-1 in LDS
// (copied in at kernel start, back at the end), the rest stay in the global block.  Small lock queues / listener
// and member lists (the common case) then never wait on global memory inside a slot's sequential walk, and a
// one-entry list (a lock with one waiter, a group with one member) never waits on LDS either.
// (2: entry 0 in registers, entry 1 in LDS -- the LDS this frees holds more event slots per walking lane, kEvLane)
constexpr uint32_t kECache = 2;
// Reads and writes select on the index, never on the pointer: each access keeps its address space (ds_read /
// global_load), so an LDS hit does not wait behind the walk's outstanding global stores as a flat access would.
typedef __attribute__((address_space(1))) CoordEnt GlbEnt;
struct Ents {
  // this lane's column of the entry planes (one pointer: three planes per cached entry, lane-minor; entry 0 lives in
  // r0, so entry p >= 1 has planes 3(p - 1) ..): x at [3(p - 1) * kLanes], idx at [(3(p - 1) + 1) * kLanes],
  // inst | pad << 32 at [(3(p - 1) + 2) * kLanes]
  LdsU64* lc;
  GlbEnt* glb;
  uint32_t cap;  // entries of the block (cc_config.coord_cap, a power of two)
  mutable CoordEnt r0;  // entry 0 (registers)
  // (the global path uses nontemporal accesses: distinct instructions the compiler cannot merge with the LDS path
  // into one flat access through a selected pointer)
  __device__ CoordEnt get(uint32_t p) const {
    if (p == 0) return r0;
    CoordEnt e;
    if (p < kECache) {
      e.x = lc[(3 * (p - 1)) * kLanes];
      e.idx = lc[(3 * (p - 1) + 1) * kLanes];
      const uint64_t ip = lc[(3 * (p - 1) + 2) * kLanes];
      e.inst = (uint32_t)ip;
      e.pad = (uint32_t)(ip >> 32);
      return e;
    }
    e.x = __builtin_nontemporal_load(&glb[p].x);
    e.idx = __builtin_nontemporal_load(&glb[p].idx);
    e.inst = __builtin_nontemporal_load(&glb[p].inst);
    e.pad = __builtin_nontemporal_load(&glb[p].pad);
    return e;
  }
  __device__ CoordEnt glb_get(uint32_t p) const {
    CoordEnt e;
    e.x = glb[p].x;
    e.idx = glb[p].idx;
    e.inst = glb[p].inst;
    e.pad = glb[p].pad;
    return e;
  }
  __device__ void glb_put(uint32_t p, const CoordEnt& v) const {
    glb[p].x = v.x;
    glb[p].idx = v.idx;
    glb[p].inst = v.inst;
    glb[p].pad = v.pad;
  }
  __device__ void put(uint32_t p, const CoordEnt& v) const {
    if (p == 0) {
      r0 = v;
      return;
    }
    if (p < kECache) {
      lc[(3 * (p - 1)) * kLanes] = v.x;
      lc[(3 * (p - 1) + 1) * kLanes] = v.idx;
      lc[(3 * (p - 1) + 2) * kLanes] = (uint64_t)v.inst | ((uint64_t)v.pad << 32);
      return;
    }
    __builtin_nontemporal_store(v.x, &glb[p].x);
    __builtin_nontemporal_store(v.idx, &glb[p].idx);
    __builtin_nontemporal_store(v.inst, &glb[p].inst);
    __builtin_nontemporal_store(v.pad, &glb[p].pad);
  }
  __device__ void load() const {  // kernel start: the slot's first kECache entries
#pragma unroll
    for (uint32_t q = 0; q < kECache; ++q) put(q, glb_get(q));
  }
  __device__ void store() const {  // kernel end
#pragma unroll
    for (uint32_t q = 0; q < kECache; ++q) glb_put(q, get(q));
  }
};

// ---- LockState ----------------------------------------------------------------------------------------
__device__ inline void lock_expire(CoordHdr& h, const Ents& q, uint64_t th) {  // silent timeouts (A7)
  uint32_t kept = 0;
  for (uint32_t i = 0; i < h.n; ++i) {
    const CoordEnt e = q.get((h.head + i) & (q.cap - 1));
    if (e.x != kNoDeadline && e.x <= th) continue;
    if (kept != i) q.put((h.head + kept) & (q.cap - 1), e);
    ++kept;
  }
  h.n = kept;
  if (!kept) h.head = 0;  // an empty ring restarts at entry 0 (kept in LDS by k_apply_coord)
}

template <uint32_t V>
struct TypeC {
  static constexpr uint32_t value = V;
};

// ---- one commit on a coordination / value slot -----------------------------------------------------------
struct Rec {
  uint32_t op, flags, inst, g;
  uint64_t a, b, key, idx, iid;
};

// T != 0: the resource type is known at compile time (a wave whose slots all hold one type walks a specialised
// copy with no code for the other types); T == 0: the runtime `type`.
template <uint32_t T>
__device__ inline uint32_t coord_apply(uint32_t type_rt, uint32_t slot, const Rec& r, CoordHdr& h, const Ents& E,
                                       uint32_t& vmeta_s, uint64_t& vval, uint64_t& rv, uint32_t& nev, const Emitter& em,
                                       uint32_t& lane_n, uint32_t& err) {
  const uint32_t type = T ? T : type_rt;
  rv = 0;
  auto ev = [&](uint32_t target, uint32_t code, uint32_t tag, uint64_t payload) {
    em.emit(lane_n, r.g, nev++, target, code, CC_EVSRC_COMMIT, tag, payload);
  };
  if (h.flags & kCoZombie) return CC_STATUS(CC_ST_NULL_POINTER, CC_TAG_NULL);
  // Small-state fast paths (type known at compile time, at most one entry, i.e. the whole list in the lane's
  // register entry E.r0): the same updates and events as the general steps below, as straight-line selects with no
  // search / shift / fan-out loops and no LDS or global entry accesses except writing entry 1 when the list grows to
  // two.  The lanes of a walking wave hold different ops, and the general steps' loops made every lane pay every
  // op's loop structure (2,700-4,500 cycles per step of a one-member group, profiles/r03/c5_diag).
  if constexpr (T == CC_RES_GROUP) {
    const bool join = r.op == CC_OP_GROUP_JOIN, leave = r.op == CC_OP_GROUP_LEAVE, exe = r.op == CC_OP_GROUP_EXECUTE;
    if (h.n <= 1 && (join || leave || exe)) {  // MembershipGroupState.join :47-64, leave :69-81, execute :108-119
      const uint64_t id = exe ? r.key : r.iid;
      const CoordEnt e0 = E.r0;
      const bool has = h.n != 0, hit = has && e0.x == id;
      const bool ins = join && !hit, rem = leave && hit;  // (coord_cap >= 64: a one-entry list is never full)
      const CoordEnt ne{r.iid, r.idx, r.inst, 0};
      const bool after = has && e0.x < id;  // members stay sorted by instance id: the joiner after the member
      CoordEnt n0 = e0;
      if (join && hit) {  // previous.clean(): the member's commit is replaced
        n0.idx = r.idx;
        n0.inst = r.inst;
      }
      if (ins && !after) n0 = ne;
      if (ins && has) E.put(1, after ? ne : e0);
      E.r0 = n0;
      h.n = ins ? h.n + 1u : (rem ? 0u : h.n);
      // "join"(id) to every other member (:55); a leave leaves no member to tell (:75)
      if (ins && has && e0.idx != r.idx) ev(e0.inst, CC_EV_JOIN, CC_TAG_LONG, r.iid);  // (as the general fan-out)
      if (join) {  // the returned Set<Long>, ascending
        em.emit(lane_n, r.g, nev++, r.inst, CC_EV_MEMBER, CC_EVSRC_RESULT, CC_TAG_LONG, n0.x);
        if (h.n == 2) em.emit(lane_n, r.g, nev++, r.inst, CC_EV_MEMBER, CC_EVSRC_RESULT, CC_TAG_LONG, after ? ne.x : e0.x);
        rv = h.n;
        return CC_STATUS(CC_ST_OK, CC_TAG_SET);
      }
      if (leave) return CC_STATUS(CC_ST_OK, CC_TAG_NULL);
      if (!hit) return CC_STATUS(CC_ST_ILLEGAL_ARGUMENT, CC_TAG_NULL);  // "unknown member"
      ev(e0.inst, CC_EV_EXECUTE, CC_FLAG_TAG_A(r.flags), r.a);
      return CC_STATUS(CC_ST_OK, CC_TAG_NULL);
    }
  }
  if constexpr (T == CC_RES_ELECTION) {
    const bool listen = r.op == CC_OP_ELECT_LISTEN, unlisten = r.op == CC_OP_ELECT_UNLISTEN;
    if (h.n <= 1 && (listen || unlisten || r.op == CC_OP_ELECT_ISLEADER)) {  // LeaderElectionState :57-98
      const bool held = (h.flags & kCoHeld) != 0, self = held && h.who == r.inst;
      if (unlisten && self && (h.flags & kCoCleaned)) return CC_STATUS(CC_ST_ILLEGAL_STATE, CC_TAG_NULL);
      const CoordEnt e0 = E.r0;
      const bool search = (listen && held) || (unlisten && !self);
      const bool found = search && h.n != 0 && e0.x == r.iid;  // the session's listener entry (entry 0)
      if (listen && !held) {  // the first listener leads
        h.flags = kCoHeld;
        h.who = r.inst;
        h.idx = r.idx;
        ev(r.inst, CC_EV_ELECT, CC_TAG_LONG, r.idx);
      }
      const bool add = listen && held && !found;  // (coord_cap >= 64: never full here)
      const CoordEnt ne{r.iid, r.idx, r.inst, 0};
      if (add && h.n == 1) E.put(1, ne);
      if (add && h.n == 0) E.r0 = ne;
      const bool promote = unlisten && self && h.n != 0;  // the leader unlistens: the next listener (entry 0) leads
      if (unlisten && self) h.flags = 0;
      h.n = add ? h.n + 1u : ((promote || (unlisten && !self && found)) ? 0u : h.n);
      if (promote) {
        h.flags = kCoHeld;
        h.who = e0.inst;
        h.idx = e0.idx;
        ev(e0.inst, CC_EV_ELECT, CC_TAG_LONG, e0.idx);
      }
      if (listen || unlisten) return CC_STATUS(CC_ST_OK, CC_TAG_NULL);
      rv = ((h.flags & kCoHeld) && h.who == r.inst && h.idx == 0) ? 1 : 0;  // isLeader (epoch 0, A3)
      return CC_STATUS(CC_ST_OK, CC_TAG_BOOL);
    }
  }
  if (!op_registered(type, r.op)) return CC_STATUS(CC_ST_UNKNOWN_OP, CC_TAG_NULL);
  switch (type) {
    case CC_RES_LOCK: {
      const uint64_t fire = r.a, clk = r.key;
      const int64_t timeout = (int64_t)r.b;
      if (r.op == CC_OP_DELETE) {
        if (h.flags & kCoHeld) {
          if (h.flags & kCoCleaned) return CC_STATUS(CC_ST_ILLEGAL_STATE, CC_TAG_NULL);  // "commit closed"
          h.flags |= kCoCleaned;
        }
        h.n = 0;
        h.head = 0;
        return CC_STATUS(CC_ST_OK, CC_TAG_NULL);
      }
      lock_expire(h, E, fire);
      if (r.op == CC_OP_LOCK_LOCK) {
        if (!(h.flags & kCoHeld)) {
          h.flags = kCoHeld;
          h.who = r.inst;
          h.idx = r.idx;
          ev(r.inst, CC_EV_LOCK, CC_TAG_BOOL, 1);
        } else if (timeout == 0) {
          ev(r.inst, CC_EV_LOCK, CC_TAG_BOOL, 0);
        } else if (h.n == E.cap) {
          err |= kErrCoordFull;
        } else {
          E.put((h.head + h.n) & (E.cap - 1), CoordEnt{timeout > 0 ? clk + (uint64_t)timeout : kNoDeadline, r.idx, r.inst, 0});
          ++h.n;
        }
        return CC_STATUS(CC_ST_OK, CC_TAG_NULL);
      }
      // unlock
      if (h.flags & kCoHeld) {
        if (h.who != r.inst) return CC_STATUS(CC_ST_ILLEGAL_STATE, CC_TAG_NULL);  // "not the lock holder"
        if (h.flags & kCoCleaned) return CC_STATUS(CC_ST_ILLEGAL_STATE, CC_TAG_NULL);
        if (h.n == 0) {
          h.flags = 0;
        } else {
          const CoordEnt e = E.get(h.head);
          h.head = (h.head + 1) & (E.cap - 1);
          if (!--h.n) h.head = 0;
          h.flags = kCoHeld;
          h.who = e.inst;
          h.idx = e.idx;
          ev(e.inst, CC_EV_LOCK, CC_TAG_BOOL, 1);
        }
      }
      return CC_STATUS(CC_ST_OK, CC_TAG_NULL);
    }
    case CC_RES_ELECTION: {
      if (r.op == CC_OP_DELETE) {
        if (h.flags & kCoHeld) {
          if (h.flags & kCoCleaned) return CC_STATUS(CC_ST_ILLEGAL_STATE, CC_TAG_NULL);
          h.flags |= kCoCleaned;
        }
        h.n = 0;
        return CC_STATUS(CC_ST_OK, CC_TAG_NULL);
      }
      // listen / unlisten as one straight-line step (shared listener search and shift; see the group step)
      const bool listen = r.op == CC_OP_ELECT_LISTEN, unlisten = r.op == CC_OP_ELECT_UNLISTEN;
      const bool held = (h.flags & kCoHeld) != 0, self = held && h.who == r.inst;
      if (unlisten && self && (h.flags & kCoCleaned)) return CC_STATUS(CC_ST_ILLEGAL_STATE, CC_TAG_NULL);
      // listen while someone leads: is the session already listening (may be the leader's own session, A9)?
      // unlisten of a listener: its entry
      const bool search = (listen && held) || (unlisten && !self);
      uint32_t fi = h.n;
      for (uint32_t i = 0; i < (search ? h.n : 0u); ++i)
        if (E.get(i).x == r.iid) {
          fi = i;
          break;
        }
      const bool found = fi < h.n;
      if (listen && !held) {  // the first listener leads
        h.flags = kCoHeld;
        h.who = r.inst;
        h.idx = r.idx;
        ev(r.inst, CC_EV_ELECT, CC_TAG_LONG, r.idx);
      }
      if (listen && held && !found) {
        if (h.n == E.cap) err |= kErrCoordFull;
        else E.put(h.n++, CoordEnt{r.iid, r.idx, r.inst, 0});
      }
      // the leader unlistens: the next listener (entry 0) leads; a listener unlistens: its entry goes
      const bool promote = unlisten && self && h.n != 0;
      if (unlisten && self) h.flags = 0;
      const CoordEnt e0 = promote ? E.get(0) : CoordEnt{0, 0, 0, 0};
      if (promote || (unlisten && !self && found)) {
        for (uint32_t k = (promote ? 0u : fi) + 1; k < h.n; ++k) E.put(k - 1, E.get(k));
        --h.n;
      }
      if (promote) {
        h.flags = kCoHeld;
        h.who = e0.inst;
        h.idx = e0.idx;
        ev(e0.inst, CC_EV_ELECT, CC_TAG_LONG, e0.idx);
      }
      if (listen || unlisten) return CC_STATUS(CC_ST_OK, CC_TAG_NULL);
      // isLeader
      rv = ((h.flags & kCoHeld) && h.who == r.inst && h.idx == 0) ? 1 : 0;
      return CC_STATUS(CC_ST_OK, CC_TAG_BOOL);
    }
    case CC_RES_GROUP: {
#ifdef CC_DIAG_GROUP_NOP  // diagnostics build only (scripts/probes/phase_timing.py): the group walk without its work
      if (r.op != 0xFF) { rv = 0; return CC_STATUS(CC_ST_OK, CC_TAG_NULL); }
#endif
      if (r.op == CC_OP_DELETE) {
        h.n = 0;
        return CC_STATUS(CC_ST_OK, CC_TAG_NULL);
      }
      if (r.op == CC_OP_GROUP_SCHEDULE) {
        err |= kErrUnsupported;
        return CC_STATUS(CC_ST_OK, CC_TAG_NULL);
      }
      // members sorted by instance id: position of `id`
      auto find = [&](uint64_t id, bool& hit) {
        uint32_t lo = 0, hi = h.n;
        while (lo < hi) {
          const uint32_t m = (lo + hi) >> 1;
          if (E.get(m).x < id) lo = m + 1; else hi = m;
        }
        hit = lo < h.n && E.get(lo).x == id;
        return lo;
      };
      // one search for every op (converged across the wave's lanes): join / leave look up the committing instance,
      // execute the target member
      bool hit;
      const uint32_t p = find(r.op == CC_OP_GROUP_EXECUTE ? r.key : r.iid, hit);
#ifdef CC_DIAG_G1  // diagnostics build only: the group step stops after the member search
      if (r.op != 0xFF) { rv = p + hit; return CC_STATUS(CC_ST_OK, CC_TAG_NULL); }
#endif
      // One straight-line step for join / leave / execute: the lanes of a walking wave hold different ops, and three
      // divergent paths cost the wave all three every step; here the entry shifts, the join / leave fan-out (one
      // loop over the members as they stand after the update) and the result share their code.
      const bool join = r.op == CC_OP_GROUP_JOIN, leave = r.op == CC_OP_GROUP_LEAVE;
      const bool full = h.n == E.cap;
      const bool ins = join && !hit && !full, rem = leave && hit;
      if (join && !hit && full) err |= kErrCoordFull;
      if (join && hit) {  // previous.clean(): the member's commit is replaced
        CoordEnt e = E.get(p);
        e.idx = r.idx;
        e.inst = r.inst;
        E.put(p, e);
      }
      if (ins) {
        for (uint32_t i = h.n; i > p; --i) E.put(i, E.get(i - 1));
        E.put(p, CoordEnt{r.iid, r.idx, r.inst, 0});
        ++h.n;
      }
      if (rem) {
        for (uint32_t i = p + 1; i < h.n; ++i) E.put(i - 1, E.get(i));
        --h.n;
      }
      // "join"(id) to every other member (:55) / "leave"(id) to every remaining member (:75)
#ifdef CC_DIAG_G2  // diagnostics build only: the group step without its fan-out and result rows
      if (r.op != 0xFF) { rv = h.n; return CC_STATUS(CC_ST_OK, CC_TAG_NULL); }
#endif
      const uint32_t fan = (ins || rem) ? h.n : 0u;
      const uint32_t code = join ? CC_EV_JOIN : CC_EV_LEAVE;
      for (uint32_t i = 0; i < fan; ++i) {
        const CoordEnt e = E.get(i);
        if (rem || e.idx != r.idx) ev(e.inst, code, CC_TAG_LONG, r.iid);
      }
      if (join) {
        for (uint32_t i = 0; i < h.n; ++i)  // the returned Set<Long>, ascending
          em.emit(lane_n, r.g, nev++, r.inst, CC_EV_MEMBER, CC_EVSRC_RESULT, CC_TAG_LONG, E.get(i).x);
        rv = h.n;
        return CC_STATUS(CC_ST_OK, CC_TAG_SET);
      }
      if (leave) return CC_STATUS(CC_ST_OK, CC_TAG_NULL);
      // execute(member = key, callback = a)
      if (!hit) return CC_STATUS(CC_ST_ILLEGAL_ARGUMENT, CC_TAG_NULL);  // "unknown member"
      ev(E.get(p).inst, CC_EV_EXECUTE, CC_FLAG_TAG_A(r.flags), r.a);
      return CC_STATUS(CC_ST_OK, CC_TAG_NULL);
    }
    case CC_RES_QUEUE: {  // QueueState.java:33-199: an ArrayDeque of (value tag in pad, payload in x), FIFO ring
      const uint32_t ta = CC_FLAG_TAG_A(r.flags);
      const uint64_t pa = ta ? r.a : 0;
      auto at = [&](uint32_t i) -> CoordEnt { return E.get((h.head + i) & (E.cap - 1)); };
      auto set_at = [&](uint32_t i, const CoordEnt& v) { E.put((h.head + i) & (E.cap - 1), v); };
      auto first_match = [&](uint32_t& pos) -> int {  // 1 match, 0 none, -1 NPE (a stored null's equals)
        for (uint32_t i = 0; i < h.n; ++i) {
          const CoordEnt e = at(i);
          const uint32_t et = e.pad & kQTagMask;
          if (et == CC_TAG_NULL) return -1;
          if (et == ta && e.x == pa) {
            pos = i;
            return 1;
          }
        }
        return 0;
      };
      auto pop = [&]() {
        h.head = (h.head + 1) & (E.cap - 1);
        if (!--h.n) h.head = 0;
      };
      switch (r.op) {
        case CC_OP_DELETE:
        case CC_OP_QUEUE_CLEAR:  // clear :184-190 / delete :191-199
          h.n = 0;
          h.head = 0;
          return CC_STATUS(CC_ST_OK, CC_TAG_NULL);
        case CC_OP_QUEUE_CONTAINS: {  // contains :36-46
          uint32_t pos = 0;
          const int m = first_match(pos);
          if (m < 0) return CC_STATUS(CC_ST_NULL_POINTER, CC_TAG_NULL);
          rv = m;
          return CC_STATUS(CC_ST_OK, CC_TAG_BOOL);
        }
        case CC_OP_QUEUE_ADD:    // add :51-59
        case CC_OP_QUEUE_OFFER:  // offer :64-72 — both answer false
          if (h.n == E.cap) {
            err |= kErrCoordFull;
          } else {
            set_at(h.n, CoordEnt{pa, r.idx, r.inst, ta});
            ++h.n;
          }
          return CC_STATUS(CC_ST_OK, CC_TAG_BOOL);
        case CC_OP_QUEUE_PEEK:  // peek :77-87
          if (!h.n) return CC_STATUS(CC_ST_OK, CC_TAG_NULL);
          rv = at(0).x;
          return CC_STATUS(CC_ST_OK, at(0).pad & kQTagMask);
        case CC_OP_QUEUE_POLL: {  // poll :92-105
          if (!h.n) return CC_STATUS(CC_ST_OK, CC_TAG_NULL);
          const CoordEnt e = at(0);
          pop();
          rv = e.x;
          return CC_STATUS(CC_ST_OK, e.pad & kQTagMask);
        }
        case CC_OP_QUEUE_ELEMENT:  // element :111-124 (throws when empty; the head stays)
          if (!h.n) return CC_STATUS(CC_ST_NO_SUCH_ELEMENT, CC_TAG_NULL);
          {
            CoordEnt e0 = at(0);
            rv = e0.x;
            const uint32_t tg = e0.pad & kQTagMask;
            e0.pad |= kQCleaned;  // value.clean() on the head it leaves in place
            set_at(0, e0);
            return CC_STATUS(CC_ST_OK, tg);
          }
        case CC_OP_QUEUE_REMOVE: {  // remove :130-157
          if (ta != CC_TAG_NULL) {
            uint32_t pos = 0;
            const int m = first_match(pos);
            if (m < 0) return CC_STATUS(CC_ST_NULL_POINTER, CC_TAG_NULL);
            if (m) {
              for (uint32_t i = pos; i + 1 < h.n; ++i) set_at(i, at(i + 1));
              --h.n;
            }
            rv = m;
            return CC_STATUS(CC_ST_OK, CC_TAG_BOOL);
          }
          if (!h.n) return CC_STATUS(CC_ST_NO_SUCH_ELEMENT, CC_TAG_NULL);  // ArrayDeque.remove()
          const CoordEnt e = at(0);
          pop();
          rv = e.x;
          return CC_STATUS(CC_ST_OK, e.pad & kQTagMask);
        }
        case CC_OP_QUEUE_SIZE:  // size :162-168 (int)
          rv = h.n;
          return CC_STATUS(CC_ST_OK, CC_TAG_INT);
        case CC_OP_QUEUE_ISEMPTY:  // isEmpty :173-179
          rv = h.n == 0;
          return CC_STATUS(CC_ST_OK, CC_TAG_BOOL);
      }
      return CC_STATUS(CC_ST_UNKNOWN_OP, CC_TAG_NULL);
    }
    case CC_RES_VALUE: {
      const uint32_t ta = CC_FLAG_TAG_A(r.flags), tb = CC_FLAG_TAG_B(r.flags);
      const uint64_t pa = ta ? r.a : 0, pb = tb ? r.b : 0;
      const uint32_t tag = vmeta_s & 0xFF, cur = (vmeta_s >> 8) & 1;
      bool write = false;
      uint32_t ntag = 0;
      uint64_t nv = 0, rvv = 0;
      uint32_t rtag = CC_TAG_NULL;
      switch (r.op) {
        case CC_OP_VALUE_GET:
          if (cur) { rtag = tag; rvv = vval; }
          break;
        case CC_OP_VALUE_SET:
          write = true; ntag = ta; nv = pa;
          break;
        case CC_OP_VALUE_CAS: {
          const bool eq = (tag == CC_TAG_NULL && ta == CC_TAG_NULL) || (tag != CC_TAG_NULL && tag == ta && vval == pa);
          write = eq; ntag = tb; nv = pb;
          rtag = CC_TAG_BOOL; rvv = eq;
          break;
        }
        case CC_OP_VALUE_GETANDSET:
          rtag = tag; rvv = vval; write = true; ntag = ta; nv = pa;
          break;
        case CC_OP_VALUE_LISTEN: {  // listeners.put(session, commit)
          bool found = false;
          for (uint32_t i = 0; i < h.n; ++i) {
            CoordEnt e = E.get(i);
            if (e.inst == r.inst) {  // the replaced commit is never clean()ed: retained for good
              em.leaked(slot, e.idx, err);
              e.idx = r.idx;
              E.put(i, e);
              found = true;
            }
          }
          if (!found) {
            if (h.n == E.cap) err |= kErrCoordFull;
            else E.put(h.n++, CoordEnt{0, r.idx, r.inst, 0});
          }
          break;
        }
        case CC_OP_VALUE_UNLISTEN:
          for (uint32_t i = 0; i < h.n; ++i)
            if (E.get(i).inst == r.inst) {
              for (uint32_t k = i + 1; k < h.n; ++k) E.put(k - 1, E.get(k));
              --h.n;
              break;
            }
          break;
        case CC_OP_DELETE:
          if (cur) { vmeta_s = 0; vval = 0; }
          break;
      }
      if (write) {
        vmeta_s = vmeta(ntag, 1);
        vval = nv;
        for (uint32_t i = 0; i < h.n; ++i) ev(E.get(i).inst, CC_EV_CHANGE, ntag, nv);  // change(value) :68-72
      }
      rv = rvv;
      return CC_STATUS(CC_ST_OK, rtag);
    }
  }
  return CC_STATUS(CC_ST_UNKNOWN_OP, CC_TAG_NULL);
}

// One workgroup per quarter super-bucket (kQ = 64 slots): the four workgroups of a super-bucket each read its list
// (the run in every tile, tile order = log order) and keep the commits of their own slots.  256 threads load a
// 512-commit chunk (the next chunk's meta words are in flight during the walk), rank their own commits per slot
// inside each wave (LDS atomics with return: lane order), one wave turns the per-wave counts into slot run starts,
// the owners' records are gathered into LDS in slot order, and wave 0 (lane = slot) applies each slot's commits in
// log order with its CoordHdr (and AtomicValueState) held in registers for the whole launch.  Small LDS
// (~48 KB) so three workgroups share a CU and hide each other's gathers.
// (Round 3 measured two 32-lane walking waves per workgroup instead of one: no change, 8.9 ms/step either way.  The
// walk is bound by each lane's sequential chain -- about 2,700-4,500 cycles per step of a group / election slot,
// phase clocks profiles/r03/c5_diag -- not by how many waves walk.)
//
// LDS hazards of the chunk loop (cf. the k_apply_map chunk-0 race): the run table (rstart / rpre) is
// written once before the loop and only read after (load_meta's rows_pos); the per-wave counters wc are read by the
// gather (each wave reads its own row) and cleared right after by that same wave's lanes (k = t covers exactly row
// w), in program order within the wave, before barrier 3; the record planes (rab ... rpos) are written by the gather
// only after barrier 2 of a chunk, which every thread reaches after the previous chunk's final barrier, i.e. after
// the walk and the result / event stores of that chunk stopped reading them.
constexpr int kQ = 64;                     // slots per workgroup
constexpr int kQPerSb = (1 << kSbShift) / kQ;
constexpr int kCT2 = 256;                  // threads per workgroup
constexpr int kCW2 = kCT2 / kWave;
constexpr int kCPer2 = 2;                  // commits per thread per chunk
constexpr int kCCh2 = kCT2 * kCPer2;       // 512 commits of the super-bucket per chunk
// LDS event slots per walking lane per chunk; more go straight to the arena, one global atomic on the arena counter
// each, which the wave waits for (a group lane publishes ~4 events per chunk on c5: with 8 slots ~6 % of lanes
// overflowed every chunk)
constexpr int kEvLane = 11;  // (LDS 52,800 B: three workgroups per CU need <= 53,248 at the 2 KiB allocation granularity)

__global__ __launch_bounds__(kCT2, 3) void k_apply_coord(const XRec* __restrict__ xr, const uint16_t* __restrict__ ttab,
                                                     uint32_t tiles, uint32_t sb, uint32_t sbq_base,
                                                     const uint8_t* __restrict__ sb_kind,
                                                     const uint8_t* __restrict__ res_type, const uint64_t* __restrict__ inst_id,
                                                     uint8_t* __restrict__ coord, uint32_t coord_cap, uint32_t* __restrict__ val_meta,
                                                     uint64_t* __restrict__ val_v, uint8_t* __restrict__ rst_status,
                                                     uint64_t* __restrict__ rst_value, uint16_t* __restrict__ ev_cnt,
                                                     EvRec* __restrict__ arena, unsigned long long* __restrict__ arena_n,
                                                     uint64_t arena_cap, LeakRec* __restrict__ leak,
                                                     unsigned long long* __restrict__ leak_n, uint64_t leak_cap,
                                                     uint32_t* __restrict__ err_out) {
  __shared__ u64x2 rab[kCCh2];
  __shared__ uint64_t rkey[kCCh2];
  __shared__ uint64_t ridx[kCCh2];
  __shared__ uint64_t riid[kCCh2];
  __shared__ uint32_t rmeta[kCCh2];
  __shared__ uint32_t rins[kCCh2];
  __shared__ uint32_t rpos[kCCh2];
  __shared__ uint32_t wc[kCW2][kQ];          // per-wave slot counts -> per-wave exclusive prefixes
  __shared__ uint32_t sstart[kQ + 1];
  __shared__ uint16_t rb0[kMaxTiles];        // run start inside tile r (staging position r * kTile + rb0[r])
  __shared__ uint32_t rpre[kMaxTiles + 1];
  __shared__ uint32_t wsum[kCW2];
  __shared__ uint64_t evp[kEvLane * 3 * kQ];    // the walkers' event buffers (lane-minor planes, see kLanes)
  __shared__ uint32_t evoff[kQ + 1];
  __shared__ uint64_t ecache[3 * (kECache - 1) * kQ];  // the walkers' entries 1 .. kECache-1 (Ents), lane-minor
  __shared__ unsigned long long evbase;

  const uint32_t s = blockIdx.x / kQPerSb, q0 = (blockIdx.x % kQPerSb) * kQ;
  if (!sb_kind[s]) return;  // value-only super-bucket: k_apply_value
  const uint32_t t = threadIdx.x, w = t >> 6, l = t & 63;
  PH_DECL
  uint32_t err = 0;
  for (uint32_t k = t; k < (uint32_t)(kCW2 * kQ); k += kCT2) (&wc[0][0])[k] = 0;
  // the list: this quarter's own bucket when the partition made quarter buckets, else the super-bucket's (filtered)
  const uint32_t bk = sbq_base ? sbq_base + blockIdx.x : s;
  {  // the list = its run in every tile, in tile order
    constexpr int PT = kMaxTiles / kCT2;
    uint32_t len[PT], sum = 0;
#pragma unroll
    for (int q = 0; q < PT; ++q) {
      const uint32_t tt = t * PT + q;
      len[q] = 0;
      if (tt < tiles) {
        const uint16_t* row = ttab + (uint64_t)tt * (sb + 1);
        const uint32_t b0 = row[bk], b1 = row[bk + 1];
        rb0[tt] = (uint16_t)b0;
        len[q] = b1 - b0;
      }
      sum += len[q];
    }
    uint32_t inc = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(inc, d, 64);
      if (l >= (uint32_t)d) inc += y;
    }
    if (l == 63) wsum[w] = inc;
    __syncthreads();
    uint32_t run = inc - sum;
    for (uint32_t q = 0; q < w; ++q) run += wsum[q];
#pragma unroll
    for (int q = 0; q < PT; ++q) {
      const uint32_t tt = t * PT + q;
      if (tt < tiles) rpre[tt] = run;
      run += len[q];
    }
    if (t == kCT2 - 1) rpre[tiles] = run;
    __syncthreads();
  }
  const uint32_t cnt = rpre[tiles];
  static_assert(kQ == (int)kLanes, "one walking lane per slot of the quarter bucket");
  const Emitter em{(LdsU64*)(evp + l), kEvLane, arena, arena_n, arena_cap, leak, leak_n, leak_cap};
  // the walker lanes (wave 0, lane = slot) keep their state machine's header in registers for the whole launch
  const uint32_t res = s * (1u << kSbShift) + q0 + l;
  uint8_t* blk = coord + (uint64_t)res * coord_block(coord_cap);
  uint32_t type = 0, vm = 0;
  uint64_t vv = 0;
  CoordHdr h{};
  const Ents E{(LdsU64*)(ecache + l), (GlbEnt*)ents(blk), coord_cap, CoordEnt{0, 0, 0, 0}};
  if (w == 0) {
    type = res_type[res];
    {  // (CoordHdr.pad is neither read nor written: two registers less across the walk)
      const CoordHdr* hp = reinterpret_cast<const CoordHdr*>(blk);
      h.who = hp->who;
      h.flags = hp->flags;
      h.idx = hp->idx;
      h.head = hp->head;
      h.n = hp->n;
    }
    if (type == CC_RES_VALUE) {
      vm = val_meta[res];
      vv = val_v[res];
    }
    E.load();
  }
  // staging position of list entry c (binary search over the tiles' prefix)
  auto pos_of = [&](uint32_t c) -> uint32_t {
    uint32_t lo = 0, hi = tiles;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (rpre[mid] <= c) lo = mid; else hi = mid;
    }
    return lo * kTile + rb0[lo] + (c - rpre[lo]);
  };
  // the next chunk's records (whole XRec: position, meta, operands, key, index, instance) stream into registers
  // during the walk; the instance-id gather is issued at the top of the chunk, ahead of the rank and scan
  uint32_t g0 = 0xFFFFFFFFu, g1 = 0xFFFFFFFFu, m0 = 0, m1 = 0, n0 = 0, n1 = 0;
  uint64_t a0x = 0, a0y = 0, a1x = 0, a1y = 0;  // the operand pairs as four words (a u64x2 pair lived in scratch)
  uint64_t k0 = 0, k1 = 0, x0 = 0, x1 = 0, i0 = 0, i1 = 0;
  // Staging positions of the wave's two rows: one 64-ary search for the run of the wave's first record, then a
  // 64-run window in the lanes (run start wS, first record wP, next run's first record wB): a row's records find
  // their runs with ballots and two lane shuffles (k_apply_value_ws); a binary search per record was ten dependent
  // LDS reads.  Many short or empty runs (the window does not cover the rows): the binary search.
  auto rows_pos = [&](uint32_t cw, uint32_t& p0, uint32_t& p1) {
    p0 = p1 = 0xFFFFFFFFu;
    if (cw >= cnt) return;  // wave-uniform
    const uint32_t step = (tiles + kWave - 1) / kWave;
    uint32_t cand = l * step;
    uint64_t bm = __ballot(cand < tiles && rpre[cand] <= cw);
    const uint32_t base = (uint32_t)(63 - __clzll((long long)bm)) * step;
    cand = base + l;
    bm = __ballot(l < step && cand < tiles && rpre[cand] <= cw);
    const uint32_t rrow = base + (uint32_t)(63 - __clzll((long long)bm));
    const uint32_t kr = rrow + l;
    const uint32_t wB = kr + 1 <= tiles ? rpre[kr + 1] : 0xFFFFFFFFu;
    const uint32_t wS = kr < tiles ? kr * kTile + rb0[kr] : 0u, wP = kr < tiles ? rpre[kr] : 0u;
    const uint32_t lastc = cw + kWave * kCPer2 - 1 < cnt ? cw + kWave * kCPer2 - 1 : cnt - 1;
    const bool win = (uint32_t)__shfl((int)wB, 63, 64) > lastc;
#pragma unroll
    for (int j = 0; j < kCPer2; ++j) {
      const uint32_t crow = cw + j * kWave, c = crow + l;
      uint32_t g = 0xFFFFFFFFu;
      if (crow < cnt) {  // wave-uniform
        if (win) {
          uint32_t ri = (uint32_t)__popcll(__ballot(wB <= crow));
          for (uint64_t mb = __ballot(wB > crow && wB <= crow + (kWave - 1)); mb; mb &= mb - 1)
            ri += c >= (uint32_t)__builtin_amdgcn_readlane((int)wB, __ffsll((long long)mb) - 1) ? 1u : 0u;
          const uint32_t rs_ = (uint32_t)__shfl((int)wS, (int)ri, 64), rp_ = (uint32_t)__shfl((int)wP, (int)ri, 64);
          if (c < cnt) g = rs_ + (c - rp_);
        } else if (c < cnt) {
          g = pos_of(c);
        }
      }
      (j == 0 ? p0 : p1) = g;
    }
  };
  static_assert(kCPer2 == 2, "two rows per wave");
  auto load_meta = [&](uint32_t c0) {
    rows_pos(c0 + w * (kWave * kCPer2), g0, g1);
    const XRec* r0 = xr + (g0 != 0xFFFFFFFFu ? g0 : 0), *r1 = xr + (g1 != 0xFFFFFFFFu ? g1 : 0);
    a0x = r0->ab.x;
    a0y = r0->ab.y;
    k0 = r0->key;
    x0 = r0->idx;
    m0 = r0->meta;
    n0 = r0->res;
    a1x = r1->ab.x;
    a1y = r1->ab.y;
    k1 = r1->key;
    x1 = r1->idx;
    m1 = r1->meta;
    n1 = r1->res;
    i0 = r0->pad;  // the instance id (k_part_ext writes it into the record on coordination engines)
    i1 = r1->pad;
  };
  load_meta(0);
#ifdef CC_PHASE_TIMING
  uint64_t ev_total_lane = 0;
  if (t == 0 && blockIdx.x < 4096) g_wg_t[4 * blockIdx.x + 3] = 0;
#endif
  PH(0);
  for (uint32_t c0 = 0; c0 < cnt; c0 += kCCh2) {
    // rank this workgroup's commits per slot inside each wave (log order = (wave, j, lane))
    // (the two rows stay in named registers: an array of the 16-byte operand pairs, indexed in the gather, was
    // promoted to scratch, and each prefetched pair was stored there right after its load, i.e. waited for)
    const uint32_t gg[kCPer2] = {g0, g1}, mm[kCPer2] = {m0, m1};
    uint32_t sl[kCPer2], rk[kCPer2];
    bool own[kCPer2];
#pragma unroll
    for (int j = 0; j < kCPer2; ++j) {
      sl[j] = ((mm[j] >> 16) & 0xFFu) - q0;
      own[j] = gg[j] != 0xFFFFFFFFu && sl[j] < (uint32_t)kQ;
    }
#pragma unroll
    for (int j = 0; j < kCPer2; ++j) rk[j] = own[j] ? atomicAdd(&wc[w][sl[j]], 1u) : 0u;
    lds_barrier();
    PH(1);
    if (w == 0) {  // lane = slot: exclusive prefixes over the waves, then the slot run starts
      uint32_t acc = 0;
#pragma unroll
      for (int q = 0; q < kCW2; ++q) {
        const uint32_t c = wc[q][l];
        wc[q][l] = acc;
        acc += c;
      }
      uint32_t inc = acc;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d, 64);
        if (l >= (uint32_t)d) inc += y;
      }
      sstart[l] = inc - acc;
      if (l == 63) sstart[kQ] = inc;
    }
    lds_barrier();
    PH(2);
    // gather the owned records into LDS, in slot order
    {
      uint32_t p[kCPer2];
#pragma unroll
      for (int j = 0; j < kCPer2; ++j) p[j] = own[j] ? sstart[sl[j]] + wc[w][sl[j]] + rk[j] : 0u;
      auto put = [&](uint32_t pj, const u64x2& abj, uint64_t kyj, uint64_t ixj, uint64_t idj, uint32_t mmj, uint32_t inj,
                     uint32_t ggj) {
        rab[pj] = abj;
        rkey[pj] = kyj;
        ridx[pj] = ixj;
        riid[pj] = idj;
        rmeta[pj] = mmj;
        rins[pj] = inj;
        rpos[pj] = ggj;
      };
      if (own[0]) put(p[0], u64x2{a0x, a0y}, k0, x0, i0, m0, n0, g0);
      if (own[1]) put(p[1], u64x2{a1x, a1y}, k1, x1, i1, m1, n1, g1);
    }
    load_meta(c0 + kCCh2);  // the next chunk's records stream in during the walk
    for (uint32_t k = t; k < (uint32_t)(kCW2 * kQ); k += kCT2) (&wc[0][0])[k] = 0;  // (read above, before the barrier)
    lds_barrier();  // LDS only: __syncthreads() would wait for the loads just issued
    PH(3);
    // the walk: lane l of wave 0 applies slot q0 + l's commits in log order
    uint32_t lane_n = 0;  // events this lane published in this chunk
    if (w == 0) {
      const uint32_t b = sstart[l], e = sstart[l + 1];
      auto walk = [&](auto tc) {
      for (uint32_t p = b; p < e; ++p) {
        const uint32_t mmr = rmeta[p];
        Rec r;
        r.op = smeta_op(mmr);
        r.flags = smeta_flags(mmr);
        r.inst = rins[p];
        r.g = rpos[p];
        r.a = rab[p].x;
        r.b = rab[p].y;
        r.key = rkey[p];
        r.idx = ridx[p];
        r.iid = riid[p];
        uint64_t rv;
        uint32_t nev = 0;
        const uint32_t st = coord_apply<decltype(tc)::value>(type, res, r, h, E, vm, vv, rv, nev, em, lane_n, err);
        rab[p] = u64x2{rv, (uint64_t)(st & 0xFFu) | ((uint64_t)(nev & 0xFFFFu) << 8)};  // the result over the record
      }
      };
      // type-specialised walk when every lane with commits in this chunk holds one type (wave-uniform).  Lanes
      // without commits do not count: a 64-slot group the allocator has not filled keeps CC_RES_NONE slots, and
      // requiring those to match sent the whole group down the generic walk (its workgroups ran 1.4-2.3x longer).
      const uint64_t act = __ballot(b < e);
      uint32_t wt = 0;
      bool uni = false;
      if (act) {
        wt = (uint32_t)__shfl((int)type, __ffsll((long long)act) - 1, 64);
        uni = __all(b >= e || type == wt) != 0;
      }
      if (!act) {
      } else if (!uni) walk(TypeC<0>{});
      else if (wt == CC_RES_LOCK) walk(TypeC<CC_RES_LOCK>{});
      else if (wt == CC_RES_ELECTION) walk(TypeC<CC_RES_ELECTION>{});
      else if (wt == CC_RES_GROUP) walk(TypeC<CC_RES_GROUP>{});
      else if (wt == CC_RES_VALUE) walk(TypeC<CC_RES_VALUE>{});
      else walk(TypeC<0>{});
#ifdef CC_PHASE_TIMING
      ev_total_lane += lane_n;
#endif
      // this chunk's event regions: exclusive prefix of the lanes' (capped) counts, one arena reservation
      const uint32_t mine = lane_n < (uint32_t)kEvLane ? lane_n : (uint32_t)kEvLane;
      uint32_t inc = mine;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d, 64);
        if (l >= (uint32_t)d) inc += y;
      }
      evoff[l] = inc - mine;
      if (l == 63) {
        evoff[kQ] = inc;
        evbase = inc ? atomicAdd(arena_n, (unsigned long long)inc) : 0ull;
      }
    }
    lds_barrier();
    for (uint32_t p = t; p < sstart[kQ]; p += kCT2) {  // results to the records' staging positions
      const uint32_t gp = rpos[p];
      const u64x2 o = rab[p];
      rst_status[gp] = (uint8_t)o.y;
      rst_value[gp] = o.x;
      ev_cnt[gp] = (uint16_t)(o.y >> 8);
    }
    PH(4);
    // flush the chunk's events (their order in the arena is free: events.hip sorts by (row, emission index))
    const uint32_t nb = evoff[kQ];
    for (uint32_t q = t; q < nb; q += kCT2) {
      uint32_t lo = 0, hi = kQ;  // lane whose region holds q: evoff[lo] <= q < evoff[lo + 1]
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (evoff[mid] <= q) lo = mid; else hi = mid;
      }
      if (evbase + q < arena_cap) {
        const uint32_t i = q - evoff[lo];
        uint64_t* dst = reinterpret_cast<uint64_t*>(arena + evbase + q);
        dst[0] = evp[(i * 3 + 0) * kQ + lo];
        dst[1] = evp[(i * 3 + 1) * kQ + lo];
        dst[2] = evp[(i * 3 + 2) * kQ + lo];
      }
    }
    lds_barrier();
    PH(5);
  }
  PH_FLUSH(g_ph_coord);
#ifdef CC_PHASE_TIMING
  if (t == 0 && blockIdx.x < 4096) {
    g_wg_t[4 * blockIdx.x] = ph_t0_;
    g_wg_t[4 * blockIdx.x + 1] = wall_clock64();
    g_wg_t[4 * blockIdx.x + 2] = cnt;
  }
  if (w == 0 && blockIdx.x < 4096) atomicAdd(&g_wg_t[4 * blockIdx.x + 3], (unsigned long long)ev_total_lane);
#endif
  if (w == 0) {
    E.store();
    CoordHdr* hp = reinterpret_cast<CoordHdr*>((uintptr_t)E.glb - sizeof(CoordHdr));  // (= blk)
    hp->who = h.who;
    hp->flags = h.flags;
    hp->idx = h.idx;
    hp->head = h.head;
    hp->n = h.n;
    if (type == CC_RES_VALUE) {
      val_meta[res] = vm;
      val_v[res] = vv;
    }
  }
  if (err) atomicOr(err_out, err);
}

// the engine clock after a batch (time is non-decreasing within a batch: checked here)
__global__ void k_time_check(const uint64_t* __restrict__ time, uint64_t n, uint64_t* __restrict__ clock,
                             uint32_t* __restrict__ err_out) {
  uint32_t bad = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x + 1; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    bad |= time[i] < time[i - 1];
  if (bad) atomicOr(err_out, kErrTime);
}
__global__ void k_clock_advance(const uint64_t* __restrict__ time, uint64_t n, uint64_t now, uint64_t* __restrict__ clock) {
  uint64_t c = *clock;
  if (time && n && time[n - 1] > c) c = time[n - 1];
  if (now > c) c = now;
  *clock = c;
}

int launch_apply_coord(const CoordArgs& a, hipStream_t st) {
  if (a.tiles == 0) return 0;
  a.mark(K_APPLY_COORD, 1, st);
  hipLaunchKernelGGL(k_apply_coord, dim3(a.sb_val * kQPerSb), dim3(kCT2), 0, st, a.xrec,
                     a.ttab, a.tiles, a.sb, a.sbq_base, a.sb_kind, a.res_type, a.inst_id, a.coord, a.coord_cap, a.val_meta, a.val_v, a.rst_status,
                     a.rst_value, a.ev_cnt, a.arena, a.arena_n, a.arena_cap, a.leak, a.leak_n, a.leak_cap, a.err);
  a.mark(K_APPLY_COORD, 0, st);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_time_check(const uint64_t* time, uint64_t n, uint64_t* clock, uint32_t* err, hipStream_t st) {
  if (!time || n < 2) return 0;
  const uint64_t blocks = (n + 255) / 256 < 1024 ? (n + 255) / 256 : 1024;
  hipLaunchKernelGGL(k_time_check, dim3((uint32_t)blocks), dim3(256), 0, st, time, n, clock, err);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ---- MembershipGroupState.schedule (op 122) :86-103: a barrier row of the batch (engine.hip) --------------
// The row's status against the group as it stands at that log position; *found tells the host to arm the timer.
__global__ void k_group_schedule(const uint8_t* __restrict__ coord, uint32_t ccap, uint32_t slot, uint64_t member, uint64_t row,
                                 uint8_t* __restrict__ out_status, uint64_t* __restrict__ out_value, uint32_t* __restrict__ found) {
  if (threadIdx.x != 0) return;
  const uint8_t* blk = coord + (uint64_t)slot * coord_block(ccap);
  const CoordHdr h = *reinterpret_cast<const CoordHdr*>(blk);
  const CoordEnt* E = reinterpret_cast<const CoordEnt*>(blk + sizeof(CoordHdr));
  uint32_t f = 0;
  for (uint32_t q = 0; q < h.n && q < ccap; ++q) f |= E[q].x == member ? 1u : 0u;
  out_status[row] = (uint8_t)(f ? CC_STATUS(CC_ST_OK, CC_TAG_NULL) : CC_STATUS(CC_ST_ILLEGAL_ARGUMENT, CC_TAG_NULL));
  out_value[row] = 0;
  *found = f;
}

// The timer fires (:92-98): publish "execute"(callback) to the member's instance if it is still in the group.
__global__ void k_group_fire(const uint8_t* __restrict__ coord, uint32_t ccap, uint32_t slot, uint64_t member, uint32_t tag, uint64_t payload,
                             uint32_t pos, unsigned long long* __restrict__ ev_total, uint64_t cap,
                             uint32_t* __restrict__ o_pos, uint32_t* __restrict__ o_target, uint8_t* __restrict__ o_code,
                             uint8_t* __restrict__ o_src, uint8_t* __restrict__ o_tag, uint64_t* __restrict__ o_payload,
                             uint32_t* __restrict__ err) {
  if (threadIdx.x != 0) return;
  const uint8_t* blk = coord + (uint64_t)slot * coord_block(ccap);
  const CoordHdr h = *reinterpret_cast<const CoordHdr*>(blk);
  const CoordEnt* E = reinterpret_cast<const CoordEnt*>(blk + sizeof(CoordHdr));
  for (uint32_t q = 0; q < h.n && q < ccap; ++q) {
    if (E[q].x != member) continue;
    if (!o_pos) {
      atomicOr(err, kErrUnsupported);  // an event with no stream to publish it to
      return;
    }
    const unsigned long long k = *ev_total;
    if (k >= cap) {
      atomicOr(err, kErrEvents);
      return;
    }
    o_pos[k] = pos;
    o_target[k] = E[q].inst;
    o_code[k] = CC_EV_EXECUTE;
    o_src[k] = CC_EVSRC_TIMER;
    o_tag[k] = (uint8_t)tag;
    o_payload[k] = payload;
    *ev_total = k + 1;
    return;
  }
}

int launch_group_schedule(const uint8_t* coord, uint32_t ccap, uint32_t slot, uint64_t member, uint64_t row, uint8_t* out_status,
                          uint64_t* out_value, uint32_t* found, hipStream_t st) {
  hipLaunchKernelGGL(k_group_schedule, dim3(1), dim3(64), 0, st, coord, ccap, slot, member, row, out_status, out_value, found);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_group_fire(const uint8_t* coord, uint32_t ccap, uint32_t slot, uint64_t member, uint32_t tag, uint64_t payload, uint32_t pos,
                      unsigned long long* ev_total, const cc_events* ev, uint32_t* err, hipStream_t st) {
  hipLaunchKernelGGL(k_group_fire, dim3(1), dim3(64), 0, st, coord, ccap, slot, member, tag, payload, pos, ev_total,
                     ev ? ev->capacity : 0, ev ? ev->pos : nullptr, ev ? ev->target : nullptr, ev ? ev->code : nullptr,
                     ev ? ev->src : nullptr, ev ? ev->tag : nullptr, ev ? ev->payload : nullptr, err);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_clock_advance(const uint64_t* time, uint64_t n, uint64_t now, uint64_t* clock, hipStream_t st) {
  hipLaunchKernelGGL(k_clock_advance, dim3(1), dim3(1), 0, st, time, n, now, clock);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace cc
