// apply_coord.hip — coordination state machines (LockState, LeaderElectionState, MembershipGroupState) and
// AtomicValue with listeners, with their published events.
//
// Same shape as apply_value.hip: one 256-thread workgroup per super-bucket (256 resource slots), thread t owns
// slot t and applies that slot's commits in log order.  The super-buckets handled here are those holding a
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
#include "common.h"
#include "engine_internal.h"

namespace cc {

constexpr int kCT = 256;            // threads = slots per super-bucket
constexpr int kCPer = 8;            // commits per thread per chunk (2048: fewer chunk barriers; 146 KB LDS)
constexpr int kCCh = kCT * kCPer;   // 2048
constexpr int kEvBuf = 2048;        // LDS event buffer per chunk

struct Emitter {
  EvRec* buf;
  uint32_t* nbuf;
  EvRec* arena;
  unsigned long long* arena_n;
  uint64_t arena_cap;
  __device__ void emit(uint32_t g, uint32_t k, uint32_t target, uint32_t code, uint32_t src, uint32_t tag,
                       uint64_t payload) const {
    EvRec e;
    e.g = g;
    e.target = target;
    e.payload = tag == CC_TAG_NULL ? 0 : payload;
    e.k = (uint16_t)k;
    e.code = (uint8_t)code;
    e.tag = (uint8_t)tag;
    e.src = (uint8_t)src;
    e.pad[0] = e.pad[1] = e.pad[2] = 0;
    const uint32_t q = atomicAdd(nbuf, 1u);
    if (q < (uint32_t)kEvBuf) {
      buf[q] = e;
    } else {  // buffer full: straight to the arena
      const unsigned long long a = atomicAdd(arena_n, 1ull);
      if (a < arena_cap) arena[a] = e;
    }
  }
};

__device__ inline CoordEnt* ents(uint8_t* blk) { return reinterpret_cast<CoordEnt*>(blk + sizeof(CoordHdr)); }

// ---- LockState ----------------------------------------------------------------------------------------
__device__ inline void lock_expire(CoordHdr& h, CoordEnt* q, uint64_t th) {  // silent timeouts (A7)
  uint32_t kept = 0;
  for (uint32_t i = 0; i < h.n; ++i) {
    const CoordEnt e = q[(h.head + i) % kCoordCap];
    if (e.x != kNoDeadline && e.x <= th) continue;
    if (kept != i) q[(h.head + kept) % kCoordCap] = e;
    ++kept;
  }
  h.n = kept;
}

// ---- one commit on a coordination / value slot -----------------------------------------------------------
struct Rec {
  uint32_t op, flags, inst, g;
  uint64_t a, b, key, idx, iid;
};

__device__ inline uint32_t coord_apply(uint32_t type, const Rec& r, CoordHdr& h, uint8_t* blk, uint32_t& vmeta_s,
                                       uint64_t& vval, uint64_t& rv, uint32_t& nev, const Emitter& em, uint32_t& err) {
  CoordEnt* E = ents(blk);
  rv = 0;
  auto ev = [&](uint32_t target, uint32_t code, uint32_t tag, uint64_t payload) {
    em.emit(r.g, nev++, target, code, CC_EVSRC_COMMIT, tag, payload);
  };
  if (h.flags & kCoZombie) return CC_STATUS(CC_ST_NULL_POINTER, CC_TAG_NULL);
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
        } else if (h.n == (uint32_t)kCoordCap) {
          err |= kErrCapacity;
        } else {
          E[(h.head + h.n) % kCoordCap] = CoordEnt{timeout > 0 ? clk + (uint64_t)timeout : kNoDeadline, r.idx, r.inst, 0};
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
          const CoordEnt e = E[h.head];
          h.head = (h.head + 1) % kCoordCap;
          --h.n;
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
      if (r.op == CC_OP_ELECT_LISTEN) {
        if (!(h.flags & kCoHeld)) {
          h.flags = kCoHeld;
          h.who = r.inst;
          h.idx = r.idx;
          ev(r.inst, CC_EV_ELECT, CC_TAG_LONG, r.idx);
        } else {
          bool found = false;
          for (uint32_t i = 0; i < h.n && !found; ++i) found = E[i].x == r.iid;
          if (!found) {  // may be the leader's own session (A9)
            if (h.n == (uint32_t)kCoordCap) err |= kErrCapacity;
            else E[h.n++] = CoordEnt{r.iid, r.idx, r.inst, 0};
          }
        }
        return CC_STATUS(CC_ST_OK, CC_TAG_NULL);
      }
      if (r.op == CC_OP_ELECT_UNLISTEN) {
        if ((h.flags & kCoHeld) && h.who == r.inst) {
          if (h.flags & kCoCleaned) return CC_STATUS(CC_ST_ILLEGAL_STATE, CC_TAG_NULL);
          h.flags = 0;
          if (h.n) {
            const CoordEnt e = E[0];
            for (uint32_t i = 1; i < h.n; ++i) E[i - 1] = E[i];
            --h.n;
            h.flags = kCoHeld;
            h.who = e.inst;
            h.idx = e.idx;
            ev(e.inst, CC_EV_ELECT, CC_TAG_LONG, e.idx);
          }
        } else {
          for (uint32_t i = 0; i < h.n; ++i)
            if (E[i].x == r.iid) {
              for (uint32_t k = i + 1; k < h.n; ++k) E[k - 1] = E[k];
              --h.n;
              break;
            }
        }
        return CC_STATUS(CC_ST_OK, CC_TAG_NULL);
      }
      // isLeader
      rv = ((h.flags & kCoHeld) && h.who == r.inst && h.idx == 0) ? 1 : 0;
      return CC_STATUS(CC_ST_OK, CC_TAG_BOOL);
    }
    case CC_RES_GROUP: {
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
          if (E[m].x < id) lo = m + 1; else hi = m;
        }
        hit = lo < h.n && E[lo].x == id;
        return lo;
      };
      bool hit;
      if (r.op == CC_OP_GROUP_JOIN) {
        const uint32_t p = find(r.iid, hit);
        if (hit) {
          E[p].idx = r.idx;  // previous.clean()
          E[p].inst = r.inst;
        } else if (h.n == (uint32_t)kCoordCap) {
          err |= kErrCapacity;
        } else {
          for (uint32_t i = h.n; i > p; --i) E[i] = E[i - 1];
          E[p] = CoordEnt{r.iid, r.idx, r.inst, 0};
          ++h.n;
          for (uint32_t i = 0; i < h.n; ++i)
            if (E[i].idx != r.idx) ev(E[i].inst, CC_EV_JOIN, CC_TAG_LONG, r.iid);
        }
        for (uint32_t i = 0; i < h.n; ++i)  // the returned Set<Long>, ascending
          em.emit(r.g, nev++, r.inst, CC_EV_MEMBER, CC_EVSRC_RESULT, CC_TAG_LONG, E[i].x);
        rv = h.n;
        return CC_STATUS(CC_ST_OK, CC_TAG_SET);
      }
      if (r.op == CC_OP_GROUP_LEAVE) {
        const uint32_t p = find(r.iid, hit);
        if (hit) {
          for (uint32_t i = p + 1; i < h.n; ++i) E[i - 1] = E[i];
          --h.n;
          for (uint32_t i = 0; i < h.n; ++i) ev(E[i].inst, CC_EV_LEAVE, CC_TAG_LONG, r.iid);
        }
        return CC_STATUS(CC_ST_OK, CC_TAG_NULL);
      }
      // execute(member = key, callback = a)
      const uint32_t p = find(r.key, hit);
      if (!hit) return CC_STATUS(CC_ST_ILLEGAL_ARGUMENT, CC_TAG_NULL);  // "unknown member"
      ev(E[p].inst, CC_EV_EXECUTE, CC_FLAG_TAG_A(r.flags), r.a);
      return CC_STATUS(CC_ST_OK, CC_TAG_NULL);
    }
    case CC_RES_QUEUE: {  // QueueState.java:33-199: an ArrayDeque of (value tag in pad, payload in x), FIFO ring
      const uint32_t ta = CC_FLAG_TAG_A(r.flags);
      const uint64_t pa = ta ? r.a : 0;
      auto at = [&](uint32_t i) -> CoordEnt& { return E[(h.head + i) % kCoordCap]; };
      auto first_match = [&](uint32_t& pos) -> int {  // 1 match, 0 none, -1 NPE (a stored null's equals)
        for (uint32_t i = 0; i < h.n; ++i) {
          const CoordEnt& e = at(i);
          if (e.pad == CC_TAG_NULL) return -1;
          if (e.pad == ta && e.x == pa) {
            pos = i;
            return 1;
          }
        }
        return 0;
      };
      auto pop = [&]() {
        h.head = (h.head + 1) % kCoordCap;
        --h.n;
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
          if (h.n == (uint32_t)kCoordCap) {
            err |= kErrCapacity;
          } else {
            at(h.n) = CoordEnt{pa, r.idx, r.inst, ta};
            ++h.n;
          }
          return CC_STATUS(CC_ST_OK, CC_TAG_BOOL);
        case CC_OP_QUEUE_PEEK:  // peek :77-87
          if (!h.n) return CC_STATUS(CC_ST_OK, CC_TAG_NULL);
          rv = at(0).x;
          return CC_STATUS(CC_ST_OK, at(0).pad);
        case CC_OP_QUEUE_POLL: {  // poll :92-105
          if (!h.n) return CC_STATUS(CC_ST_OK, CC_TAG_NULL);
          const CoordEnt e = at(0);
          pop();
          rv = e.x;
          return CC_STATUS(CC_ST_OK, e.pad);
        }
        case CC_OP_QUEUE_ELEMENT:  // element :111-124 (throws when empty; the head stays)
          if (!h.n) return CC_STATUS(CC_ST_NO_SUCH_ELEMENT, CC_TAG_NULL);
          rv = at(0).x;
          return CC_STATUS(CC_ST_OK, at(0).pad);
        case CC_OP_QUEUE_REMOVE: {  // remove :130-157
          if (ta != CC_TAG_NULL) {
            uint32_t pos = 0;
            const int m = first_match(pos);
            if (m < 0) return CC_STATUS(CC_ST_NULL_POINTER, CC_TAG_NULL);
            if (m) {
              for (uint32_t i = pos; i + 1 < h.n; ++i) at(i) = at(i + 1);
              --h.n;
            }
            rv = m;
            return CC_STATUS(CC_ST_OK, CC_TAG_BOOL);
          }
          if (!h.n) return CC_STATUS(CC_ST_NO_SUCH_ELEMENT, CC_TAG_NULL);  // ArrayDeque.remove()
          const CoordEnt e = at(0);
          pop();
          rv = e.x;
          return CC_STATUS(CC_ST_OK, e.pad);
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
          for (uint32_t i = 0; i < h.n; ++i)
            if (E[i].inst == r.inst) { E[i].idx = r.idx; found = true; }
          if (!found) {
            if (h.n == (uint32_t)kCoordCap) err |= kErrCapacity;
            else E[h.n++] = CoordEnt{0, r.idx, r.inst, 0};
          }
          break;
        }
        case CC_OP_VALUE_UNLISTEN:
          for (uint32_t i = 0; i < h.n; ++i)
            if (E[i].inst == r.inst) {
              for (uint32_t k = i + 1; k < h.n; ++k) E[k - 1] = E[k];
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
        for (uint32_t i = 0; i < h.n; ++i) ev(E[i].inst, CC_EV_CHANGE, ntag, nv);  // change(value) :68-72
      }
      rv = rvv;
      return CC_STATUS(CC_ST_OK, rtag);
    }
  }
  return CC_STATUS(CC_ST_UNKNOWN_OP, CC_TAG_NULL);
}

__global__ __launch_bounds__(kCT) void k_apply_coord(const uint32_t* __restrict__ st_meta, const u64x2* __restrict__ st_ab,
                                                    const uint32_t* __restrict__ st_res, const uint64_t* __restrict__ st_key,
                                                    const uint64_t* __restrict__ st_idx, const uint16_t* __restrict__ ttab,
                                                    uint32_t tiles, uint32_t sb, const uint8_t* __restrict__ sb_kind,
                                                    const uint8_t* __restrict__ res_type, const uint64_t* __restrict__ inst_id,
                                                    uint8_t* __restrict__ coord, uint32_t* __restrict__ val_meta,
                                                    uint64_t* __restrict__ val_v, uint8_t* __restrict__ rst_status,
                                                    uint64_t* __restrict__ rst_value, uint16_t* __restrict__ ev_cnt,
                                                    EvRec* __restrict__ arena, unsigned long long* __restrict__ arena_n,
                                                    uint64_t arena_cap, uint32_t* __restrict__ err_out) {
  __shared__ u64x2 rab[kCCh];
  __shared__ uint64_t rkey[kCCh];
  __shared__ uint64_t ridx[kCCh];
  __shared__ uint32_t rmeta[kCCh];
  __shared__ uint32_t rins[kCCh];
  __shared__ uint32_t rpos[kCCh];
  __shared__ uint32_t scnt[kCT + 1];
  __shared__ uint32_t rstart[kMaxTiles];
  __shared__ uint32_t rpre[kMaxTiles + 1];
  __shared__ uint32_t wsum[kCT / kWave];
  __shared__ EvRec evbuf[kEvBuf];
  __shared__ uint32_t evn;
  __shared__ unsigned long long evbase;

  const uint32_t s = blockIdx.x;
  if (!sb_kind[s]) return;  // value-only super-bucket: k_apply_value
  const uint32_t t = threadIdx.x, w = t >> 6, l = t & 63;
  const uint32_t res = s * kCT + t, type = res_type[res];
  uint32_t err = 0;
  scnt[t] = 0;
  if (t == 0) {
    scnt[kCT] = 0;
    evn = 0;
  }
  {  // this super-bucket's list = its run in every tile, in tile order
    constexpr int PT = kMaxTiles / kCT;
    uint32_t len[PT], sum = 0;
#pragma unroll
    for (int q = 0; q < PT; ++q) {
      const uint32_t tt = t * PT + q;
      len[q] = 0;
      if (tt < tiles) {
        const uint16_t* row = ttab + (uint64_t)tt * (sb + 1);
        const uint32_t b0 = row[s], b1 = row[s + 1];
        rstart[tt] = tt * kTile + b0;
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
    if (t == kCT - 1) rpre[tiles] = run;
    __syncthreads();
  }
  const uint32_t cnt = rpre[tiles];
  const Emitter em{evbuf, &evn, arena, arena_n, arena_cap};
  uint8_t* blk = coord + (uint64_t)res * kCoordBlock;

  for (uint32_t c0 = 0; c0 < cnt; c0 += kCCh) {
    uint32_t m[kCPer], g[kCPer], rk[kCPer];
#pragma unroll
    for (int j = 0; j < kCPer; ++j) {
      const uint32_t c = c0 + w * (kWave * kCPer) + j * kWave + l;
      g[j] = 0xFFFFFFFFu;
      if (c < cnt) {
        uint32_t lo = 0, hi = tiles;
        while (hi - lo > 1) {
          const uint32_t mid = (lo + hi) >> 1;
          if (rpre[mid] <= c) lo = mid; else hi = mid;
        }
        g[j] = rstart[lo] + (c - rpre[lo]);
        m[j] = st_meta[g[j]];
      }
    }
    // stable counting sort by slot, one wave at a time (log order = (wave, j, lane))
    for (uint32_t q = 0; q < kCT / kWave; ++q) {
      if (w == q) {
#pragma unroll
        for (int j = 0; j < kCPer; ++j)
          if (g[j] != 0xFFFFFFFFu) rk[j] = atomicAdd(&scnt[(m[j] >> 16) & 0xFF], 1u);
      }
      __syncthreads();
    }
    const uint32_t mine = scnt[t];
    uint32_t inc = mine;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(inc, d, 64);
      if (l >= (uint32_t)d) inc += y;
    }
    if (l == 63) wsum[w] = inc;
    __syncthreads();
    uint32_t start = inc - mine;
    for (uint32_t q = 0; q < w; ++q) start += wsum[q];
    __syncthreads();
    scnt[t] = start;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kCPer; ++j) {
      if (g[j] == 0xFFFFFFFFu) continue;
      const uint32_t p = scnt[(m[j] >> 16) & 0xFF] + rk[j];
      rab[p] = st_ab[g[j]];
      rkey[p] = st_key[g[j]];
      ridx[p] = st_idx[g[j]];
      rmeta[p] = m[j];
      rins[p] = st_res[g[j]];
      rpos[p] = g[j];
    }
    __syncthreads();
    // this slot's commits, in log order
    if (mine) {
      CoordHdr h = *reinterpret_cast<const CoordHdr*>(blk);
      uint32_t vm = 0;
      uint64_t vv = 0;
      if (type == CC_RES_VALUE) {
        vm = val_meta[res];
        vv = val_v[res];
      }
      for (uint32_t p = start; p < start + mine; ++p) {
        const uint32_t mm = rmeta[p];
        Rec r;
        r.op = smeta_op(mm);
        r.flags = smeta_flags(mm);
        r.inst = rins[p];
        r.g = rpos[p];
        r.a = rab[p].x;
        r.b = rab[p].y;
        r.key = rkey[p];
        r.idx = ridx[p];
        r.iid = inst_id[r.inst];
        uint64_t rv;
        uint32_t nev = 0;
        const uint32_t st = coord_apply(type, r, h, blk, vm, vv, rv, nev, em, err);
        rst_status[r.g] = (uint8_t)st;
        rst_value[r.g] = rv;
        ev_cnt[r.g] = (uint16_t)nev;
      }
      *reinterpret_cast<CoordHdr*>(blk) = h;
      if (type == CC_RES_VALUE) {
        val_meta[res] = vm;
        val_v[res] = vv;
      }
    }
    __syncthreads();
    // flush the chunk's events: one arena reservation per chunk
    const uint32_t nb = evn < (uint32_t)kEvBuf ? evn : (uint32_t)kEvBuf;
    if (t == 0) evbase = nb ? atomicAdd(arena_n, (unsigned long long)nb) : 0ull;
    __syncthreads();
    for (uint32_t q = t; q < nb; q += kCT)
      if (evbase + q < arena_cap) arena[evbase + q] = evbuf[q];
    __syncthreads();
    scnt[t] = 0;
    if (t == 0) evn = 0;
    __syncthreads();
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
  hipLaunchKernelGGL(k_apply_coord, dim3(a.sb_val), dim3(kCT), 0, st, a.st_meta, a.st_ab, a.st_res, a.st_key, a.st_idx,
                     a.ttab, a.tiles, a.sb, a.sb_kind, a.res_type, a.inst_id, a.coord, a.val_meta, a.val_v, a.rst_status,
                     a.rst_value, a.ev_cnt, a.arena, a.arena_n, a.arena_cap, a.err);
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
__global__ void k_group_schedule(const uint8_t* __restrict__ coord, uint32_t slot, uint64_t member, uint64_t row,
                                 uint8_t* __restrict__ out_status, uint64_t* __restrict__ out_value, uint32_t* __restrict__ found) {
  if (threadIdx.x != 0) return;
  const uint8_t* blk = coord + (uint64_t)slot * kCoordBlock;
  const CoordHdr h = *reinterpret_cast<const CoordHdr*>(blk);
  const CoordEnt* E = reinterpret_cast<const CoordEnt*>(blk + sizeof(CoordHdr));
  uint32_t f = 0;
  for (uint32_t q = 0; q < h.n && q < (uint32_t)kCoordCap; ++q) f |= E[q].x == member ? 1u : 0u;
  out_status[row] = (uint8_t)(f ? CC_STATUS(CC_ST_OK, CC_TAG_NULL) : CC_STATUS(CC_ST_ILLEGAL_ARGUMENT, CC_TAG_NULL));
  out_value[row] = 0;
  *found = f;
}

// The timer fires (:92-98): publish "execute"(callback) to the member's instance if it is still in the group.
__global__ void k_group_fire(const uint8_t* __restrict__ coord, uint32_t slot, uint64_t member, uint32_t tag, uint64_t payload,
                             uint32_t pos, unsigned long long* __restrict__ ev_total, uint64_t cap,
                             uint32_t* __restrict__ o_pos, uint32_t* __restrict__ o_target, uint8_t* __restrict__ o_code,
                             uint8_t* __restrict__ o_src, uint8_t* __restrict__ o_tag, uint64_t* __restrict__ o_payload,
                             uint32_t* __restrict__ err) {
  if (threadIdx.x != 0) return;
  const uint8_t* blk = coord + (uint64_t)slot * kCoordBlock;
  const CoordHdr h = *reinterpret_cast<const CoordHdr*>(blk);
  const CoordEnt* E = reinterpret_cast<const CoordEnt*>(blk + sizeof(CoordHdr));
  for (uint32_t q = 0; q < h.n && q < (uint32_t)kCoordCap; ++q) {
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

int launch_group_schedule(const uint8_t* coord, uint32_t slot, uint64_t member, uint64_t row, uint8_t* out_status,
                          uint64_t* out_value, uint32_t* found, hipStream_t st) {
  hipLaunchKernelGGL(k_group_schedule, dim3(1), dim3(64), 0, st, coord, slot, member, row, out_status, out_value, found);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_group_fire(const uint8_t* coord, uint32_t slot, uint64_t member, uint32_t tag, uint64_t payload, uint32_t pos,
                      unsigned long long* ev_total, const cc_events* ev, uint32_t* err, hipStream_t st) {
  hipLaunchKernelGGL(k_group_fire, dim3(1), dim3(64), 0, st, coord, slot, member, tag, payload, pos, ev_total,
                     ev ? ev->capacity : 0, ev ? ev->pos : nullptr, ev ? ev->target : nullptr, ev ? ev->code : nullptr,
                     ev ? ev->src : nullptr, ev ? ev->tag : nullptr, ev ? ev->payload : nullptr, err);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_clock_advance(const uint64_t* time, uint64_t n, uint64_t now, uint64_t* clock, hipStream_t st) {
  hipLaunchKernelGGL(k_clock_advance, dim3(1), dim3(1), 0, st, time, n, now, clock);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace cc
