// close.hip — the session close / expire fan-out of ResourceManager on the GPU.
//
// Reference: ResourceManager.close(Session) :250-264 and expire(Session) :238-247
// (manager/src/main/java/io/atomix/manager/ResourceManager.java).  For one client session the manager walks
// ResourceManager.sessions (a HashMap<Long instanceId, SessionHolder>) and, for every instance the session
// owns, calls the resource state machine's close(instanceSession), then drops the instance.  expire() calls
// StateMachine.expire, which none of the covered state machines override; Copycat then closes the session
// [not vendored], so an expiry is a close.
//
// State-machine close overrides restated here:
//   AtomicValueState — the Listen commit's session close listener drops the listener (AtomicValueState.java:43-48);
//   LeaderElectionState.close :35-52 — the leader's session: leader.clean() (throws "commit closed" when delete()
//                      already cleaned it), the first listener becomes leader and is told "elect"(its Listen
//                      index); any other session: its listener entry is removed;
//   MembershipGroupState.close :36-42 — members.remove(id) and "leave"(id) to every remaining member, even when
//                      the session was not a member;
//   LockState / MapState — no close handler (A11): nothing.
//
// engine.hip turns the closing client sessions into the ordered list of instance slots (client order, then the
// Java HashMap order of ResourceManager.sessions) and groups the list positions by resource.  Then:
//   k_close_check   : one thread per position: per client, the first position whose close throws (an election
//                     whose cleaned leader commit belongs to that instance — a cleaned leader can never be
//                     replaced, so the pre-state decides); that client's ResourceManager.close loop stops there;
//   k_close_apply   : one thread per resource: its closes in fan-out order, positions before the stop; events
//                     to the arena tagged (position, emission index), per-position event counts;
//   k_close_scan    : one workgroup: exclusive scan of the per-position counts, capacity checks;
//   k_close_scatter : arena -> the caller's event stream, ordered by (position, emission index);
//   k_close_unreg   : closed instances leave the dispatch table (ResourceManager.sessions.remove).
#include "common.h"
#include "engine_internal.h"

namespace cc {

__global__ void k_close_check(const uint32_t* __restrict__ cinst, uint32_t m, const uint32_t* __restrict__ inst_res,
                              const uint8_t* __restrict__ res_type, const uint8_t* __restrict__ coord, uint32_t ccap,
                              const uint32_t* __restrict__ pcl, uint32_t* __restrict__ fail) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= m || !coord) return;
  const uint32_t islot = cinst[p], r = inst_res[islot];
  if (r == kNoRes || res_type[r] != CC_RES_ELECTION) return;
  const CoordHdr h = *reinterpret_cast<const CoordHdr*>(coord + (uint64_t)r * coord_block(ccap));
  if (h.flags & kCoZombie) return;  // not in ResourceManager.resources: no close handler runs
  if ((h.flags & kCoHeld) && (h.flags & kCoCleaned) && h.who == islot) atomicMin(&fail[pcl[p]], p);
}

__global__ void k_close_apply(const uint32_t* __restrict__ cinst, const uint32_t* __restrict__ rlist,
                              const uint32_t* __restrict__ rstart, const uint32_t* __restrict__ items, uint32_t nr,
                              const uint32_t* __restrict__ pcl, const uint32_t* __restrict__ fail,
                              const uint8_t* __restrict__ res_type,
                              const uint64_t* __restrict__ inst_id, uint8_t* __restrict__ coord, uint32_t ccap,
                              uint32_t* __restrict__ cnt,
                              EvRec* __restrict__ arena, unsigned long long* __restrict__ arena_n, uint64_t arena_cap,
                              LeakRec* __restrict__ leak, unsigned long long* __restrict__ leak_n, uint64_t leak_cap,
                              uint32_t* __restrict__ err) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nr) return;
  const uint32_t r = rlist[k], type = res_type[r];
  uint8_t* blk = coord + (uint64_t)r * coord_block(ccap);
  CoordHdr h = *reinterpret_cast<const CoordHdr*>(blk);
  CoordEnt* E = reinterpret_cast<CoordEnt*>(blk + sizeof(CoordHdr));
  for (uint32_t q = rstart[k]; q < rstart[k + 1]; ++q) {
    const uint32_t p = items[q];
    if (p >= fail[pcl[p]]) continue;  // this client's ResourceManager.close loop ended before this close
    const uint32_t islot = cinst[p];
    const uint64_t iid = inst_id[islot];
    uint32_t nev = 0;
    auto ev = [&](uint32_t target, uint32_t code, uint64_t payload) {
      const unsigned long long a = atomicAdd(arena_n, 1ull);
      if (a < arena_cap) {
        EvRec e;
        e.g = p;
        e.target = target;
        e.payload = payload;
        e.k = (uint16_t)nev;
        e.code = (uint8_t)code;
        e.tag = CC_TAG_LONG;
        e.src = CC_EVSRC_CLOSE;
        e.pad[0] = e.pad[1] = e.pad[2] = 0;
        arena[a] = e;
      }
      ++nev;
    };
    if (type == CC_RES_VALUE) {  // AtomicValueState.java:43-48
      for (uint32_t i = 0; i < h.n; ++i)
        if (E[i].inst == islot) {
          for (uint32_t j = i + 1; j < h.n; ++j) E[j - 1] = E[j];
          --h.n;
          break;
        }
    } else if (type == CC_RES_ELECTION) {  // LeaderElectionState.close :35-52
      if ((h.flags & kCoHeld) && h.who == islot) {
        h.flags = 0;
        if (h.n) {
          const CoordEnt e = E[0];
          for (uint32_t i = 1; i < h.n; ++i) E[i - 1] = E[i];
          --h.n;
          h.flags = kCoHeld;
          h.who = e.inst;
          h.idx = e.idx;
          ev(e.inst, CC_EV_ELECT, e.idx);
        }
      } else {
        for (uint32_t i = 0; i < h.n; ++i)
          if (E[i].x == iid) {
            for (uint32_t j = i + 1; j < h.n; ++j) E[j - 1] = E[j];
            --h.n;
            break;
          }
      }
    } else if (type == CC_RES_GROUP) {  // MembershipGroupState.close :36-42 (members sorted by instance id)
      uint32_t lo = 0, hi = h.n;
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (E[mid].x < iid) lo = mid + 1; else hi = mid;
      }
      if (lo < h.n && E[lo].x == iid) {  // members.remove without clean(): the join commit stays in the log
        const unsigned long long a = atomicAdd(leak_n, 1ull);
        if (a < leak_cap) {
          leak[a].idx = E[lo].idx;
          leak[a].slot = r;
          leak[a].pad = 0;
        } else {
          atomicOr(err, kErrCapacity);
        }
        for (uint32_t j = lo + 1; j < h.n; ++j) E[j - 1] = E[j];
        --h.n;
      }
      for (uint32_t i = 0; i < h.n; ++i) ev(E[i].inst, CC_EV_LEAVE, iid);
    }
    cnt[p] = nev;
  }
  *reinterpret_cast<CoordHdr*>(blk) = h;
}

// exclusive scan of cnt[0, min(m, stop)) -> off[0..m]; the event count; capacity checks
constexpr int kCS = 1024;
__global__ __launch_bounds__(kCS) void k_close_scan(const uint32_t* __restrict__ cnt, uint32_t m,
                                                    const uint32_t* __restrict__ pcl, const uint32_t* __restrict__ fail,
                                                    uint64_t* __restrict__ off, const unsigned long long* __restrict__ arena_n,
                                                    uint64_t arena_cap, uint64_t out_cap, int has_out,
                                                    uint64_t* __restrict__ out_count, uint32_t* __restrict__ err_out) {
  __shared__ unsigned long long wsum[kCS / kWave];
  __shared__ unsigned long long carry;
  const uint32_t t = threadIdx.x, w = t >> 6, l = t & 63;
  if (t == 0) carry = 0;
  __syncthreads();
  for (uint32_t b = 0; b < m; b += kCS) {
    const uint32_t p = b + t;
    const unsigned long long v = p < m && p < fail[pcl[p]] ? cnt[p] : 0ull;
    unsigned long long inc = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const unsigned long long y = __shfl_up(inc, d, 64);
      if (l >= (uint32_t)d) inc += y;
    }
    if (l == 63) wsum[w] = inc;
    __syncthreads();
    unsigned long long pre = carry, tot = 0;
    for (uint32_t q = 0; q < kCS / kWave; ++q) {
      if (q < w) pre += wsum[q];
      tot += wsum[q];
    }
    if (p < m) off[p] = pre + inc - v;
    __syncthreads();
    if (t == 0) carry += tot;
    __syncthreads();
  }
  if (t == 0) {
    off[m] = carry;
    if (out_count) *out_count = carry;
    uint32_t err = 0;
    if (*arena_n > arena_cap || (has_out && carry > out_cap)) err |= kErrEvents;
    if (!has_out && carry) err |= kErrUnsupported;  // events published but no stream to publish them to
    if (err) atomicOr(err_out, err);
  }
}

__global__ void k_close_scatter(const EvRec* __restrict__ arena, const unsigned long long* __restrict__ arena_n,
                                uint64_t arena_cap, const uint64_t* __restrict__ off, uint64_t out_cap,
                                uint32_t* __restrict__ pos, uint32_t* __restrict__ target, uint8_t* __restrict__ code,
                                uint8_t* __restrict__ src, uint8_t* __restrict__ tag, uint64_t* __restrict__ payload) {
  const uint64_t ne = *arena_n < arena_cap ? *arena_n : arena_cap;
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < ne; e += (uint64_t)gridDim.x * blockDim.x) {
    const EvRec r = arena[e];
    const uint64_t dst = off[r.g] + r.k;
    if (dst >= out_cap) continue;
    pos[dst] = 0xFFFFFFFFu;  // not a log row: published by the close fan-out
    target[dst] = r.target;
    code[dst] = r.code;
    src[dst] = r.src;
    tag[dst] = r.tag;
    payload[dst] = r.payload;
  }
}

__global__ void k_close_unreg(const uint32_t* __restrict__ cinst, uint32_t m, const uint32_t* __restrict__ pcl,
                              const uint32_t* __restrict__ fail, uint32_t* __restrict__ inst_res) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < m && p < fail[pcl[p]]) inst_res[cinst[p]] = kNoRes;
}

int launch_close(const CloseArgs& a, hipStream_t st) {
  if (a.m == 0) return 0;
  const uint32_t gm = (a.m + 255) / 256;
  hipLaunchKernelGGL(k_close_check, dim3(gm), dim3(256), 0, st, a.cinst, a.m, a.inst_res, a.res_type, a.coord, a.coord_cap, a.pcl, a.fail);
  if (a.nr && a.coord)
    hipLaunchKernelGGL(k_close_apply, dim3((a.nr + 63) / 64), dim3(64), 0, st, a.cinst, a.rlist, a.rstart, a.items, a.nr,
                       a.pcl, a.fail, a.res_type, a.inst_id, a.coord, a.coord_cap, a.cnt, a.arena, a.arena_n, a.arena_cap,
                       a.leak, a.leak_n, a.leak_cap, a.err);
  hipLaunchKernelGGL(k_close_scan, dim3(1), dim3(kCS), 0, st, a.cnt, a.m, a.pcl, a.fail, a.off, a.arena_n, a.arena_cap, a.out_cap,
                     a.out_pos ? 1 : 0, a.out_count, a.err);
  if (a.out_pos)
    hipLaunchKernelGGL(k_close_scatter, dim3(256), dim3(256), 0, st, a.arena, a.arena_n, a.arena_cap, a.off, a.out_cap,
                       a.out_pos, a.out_target, a.out_code, a.out_src, a.out_tag, a.out_payload);
  hipLaunchKernelGGL(k_close_unreg, dim3(gm), dim3(256), 0, st, a.cinst, a.m, a.pcl, a.fail, a.inst_res);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace cc
