// map_wide.hip — MapState operations that read or reset a whole map: containsValue :49-60, isEmpty :244-250,
// size :233-239, clear :255-261 and the map's DeleteCommand (ResourceStateMachine.java:34-40 -> MapState.delete
// :264-274) (collections/src/main/java/io/atomix/collections/state/MapState.java).
//
// A map's keys are spread over every table region (apply_map.hip), so these ops cannot run inside the region
// kernel.  They are *barriers*: cc_apply_batch finds them first (k_map_barriers), applies the rows between two
// barriers as an ordinary segment (partition + region apply), then applies the barrier row against the table as
// it stands at that log position:
//   k_mw_count   every entry of the map: live size, bound entries, stored nulls, values equal to the operand;
//   k_mw_order   containsValue only, when the answer depends on java.util.HashMap iteration order (the map
//                stores a null AND a match: the first of them in iteration order decides NPE vs true, A5);
//   k_mw_finish  the row's status/value, the map's peak-size bound; clear/Delete then drop the entries
//                (k_map_drop, apply_map.hip).
//
// Iteration order (oracle/oracle.cpp JavaOrder): bucket = Java hash & (capacity - 1), then insertion order in
// the bucket (= the commit index that created the node, tbl_ins).  The capacity is a function of the map's peak
// size (HashMap.resize doubles it when ++size > 0.75 * capacity and never shrinks it; clear() keeps the table).
// The engine tracks every map's size and capacity exactly (launch_map_size, after each sub-batch's map kernels:
// per-commit size deltas -> per (tile, map) insert/remove counts -> per map the sizes at tile starts; a tile
// whose counts straddle a resize threshold is replayed in log order).  In TTL mode (entries also leave when
// their timers fire) the sub-batch's commits and timer expiries become events in log order and are replayed per
// map instead (map_small.hip k_ttl_replay, common.h TtlEmit).  The peak-size bounds below (lower = sizes seen at
// barriers, upper = bound entries + entries dropped by compaction or clear) remain only for a capacity marked
// inexact (kMpInexact: the exact list overflowed), where a straddling order-dependent answer fails with CC_ERR_STATE.
#include <algorithm>

#include "common.h"
#include "engine_internal.h"
#include "big_jhm.h"
#include "small_jhm.h"

namespace cc {

constexpr int kMwT = 256;

__device__ inline bool map_wide_op(uint32_t op) {
  return op == CC_OP_DELETE || op == CC_OP_MAP_CONTAINSVALUE || op == CC_OP_MAP_ISEMPTY || op == CC_OP_MAP_SIZE ||
         op == CC_OP_MAP_CLEAR;
}

__device__ inline bool set_wide_op(uint32_t op) {
  return op == CC_OP_DELETE || op == CC_OP_SET_SIZE || op == CC_OP_SET_ISEMPTY || op == CC_OP_SET_CLEAR;
}
__device__ inline bool mmap_wide_op(uint32_t op) {  // MultiMapState.removeValue / isEmpty / clear / delete
  return op == CC_OP_DELETE || op == CC_OP_MMAP_REMOVEVALUE || op == CC_OP_MMAP_ISEMPTY || op == CC_OP_MMAP_CLEAR;
}
__device__ inline bool ttl_op(uint32_t op) {
  return op == CC_OP_MAP_PUT || op == CC_OP_MAP_PUTIFABSENT || op == CC_OP_MAP_REPLACE || op == CC_OP_MAP_REPLACEIFPRESENT ||
         op == CC_OP_SET_ADD;
}

// The row lists k_map_barriers fills: barrier rows, then (null: not listed) in-stream size / isEmpty, containsValue
// candidates and clears.
enum { kLsBar = 0, kLsSz, kLsCv, kLsClr, kLists };
// One candidate row (its op is whole-map / set / multimap / schedule, or may arm a TTL timer): resolve its resource.
// push(list, row) appends the row to a list.
template <class Push>
__device__ inline void map_barrier_row(uint64_t i, uint32_t o, const uint32_t* __restrict__ inst,
                                       const uint64_t* __restrict__ aux, const uint32_t* __restrict__ inst_res,
                                       const uint8_t* __restrict__ res_type, uint32_t max_inst,
                                       uint32_t* __restrict__ ttl_seen, bool szq, uint8_t* __restrict__ mflag, bool cvq,
                                       uint32_t* __restrict__ mfirst, bool clrq, Push push) {
  bool wide = map_wide_op(o) || set_wide_op(o) || mmap_wide_op(o) || o == CC_OP_GROUP_SCHEDULE;
  const bool ttl = aux && ttl_op(o);
  if (!wide && !ttl) return;
  if (ttl && (int64_t)aux[i] <= 0) {
    if (!wide) return;
  }
  const uint32_t in = inst[i];
  if (in >= max_inst) return;
  const uint32_t r = inst_res[in];
  if (r == kNoRes) return;
  const uint32_t ty = res_type[r];
  if (ty == CC_RES_MAP) wide = map_wide_op(o);
  else if (ty == CC_RES_SET) wide = set_wide_op(o);
  else if (ty == CC_RES_MULTIMAP) wide = mmap_wide_op(o);  // (its Put arms no map TTL timer: A18)
  else if (ty == CC_RES_GROUP) wide = o == CC_OP_GROUP_SCHEDULE;  // MembershipGroupState.schedule: a timer
  else return;
  if ((ty == CC_RES_GROUP || ty == CC_RES_MULTIMAP) && !wide) return;
  if (szq && ty == CC_RES_MAP && (o == CC_OP_MAP_SIZE || o == CC_OP_MAP_ISEMPTY)) {
    // MapState.size / isEmpty (:233-250): an ordinary row, answered from the exact size tracking (k_size_answer; in
    // TTL mode from the event replay, k_ttl_replay); its map's insertions and removals of the batch are followed
    // (mflag bit 1)
    push(kLsSz, (uint32_t)i);
    if (!(mflag[r] & kMfSize)) mflag_or(mflag, r, kMfSize);
    return;
  }
  if (cvq && ty == CC_RES_MAP && o == CC_OP_MAP_CONTAINSVALUE) {
    // MapState.containsValue (:49-60) outside TTL mode: a candidate for an answer in the stream (map_cv.hip
    // k_cv_classify decides: a map that may hold a null at the row keeps it a barrier)
    push(kLsCv, (uint32_t)i);
    if (!(mflag[r] & kMfCv)) mflag_or(mflag, r, kMfCv);
    return;
  }
  if (clrq && ty == CC_RES_MAP && o == CC_OP_MAP_CLEAR) {
    // MapState.clear (:255-274) outside TTL mode: applied in the stream as an epoch (map_clear.hip)
    push(kLsClr, (uint32_t)i);  // (k_clr_sub flags the map in the sub-batches that clear it)
    return;
  }
  if (mfirst && ty == CC_RES_MAP && o == CC_OP_DELETE) atomicMin(&mfirst[r], (uint32_t)i);  // (k_cv_classify)
  if (!wide) {
    // not a barrier here: a row that arms a TTL timer on this map / set?
    if (!aux || !(ty == CC_RES_MAP ? ttl_op(o) && o != CC_OP_SET_ADD : o == CC_OP_SET_ADD) || (int64_t)aux[i] <= 0) return;
    *ttl_seen = 1u;
    return;
  }
  push(kLsBar, (uint32_t)i);
}

// Rows whose instance is open on a live map and whose op reads or resets the whole map; and whether any map row
// arms a TTL timer (the engine then switches to TTL mode for good).  A persistent grid-stride scan of the op column:
// each wave reads 4 KB per step (four fully coalesced 16-byte loads per lane, 64 rows per thread), every op byte is
// looked up in a 256-entry LDS table of candidate ops, and only a wave holding a candidate row (rare) leaves the fast
// path to resolve it.  (One 16-row thread per 16-byte load, each row tested by a chain of compares behind a divergent
// branch, was 976,564 waves and 1.38 G scalar instructions per 1e9 rows: 2.30 ms.)
constexpr int kMwLd = 4;                      // 16-byte loads per thread and step
constexpr int kMwRows = 16 * kMwLd;           // rows per thread and step
constexpr uint32_t kMwWaveBytes = kWave * kMwRows;  // op bytes per wave and step
// The lists are staged per workgroup in LDS and reserved with one global atomic per list and workgroup (an atomic
// per listed row on one counter was ~11 ms per 1B-row batch with 0.1 % in-stream containsValue rows).
constexpr uint32_t kMwStage = 256;  // staged rows per list and workgroup (more: appended one by one)
__global__ __launch_bounds__(kMwT) void k_map_barriers(const uint32_t* __restrict__ inst, const uint8_t* __restrict__ op,
                                                      const uint64_t* __restrict__ aux, uint64_t n,
                                                      const uint32_t* __restrict__ inst_res,
                                                      const uint8_t* __restrict__ res_type, uint32_t max_inst,
                                                      uint32_t* __restrict__ bar, uint32_t* __restrict__ bar_n, uint32_t cap,
                                                      uint32_t* __restrict__ ttl_seen, uint32_t* __restrict__ szq,
                                                      uint32_t* __restrict__ szq_n, uint32_t szq_cap,
                                                      uint8_t* __restrict__ mflag, uint32_t* __restrict__ cvq,
                                                      uint32_t* __restrict__ cvq_n, uint32_t cvq_cap,
                                                      uint32_t* __restrict__ mfirst, uint32_t* __restrict__ clrq,
                                                      uint32_t* __restrict__ clrq_n, uint32_t clrq_cap) {
  static_assert(kMwT == 256, "one candidate-table entry per thread");
  __shared__ uint32_t lrow[kLists][kMwStage];
  __shared__ uint32_t lcnt[kLists], lbase[kLists];
  __shared__ uint8_t lut[256];  // 1: the op may make its row a listed row (resolved by map_barrier_row)
  uint32_t* const gl[kLists] = {bar, szq, cvq, clrq};
  uint32_t* const gn[kLists] = {bar_n, szq_n, cvq_n, clrq_n};
  const uint32_t gcap[kLists] = {cap, szq_cap, cvq_cap, clrq_cap};
  const uint32_t t = threadIdx.x, l = t & 63;
  {
    const uint32_t o = t;
    lut[t] = (map_wide_op(o) || set_wide_op(o) || mmap_wide_op(o) || o == CC_OP_GROUP_SCHEDULE || (aux && ttl_op(o))) ? 1 : 0;
  }
  if (t < kLists) lcnt[t] = 0;
  __syncthreads();
  auto push = [&](int ls, uint32_t row) {
    const uint32_t k = atomicAdd(&lcnt[ls], 1u);
    if (k < kMwStage) {
      lrow[ls][k] = row;
    } else {  // (the workgroup's stage is full: this row goes straight to the list)
      const uint32_t g = atomicAdd(gn[ls], 1u);
      if (g < gcap[ls]) gl[ls][g] = row;
    }
  };
  const bool al = (reinterpret_cast<uintptr_t>(op) & 15) == 0;
  const uint64_t waves = (uint64_t)gridDim.x * (kMwT / kWave);
  // wave step s covers op bytes [s * kMwWaveBytes, +kMwWaveBytes); lane l's load k reads bytes k * 1024 + 16 l .. +15
  for (uint64_t s = (uint64_t)blockIdx.x * (kMwT / kWave) + (t >> 6); s * kMwWaveBytes < n; s += waves) {
    const uint64_t b0 = s * kMwWaveBytes;
    uint4 v[kMwLd];
    if (al && b0 + kMwWaveBytes <= n) {
#pragma unroll
      for (int k = 0; k < kMwLd; ++k) v[k] = *reinterpret_cast<const uint4*>(op + b0 + k * (16 * kWave) + 16 * l);
    } else {  // the last, partial step: bytes past the end read as op 0 (no candidate)
#pragma unroll
      for (int k = 0; k < kMwLd; ++k) {
        uint32_t w4[4] = {0, 0, 0, 0};
        for (int q = 0; q < 16; ++q) {
          const uint64_t i = b0 + k * (16 * kWave) + 16 * l + q;
          if (i < n) w4[q / 4] |= (uint32_t)op[i] << (8 * (q % 4));
        }
        v[k] = make_uint4(w4[0], w4[1], w4[2], w4[3]);
      }
    }
    uint32_t any = 0;  // a candidate op among the thread's 64 rows
#pragma unroll
    for (int k = 0; k < kMwLd; ++k) {
      const uint32_t w4[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
      for (int q = 0; q < 16; ++q) any |= lut[(w4[q / 4] >> (8 * (q % 4))) & 0xFFu];
    }
    if (__ballot(any != 0) == 0) continue;  // (wave-uniform: the common case)
    if (any) {  // (rare per thread) its candidate rows: a bit mask, then each row's op byte again from the cache
      uint64_t cm = 0;
#pragma unroll
      for (int k = 0; k < kMwLd; ++k) {
        const uint32_t w4[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
        for (int q = 0; q < 16; ++q) cm |= (uint64_t)lut[(w4[q / 4] >> (8 * (q % 4))) & 0xFFu] << (16 * k + q);
      }
      while (cm) {
        const uint32_t bit = (uint32_t)__ffsll((long long)cm) - 1;
        cm &= cm - 1;
        const uint64_t i = b0 + (bit >> 4) * (16 * kWave) + 16 * l + (bit & 15u);
        if (i >= n) continue;
        const uint32_t o = op[i];
        map_barrier_row(i, o, inst, aux, inst_res, res_type, max_inst, ttl_seen, szq != nullptr, mflag, cvq != nullptr,
                        mfirst, clrq != nullptr, push);
      }
    }
  }
  __syncthreads();
  if (t < kLists) {
    const uint32_t c = lcnt[t] < kMwStage ? lcnt[t] : kMwStage;
    lbase[t] = c ? atomicAdd(gn[t], c) : 0u;
  }
  __syncthreads();
#pragma unroll
  for (int ls = 0; ls < kLists; ++ls) {
    const uint32_t c = lcnt[ls] < kMwStage ? lcnt[ls] : kMwStage;
    for (uint32_t q = t; q < c; q += kMwT)
      if (lbase[ls] + q < gcap[ls]) gl[ls][lbase[ls] + q] = lrow[ls][q];
  }
}

// The barrier rows' columns in one launch (the host then reads them with one copy per batch).
__global__ void k_bar_fields(const uint32_t* __restrict__ rows, uint32_t nb, const uint32_t* __restrict__ inst,
                             const uint8_t* __restrict__ op, const uint8_t* __restrict__ flags,
                             const uint64_t* __restrict__ a, const uint64_t* __restrict__ key,
                             const uint64_t* __restrict__ aux, const uint64_t* __restrict__ index,
                             const uint64_t* __restrict__ time, BarRow* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nb) return;
  const uint32_t r = rows[i];
  BarRow b{};
  b.inst = inst[r];
  b.op = op[r];
  b.flags = flags[r];
  b.a = a[r];
  b.key = key ? key[r] : 0;
  b.aux = aux ? aux[r] : 0;
  b.idx = index ? index[r] : 0;
  b.t_row = time ? time[r] : 0;
  b.t_prev = time && r > 0 ? time[r - 1] : 0;
  out[i] = b;
}

int launch_bar_fields(const uint32_t* rows, uint32_t nb, const uint32_t* inst, const uint8_t* op, const uint8_t* flags,
                      const uint64_t* a, const uint64_t* key, const uint64_t* aux, const uint64_t* index,
                      const uint64_t* time, BarRow* out, hipStream_t st) {
  if (nb == 0) return 0;
  hipLaunchKernelGGL(k_bar_fields, dim3((nb + 255) / 256), dim3(256), 0, st, rows, nb, inst, op, flags, a, key, aux, index,
                     time, out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// The clock at row r is max(clock_before, time[r]) (non-decreasing: k_time_check / k_part_ext fail a batch whose
// time column goes backwards), so the first row reaching a deadline is a binary search.
__global__ void k_fire_bounds(const uint64_t* __restrict__ time, uint64_t n, uint64_t clock_before,
                              const uint64_t* __restrict__ deadline, const uint64_t* __restrict__ from, uint32_t m,
                              bool deferred, uint64_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const uint64_t d = deadline[i];
  uint64_t lo = from[i], hi = n;  // search [lo, hi)
  while (lo < hi) {
    const uint64_t mid = lo + (hi - lo) / 2;
    const uint64_t t = time ? (time[mid] > clock_before ? time[mid] : clock_before) : clock_before;
    if (t >= d) hi = mid;
    else lo = mid + 1;
  }
  out[i] = lo < n ? (deferred ? lo + 1 : lo) : ~0ull;
}

int launch_fire_bounds(const uint64_t* time, uint64_t n, uint64_t clock_before, const uint64_t* deadline,
                       const uint64_t* from, uint32_t m, bool deferred, uint64_t* out, hipStream_t st) {
  if (m == 0) return 0;
  hipLaunchKernelGGL(k_fire_bounds, dim3((m + 255) / 256), dim3(256), 0, st, time, n, clock_before, deadline, from, m,
                     deferred, out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// An entry is live at the barrier row: present, and no TTL timer of it has fired by then.
__device__ inline bool live_at(uint32_t w, const uint64_t* __restrict__ dl, uint64_t e, uint64_t fire) {
  if (!(w & kMwPresent)) return false;
  if (!dl) return true;
  const uint64_t d = dl[e];
  return d == 0 || d > fire;
}

// HashMap capacity after the map's size peaked at p (16, doubled while p > 0.75 * capacity).
__device__ inline uint64_t java_cap(uint64_t p) {
  uint64_t cap = 16, thr = 12;
  while (p > thr) {
    cap <<= 1;
    thr <<= 1;
  }
  return cap;
}

// ctl layout (u64): 0 present, 1 bound (used, not dead), 2 stored nulls, 3 matches, 4/5 min bucket of a
// null / a match, 6/7 min insertion index of a null / a match inside that bucket, 8 capacity (0 = undetermined)
// 9.. per capacity level L >= 3 (128 << (L - 3)): bound keys of the map whose hash is the deciding bucket's modulo
// that capacity (a tree bin can have formed there only if >= 9 keys ever shared it)
enum { C_PRES = 0, C_USED, C_NULLS, C_MATCH, C_BN, C_BM, C_IN, C_IM, C_CAP, C_TR0, C_N = C_TR0 + 32 };

// the log index at which map `slot`'s table left level L (grew to L + 1; ~0 while it has not): a key whose entry was
// claimed later never shared a bin of that width with the others
__device__ inline uint64_t lvl_left(const unsigned long long* __restrict__ lvl_at, uint32_t slot, uint32_t L) {
  return L + 1 < kLvlSlots ? (uint64_t)lvl_at[(uint64_t)slot * kLvlSlots + L + 1] : ~0ull;
}

__global__ void k_mw_reset(unsigned long long* ctl) {
  const int t = threadIdx.x;
  for (int q = t; q < C_N; q += blockDim.x) ctl[q] = (q >= C_BN && q <= C_IM) ? ~0ull : 0ull;
}

__device__ inline unsigned long long wave_sum(unsigned long long x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
  return x;
}

__global__ __launch_bounds__(kMwT) void k_mw_count(const uint32_t* __restrict__ word, const uint64_t* __restrict__ val,
                                                  const uint64_t* __restrict__ dl, uint64_t fire, uint64_t entries, uint32_t slot, uint32_t op, uint32_t atag,
                                                  uint64_t apay, unsigned long long* __restrict__ ctl) {
  unsigned long long pres = 0, used = 0, nulls = 0, match = 0;
  for (uint64_t e = (uint64_t)blockIdx.x * kMwT + threadIdx.x; e < entries; e += (uint64_t)gridDim.x * kMwT) {
    const uint32_t w = word[e];
    if (!(w & kMwUsed) || (w & kMwDead) || (w & kMwSlotMask) != slot) continue;
    if (!(w & kMwUnseen)) ++used;  // (a hot-key placeholder no commit stored into is no key the map ever held)
    if (!live_at(w, dl, e, fire)) continue;
    ++pres;
    if (op == CC_OP_MAP_CONTAINSVALUE) {
      const uint32_t vt = mw_vtag(w);
      if (vt == CC_TAG_NULL) ++nulls;
      else if (vt == atag && val[e] == apay) ++match;
    }
  }
  pres = wave_sum(pres);
  used = wave_sum(used);
  nulls = wave_sum(nulls);
  match = wave_sum(match);
  if ((threadIdx.x & 63) == 0 && used) {
    atomicAdd(&ctl[C_PRES], pres);
    atomicAdd(&ctl[C_USED], used);
    if (nulls) atomicAdd(&ctl[C_NULLS], nulls);
    if (match) atomicAdd(&ctl[C_MATCH], match);
  }
}

// pass 0: the capacity, then the first bucket holding a null / a match; pass 1: inside the common first bucket,
// the first insertion of each.  Runs only for an order-dependent containsValue (all threads read the same ctl).

__global__ __launch_bounds__(kMwT) void k_mw_order(const uint32_t* __restrict__ word, const uint64_t* __restrict__ key,
                                                  const uint64_t* __restrict__ val, const uint64_t* __restrict__ ins,
                                                  const uint64_t* __restrict__ dl, uint64_t fire, uint64_t entries, uint32_t slot, uint32_t op, uint32_t atag, uint64_t apay,
                                                  const uint32_t* __restrict__ peak_lo, const unsigned long long* __restrict__ dropped,
                                                  const uint32_t* __restrict__ mpcap, bool exact, const SmallMap* __restrict__ small,
                                                  const BigMap* __restrict__ big,
                                                  const uint64_t* __restrict__ hh_key, const int32_t* __restrict__ hh_val,
                                                  uint32_t hh_n, int pass, const uint64_t* __restrict__ claim,
                                                  const unsigned long long* __restrict__ lvl_at,
                                                  unsigned long long* __restrict__ ctl, uint32_t* __restrict__ err) {
  if (op != CC_OP_MAP_CONTAINSVALUE || ctl[C_NULLS] == 0 || ctl[C_MATCH] == 0) return;
  const uint32_t mp = mpcap ? mpcap[slot] : 0u, lv = mp & ~kMpInexact;
  const uint32_t sflags = small ? small[slot].flags : 0u;
  uint64_t cap;
  if (exact && !(mp & kMpInexact)) {
    cap = 16ull << lv;  // the tracked capacity (size-driven resizes, and treeifyBin's below 64: map_small.hip)
  } else {
    // bounds: the level reached while tracking was exact means a peak above the previous level's threshold
    const uint64_t lo = max(max((uint64_t)peak_lo[slot], (uint64_t)ctl[C_PRES]), lv ? (12ull << (lv - 1)) + 1 : 0ull);
    const uint64_t hi = ctl[C_USED] + dropped[slot];
    cap = max(java_cap(lo), 16ull << lv);
    uint64_t cap_hi = java_cap(hi);
    if ((sflags & kSmUnknown) && hi >= 9) cap_hi = max(cap_hi, 64ull);  // an untracked early resize (treeifyBin)
    if (max(cap_hi, 16ull << lv) != cap) {
      if (blockIdx.x == 0 && threadIdx.x == 0 && pass == 0) atomicOr(err, kErrMapOrder);
      return;
    }
  }
  if (pass == 1 && ctl[C_BN] != ctl[C_BM]) return;  // decided by the buckets
  const uint64_t bb = ctl[C_BN];                     // (pass 1: the bucket holding the first null and the first match)
  for (uint64_t e = (uint64_t)blockIdx.x * kMwT + threadIdx.x; e < entries; e += (uint64_t)gridDim.x * kMwT) {
    const uint32_t w = word[e];
    if ((w & kMwDead) || !(w & kMwUsed) || (w & kMwUnseen) || (w & kMwSlotMask) != slot) continue;
    const bool present = live_at(w, dl, e, fire);
    const uint32_t vt = mw_vtag(w);
    const bool isnull = vt == CC_TAG_NULL;
    const bool cand = present && (isnull || (vt == atag && val[e] == apay));
    if (pass == 0 && !cand) continue;
    bool ok;
    const uint32_t jh = java_key_hash((w >> 17) & 3, key[e], hh_key, hh_val, hh_n, ok);
    if (!ok) {
      atomicOr(err, kErrHandleHash);
      continue;
    }
    const uint64_t b = jh & (cap - 1);
    if (pass == 0) {
      atomicMin(&ctl[isnull ? C_BN : C_BM], (unsigned long long)b);
    } else {
      if (cand && b == bb) {
        // the order inside the bin: creation order (tbl_ins) for a list bin; a small map's bin chain from its HashMap
        // model (small_jhm.h), tree bins included; past the window, a map with a tree bin from its big model
        uint64_t ord = ins[e];
        if (sflags & kSmIn) {
          bool dup;
          ord = small_chain_pos(small[slot], jh, (w >> 17) & 3, key[e], dup);
          // (and a model that does not hold the map's live keys -- an engine fault -- refuses rather than guesses)
          if (dup || (16ull << small[slot].lvl) != cap || (!dl && small[slot].n != ctl[C_PRES])) atomicOr(err, kErrMapOrder);
        } else if (sflags & kSmBig) {
          const BigMap& B = big[small[slot].pad];
          bool dup;
          ord = big_chain_pos(B, jh, (w >> 17) & 3, key[e], dup);
          if (dup || (16ull << B.h.lvl) != cap || (!dl && B.h.n != ctl[C_PRES])) atomicOr(err, kErrMapOrder);
        }
        atomicMin(&ctl[isnull ? C_IN : C_IM], (unsigned long long)ord);
      }
      if (sflags & kSmBig) continue;  // (every bin followed: no bounds test)
      // every key the map bound since its last clear (present or not) that shares the deciding bin at a capacity
      // >= 128 and was bound before the table grew past that capacity: a tree bin there needs >= 9 of them at once
      // (HashMap.treeifyBin, TREEIFY_THRESHOLD)
      for (uint32_t L = 3; L <= lv && L - 3 < 32; ++L) {
        const uint64_t mk = (16ull << L) - 1;
        if ((jh & mk) == (bb & mk) && claim[e] <= lvl_left(lvl_at, slot, L)) atomicAdd(&ctl[C_TR0 + (L - 3)], 1ull);
      }
    }
  }
  if (pass == 0 && blockIdx.x == 0 && threadIdx.x == 0) ctl[C_CAP] = cap;
}

// The deciding bin's keys that the map bound since its last clear and that compaction dropped since (the set of
// common.h CsetEnt, with each key's earliest claim): added to the per-level counts of the tree-bin test, except at
// the levels where k_mw_order pass 1 already counted the key's entry bound now (by that entry's own claim).  A key
// bound again after a compaction thus counts once, by its earliest claim.  Runs only for an order-dependent containsValue decided inside one bin of a
// table above 64 (all threads read the same ctl).  A set that overflowed counts as 9 (refuse).
__global__ __launch_bounds__(kMwT) void k_mw_cset(const CsetEnt* __restrict__ set, uint64_t n, const uint32_t* __restrict__ full,
                                                 const uint64_t* __restrict__ cgen, uint32_t slot,
                                                 const uint32_t* __restrict__ word, const uint64_t* __restrict__ tkey,
                                                 const uint64_t* __restrict__ claim, uint32_t map_bits,
                                                 const uint32_t* __restrict__ mpcap,
                                                 const SmallMap* __restrict__ small, const uint64_t* __restrict__ hh_key,
                                                 const int32_t* __restrict__ hh_val, uint32_t hh_n,
                                                 const unsigned long long* __restrict__ lvl_at,
                                                 unsigned long long* __restrict__ ctl, uint32_t* __restrict__ err) {
  if (ctl[C_NULLS] == 0 || ctl[C_MATCH] == 0 || ctl[C_BN] != ctl[C_BM]) return;
  if (small && (small[slot].flags & (kSmIn | kSmBig))) return;  // (a followed table's order is its model's)
  const uint32_t lv = mpcap ? (mpcap[slot] & ~kMpInexact) : 0u;
  if (lv < 3) return;
  if (*full) {
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&ctl[C_TR0], 9ull);
    return;
  }
  const uint64_t bb = ctl[C_BN], gen = cgen[slot];
  const uint32_t want = cset_meta(slot, 0, gen) & ~(3u << 17);
  for (uint64_t e = (uint64_t)blockIdx.x * kMwT + threadIdx.x; e < n; e += (uint64_t)gridDim.x * kMwT) {
    const uint32_t m = set[e].meta;
    if ((m & ~(3u << 17)) != want) continue;  // another map / generation, or an empty entry
    const uint32_t kt = (m >> 17) & 3u;
    const uint64_t k = set[e].key;
    bool ok;
    const uint32_t jh = java_key_hash(kt, k, hh_key, hh_val, hh_n, ok);
    if (!ok) {
      atomicOr(err, kErrHandleHash);
      continue;
    }
    if ((jh & 127u) != (bb & 127u)) continue;  // not in the bin even at 128 (bins only split further above)
    // its entry bound now, as k_mw_order pass 1 counts entries (used, not dead, not unseen): that entry's claim
    const uint64_t te = tbl_find(word, tkey, map_bits, slot, kt, k);
    uint64_t tcl = ~0ull;
    if (te != ~0ull) {
      const uint32_t tw = word[te];
      if (!(tw & kMwDead) && (tw & kMwUsed) && !(tw & kMwUnseen)) tcl = claim[te];
    }
    const uint64_t cl = set[e].claim;
    for (uint32_t L = 3; L <= lv && L - 3 < 32; ++L) {
      const uint64_t mk = (16ull << L) - 1, left = lvl_left(lvl_at, slot, L);
      if ((jh & mk) == (bb & mk) && cl <= left && !(tcl <= left)) atomicAdd(&ctl[C_TR0 + (L - 3)], 1ull);
    }
  }
}

// The barrier row's result (MapState.java :49-60 / :233-239 / :244-250 / :255-261 / :264-274) and the map's
// peak-size bounds.
// Exact tracking (not in TTL mode): the tracked size must be what the table holds; clear / Delete empty the map.
// (Its own launch: folded into k_mw_finish behind an `if (msize)`, hipcc 7.2 at -O3 lost the slot register on the
// msize == null path of the clear / Delete case and k_mw_finish wrote dropped[] through a garbage index.)
__global__ void k_mw_size(uint32_t slot, uint32_t op, const unsigned long long* __restrict__ ctl, uint32_t* __restrict__ msize,
                          uint32_t* __restrict__ err) {
  if (threadIdx.x != 0) return;
  if (msize[slot] != ctl[C_PRES]) atomicOr(err, kErrMapSize);
  if (op == CC_OP_MAP_CLEAR || op == CC_OP_DELETE) msize[slot] = 0;
}

__global__ void k_mw_finish(uint32_t slot, uint32_t op, uint64_t row, const unsigned long long* __restrict__ ctl,
                            uint32_t* __restrict__ peak_lo, unsigned long long* __restrict__ dropped,
                            uint8_t* __restrict__ out_status,
                            uint64_t* __restrict__ out_value, const SmallMap* __restrict__ small,
                            const BigMap* __restrict__ big, uint32_t* __restrict__ err) {
  if (threadIdx.x != 0) return;
  const uint64_t pres = ctl[C_PRES];
  uint32_t st = CC_STATUS(CC_ST_OK, CC_TAG_NULL);
  uint64_t v = 0;
  switch (op) {
    case CC_OP_MAP_SIZE:  // int
      st = CC_STATUS(CC_ST_OK, CC_TAG_INT);
      v = (uint64_t)(int64_t)(int32_t)(uint32_t)pres;
      break;
    case CC_OP_MAP_ISEMPTY:
      st = CC_STATUS(CC_ST_OK, CC_TAG_BOOL);
      v = pres == 0;
      break;
    case CC_OP_MAP_CONTAINSVALUE: {
      const uint64_t nulls = ctl[C_NULLS], match = ctl[C_MATCH];
      bool npe;
      if (nulls == 0 || match == 0) {
        npe = nulls != 0;
      } else {  // the first of (null, match) in HashMap iteration order
        const uint64_t bn = ctl[C_BN], bm = ctl[C_BM];
        npe = bn != bm ? bn < bm : ctl[C_IN] < ctl[C_IM];
        if (bn == bm) {  // decided inside one bin: by the bin's chain order
          bool tree = false, followed = false;
          if (small) {
            const SmallMap& sm = small[slot];
            if (sm.flags & kSmIn) {
              tree = (sm.flags & kSmAmbig) != 0;  // the chain read from the map's HashMap model (k_mw_order)
            } else if (sm.flags & kSmBig) {  // the chain read from the map's big model (k_mw_order)
              tree = (big[sm.pad].h.flags & kSmAmbig) != 0;
              followed = true;
            } else {  // a bin that was a tree bin while the table was small (mod 64)
              tree = ((sm.flags & kSmTree) && ((sm.tree_bins >> (bn & 63u)) & 1ull)) || (sm.flags & kSmUnknown);
            }
          }
          // above capacity 64: creation order unless the bin could have been a tree bin, which needs 9 keys in it at
          // once since the last clear (that wipes every bin); the bin's distinct keys since then are at most its
          // bound keys plus the keys compacted away (k_mw_order pass 1, k_mw_cset)
          for (int q = 0; q < 32 && !followed; ++q) tree |= ctl[C_TR0 + q] >= 9;
          if (tree) atomicOr(err, kErrMapOrder);
        }
      }
      if (npe) {
        st = CC_STATUS(CC_ST_NULL_POINTER, CC_TAG_NULL);
      } else {
        st = CC_STATUS(CC_ST_OK, CC_TAG_BOOL);
        v = match != 0;
      }
      break;
    }
    default:  // clear / Delete: every entry is dropped; the keys they held count toward the peak bound; no bin is left
      dropped[slot] += ctl[C_USED];  // (k_map_drop moves the map's generation on: its compacted keys stop counting)
      break;
  }
  if (pres > peak_lo[slot]) peak_lo[slot] = (uint32_t)min(pres, (uint64_t)0xFFFFFFFFu);
  out_status[row] = (uint8_t)st;
  out_value[row] = v;
}

// Results of the set / multimap ops that ran as map ops.
// SetState (SetState.java:49-87): add returns false whatever happened; remove returns whether the element was
// present (the map remove it ran as returned the stored Boolean TRUE, or null).
// MultiMapState (MultiMapState.java:48-183): put returns true (its value is never stored, so never "contained")
// and its commit is never cleaned (-> the leak log); get and remove(key) return an empty collection;
// remove(key, value) false; size(key) 0.
__global__ __launch_bounds__(kMwT) void k_keyed_results(const uint32_t* __restrict__ inst, const uint8_t* __restrict__ op,
                                                       const uint8_t* __restrict__ flags, const uint64_t* __restrict__ index,
                                                       uint64_t n, const uint32_t* __restrict__ inst_res,
                                                       const uint8_t* __restrict__ res_type, uint32_t max_inst,
                                                       uint8_t* __restrict__ status, uint64_t* __restrict__ value,
                                                       LeakRec* __restrict__ leak, unsigned long long* __restrict__ leak_n,
                                                       uint64_t leak_cap, uint32_t* __restrict__ err) {
  const uint64_t i = (uint64_t)blockIdx.x * kMwT + threadIdx.x;
  if (i >= n) return;
  const uint32_t o = op[i];
  const bool set_op = o == CC_OP_SET_ADD || o == CC_OP_SET_REMOVE;
  const bool mm_op = o == CC_OP_MMAP_PUT || o == CC_OP_MMAP_GET || o == CC_OP_MMAP_REMOVE || o == CC_OP_MMAP_SIZE;
  if (!set_op && !mm_op) return;
  const uint32_t in = inst[i];
  if (in >= max_inst) return;
  const uint32_t r = inst_res[in];
  if (r == kNoRes || res_type[r] != (set_op ? CC_RES_SET : CC_RES_MULTIMAP)) return;
  const uint8_t s = status[i];
  if (CC_STATUS_CODE(s) != CC_ST_OK) return;
  uint32_t tag = CC_TAG_BOOL;
  uint64_t v = 0;
  if (set_op) {
    v = o == CC_OP_SET_ADD ? 0ull : (CC_STATUS_TAG(s) != CC_TAG_NULL ? 1ull : 0ull);
  } else if (o == CC_OP_MMAP_PUT) {
    v = 1;
    const unsigned long long a = atomicAdd(leak_n, 1ull);
    if (a < leak_cap) {
      leak[a].idx = index ? index[i] : 0;
      leak[a].slot = r;
      leak[a].pad = 0;
    } else {
      atomicOr(err, kErrCapacity);
    }
  } else if (o == CC_OP_MMAP_SIZE) {
    tag = CC_TAG_INT;
  } else if (o == CC_OP_MMAP_GET || CC_FLAG_TAG_A(flags[i]) == CC_TAG_NULL) {
    tag = CC_TAG_LIST;  // an empty collection
  }
  value[i] = v;
  status[i] = CC_STATUS(CC_ST_OK, tag);
}

int launch_keyed_results(const KeyedResultArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(k_keyed_results, dim3((uint32_t)((a.n + kMwT - 1) / kMwT)), dim3(kMwT), 0, st, a.inst, a.op, a.flags,
                     a.index, a.n, a.inst_res, a.res_type, a.max_inst, a.status, a.value, a.leak, a.leak_n, a.leak_cap,
                     a.err);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_map_barriers(const uint32_t* inst, const uint8_t* op, const uint64_t* aux, uint64_t n, const uint32_t* inst_res,
                        const uint8_t* res_type, uint32_t max_inst, uint32_t* bar, uint32_t* bar_n, uint32_t cap,
                        uint32_t* ttl_seen, uint32_t* szq, uint32_t* szq_n, uint32_t szq_cap, uint8_t* mflag,
                        uint32_t* cvq, uint32_t* cvq_n, uint32_t cvq_cap, uint32_t* mfirst, uint32_t R,
                        uint32_t* clrq, uint32_t* clrq_n, uint32_t clrq_cap, hipStream_t st) {
  if (hipMemsetAsync(bar_n, 0, sizeof(uint32_t), st) != hipSuccess) return -1;
  if (szq_n && hipMemsetAsync(szq_n, 0, sizeof(uint32_t), st) != hipSuccess) return -1;
  if (cvq_n && hipMemsetAsync(cvq_n, 0, sizeof(uint32_t), st) != hipSuccess) return -1;
  if (clrq_n && hipMemsetAsync(clrq_n, 0, sizeof(uint32_t), st) != hipSuccess) return -1;
  if (mfirst && hipMemsetAsync(mfirst, 0xFF, sizeof(uint32_t) * R, st) != hipSuccess) return -1;
  // persistent: 8 workgroups per CU at most (each wave then takes ~30 4-KB steps of a 1e9-row batch)
  const uint64_t steps = (n + kMwWaveBytes - 1) / kMwWaveBytes, wpg = kMwT / kWave;
  const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(8 * kPersistGrid, (steps + wpg - 1) / wpg));
  hipLaunchKernelGGL(k_map_barriers, dim3(grid), dim3(kMwT), 0, st, inst, op, aux, n, inst_res,
                     res_type, max_inst, bar, bar_n, cap, ttl_seen, szq, szq_n, szq_cap, mflag, cvq, cvq_n, cvq_cap, mfirst,
                     clrq, clrq_n, clrq_cap);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_map_wide(const MapWideArgs& a, hipStream_t st) {
  const uint32_t grid = (uint32_t)std::min<uint64_t>(2048, (a.entries + kMwT - 1) / kMwT);
  const uint32_t atag = a.atag, op = a.op;
  const uint64_t apay = atag == CC_TAG_NULL ? 0 : a.apay;  // canonical NULL payload
  hipLaunchKernelGGL(k_mw_reset, dim3(1), dim3(64), 0, st, a.ctl);  // (C_N <= 64 entries)
  hipLaunchKernelGGL(k_mw_count, dim3(grid), dim3(kMwT), 0, st, a.tbl_word, a.tbl_val, a.tbl_dl, a.fire_clock, a.entries, a.slot, op,
                     atag, apay, a.ctl);
  if (op == CC_OP_MAP_CONTAINSVALUE) {
    for (int pass = 0; pass < 2; ++pass)
      hipLaunchKernelGGL(k_mw_order, dim3(grid), dim3(kMwT), 0, st, a.tbl_word, a.tbl_key, a.tbl_val, a.tbl_ins, a.tbl_dl,
                         a.fire_clock, a.entries, a.slot, op, atag, apay, a.peak_lo,
                         (const unsigned long long*)a.dropped, a.mpcap, a.msize != nullptr, a.small, a.big, a.hh_key, a.hh_val,
                         a.hh_n, pass, a.tbl_claim, a.lvl_at, a.ctl, a.err);
    if (a.cset) {
      const uint32_t cg = (uint32_t)std::min<uint64_t>(2048, (a.cset_n + kMwT - 1) / kMwT);
      hipLaunchKernelGGL(k_mw_cset, dim3(cg), dim3(kMwT), 0, st, a.cset, a.cset_n, a.cset_full, a.cgen, a.slot, a.tbl_word,
                         a.tbl_key, a.tbl_claim, a.map_bits, a.mpcap, a.small, a.hh_key, a.hh_val, a.hh_n, a.lvl_at, a.ctl, a.err);
    }
  }
  if (a.msize) hipLaunchKernelGGL(k_mw_size, dim3(1), dim3(64), 0, st, a.slot, op, a.ctl, a.msize, a.err);
  hipLaunchKernelGGL(k_mw_finish, dim3(1), dim3(64), 0, st, a.slot, op, a.row, a.ctl, a.peak_lo,
                     (unsigned long long*)a.dropped, a.out_status, a.out_value, a.small, a.big, a.err);
  if (hipGetLastError() != hipSuccess) return -1;
  if (op == CC_OP_MAP_CLEAR || op == CC_OP_DELETE)
    return launch_map_drop_resource(a.tbl_word, a.entries, a.slot, a.cgen, st);
  return 0;
}

// ---- exact map sizes and capacities (MapState's java.util.HashMap: size, and the table capacity its peak size
//      set, HashMap.putVal / resize) ----
// k_apply_map writes one word per region record (msz_word: the map slot and whether the commit inserted or removed a
// key); k_hot_apply writes 2-bit codes per position of each hot key's list, 16 per word (one coalesced word per
// thread and piece: a word per commit at the hot commits' staging positions cost ~7 ms per c3 step in partial-line
// writes).  Then, per sub-batch:
// 1. k_msize_count, one workgroup per partition tile: the region records' words (one coalesced span) and each hot
//    key's codes for its run in the tile (popcounts) counted per map in LDS (direct-indexed, 16384 maps per pass);
//    the tile's row of tcnt written whole (coalesced, zeros included).
// 2. k_msize_scan, one workgroup per 64 maps (lane = map, wave = a chunk of tiles): the size at every tile start (a
//    prefix sum of inserts - removes in log order), per tile the capacity level bounds [level(max(size before, size
//    after)), level(size before + inserts)], L = the highest lower bound (and the level so far).  Only a tile whose
//    upper bound exceeds L can raise the capacity beyond L: it goes to the exact list.  Order-free: no serial walk.
// 3. k_msize_exact, one workgroup per listed (tile, map): the tile's rows in log order (cpos), the map's size
//    changes among them, the running maximum -> the tile's true peak -> atomicMax on the level.
// Traffic per sub-batch: 4 B written + 4 B read per map record, 4 B x maps per tile (the counter rows, written and
// read once); the exact pass reads a tile's cpos (32 KB) plus its gathers per listed pair.
constexpr int kMszT = 1024;
constexpr uint32_t kMszPass = 16384;  // maps counted per LDS pass (64 KB)

// hot-key list helpers: word of list position lp of key h (pfx: the keys' piece prefix, as k_hot_apply's)
constexpr uint32_t kHotWords = kHotPiece / 16;  // code words per hot piece
__device__ inline uint32_t hot_code(const uint32_t* __restrict__ hot_msz, const uint32_t* pfx, uint32_t h, uint32_t lp) {
  return (hot_msz[(uint64_t)pfx[h] * kHotWords + lp / 16] >> (2 * (lp % 16))) & 3u;
}
__device__ inline void hot_pfx(const uint32_t* __restrict__ hot_n, const uint32_t* __restrict__ hot_len, uint32_t* pfx,
                               uint32_t& nh) {
  nh = hot_n ? *hot_n : 0u;
  hot_piece_prefix(hot_len, nh, pfx);
  lds_barrier();
}

// A map commit's insertion / removal as an event (map_small.hip): its position (the log index's offset in the
// sub-batch, or in TTL mode 2 * row offset + 1: common.h TtlEmit) and the key's HashMap hash.
// (at: its slot in the event buffer)
__device__ inline void map_event(uint32_t at, uint32_t m, uint32_t code, uint64_t d, const MRec& xr,
                                 const uint64_t* __restrict__ hh_key, const int32_t* __restrict__ hh_val, uint32_t hh_n,
                                 uint64_t* __restrict__ ev_key, uint32_t* __restrict__ ev_val, EvPay* __restrict__ ev_pay,
                                 uint32_t ev_cap, uint32_t* __restrict__ err) {
  bool ok;
  const uint32_t kt = CC_FLAG_KTAG(smeta_flags(xr.meta));
  const uint32_t jh = java_key_hash(kt, xr.key, hh_key, hh_val, hh_n, ok);
  if (!ok) atomicOr(err, kErrHandleHash);  // an unregistered String key
  if (d >> kEvPosBits) atomicOr(err, kErrSpan);  // a sub-batch spanning 2^32 indices (the host cuts them: never)
  if (at < ev_cap) {
    ev_key[at] = ((uint64_t)m << kEvMapShift) | ((d & kEvPosMask) << 4) | code;
    ev_val[at] = at;
    ev_pay[at] = EvPay{xr.key, jh, kt};
  }
}

__global__ __launch_bounds__(kMszT) void k_msize_count(const uint16_t* __restrict__ ttab, uint32_t sb, uint32_t k0,
                                                      uint32_t sb_hot, const uint32_t* __restrict__ msz,
                                                      const HotKey* __restrict__ hot, const uint32_t* __restrict__ hot_n,
                                                      const uint32_t* __restrict__ hot_len, const uint32_t* __restrict__ hot_rpre,
                                                      const uint32_t* __restrict__ hot_msz, uint32_t R,
                                                      uint32_t* __restrict__ tcnt, uint32_t* __restrict__ list_n,
                                                      const uint8_t* __restrict__ msmall, const MRec* __restrict__ xrec,
                                                      const uint64_t* __restrict__ idx0p, const uint64_t* __restrict__ hh_key,
                                                      const int32_t* __restrict__ hh_val, uint32_t hh_n,
                                                      uint64_t* __restrict__ ev_key, uint32_t* __restrict__ ev_val,
                                                      EvPay* __restrict__ ev_pay, uint32_t ev_cap, uint32_t* __restrict__ sm_ctl,
                                                      const uint32_t* __restrict__ map_row, uint64_t lo,
                                                      uint32_t* __restrict__ err) {
  __shared__ uint32_t cnt[kMszPass];
  if (blockIdx.x == 0 && threadIdx.x == 0) *list_n = 0;  // (k_msize_scan, the next launch, appends to the list)
  __shared__ uint32_t pfx[kHotMax + 1];
  // each hot key's run in this tile (list positions [hl0, hl1)) and the prefix of its 2-bit code words (wpfx): the
  // words are then shared out over all threads (one thread per key walked the heaviest key's ~70 words per tile as
  // a chain of dependent global loads)
  __shared__ uint32_t hl0[kHotMax], hl1[kHotMax], hsl[kHotMax], wpfx[kHotMax + 1];
  const uint32_t t = blockIdx.x;
  uint32_t nh;
  hot_pfx(hot_n, hot_len, pfx, nh);
  if (threadIdx.x < kWave) {
    constexpr int PL = (kHotMax + kWave - 1) / kWave;
    const uint32_t l = threadIdx.x;
    uint32_t c[PL], sum = 0;
#pragma unroll
    for (int q = 0; q < PL; ++q) {
      const uint32_t h = l * PL + q;
      c[q] = 0;
      if (h < nh) {
        const uint32_t* rp = hot_rpre + (uint64_t)h * (kMaxTiles + 1);
        const uint32_t a = rp[t], b = rp[t + 1];
        hl0[h] = a;
        hl1[h] = b;
        hsl[h] = hot[h].ident & kMwSlotMask;
        c[q] = a < b ? (b - 1) / 16 - a / 16 + 1 : 0u;
      }
      sum += c[q];
    }
    uint32_t inc = sum;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
      const uint32_t y = __shfl_up(inc, d, kWave);
      if (l >= (uint32_t)d) inc += y;
    }
    uint32_t run = inc - sum;
#pragma unroll
    for (int q = 0; q < PL; ++q) {
      const uint32_t h = l * PL + q;
      if (h < nh) wpfx[h] = run;
      run += c[q];
    }
    if (l == kWave - 1) wpfx[kHotMax] = inc;  // all words of the tile
  }
  lds_barrier();
  const uint32_t nwords = wpfx[kHotMax];
  const uint16_t* row = ttab + (uint64_t)t * (sb + 1);
  const uint32_t b0 = row[k0], b1 = row[sb_hot];
  const uint32_t* w = msz + (uint64_t)t * kTile;
  uint32_t* out = tcnt + (uint64_t)t * R;
  if (map_row || msmall) {
    // the tile's map events: counted per thread, one event-buffer reservation for the workgroup, then written (one
    // global atomic per tile: a wave_append per wave and step was ~250K atomics on one counter per c3 sub-batch)
    auto evm = [&](uint32_t x) {
      return (x & 3u) && (map_row || (msmall[x >> 2] & (kMfSmall | kMfSize | kMfClr)));
    };
    // (each position's decision is taken once and kept in a bit mask, so the writes match the reservation by
    // construction; the flags are the engine stream's snapshot and do not change during the launch, common.h)
    static_assert(kTile / kMszT <= 32, "one mask bit per position of a thread");
    uint32_t my = 0, emask = 0;
    for (uint32_t p = b0 + threadIdx.x, j = 0; p < b1; p += kMszT, ++j)
      if (evm(w[p])) {
        ++my;
        emask |= 1u << j;
      }
    __shared__ uint32_t wsum[kMszT / kWave], ebase;
    const uint32_t l = __lane_id(), wv = threadIdx.x / kWave;
    uint32_t inc = my;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
      const uint32_t y = __shfl_up(inc, d, kWave);
      if (l >= (uint32_t)d) inc += y;
    }
    if (l == kWave - 1) wsum[wv] = inc;
    lds_barrier();
    if (threadIdx.x == 0) {
      uint32_t tot = 0;
      for (uint32_t q = 0; q < kMszT / kWave; ++q) {
        const uint32_t c = wsum[q];
        wsum[q] = tot;
        tot += c;
      }
      ebase = tot ? atomicAdd(sm_ctl, tot) : 0u;
    }
    lds_barrier();
    uint32_t at = ebase + wsum[wv] + inc - my;
    for (uint32_t p = b0 + threadIdx.x, j = 0; p < b1; p += kMszT, ++j) {
      if (!((emask >> j) & 1u)) continue;
      const uint32_t x = w[p];
      const uint64_t g = (uint64_t)t * kTile + p;
      // TTL mode: every map's commits, positioned by row (expiries join them: map_small.hip); else small,
      // size-queried or cleared maps' commits by log index
      const uint64_t d = map_row ? 2 * ((uint64_t)map_row[g] - lo) + 1 : xrec[g].idx - *idx0p;
      map_event(at++, x >> 2, x & 3u, d, xrec[g], hh_key, hh_val, hh_n, ev_key, ev_val, ev_pay, ev_cap, err);
    }
  }
  for (uint32_t base = 0; base < R; base += kMszPass) {
    const uint32_t span = min(kMszPass, R - base);
    for (uint32_t q = threadIdx.x; q < span; q += kMszT) cnt[q] = 0;
    lds_barrier();
    for (uint32_t p = b0 + threadIdx.x; p < b1; p += kMszT) {
      const uint32_t x = w[p], code = x & 3u, m = (x >> 2) - base;
      // (a map cleared in the stream: its sizes come from event replay, map_clear.hip k_clr_replay)
      if (code && m < span && !(msmall && (msmall[x >> 2] & kMfClr)))
        atomicAdd(&cnt[m], code == 1u ? 1u : 0x10000u);  // <= 16384 each: halves never carry
    }
    for (uint32_t i = threadIdx.x; i < nwords; i += kMszT) {  // one code word (16 list positions) per thread
      uint32_t h = 0, hb = nh;  // the last key whose words start at or before i (keys without words are skipped)
      while (hb - h > 1) {
        const uint32_t c = (h + hb) >> 1;
        if (wpfx[c] <= i) h = c; else hb = c;
      }
      const uint32_t m = hsl[h] - base;
      if (m >= span) continue;
      if (msmall && (msmall[hsl[h]] & kMfClr)) continue;  // (a cleared map: k_hot_apply emits its size events)
      const uint32_t lp0 = hl0[h], lp1 = hl1[h], wd = lp0 / 16 + (i - wpfx[h]);
      uint32_t x = hot_msz[(uint64_t)pfx[h] * kHotWords + wd];
      const uint32_t a = wd * 16 < lp0 ? lp0 - wd * 16 : 0u, b = lp1 - wd * 16 < 16u ? lp1 - wd * 16 : 16u;
      x &= (b == 16u ? ~0u : (1u << (2 * b)) - 1u) & ~((1u << (2 * a)) - 1u);  // positions [a, b) of the word
      const uint32_t lo = x & 0x55555555u, hi = (x >> 1) & 0x55555555u;
      const uint32_t ins = __popc(lo & ~hi), rem = __popc(hi & ~lo);
      if (ins | rem) atomicAdd(&cnt[m], ins | (rem << 16));
    }
    lds_barrier();
    for (uint32_t q = threadIdx.x; q < span; q += kMszT) out[base + q] = cnt[q];
    lds_barrier();  // (the next pass clears cnt)
  }
}

__device__ inline int32_t msz_net(uint32_t c) { return (int32_t)(c & 0xFFFFu) - (int32_t)(c >> 16); }

constexpr int kMszScanW = 16;  // waves per scan workgroup
constexpr int kMszMaps = 16;   // maps per scan workgroup: lane = map (l % 16) and quarter (l / 16) of its wave's tiles
constexpr int kMszSub = (kWave / kMszMaps) * kMszScanW;  // tile sub-chunks in log order: (wave, quarter)
__global__ __launch_bounds__(kMszScanW * kWave) void k_msize_scan(const uint8_t* __restrict__ res_type, uint32_t R,
                                                                 uint32_t tiles, const uint32_t* __restrict__ tcnt,
                                                                 uint32_t* __restrict__ msize, uint32_t* __restrict__ mpcap,
                                                                 uint4* __restrict__ list, uint32_t* __restrict__ list_n) {
  __shared__ int32_t csum[kMszSub][kMszMaps];
  __shared__ uint32_t clv[kMszSub][kMszMaps];
  const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63, ml = l % kMszMaps, h = l / kMszMaps;
  const uint32_t m = blockIdx.x * kMszMaps + ml, sc = (kWave / kMszMaps) * w + h;  // this lane's map and sub-chunk
  const bool ok = m < R && is_keyed(res_type[m]);
  const uint32_t per = (tiles + kMszSub - 1) / kMszSub, t0 = min(sc * per, tiles), t1 = min(t0 + per, tiles);
  // sub-chunk sc's tiles [t0, t1) in log order (row t of tcnt: 16 maps' words per quarter-wave), loaded once into
  // registers, all in flight together, for the three passes below (64 maps per workgroup re-reading the rows per pass
  // was ~53 us per c3 sub-batch on 64 workgroups)
  constexpr int kPerMax = kMaxTiles / kMszSub;
  const uint32_t* c = tcnt + m;
  uint32_t xc[kPerMax];
#pragma unroll
  for (int q = 0; q < kPerMax; ++q) xc[q] = ok && t0 + q < t1 ? c[(uint64_t)(t0 + q) * R] : 0u;
  int32_t sum = 0;
#pragma unroll
  for (int q = 0; q < kPerMax; ++q) sum += msz_net(xc[q]);
  csum[sc][ml] = sum;
  lds_barrier();
  // (mpcap is raised atomically by an overlapped small-map replay on the side stream: an atomic load here; a stale
  // level only lists more tiles for the exact pass, and the CAS merge below keeps the higher one)
  const uint32_t s0 = ok ? msize[m] : 0u, mp = ok ? __hip_atomic_load(&mpcap[m], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
  int32_t start = (int32_t)s0;  // (sizes are < 2^31: map_capacity <= 2M live entries)
  for (uint32_t q = 0; q < sc; ++q) start += csum[q][ml];
  // lower bounds: the highest level every tile's counts prove (with the level reached so far)
  uint32_t lv = mp & ~kMpInexact;
  if (ok) {
    int32_t s = start;
#pragma unroll
    for (int q = 0; q < kPerMax; ++q) {
      const uint32_t x = xc[q];
      const int32_t fin = s + msz_net(x);
      if (x) lv = max(lv, cap_level((uint64_t)(int64_t)max(s, fin)));
      s = fin;
    }
  }
  clv[sc][ml] = lv;
  lds_barrier();
  uint32_t lr = mp & ~kMpInexact;  // the level proven at this sub-chunk's start: before the sub-batch, and earlier ones
#pragma unroll 4
  for (uint32_t q = 0; q < (uint32_t)kMszSub; ++q) {  // (one pass: the values are not kept for a second)
    const uint32_t x = clv[q][ml];
    lv = max(lv, x);
    if (q < sc) lr = max(lr, x);
  }
  // tiles that may cross a resize threshold above the level proven before them: replayed by k_msize_exact, which
  // also records where each resize happened (the capacity-level timeline of the tree-bin test, common.h)
  uint32_t inexact = 0;
  if (ok) {
    int32_t s = start;
#pragma unroll
    for (int q = 0; q < kPerMax; ++q) {
      const uint32_t x = xc[q], t = t0 + q;
      if (t < t1 && (int64_t)s + (int64_t)(x & 0xFFFFu) > (int64_t)(12ull << lr)) {  // level(p) <= lr  <=>  p <= 12 << lr
        const uint32_t k = atomicAdd(list_n, 1u);
        if (k < kMszListCap) list[k] = make_uint4(t, m, (uint32_t)s, 0u);
        else inexact = kMpInexact;
      }
      const int32_t fin = s + msz_net(x);
      if (x) lr = max(lr, cap_level((uint64_t)(int64_t)max(s, fin)));
      s = fin;
    }
  }
  lds_barrier();  // every lane read clv
  clv[sc][ml] = inexact;
  lds_barrier();
  if (sc == 0 && ok) {
    for (int q = 0; q < kMszSub; ++q) inexact |= clv[q][ml];
    int64_t total = 0;
    for (int q = 0; q < kMszSub; ++q) total += csum[q][ml];
    msize[m] = (uint32_t)((int64_t)s0 + total);
    // (merged: an overlapped small-map replay may raise the level meanwhile, map_small.hip)
    for (uint32_t old = mp;;) {
      const uint32_t nv = max(old & ~kMpInexact, lv) | inexact | (old & kMpInexact);
      const uint32_t got = atomicCAS(&mpcap[m], old, nv);
      if (got == old) break;
      old = got;
    }
  }
}

__global__ __launch_bounds__(kMszT) void k_msize_exact(const uint16_t* __restrict__ ttab, const uint16_t* __restrict__ cpos,
                                                      uint64_t rows, uint32_t sb, uint32_t k0, uint32_t k1, uint32_t sb_hot,
                                                      const uint32_t* __restrict__ msz, const HotKey* __restrict__ hot,
                                                      const uint32_t* __restrict__ hot_n, const uint32_t* __restrict__ hot_len,
                                                      const uint32_t* __restrict__ hot_rpre, const uint32_t* __restrict__ hot_msz,
                                                      const uint4* __restrict__ list,
                                                      const uint32_t* __restrict__ list_n, uint32_t* __restrict__ mpcap,
                                                      unsigned long long* __restrict__ lvl_at, const uint64_t* __restrict__ index,
                                                      uint64_t lo) {
  constexpr int kPer = kTile / kMszT;
  __shared__ int32_t wsum[kMszT / kWave], wmax[kMszT / kWave];
  __shared__ uint32_t pfx[kHotMax + 1];
  __shared__ uint32_t hb[kHotMax + 1], hslot[kHotMax], hlp[kHotMax];  // per item: the tile's hot runs (LDS lookups)
  const uint32_t n = min(*list_n, kMszListCap), w = threadIdx.x >> 6, l = threadIdx.x & 63;
  uint32_t nh;
  hot_pfx(hot_n, hot_len, pfx, nh);
  for (uint32_t it = blockIdx.x; it < n; it += gridDim.x) {
    const uint4 e = list[it];
    const uint32_t t = e.x, m = e.y;
    const uint16_t* row = ttab + (uint64_t)t * (sb + 1);
    const uint32_t b0 = row[k0], bh = row[sb_hot], b1 = row[k1];
    const uint64_t base = (uint64_t)t * kTile;
    for (uint32_t h = threadIdx.x; h <= nh; h += kMszT) {
      hb[h] = row[sb_hot + h];
      if (h < nh) {
        hslot[h] = hot[h].ident & kMwSlotMask;
        hlp[h] = hot_rpre[(uint64_t)h * (kMaxTiles + 1) + t];
      }
    }
    lds_barrier();
    // the size change of this thread's j-th row (consecutive rows, log order): +1 insert, -1 removal, 0 other
    auto delta = [&](int j, uint64_t& r) -> int32_t {
      r = base + (uint64_t)threadIdx.x * kPer + j;
      if (r >= rows) return 0;
      const uint32_t p = cpos[r];
      if (p < b0 || p >= b1) return 0;  // unknown session (0xFFFF) or not a map record
      uint32_t code;
      if (p < bh) {  // a region record
        const uint32_t x = msz[base + p];
        if ((x >> 2) != m) return 0;
        code = x & 3u;
      } else {  // a hot key's record: its bucket (the last hot bucket starting at or before p), list position
        uint32_t a = 0, b = nh;
        while (b - a > 1) {
          const uint32_t c = (a + b) >> 1;
          if (hb[c] <= p) a = c; else b = c;
        }
        if (hslot[a] != m) return 0;
        code = hot_code(hot_msz, pfx, a, hlp[a] + (p - hb[a]));
      }
      return code == 1u ? 1 : code == 2u ? -1 : 0;
    };
    int32_t sum = 0, mx = 0;  // this thread's rows: net change, highest running value
    for (int j = 0; j < kPer; ++j) {
      uint64_t r;
      sum += delta(j, r);
      mx = max(mx, sum);
    }
    int32_t inc = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int32_t y = __shfl_up(inc, d, 64);
      if (l >= (uint32_t)d) inc += y;
    }
    int32_t best = inc - sum + mx;  // the highest running value inside this thread's rows, from the wave's start
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) best = max(best, __shfl_xor(best, d, 64));
    if (l == 63) wsum[w] = inc;
    if (l == 0) wmax[w] = best;
    lds_barrier();
    if (threadIdx.x == 0) {
      int32_t run = 0, peak = 0;
      for (int q = 0; q < kMszT / kWave; ++q) {
        peak = max(peak, run + wmax[q]);
        run += wsum[q];
      }
      atomicMax(&mpcap[m], cap_level((uint64_t)e.z + (uint64_t)peak));
    }
    if (lvl_at && index && mx > 0) {  // rows that raise the running peak: the log index of each resize (timeline)
      int64_t sz = (int64_t)e.z + (inc - sum);  // this thread's start size
      for (uint32_t q = 0; q < w; ++q) sz += wsum[q];
      int64_t pk = sz;
      for (int j = 0; j < kPer; ++j) {
        uint64_t r;
        sz += delta(j, r);
        if (sz > pk) {
          if (cap_level((uint64_t)sz) > cap_level((uint64_t)max<int64_t>(pk, 0)))
            lvl_reached(lvl_at, m, cap_level((uint64_t)max<int64_t>(pk, 0)), cap_level((uint64_t)sz), index[lo + r]);
          pk = sz;
        }
      }
    }
    lds_barrier();  // wsum / wmax are rewritten by the next item
  }
}

int launch_map_size(const MapSizeArgs& a, hipStream_t st) {
  if (a.tiles == 0) return 0;
  hipLaunchKernelGGL(k_msize_count, dim3(a.tiles), dim3(kMszT), 0, st, a.ttab, a.sb, a.k0, a.sb_hot, a.rst_msz, a.hot,
                     a.hot_n, a.hot_len, a.hot_rpre, a.hot_msz, a.max_resources, a.tcnt, a.list_n, a.msmall, a.mrec,
                     a.idx0, a.hh_key, a.hh_val, a.hh_n, a.ev_key, a.ev_val, a.ev_pay, a.ev_cap, a.sm_ctl, a.map_row, a.lo,
                     a.err);
  if (a.map_row) return hipGetLastError() == hipSuccess ? 0 : -1;  // TTL mode: sizes from the events (k_ttl_replay)
  hipLaunchKernelGGL(k_msize_scan, dim3((a.max_resources + kMszMaps - 1) / kMszMaps), dim3(kMszScanW * kWave), 0, st,
                     a.res_type, a.max_resources, a.tiles, a.tcnt, a.msize, a.mpcap, a.list, a.list_n);
  hipLaunchKernelGGL(k_msize_exact, dim3(256), dim3(kMszT), 0, st, a.ttab, a.cpos, a.rows, a.sb, a.k0, a.k1, a.sb_hot,
                     a.rst_msz, a.hot, a.hot_n, a.hot_len, a.hot_rpre, a.hot_msz, a.list, a.list_n, a.mpcap, a.lvl_at,
                     a.index, a.lo);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace cc
