// apply_value.hip — AtomicValueState apply (also DistributedAtomicLong, whose add is a client-side CAS loop).
//
// One 1024-thread workgroup owns one super-bucket = 256 AtomicValueState instances: thread t < 256 holds slot
// t's state in registers for the whole launch.  The workgroup walks the super-bucket's staging list (its run
// in every tile, tile order = log order; built by partition.hip) in chunks of 4096 records:
//   1. all 16 waves load the chunk (the next chunk's loads are in flight while the current one is resolved)
//      and sort it stably by slot: ranking inside each wave with LDS atomics with return (same-address lanes
//      of one instruction resolve in lane order on gfx950 — checked at engine start), per-wave prefixes per
//      slot, a scan over the 256 slots;
//   2. threads 0..255 each apply their slot's commits sequentially, in log order — the same order the
//      reference's single state-machine thread would (ResourceManager.java:56-72);
//   3. results go back to the records' staging positions; k_unpermute returns them to log order.
//
// The partition encodes every value record for this walk (common.h value_encode): the op becomes flag bits
// plus the precomputed status byte, the operands the canonical compare value and the canonical new value.
// Per-op semantics restate AtomicValueState (atomic/src/main/java/io/atomix/atomic/state/AtomicValueState.java):
//   get :77-83, set :114-118, compareAndSet :123-133, getAndSet :138-144, delete :146-157.
// `ttl` is never serialized for these commands (AtomicValueCommands.java:125-133,181-191,227-235),
// so no TTL timer can exist.  Listen/Unlisten (:41-63) publish events: applied by apply_coord.hip under
// CC_CFG_VALUE_EVENTS, flagged as unsupported here.
#include "common.h"
#include "engine_internal.h"

namespace cc {

constexpr int kVT = 1024;                  // threads per workgroup (16 waves)
constexpr int kVW = kVT / kWave;
constexpr int kVPer = 4;                   // records per thread per chunk
constexpr int kVCh = kVT * kVPer;          // 4096 records per chunk
constexpr int kVWaveRecs = kWave * kVPer;  // records of a chunk per wave (contiguous in log order)
constexpr int kVSlots = 1 << kSbShift;     // 256 slots per super-bucket
constexpr int kVPairs = kVSlots / 2;       // per-wave slot counters: packed u16 pairs
constexpr uint32_t kNoPos = 0xFFFFFFFFu;

// One step of a slot's chain.  State: ms = tag | has_current << 8, v = payload (0 when the tag is NULL: every
// write stores a canonical payload and delete clears both, so current == null implies value == null, and get's
// `current != null ? value : null` is the value itself).  Returns the status byte; rv = result payload.
__device__ inline uint32_t value_walk(uint32_t m, uint64_t x, uint64_t y, uint32_t& ms, uint64_t& v, uint64_t& rv) {
  const uint32_t tag = ms & 0xFFu;
  // compareAndSet :124 (value == null && expect == null) || (value != null && value.equals(expect))
  const bool eq = vrec_ctag(m) == tag && v == x;
  const bool is_c = (m & kVrC) != 0, is_r = (m & kVrR) != 0, is_d = (m & kVrD) != 0;
  const bool w = (m & kVrW) != 0 || (is_c && eq);
  rv = is_r ? v : ((is_c && eq) ? 1ull : 0ull);
  const uint32_t st = is_r ? (tag << 4) : (m & 0xFFu);
  ms = w ? (vrec_ntag(m) | 0x100u) : (is_d ? 0u : ms);
  v = w ? y : (is_d ? 0ull : v);
  return st;
}

// Largest r in [0, tiles) with rpre[r] <= c (rpre non-decreasing, rpre[0] = 0): a two-round 64-ary search by
// the whole wave (c is wave-uniform; every lane must be active).  Record c lies in run r when c < rpre[tiles].
__device__ inline uint32_t find_run(const uint32_t* rpre, uint32_t tiles, uint32_t c) {
  const uint32_t l = __lane_id();
  const uint32_t step = (tiles + kWave - 1) / kWave;
  uint32_t cand = l * step;
  uint64_t b = __ballot(cand < tiles && rpre[cand] <= c);
  const uint32_t base = (uint32_t)(63 - __clzll((long long)b)) * step;
  cand = base + l;
  b = __ballot(l < step && cand < tiles && rpre[cand] <= c);
  return base + (uint32_t)(63 - __clzll((long long)b));
}

__global__ __launch_bounds__(kVT) void k_apply_value(const uint32_t* __restrict__ st_meta, const u64x2* __restrict__ st_ab,
                                                    const uint16_t* __restrict__ ttab, uint32_t tiles, uint32_t sb,
                                                    const uint8_t* __restrict__ sb_kind,
                                                    uint32_t* __restrict__ val_meta, uint64_t* __restrict__ val_v,
                                                    uint8_t* __restrict__ rst_status, uint64_t* __restrict__ rst_value,
                                                    uint32_t* __restrict__ err_out) {
  __shared__ u64x2 sab[kVCh];                  // the chunk sorted by slot
  __shared__ uint32_t sm[kVCh];
  __shared__ uint64_t rval[kVCh];              // results, sorted order
  __shared__ uint8_t rstat[kVCh];
  __shared__ uint32_t wcnt[kVW][kVPairs];      // per-wave slot counts -> per-wave exclusive prefixes (u16 pairs)
  __shared__ uint32_t qsum[kVW / 2][kVPairs];  // counts of wave pairs
  __shared__ uint32_t ctot[kVPairs];           // slot totals of the chunk (u16 pairs)
  __shared__ uint32_t sstart[kVSlots];
  __shared__ uint32_t wsum[kVW];
  __shared__ uint32_t rstart[kMaxTiles];       // staging position of this super-bucket's run in tile t
  __shared__ uint32_t rpre[kMaxTiles + 1];     // records of this super-bucket before tile t

  const uint32_t s = blockIdx.x, t = threadIdx.x, w = t >> 6, l = t & 63;
  if (sb_kind && sb_kind[s]) return;  // holds coordination resources / value events: k_apply_coord
  uint32_t ms = 0;
  uint64_t sv = 0;
  if (t < (uint32_t)kVSlots) {
    ms = val_meta[(uint64_t)s * kVSlots + t];
    sv = val_v[(uint64_t)s * kVSlots + t];
  }
  for (uint32_t k = t; k < (uint32_t)(kVW * kVPairs); k += kVT) (&wcnt[0][0])[k] = 0;
  // the super-bucket's list = its run in every tile, in tile order (tile-local layout of partition.hip)
  {
    uint32_t len = 0;
    if (t < tiles) {
      const uint16_t* row = ttab + (uint64_t)t * (sb + 1);
      const uint32_t b0 = row[s], b1 = row[s + 1];
      rstart[t] = t * kTile + b0;
      len = b1 - b0;
    }
    uint32_t inc = len;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(inc, d, 64);
      if (l >= (uint32_t)d) inc += y;
    }
    if (l == 63) wsum[w] = inc;
    lds_barrier();
    uint32_t pre = inc - len, all = 0;
    for (uint32_t q = 0; q < (uint32_t)kVW; ++q) {
      const uint32_t x = wsum[q];
      if (q < w) pre += x;
      all += x;
    }
    if (t < tiles) rpre[t] = pre;
    if (t == 0) rpre[tiles] = all;
    lds_barrier();
  }
  const uint32_t cnt = rpre[tiles];
  uint32_t err = 0;

  // thread (w, j, l) holds record c0 + w*256 + j*64 + l of a chunk: log order = (w, j, l)
  uint32_t m[kVPer], nm[kVPer], g[kVPer], ng[kVPer];
  u64x2 ab[kVPer], nab[kVPer];
  auto load = [&](uint32_t c0, uint32_t (&mm)[kVPer], u64x2 (&aa)[kVPer], uint32_t (&gg)[kVPer]) {
#pragma unroll
    for (int j = 0; j < kVPer; ++j) {
      const uint32_t crow = c0 + w * kVWaveRecs + j * kWave, c = crow + l;
      mm[j] = 0;
      aa[j] = u64x2{0, 0};
      gg[j] = kNoPos;
      if (crow < cnt) {  // wave-uniform
        uint32_t r = find_run(rpre, tiles, crow);
        if (c < cnt) {
          while (rpre[r + 1] <= c) ++r;  // a lane is at most 63 records past its row's start
          const uint32_t gp = rstart[r] + (c - rpre[r]);
          gg[j] = gp;
          mm[j] = st_meta[gp];
          aa[j] = st_ab[gp];
        }
      }
    }
  };
  load(0, m, ab, g);
  for (uint32_t c0 = 0; c0 < cnt; c0 += kVCh) {
    // the next chunk's records stream in during this whole chunk
    load(c0 + kVCh, nm, nab, ng);
    // 1a. rank each record among the wave's earlier records of its slot
    uint32_t rank[kVPer], slot[kVPer];
#pragma unroll
    for (int j = 0; j < kVPer; ++j) {
      slot[j] = smeta_slot(m[j]) & (kVSlots - 1);
      const uint32_t sh = 16 * (slot[j] & 1);
      rank[j] = g[j] != kNoPos ? (atomicAdd(&wcnt[w][slot[j] >> 1], 1u << sh) >> sh) & 0xFFFFu : 0u;
    }
    lds_barrier();
    // 1b. exclusive prefixes over the 16 waves, per slot (thread = slot pair x wave pair; u16 halves never carry:
    //     a chunk holds 4096 records)
    {
      const uint32_t pr = t & (kVPairs - 1), q = t >> 7;
      const uint32_t c0v = wcnt[2 * q][pr], c1v = wcnt[2 * q + 1][pr];
      qsum[q][pr] = c0v + c1v;
      lds_barrier();
      uint32_t base = 0;
      for (uint32_t qq = 0; qq < q; ++qq) base += qsum[qq][pr];
      wcnt[2 * q][pr] = base;
      wcnt[2 * q + 1][pr] = base + c0v;
      if (q == kVW / 2 - 1) ctot[pr] = base + c0v + c1v;
      lds_barrier();
    }
    // 1c. run start of every slot (exclusive scan over the 256 slots by waves 0..3)
    uint32_t run = 0, start = 0;
    if (t < (uint32_t)kVSlots) {
      run = (ctot[t >> 1] >> (16 * (t & 1))) & 0xFFFFu;
      uint32_t inc = run;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d, 64);
        if (l >= (uint32_t)d) inc += y;
      }
      if (l == 63) wsum[w] = inc;
      start = inc - run;
    }
    lds_barrier();
    if (t < (uint32_t)kVSlots) {
      for (uint32_t q = 0; q < w; ++q) start += wsum[q];
      sstart[t] = start;
    }
    lds_barrier();
    // 1d. place records in slot order; p[j] = sorted position (results come back from there)
    uint32_t p[kVPer];
#pragma unroll
    for (int j = 0; j < kVPer; ++j) {
      p[j] = 0;
      if (g[j] == kNoPos) continue;
      const uint32_t sl = slot[j];
      const uint32_t pre = (wcnt[w][sl >> 1] >> (16 * (sl & 1))) & 0xFFFFu;
      p[j] = sstart[sl] + pre + rank[j];
      sm[p[j]] = m[j];
      sab[p[j]] = ab[j];
    }
    lds_barrier();
    for (uint32_t k = t; k < (uint32_t)(kVW * kVPairs); k += kVT) (&wcnt[0][0])[k] = 0;
    // 2. thread t applies its slot's commits in log order, state in registers (the next record's LDS reads
    //    are issued before the current one is applied)
    if (t < (uint32_t)kVSlots && run) {
      uint32_t mm = sm[start];
      u64x2 xy = sab[start];
      for (uint32_t k = 0; k < run; ++k) {
        const uint32_t pn = k + 1 < run ? start + k + 1 : start + k;
        const uint32_t mm2 = sm[pn];
        const u64x2 xy2 = sab[pn];
        uint64_t rv;
        const uint32_t stt = value_walk(mm, xy.x, xy.y, ms, sv, rv);
        if (mm & kVrL) err |= kErrUnsupported;
        rstat[start + k] = (uint8_t)stt;
        rval[start + k] = rv;
        mm = mm2;
        xy = xy2;
      }
    }
    lds_barrier();
    // 3. results back to the records' staging positions (contiguous within each run)
#pragma unroll
    for (int j = 0; j < kVPer; ++j) {
      if (g[j] == kNoPos) continue;
      rst_status[g[j]] = rstat[p[j]];
      rst_value[g[j]] = rval[p[j]];
    }
#pragma unroll
    for (int j = 0; j < kVPer; ++j) {
      m[j] = nm[j];
      ab[j] = nab[j];
      g[j] = ng[j];
    }
  }
  if (t < (uint32_t)kVSlots) {
    val_meta[(uint64_t)s * kVSlots + t] = ms;
    val_v[(uint64_t)s * kVSlots + t] = sv;
  }
  if (err) atomicOr(err_out, err);
}

// Engine-start self-check of the hardware property the stable rankings rely on: LDS atomics with return
// from one wave instruction that hit the same address are resolved in lane order.  *bad counts violations.
__global__ __launch_bounds__(256) void k_selfcheck_lds_order(uint32_t* __restrict__ bad) {
  __shared__ uint32_t tbl[256];
  const uint32_t t = threadIdx.x, l = t & 63;
  uint32_t x = 0x9E3779B9u ^ (t * 2654435761u) ^ (blockIdx.x * 40503u);
  uint32_t v = 0;
  for (uint32_t it = 0; it < 32; ++it) {
    tbl[t] = 0;
    lds_barrier();
    x = x * 1664525u + 1013904223u;
    const uint32_t key = ((x >> 8) & ((1u << (it & 3)) - 1)) + (t >> 6) * 64;
    const uint32_t old = atomicAdd(&tbl[key], 1u);
    for (uint32_t j = 0; j < 64; ++j) {  // uniform loop: every lane takes part in each shuffle
      const uint32_t kj = __shfl(key, j, 64), oj = __shfl(old, j, 64);
      if (j < l && kj == key && oj >= old) ++v;
    }
    lds_barrier();
  }
  if (v) atomicAdd(bad, v);
}

int launch_selfcheck(uint32_t* d_bad, hipStream_t st) {
  hipLaunchKernelGGL(k_selfcheck_lds_order, dim3(64), dim3(256), 0, st, d_bad);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_apply_value(const ValueArgs& a, hipStream_t st) {
  a.mark(K_APPLY_VALUE, 1, st);
  hipLaunchKernelGGL(k_apply_value, dim3(a.sb_val), dim3(kVT), 0, st, a.st_meta, a.st_ab, a.ttab, a.tiles, a.sb, a.sb_kind,
                     a.val_meta, a.val_v, a.rst_status, a.rst_value, a.err);
  a.mark(K_APPLY_VALUE, 0, st);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace cc
