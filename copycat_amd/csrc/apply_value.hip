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

#ifdef CC_PHASE_TIMING
__device__ unsigned long long g_ph_value[kPhases];
int phase_read_value(uint64_t* out) {
  unsigned long long z[kPhases] = {};
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ph_value), sizeof z) != hipSuccess ||
      hipMemcpyToSymbol(HIP_SYMBOL(g_ph_value), z, sizeof z) != hipSuccess)
    return CC_ERR_HIP;
  return CC_OK;
}
#endif

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

// ---- k_apply_value_ws: the same walk with the sort pipelined behind it (loader / walker waves) -------------------
// (Round 1's k_apply_value ran its phases in turn: 12 of its 16 waves idled through the walk and the 4 walking
// waves through the sort.)  Here waves 0-3 only walk (thread t = slot t, state in registers) and waves 4-15 only load,
// sort and store: while the walkers apply chunk i (3072 records) out of one LDS buffer, the loaders store chunk
// i-1's results, rank / place chunk i+1 into the other buffer and issue chunk i+2's loads.  One workgroup barrier
// per chunk hands the buffers over; the loaders' own rank -> place step synchronises the 12 loader waves through an
// LDS arrival counter, so the walkers never stop mid-walk for it.  Every loader wave derives its own per-slot
// placement base from the 12 waves' counters (no second barrier).  Results overwrite their records in place (status
// into the meta word, value into the first operand).  Order and semantics are k_apply_value's: a record's sorted
// position is (slot run start) + (earlier loader waves' records of the slot) + (its rank inside its wave).
#ifndef CC_DIAG_NO_WALK
#define CC_DIAG_NO_WALK 0  // diagnostics only: the walkers skip the walk (wrong results)
#endif
#ifndef CC_DIAG_FAKE_POS
#define CC_DIAG_FAKE_POS 0  // diagnostics only: staging positions without the run lookup (wrong results)
#endif
constexpr int kWsLW = 12;                   // loader waves (waves 4..15)
constexpr int kWsPer = 4;                   // records per loader thread per chunk
constexpr int kWsCh = kWsLW * kWave * kWsPer;  // 3072 records per chunk

// Arrival barrier of the loader waves only: `target` = arrivals expected so far (monotonic counter in LDS).
__device__ inline void loader_barrier(uint32_t* ctr, uint32_t target) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  if (__lane_id() == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < target) __builtin_amdgcn_s_sleep(1);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__global__ __launch_bounds__(kVT) void k_apply_value_ws(const uint32_t* __restrict__ st_meta, const u64x2* __restrict__ st_ab,
                                                       const uint16_t* __restrict__ ttab, uint32_t tiles, uint32_t sb,
                                                       const uint8_t* __restrict__ sb_kind,
                                                       uint32_t* __restrict__ val_meta, uint64_t* __restrict__ val_v,
                                                       uint8_t* __restrict__ rst_status, uint64_t* __restrict__ rst_value,
                                                       uint64_t dummy, uint32_t* __restrict__ err_out) {
  __shared__ u64x2 sab[2][kWsCh];             // chunk buffers sorted by slot; results in place (value -> .x)
  __shared__ uint32_t sm[2][kWsCh];           //   meta words; results in place (status)
  __shared__ uint32_t wcnt[2][kWsLW][kVPairs];  // per-loader-wave slot counts (packed u16 pairs), double-buffered
  __shared__ uint16_t pbase[kWsLW][kVSlots];  // per loader wave: sorted position of its first record of each slot
  __shared__ uint32_t sstart[2][kVSlots + 1];  // slot run starts of each buffer (+ total)
  __shared__ uint32_t rstart[kMaxTiles];
  __shared__ uint32_t rpre[kMaxTiles + 1];
  __shared__ uint32_t wsum[kVW];
  __shared__ uint32_t lbar;

  const uint32_t s = blockIdx.x, t = threadIdx.x, w = t >> 6, l = t & 63;
  if (sb_kind && sb_kind[s]) return;  // holds coordination resources / value events: k_apply_coord
  const bool walker = w < 4;
  const uint32_t lw = walker ? 0u : w - 4;
  uint32_t ms = 0;
  uint64_t sv = 0;
  if (walker) {
    ms = val_meta[(uint64_t)s * kVSlots + t];
    sv = val_v[(uint64_t)s * kVSlots + t];
  }
  for (uint32_t k = t; k < (uint32_t)(2 * kWsLW * kVPairs); k += kVT) (&wcnt[0][0][0])[k] = 0;
  if (t == 0) lbar = 0;
  {  // the super-bucket's list = its run in every tile, in tile order
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
  const uint32_t nch = (cnt + kWsCh - 1) / kWsCh;
#ifdef CC_PHASE_TIMING
  // diagnostics: thread 0 (walker) phases 0 walk, 1 wait; thread 256 (loader) phases 2 result store, 3 rank,
  // 4 loader barrier + workgroup barrier, 5 clear + placement bases, 6 place, 7 load issue
  uint64_t wph_last = wall_clock64(), wph[kPhases] = {0, 0, 0, 0, 0, 0, 0, 0};
  auto WPH = [&](int k) {
    if (t == 0 || t == 4 * kWave) {
      const uint64_t n_ = wall_clock64();
      wph[k] += n_ - wph_last;
      wph_last = n_;
    }
  };
#else
  auto WPH = [&](int) {};
#endif
  uint32_t err = 0;

  // loader registers: the chunk to place next (m, g, ab; loaded one chunk ahead), the sorted / staging positions of
  // the chunk being walked (pp, gp) and of the chunk before it (qp, gq: its results are stored during the walk).
  // Named scalars: register arrays would live in scratch.
#define CC_J4(X) X(0) X(1) X(2) X(3)
#define CC_DECL(J) uint32_t m##J = 0, g##J = kNoPos, pp##J = 0, gp##J = kNoPos, qp##J = 0, gq##J = kNoPos; uint4 ab##J = make_uint4(0, 0, 0, 0);
  CC_J4(CC_DECL)
#undef CC_DECL
  // record c0 + lw*256 + j*64 + l of the list (log order = (loader wave, j, lane)); past the end: staging position 0
  // Staging position of list record c: the run r holding it (rpre[r] <= c < rpre[r+1]) gives rstart[r] + c - rpre[r].
  // Per wave and chunk, one 64-ary search finds the run of the wave's first record; lane k then holds the window
  // run rrow + k (its start wS, its first record wP) and the next run's first record wB.  When the window covers the
  // wave's 256 records (runs average 64 records), a row's records find their runs with ballots over wB and a scalar
  // loop over the (one or two) run starts inside the row, and their positions with two lane shuffles: no dependent
  // LDS lookups.  Otherwise (many short or empty runs) every row searches as in k_apply_value.
#define CC_LOAD1(J)                                                                               \
  {                                                                                               \
    const uint32_t crow = c0w + (J) * kWave, c = crow + l;                                        \
    uint32_t gpos = 0;                                                                            \
    if (CC_DIAG_FAKE_POS) { gpos = c < cnt ? c : 0; } else                                       \
    if (crow < cnt) { /* wave-uniform */                                                          \
      if (win) {                                                                                  \
        uint32_t ri = (uint32_t)__popcll(__ballot(wB <= crow));                                   \
        uint64_t mb = __ballot(wB > crow && wB <= crow + (kWave - 1));                            \
        while (mb) {                                                                              \
          const uint32_t bk = (uint32_t)__builtin_amdgcn_readlane((int)wB, __ffsll((long long)mb) - 1); \
          ri += c >= bk ? 1u : 0u;                                                                \
          mb &= mb - 1;                                                                           \
        }                                                                                         \
        const uint32_t rs_ = (uint32_t)__shfl((int)wS, (int)ri, 64);                              \
        const uint32_t rp_ = (uint32_t)__shfl((int)wP, (int)ri, 64);                              \
        if (c < cnt) gpos = rs_ + (c - rp_);                                                      \
      } else {                                                                                    \
        uint32_t r = find_run(rpre, tiles, crow);                                                 \
        if (c < cnt) {                                                                            \
          while (rpre[r + 1] <= c) ++r;                                                           \
          gpos = rstart[r] + (c - rpre[r]);                                                       \
        }                                                                                         \
      }                                                                                           \
    }                                                                                             \
    g##J = c < cnt ? gpos : kNoPos;                                                               \
    m##J = st_meta[gpos];                                                                         \
    ab##J = reinterpret_cast<const uint4*>(st_ab)[gpos];                                          \
  }
#define CC_LOAD_CHUNK(C0)                                                                         \
  {                                                                                               \
    const uint32_t c0w = (C0) + lw * (kWave * kWsPer);                                            \
    uint32_t wB = 0xFFFFFFFFu, wS = 0, wP = 0;                                                    \
    bool win = false;                                                                             \
    if (!CC_DIAG_FAKE_POS && c0w < cnt) {                                                         \
      const uint32_t rrow = find_run(rpre, tiles, c0w);                                           \
      const uint32_t kr = rrow + l;                                                               \
      wB = kr + 1 <= tiles ? rpre[kr + 1] : 0xFFFFFFFFu;                                          \
      wS = kr < tiles ? rstart[kr] : 0u;                                                          \
      wP = kr < tiles ? rpre[kr] : 0u;                                                            \
      const uint32_t lastc = c0w + kWave * kWsPer - 1 < cnt ? c0w + kWave * kWsPer - 1 : cnt - 1; \
      win = (uint32_t)__shfl((int)wB, 63, 64) > lastc;                                            \
    }                                                                                             \
    CC_J4(CC_LOAD1)                                                                               \
  }
  uint32_t bar_n = 0;  // loader-barrier arrivals expected so far
  // rank / place the registers' chunk into buffer b (loaders only)
  auto prepare = [&](uint32_t b) {
    uint32_t rank[kWsPer], slot[kWsPer];
    const uint32_t mv[kWsPer] = {m0, m1, m2, m3}, gv[kWsPer] = {g0, g1, g2, g3};
#pragma unroll
    for (int j = 0; j < kWsPer; ++j) {
      slot[j] = smeta_slot(mv[j]) & (kVSlots - 1);
      const uint32_t sh = 16 * (slot[j] & 1);
      rank[j] = gv[j] != kNoPos ? (atomicAdd(&wcnt[b][lw][slot[j] >> 1], 1u << sh) >> sh) & 0xFFFFu : 0u;
    }
    WPH(3);
    bar_n += kWsLW;
    loader_barrier(&lbar, bar_n);
    WPH(4);
    // the other counter buffer was last read before the previous workgroup barrier: clear it for the next chunk
    for (uint32_t k = t - 4 * kWave; k < (uint32_t)(kWsLW * kVPairs); k += kWsLW * kWave) (&wcnt[b ^ 1][0][0])[k] = 0;
    // this wave's placement bases: lane l owns slots 4l..4l+3 (counter pairs 2l, 2l+1)
    uint32_t a0 = 0, a1 = 0, p0 = 0, p1 = 0;
#pragma unroll
    for (int q = 0; q < kWsLW; ++q) {
      const uint32_t c0v = wcnt[b][q][2 * l], c1v = wcnt[b][q][2 * l + 1];
      if ((uint32_t)q == lw) {
        p0 = a0;
        p1 = a1;
      }
      a0 += c0v;
      a1 += c1v;
    }
    const uint32_t r0 = a0 & 0xFFFFu, r1 = a0 >> 16, r2 = a1 & 0xFFFFu, r3 = a1 >> 16;
    const uint32_t mine = r0 + r1 + r2 + r3;
    uint32_t inc = mine;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(inc, d, 64);
      if (l >= (uint32_t)d) inc += y;
    }
    const uint32_t ex = inc - mine;
    const uint32_t s0 = ex, s1 = ex + r0, s2 = s1 + r1, s3 = s2 + r2;
    pbase[lw][4 * l] = (uint16_t)(s0 + (p0 & 0xFFFFu));
    pbase[lw][4 * l + 1] = (uint16_t)(s1 + (p0 >> 16));
    pbase[lw][4 * l + 2] = (uint16_t)(s2 + (p1 & 0xFFFFu));
    pbase[lw][4 * l + 3] = (uint16_t)(s3 + (p1 >> 16));
    if (lw == 0) {  // the walkers' run starts (read after the workgroup barrier)
      sstart[b][4 * l] = s0;
      sstart[b][4 * l + 1] = s1;
      sstart[b][4 * l + 2] = s2;
      sstart[b][4 * l + 3] = s3;
      if (l == 63) sstart[b][kVSlots] = inc;
    }
    WPH(5);
    // lanes read bases other lanes of this wave just wrote: LDS keeps one wave's accesses in order
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
#define CC_PLACE1(J)                                                                \
    {                                                                               \
      pp##J = 0;                                                                    \
      gp##J = g##J;                                                                 \
      if (g##J != kNoPos) {                                                         \
        pp##J = pbase[lw][slot[J]] + rank[J];                                       \
        sm[b][pp##J] = m##J;                                                        \
        reinterpret_cast<uint4*>(sab[b])[pp##J] = ab##J;                            \
      }                                                                             \
    }
    CC_J4(CC_PLACE1)
#undef CC_PLACE1
    WPH(6);
  };
  // the previous chunk's results (buffer b) back to the records' staging positions; unconditional stores
  auto store_results = [&](uint32_t b) {
#define CC_STORE1(J)                                                                \
    {                                                                               \
      const uint64_t gx = gq##J != kNoPos ? (uint64_t)gq##J : dummy + t;            \
      rst_status[gx] = (uint8_t)sm[b][qp##J];                                       \
      rst_value[gx] = sab[b][qp##J].x;                                              \
    }
    CC_J4(CC_STORE1)
#undef CC_STORE1
  };

  if (!walker) {
    CC_LOAD_CHUNK(0)
    prepare(0);
    CC_LOAD_CHUNK(kWsCh)
  }
  lds_barrier();
  for (uint32_t i = 0; i < nch; ++i) {
    const uint32_t b = i & 1;
    if (walker) {
      const uint32_t start = sstart[b][t], run = CC_DIAG_NO_WALK ? 0u : sstart[b][t + 1] - start;
      if (run) {
        uint32_t mA[4], mB[4];
        u64x2 xA[4], xB[4];
        const uint32_t last = start + run - 1;
        auto fetch = [&](uint32_t k0, uint32_t (&mm)[4], u64x2 (&xx)[4]) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint32_t pq = start + k0 + q <= last ? start + k0 + q : last;
            mm[q] = sm[b][pq];
            xx[q] = sab[b][pq];
          }
        };
        auto walk4 = [&](uint32_t k0, const uint32_t (&mm)[4], const u64x2 (&xx)[4]) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            if (k0 + q < run) {
              uint64_t rv;
              const uint32_t stt = value_walk(mm[q], xx[q].x, xx[q].y, ms, sv, rv);
              if (mm[q] & kVrL) err |= kErrUnsupported;
              sm[b][start + k0 + q] = stt;
              sab[b][start + k0 + q].x = rv;
            }
          }
        };
        fetch(0, mA, xA);
        for (uint32_t k0 = 0; k0 < run; k0 += 8) {
          fetch(k0 + 4, mB, xB);
          walk4(k0, mA, xA);
          if (k0 + 4 >= run) break;
          fetch(k0 + 8, mA, xA);
          walk4(k0 + 4, mB, xB);
        }
      }
    } else {
      store_results(b ^ 1);  // chunk i-1 (i = 0: the dummy rows)
      WPH(2);
#define CC_SHIFT1(J) qp##J = pp##J; gq##J = gp##J;
      CC_J4(CC_SHIFT1)
#undef CC_SHIFT1
      prepare(b ^ 1);        // chunk i+1 (past the end: no live records)
      CC_LOAD_CHUNK((i + 2) * kWsCh)
      WPH(7);
    }
    if (walker) WPH(0);
    lds_barrier();
    WPH(walker ? 1 : 4);
  }
  if (!walker && nch) store_results((nch - 1) & 1);  // the last chunk (qp / gq since its walk)
#ifdef CC_PHASE_TIMING
  if (t == 0 || t == 4 * kWave)
    for (int q = 0; q < kPhases; ++q) atomicAdd(&g_ph_value[q], (unsigned long long)wph[q]);
#endif
#undef CC_LOAD_CHUNK
#undef CC_LOAD1
#undef CC_J4
  if (walker) {
    val_meta[(uint64_t)s * kVSlots + t] = ms;
    val_v[(uint64_t)s * kVSlots + t] = sv;
  }
  if (err) atomicOr(err_out, err);
}

// Engine-start self-check of the hardware property the stable rankings rely on: LDS atomics with return
// from one wave instruction that hit the same address are resolved in lane order.  *bad counts violations.
// Shaped like the kernels' rankings: 1024-thread workgroups (16 waves contending for the LDS at once), each wave
// on its own counter row, packed u16 pair counters bumped by 1 << 16 * (key & 1) as well as plain counters, and
// per-wave key sets from 1 to 256 distinct keys (the value apply's 256 slots, the partition's super-buckets).
__global__ __launch_bounds__(1024) void k_selfcheck_lds_order(uint32_t* __restrict__ bad) {
  __shared__ uint32_t tbl[16][256];
  const uint32_t t = threadIdx.x, l = t & 63, w = t >> 6;
  uint32_t x = 0x9E3779B9u ^ (t * 2654435761u) ^ (blockIdx.x * 40503u);
  uint32_t v = 0;
  for (uint32_t it = 0; it < 32; ++it) {
    for (uint32_t k = l; k < 256; k += 64) tbl[w][k] = 0;
    lds_barrier();
    x = x * 1664525u + 1013904223u;
    const uint32_t nkeys = 1u << (it & 7);                      // 1 .. 128 keys, then (it & 8) the skewed form
    uint32_t key = (x >> 8) & (nkeys * 2 - 1) & 255u;
    if (it & 8) key = ((x >> 8) & 7u) == 0 ? (x >> 12) & 255u : 0u;  // one hot key plus a tail
    const bool packed = (it & 16) != 0;
    const uint32_t sh = packed ? 16 * (key & 1) : 0;
    const uint32_t addr = packed ? key >> 1 : key;
    const uint32_t old = (atomicAdd(&tbl[w][addr], 1u << sh) >> sh) & 0xFFFFu;
    for (uint32_t j = 0; j < 64; ++j) {  // uniform loop: every lane takes part in each shuffle
      const uint32_t kj = __shfl(key, j, 64), oj = __shfl(old, j, 64);
      if (j < l && kj == key && oj >= old) ++v;
    }
    lds_barrier();
  }
  if (v) atomicAdd(bad, v);
}

int launch_selfcheck(uint32_t* d_bad, hipStream_t st) {
  hipLaunchKernelGGL(k_selfcheck_lds_order, dim3(256), dim3(1024), 0, st, d_bad);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_apply_value(const ValueArgs& a, hipStream_t st) {
  a.mark(K_APPLY_VALUE, 1, st);
  if (a.v3) {
    if (launch_apply_value_v3(a, st)) return -1;
  } else
    hipLaunchKernelGGL(k_apply_value_ws, dim3(a.sb_val), dim3(kVT), 0, st, a.st_meta, a.st_ab, a.ttab, a.tiles, a.sb,
                       a.sb_kind, a.val_meta, a.val_v, a.rst_status, a.rst_value, a.dummy, a.err);
  a.mark(K_APPLY_VALUE, 0, st);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace cc
