// partition_ext.hip — the tile-local partition (partition.hip) for batches with extended staging: maps (keys routed
// to their table region or to a hot key's bucket), coordination resources (quarter buckets) and value events.
//
// Same output as k_part_tile<J, true> (staging records per super-bucket run, ttab rows, cpos), restructured so no
// wave waits on a chain of dependent gathers:
//   (0) the tile's 16 commits per thread are resolved in one batch — instance column, instance -> resource,
//       resource -> type, then the map commits' key / flags — and each commit's route (super-bucket) is kept in a
//       register with its resource slot and type for the whole tile: the histogram comes from those registers and
//       the chunks never recompute a route (no second map_hash or hot-key probe);
//   (1..) chunks of 2048 commits (fully unrolled: the route registers are indexed at compile time); a chunk's raw
//       columns are requested at the top of the previous chunk, and with the type already known every column
//       the record needs (key, index, ttl / timeout, clock) is in that one batch of loads.
// Ranking, the per-wave prefix, run starts, placement and the run-by-run write-out are those of k_part_tile.
#include <cstdlib>

#include "common.h"
#include "engine_internal.h"

namespace cc {

#ifndef CC_PART_EXT_UNCOND
#define CC_PART_EXT_UNCOND 1  // every present column loaded for every row under the full wave mask (0: per-type loads)
#endif
#ifndef CC_PART_EXT_LATE
#define CC_PART_EXT_LATE 1  // the next chunk's columns loaded into the working registers after the placement (0: at
                            // the top of the chunk, into a second register set)
#endif
#ifndef CC_PART_EXT_UNROLL
#define CC_PART_EXT_UNROLL 0  // 1: the chunk loop fully unrolled (bigger code, fewer spills)
#endif
namespace {
enum : uint32_t { kRgXRec = 0, kRgValue = 1, kRgMap = 2, kRgHot = 3 };  // record kinds of the write-out plane (rg)
constexpr uint32_t kRgPos = (1u << 14) - 1;
static_assert(kTile <= (int)kRgPos + 1, "tile-local staging positions in 14 bits");
constexpr int kXQ = kTile / kPT;  // commits per thread per tile (16)
constexpr uint32_t kRpDead = 0xFFFFFFFFu;
constexpr uint32_t kTpWalk = 0x80u;  // type byte flag: a value commit of a super-bucket k_apply_value walks
}  // namespace

#ifdef CC_PHASE_TIMING
__device__ unsigned long long g_ph_partx[kPhases];
int phase_read_partx(uint64_t* out) {
  unsigned long long z[kPhases] = {};
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ph_partx), sizeof z) != hipSuccess ||
      hipMemcpyToSymbol(HIP_SYMBOL(g_ph_partx), z, sizeof z) != hipSuccess)
    return CC_ERR_HIP;
  return CC_OK;
}
#endif

// C: commits per LDS-staged chunk (2048; 1024 when the buckets' per-wave counters need the room: > 1024 map regions)
// IDS: coordination engines (instance ids into XRec.pad; a compile-time switch, so map-only engines pay no registers)
// TCK: the batch's clock column is checked (kExtTimeCheck; its two clocks per row ride with the chunk's loads)
template <int C, bool IDS, bool TCK>
__global__ __launch_bounds__(kPT, 4) void k_part_ext(
    const uint32_t* __restrict__ inst, const uint8_t* __restrict__ op, const uint8_t* __restrict__ flags,
    const uint64_t* __restrict__ ca, const uint64_t* __restrict__ cb, const uint64_t* __restrict__ ckey,
    const uint64_t* __restrict__ cidx, const uint64_t* __restrict__ caux, const uint64_t* __restrict__ ctime,
    const uint64_t* __restrict__ clock_base, uint32_t ext_flags, uint64_t lo, uint64_t hi,
    const uint64_t* __restrict__ inst_id, const uint32_t* __restrict__ inst_res, const uint8_t* __restrict__ res_type, const uint8_t* __restrict__ sb_kind,
    uint32_t max_inst, uint32_t sb, uint32_t sb_val, uint32_t map_bits, uint32_t sbq_base,
    const HotKey* __restrict__ hot, const uint32_t* __restrict__ hot_n, uint32_t* __restrict__ st_meta,
    u64x2* __restrict__ st_ab, XRec* __restrict__ xrec, MRec* __restrict__ mrec, uint32_t* __restrict__ hot_meta,
    uint16_t* __restrict__ cpos,
    uint16_t* __restrict__ ttab, ClrCtx clr, uint32_t* __restrict__ err_out) {
  constexpr int J = C / kPT;       // commits per thread per chunk
  constexpr int kXCh = kTile / C;  // chunks per tile
  static_assert(J * kXCh == kXQ && (J == 1 || J == 2), "chunk geometry");
  extern __shared__ __align__(16) uint8_t smem[];  // layout: partition.hip tile_lds_bytes(sb, true, C)
  u64x2* rab = reinterpret_cast<u64x2*>(smem);
  uint64_t* rkey = reinterpret_cast<uint64_t*>(rab + C);
  uint64_t* ridx = rkey + C;
  uint32_t* rres = reinterpret_cast<uint32_t*>(ridx + C);
  uint32_t* rmeta = rres + C;
  // per sorted record: its tile-local staging position | kind << 14 (kRgXRec / kRgValue / kRgMap / kRgHot), written by
  // the thread that places it: the write-out's pieces find their destination with one LDS read instead of the bucket
  // lookups bucket -> toff / trun / kstart / skind (three dependent LDS levels per 16-byte piece)
  uint16_t* rsb = reinterpret_cast<uint16_t*>(rmeta + C);
  uint32_t* wc = reinterpret_cast<uint32_t*>(rsb + C);  // [kPW][hw] packed u16 pairs
  const uint32_t hw = (sb + 1) / 2;
  uint16_t* toff = reinterpret_cast<uint16_t*>(wc + kPW * hw);
  uint16_t* trun = toff + 2 * hw;
  uint16_t* ctot = trun + 2 * hw;
  uint16_t* kstart = ctot + 2 * hw;
  uint32_t* wsum = reinterpret_cast<uint32_t*>(kstart + 2 * hw);
  uint32_t* ctot32 = reinterpret_cast<uint32_t*>(ctot);
  uint32_t* hslot = wsum + 16;
  uint64_t* hh64 = reinterpret_cast<uint64_t*>(hslot + kHotSlots);
  uint64_t* hkey = hh64 + kHotMax;
  uint32_t* hident = reinterpret_cast<uint32_t*>(hkey + kHotMax);
  // coordination engines (inst_id): each record's instance id, written into XRec.pad so k_apply_coord gets it with the
  // record instead of a dependent gather per chunk (tile_lds_bytes(..., ids) appends this plane)
  uint64_t* rpad = reinterpret_cast<uint64_t*>(hident + kHotMax);

  // sb_kind in LDS: a global load whose value is used right away waits for every load issued before it (one
  // in-order counter)
  __shared__ uint8_t skind[kMaxSb];
  PH_DECL
  const uint32_t t = threadIdx.x, w = t >> 6, l = t & 63;
  for (uint32_t q = t; q < sb_val; q += kPT) skind[q] = sb_kind[q];
  const uint64_t cbase0 = clock_base ? *clock_base : 0;
  const bool deferred = (ext_flags & kExtDeferred) != 0;
  // the log clock must not go backwards (each row against the row before it; replaces k_time_check when the batch
  // has no barrier rows, which are not partitioned)
  const bool tcheck = TCK && ctime && (ext_flags & kExtTimeCheck);
  uint32_t tbad = 0;
  uint32_t nhot = 0;
  if (map_bits) {
    nhot = *hot_n;
    for (uint32_t q = t; q < kHotSlots; q += kPT) hslot[q] = 0xFFFFFFFFu;
    if (t < nhot) {
      const HotKey hk = hot[t];
      hh64[t] = hk.h64;
      hkey[t] = hk.key;
      hident[t] = hk.ident;
    }
  }
  for (uint32_t k = t; k < hw; k += kPT) ctot32[k] = 0;
  lds_barrier();
  if (t < nhot) {
    uint32_t q = (uint32_t)(hh64[t] >> 32) & (kHotSlots - 1);
    while (atomicCAS(&hslot[q], 0xFFFFFFFFu, t) != 0xFFFFFFFFu) q = (q + 1) & (kHotSlots - 1);
  }
  lds_barrier();
  const uint32_t sb_hot = sb_val + (map_bits ? (1u << map_bits) : 0u);
  const uint32_t map_lim = sb_hot + (map_bits ? (uint32_t)kHotMax : 0u);  // map regions + hot-key buckets
  const uint64_t tile0 = lo + (uint64_t)blockIdx.x * kTile;
  const uint64_t tile1 = tile0 + kTile < hi ? tile0 + kTile : hi;
  const uint32_t tbase = blockIdx.x * kTile;
  auto row_of = [&](int q) -> uint64_t {  // commit q of this thread: chunk q / J, slot (w, q % J, l)
    return tile0 + (uint64_t)(q / J) * C + (uint64_t)w * (kWave * J) + (uint64_t)(q % J) * kWave + l;
  };

  // ---- 0. route every commit of the tile (one batch of loads per stage), histogram from registers ----
  uint32_t rp[kXQ];     // resource slot | super-bucket << 17; kRpDead: unknown session / past the batch
  uint32_t tp[kXQ / 4]; // resource type | kTpWalk (a k_apply_value record), 4 per word
#pragma unroll
  for (int q = 0; q < kXQ / 4; ++q) tp[q] = 0;
#pragma unroll
#ifndef CC_PART_EXT_ROUTE_SPLIT
#define CC_PART_EXT_ROUTE_SPLIT 2  // route stages in two halves of 8 rows (1: all 16 at once, measured no faster)
#endif
  for (int hq = 0; hq < kXQ; hq += kXQ / CC_PART_EXT_ROUTE_SPLIT) {
    constexpr int H = kXQ / CC_PART_EXT_ROUTE_SPLIT;
    uint32_t rr[H], fl[H];
    uint64_t ky[H];
    // an engine with maps loads every row's key and flags with its instance (one HBM round trip, not a fourth one
    // after the instance -> resource -> type gathers; rows that are not keyed ignore them)
#pragma unroll
    for (int u = 0; u < H; ++u) {
      const uint64_t i = row_of(hq + u);
      rr[u] = i < tile1 ? inst[i] : kNoRes;
      fl[u] = 0;
      ky[u] = 0;
      if (map_bits) {  // (block-uniform)
        const uint64_t ic = i < tile1 ? i : tile0;
        fl[u] = flags[ic];
        ky[u] = ckey[ic];
      }
    }
#pragma unroll
    for (int u = 0; u < H; ++u) rr[u] = rr[u] < max_inst ? inst_res[rr[u]] : kNoRes;
    uint32_t ty[H];
#pragma unroll
    for (int u = 0; u < H; ++u) ty[u] = rr[u] != kNoRes ? res_type[rr[u]] : 0u;
#pragma unroll
    for (int u = 0; u < H; ++u) {
      const int q = hq + u;
      rp[q] = kRpDead;
      if (rr[u] == kNoRes) continue;
      const uint32_t r = rr[u];
      uint32_t k;
      if (is_keyed(ty[u])) {
        const uint32_t kt = CC_FLAG_KTAG(fl[u]);
        const uint64_t h = map_hash(r, kt, ky[u]);
        k = sb_val + (uint32_t)(h >> (64 - map_bits));
        if (nhot) {
          const uint32_t id = mw_ident(r, kt);
          for (uint32_t s = (uint32_t)(h >> 32) & (kHotSlots - 1);; s = (s + 1) & (kHotSlots - 1)) {
            const uint32_t x = hslot[s];
            if (x == 0xFFFFFFFFu) break;
            if (hh64[x] == h && hident[x] == id && hkey[x] == ky[u]) {
              k = sb_hot + x;
              break;
            }
          }
        }
      } else if (sbq_base && skind[r >> kSbShift]) {
        k = sbq_base + (r >> 6);  // quarter bucket (k_apply_coord)
      } else {
        k = r >> kSbShift;
      }
      rp[q] = r | (k << 17);
      const uint32_t vw = ty[u] == CC_RES_VALUE && !skind[r >> kSbShift] ? kTpWalk : 0u;
      tp[q / 4] |= (ty[u] | vw) << (8 * (q % 4));
      atomicAdd(&ctot32[k >> 1], 1u << (16 * (k & 1)));
    }
  }
  lds_barrier();
  {
    uint16_t* row = ttab + (uint64_t)blockIdx.x * (sb + 1);
    uint32_t run = 0;
    for (uint32_t k0 = 0; k0 < sb; k0 += kPT) {  // block-uniform
      const uint32_t k = k0 + t;
      uint32_t inc = k < sb ? ctot[k] : 0, v = inc;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d, 64);
        if (l >= (uint32_t)d) inc += y;
      }
      lds_barrier();
      if (l == 63) wsum[w] = inc;
      lds_barrier();
      uint32_t pre = 0, all = 0;
      for (uint32_t q = 0; q < (uint32_t)kPW; ++q) {
        const uint32_t x = wsum[q];
        pre += q < w ? x : 0;
        all += x;
      }
      if (k < sb) {
        toff[k] = run + pre + inc - v;
        trun[k] = 0;
        row[k] = (uint16_t)(run + pre + inc - v);
      }
      run += all;
    }
    if (t == 0) row[sb] = (uint16_t)run;  // live commits of the tile (<= 16384)
  }
  PH(0);

  // ---- chunks: raw columns of chunk ch + 1 requested at the top of chunk ch ----
  uint32_t in[J], mt[J], fl[J];
  u64x2 ab[J];
  uint64_t kk[J], ii[J], xa[J], t0v[J], t1v[J];
#if !CC_PART_EXT_LATE
  uint32_t nin[J], nmt[J], nfl[J];
  u64x2 nab[J];
  uint64_t nkk[J], nii[J], nxa[J], nt0[J], nt1[J];
#endif
  // a lock record's raw columns ride in the slots it does not use: ab = (clock, clock of the commit before), kk
  // unused, xa = timeout
  // the route registers rotate by J per chunk: rp[0..J) = this chunk, rp[J..2J) = the next (compile-time indices
  // in a rolled loop)
  // Raw loads only: a select or an ALU op on a loaded value makes the wave wait for that load right there (one
  // in-order counter), i.e. for the whole next chunk's columns at the top of this chunk.  So op and flags stay in
  // two registers until the take, a lock's clocks arrive in ab by address (ctime instead of ca / cb), and the
  // fields a dead row or a type does not use keep whatever was loaded (nothing reads them: placement skips dead
  // rows, the record's fields are picked by type at use).
  auto load_raw = [&](uint32_t ch, int qb, uint32_t (&in_)[J], uint32_t (&mt_)[J], uint32_t (&fl_)[J], u64x2 (&ab_)[J],
                      uint64_t (&kk_)[J], uint64_t (&ii_)[J], uint64_t (&xa_)[J], uint64_t (&t0_)[J], uint64_t (&t1_)[J]) {
#if CC_PART_EXT_UNCOND
    // every column the batch has, for every row (loads under the wave's full mask: no per-type divergent loads)
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int q = qb + j;
      const uint64_t i0 = tile0 + (uint64_t)ch * C + (uint64_t)w * (kWave * J) + (uint64_t)j * kWave + l;
      const uint64_t i = i0 < tile1 ? i0 : lo;
      const uint32_t ty = ((tp[q / 4] >> (8 * (q % 4))) & 0xFFu) & ~kTpWalk;
      const bool lock = ty == CC_RES_LOCK;
      in_[j] = inst[i];
      mt_[j] = op[i];
      fl_[j] = flags[i];
      const uint64_t* pa = lock ? (ctime ? ctime + i : nullptr) : (ca ? ca + i : nullptr);
      // (a keyed record's b is not staged: MRec drops it, and replaceIfPresent reads it from the batch by row)
      const uint64_t* pb = lock ? (ctime && i > 0 ? ctime + (i - 1) : nullptr) : (cb && !is_keyed(ty) ? cb + i : nullptr);
      uint64_t av = 0, bv = 0;
      if (pa) av = *pa;
      if (pb) bv = *pb;
      ab_[j] = u64x2{av, bv};
      kk_[j] = ckey ? ckey[i] : 0;
      xa_[j] = caux ? caux[i] : 0;
      ii_[j] = cidx ? cidx[i] : 0;
      if (TCK) {  // compared at the take (kErrTime)
        t0_[j] = ctime ? ctime[i] : 0;
        t1_[j] = ctime ? ctime[i > 0 ? i - 1 : i] : 0;
      }
    }
    return;
#endif
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int q = qb + j;
      const uint64_t i = tile0 + (uint64_t)ch * C + (uint64_t)w * (kWave * J) + (uint64_t)j * kWave + l;
      in_[j] = kNoRes;
      mt_[j] = 0;
      fl_[j] = 0;
      ab_[j] = u64x2{0, 0};
      kk_[j] = ii_[j] = xa_[j] = 0;
      if (rp[q] == kRpDead) continue;
      const uint32_t tyb = (tp[q / 4] >> (8 * (q % 4))) & 0xFFu, ty = tyb & ~kTpWalk;
      in_[j] = inst[i];
      mt_[j] = op[i];
      fl_[j] = flags[i];
      if (ty == CC_RES_LOCK) {  // clock of this commit and of the one before it (deterministic log time)
        ab_[j].x = ctime ? ctime[i] : 0;
        ab_[j].y = ctime && i > 0 ? ctime[i - 1] : 0;
        xa_[j] = caux ? caux[i] : 0;
        ii_[j] = cidx ? cidx[i] : 0;
        continue;
      }
      ab_[j].x = ca[i];
      ab_[j].y = cb[i];
      if (tyb & kTpWalk) continue;  // k_apply_value records: the encoded operands only
      ii_[j] = cidx ? cidx[i] : 0;
      {
        kk_[j] = ckey ? ckey[i] : 0;
        if (is_keyed(ty)) xa_[j] = caux ? caux[i] : 0;
      }
    }
  };
  load_raw(0, 0, in, mt, fl, ab, kk, ii, xa, t0v, t1v);
  // the clock check of a chunk's rows (TCK), at its take
  auto tcheck_rows = [&](uint32_t ch, const uint64_t (&a_)[J], const uint64_t (&b_)[J]) {
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const uint64_t i0 = tile0 + (uint64_t)ch * C + (uint64_t)w * (kWave * J) + (uint64_t)j * kWave + l;
      tbad |= tcheck && i0 < tile1 && i0 > 0 && a_[j] < b_[j] ? 1u : 0u;
    }
  };
  // instance ids of the working chunk's records: requested when its instance slots are taken into the working
  // registers (here for chunk 0, at the take for the others; CC_PART_EXT_LATE: after the previous chunk's write-out,
  // whose stores were issued after the loads they wait for, so that wait never covers them), used at
  // the placement
  uint64_t idv[J];
  auto issue_ids = [&]() {
#pragma unroll
    for (int j = 0; j < J; ++j) idv[j] = IDS ? inst_id[in[j] < max_inst ? in[j] : 0u] : 0ull;
  };
#if !CC_PART_EXT_LATE
#pragma unroll
  for (int j = 0; j < J; ++j) mt[j] |= fl[j] << 8;
  if (TCK) tcheck_rows(0, t0v, t1v);
#endif
  issue_ids();
#if CC_PART_EXT_UNROLL
#pragma unroll
#else
#pragma unroll 1
#endif
  for (uint32_t ch = 0; ch < (uint32_t)kXCh; ++ch) {
    const uint64_t cbase = tile0 + (uint64_t)ch * C;
    if (cbase >= tile1) break;  // block-uniform
    const bool more = ch + 1 < (uint32_t)kXCh && cbase + C < tile1;
#if !CC_PART_EXT_LATE
    if (more) load_raw(ch + 1, J, nin, nmt, nfl, nab, nkk, nii, nxa, nt0, nt1);
#endif
    for (uint32_t k = t; k < kPW * hw; k += kPT) wc[k] = 0;
    lds_barrier();
    PH(6);
#if CC_PART_EXT_LATE
    // this chunk's columns (loaded before the loop, or after the previous chunk's placement)
#pragma unroll
    for (int j = 0; j < J; ++j) mt[j] |= fl[j] << 8;
    if (TCK) tcheck_rows(ch, t0v, t1v);
#endif
    // the records of this chunk (compute only: every column arrived with the chunk's loads)
    uint32_t sk[J], loc[J], res[J], meta[J], xs[J];
    bool live[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int q = j;
      live[j] = rp[q] != kRpDead;
      res[j] = rp[q] & 0x1FFFFu;
      sk[j] = live[j] ? rp[q] >> 17 : 0u;
      meta[j] = mt[j];
      xs[j] = in[j];
      if (!live[j]) continue;
      const uint32_t tyb = (tp[q / 4] >> (8 * (q % 4))) & 0xFFu, ty = tyb & ~kTpWalk;
      if (is_keyed(ty)) {
        if (ty == CC_RES_SET || ty == CC_RES_MULTIMAP) {  // an element / multimap key holds Boolean TRUE
          uint32_t fl = (meta[j] >> 8) & 0xFF;
          const uint32_t mop = ty == CC_RES_SET ? set_as_map_op(meta[j] & 0xFF) : mmap_as_map_op(meta[j] & 0xFF, fl & 7u);
          if (mop == CC_OP_MAP_PUTIFABSENT) {
            fl = (fl & ~7u) | CC_TAG_BOOL;
            ab[j].x = 1;
          }
          meta[j] = (meta[j] & ~0xFFFFu) | mop | (fl << 8);
        }
        // map slot | row in the tile << 17 (MRec.rr: replaceIfPresent's b is read from the batch by row)
        xs[j] = res[j] | ((uint32_t)(w * (kWave * J) + j * kWave + l + ch * C) << 17);
        if ((int64_t)xa[j] > 0 && ty != CC_RES_MULTIMAP) meta[j] |= kMetaTtl;
        // a map cleared in this sub-batch: the commit's clear epoch (the map kernels read it from the meta word)
        if (clr.mflag && ty == CC_RES_MAP)  // (0 for a map not cleared in the sub-batch: one load, no flag test)
          meta[j] |= clr_epoch(clr, res[j], cbase + (uint64_t)w * (kWave * J) + (uint64_t)j * kWave + l) << kMetaEpochShift;
      } else if (tyb & kTpWalk) {
        value_encode(meta[j] & 0xFF, (meta[j] >> 8) & 0xFF, ab[j].x, ab[j].y, meta[j], ab[j]);
      } else if (ty == CC_RES_LOCK) {
        const uint64_t i = cbase + (uint64_t)w * (kWave * J) + (uint64_t)j * kWave + l;
        const uint64_t clk = ab[j].x > cbase0 ? ab[j].x : cbase0;
        const uint64_t prev = i > 0 && ctime ? (ab[j].y > cbase0 ? ab[j].y : cbase0) : cbase0;
        ab[j].x = deferred ? prev : clk;
        ab[j].y = xa[j];
        kk[j] = clk;
      }
      const uint32_t sh = 16 * (sk[j] & 1);
      loc[j] = (atomicAdd(&wc[w * hw + (sk[j] >> 1)], 1u << sh) >> sh) & 0xFFFF;
    }
    lds_barrier();
    PH(1);
    // per super-bucket: exclusive prefix over waves (packed halves) and chunk totals; chunk-sorted starts
    for (uint32_t kw = t; kw < hw; kw += kPT) {
      uint32_t r0 = 0, r1 = 0;
      for (uint32_t q = 0; q < (uint32_t)kPW; ++q) {
        const uint32_t c = wc[q * hw + kw];
        wc[q * hw + kw] = r0 | (r1 << 16);
        r0 += c & 0xFFFF;
        r1 += c >> 16;
      }
      ctot32[kw] = r0 | (r1 << 16);
    }
    lds_barrier();
    PH(2);
    uint32_t nlive = 0;
    for (uint32_t k0 = 0; k0 < sb; k0 += kPT) {  // block-uniform
      const uint32_t k = k0 + t;
      const uint32_t v = k < sb ? ctot[k] : 0;
      uint32_t inc = v;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d, 64);
        if (l >= (uint32_t)d) inc += y;
      }
      lds_barrier();
      if (l == 63) wsum[w] = inc;
      lds_barrier();
      uint32_t pre = 0, all = 0;
      for (uint32_t q = 0; q < (uint32_t)kPW; ++q) {
        const uint32_t x = wsum[q];
        pre += q < w ? x : 0;
        all += x;
      }
      if (k < sb) kstart[k] = nlive + pre + inc - v;
      nlive += all;
    }
    lds_barrier();
    PH(3);
    // place records in LDS in sorted order; per-commit tile-local position (stored below)
    uint32_t cp[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
      cp[j] = 0xFFFF;
      const uint64_t i = cbase + (uint64_t)w * (kWave * J) + (uint64_t)j * kWave + l;
      if (i >= tile1 || !live[j]) continue;
      const uint32_t pre = (wc[w * hw + (sk[j] >> 1)] >> (16 * (sk[j] & 1))) & 0xFFFF;
      const uint32_t within = pre + loc[j];
      const uint32_t s = kstart[sk[j]] + within;
      rab[s] = ab[j];
      rmeta[s] = meta[j] | ((res[j] & ((1u << kSbShift) - 1)) << 16);
      rres[s] = xs[j];
      rkey[s] = kk[j];
      ridx[s] = ii[j];
      if (IDS) rpad[s] = idv[j];
      cp[j] = toff[sk[j]] + trun[sk[j]] + within;
      const uint32_t k = sk[j];
      const uint32_t kind = k < sb_val && !skind[k] ? kRgValue : (k >= sb_val && k < map_lim ? (k >= sb_hot ? kRgHot : kRgMap) : kRgXRec);
      rsb[s] = (uint16_t)(cp[j] | (kind << 14));
    }
    lds_barrier();
    PH(4);
    // The next chunk's columns are taken into the working registers HERE, before this chunk's stores: waiting for
    // a load also waits for every memory op issued before it (one in-order counter), so the wait covers only the
    // previous chunk's stores, long done, and not the ones below.
#if CC_PART_EXT_LATE
    // the working registers are free (the chunk's records are in LDS): the next chunk's columns fly during the
    // write-out below (its stores are issued after these loads, so waiting for the loads never waits for them)
    if (more) load_raw(ch + 1, J, in, mt, fl, ab, kk, ii, xa, t0v, t1v);
#else
    if (more) {
#pragma unroll
      for (int j = 0; j < J; ++j) {
        in[j] = nin[j];
        mt[j] = nmt[j] | (nfl[j] << 8);
        ab[j] = nab[j];
        kk[j] = nkk[j];
        ii[j] = nii[j];
        xa[j] = nxa[j];
      }
      issue_ids();
      if (TCK) tcheck_rows(ch + 1, nt0, nt1);
    }
#endif
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const uint64_t i = cbase + (uint64_t)w * (kWave * J) + (uint64_t)j * kWave + l;
      if (i < tile1) cpos[i - lo] = (uint16_t)cp[j];
    }
    // write the chunk out run by run (contiguous): k_apply_value records as (meta, operands) columns, map records as
    // one 32-byte MRec (2 pieces), every other record as one 48-byte XRec.  Lanes take consecutive 16-byte pieces
    // (piece p = part p % np of sorted record p / np), so a wave's store covers a run contiguously; one lane per record
    // (three stores at a 48-byte stride) left every piece its own partial-line write request (WRITE_SIZE 99 B per
    // commit against 50).  np = 2 when no record is an XRec (no coordination, no value events): a map record's two
    // pieces then take two lanes, not three with one idle (c3: the write-out was 37 % of the partition).
    const uint32_t np = (IDS || sbq_base || (ext_flags & kExtValue)) ? 3u : 2u;  // (block-uniform)
    for (uint32_t p = t; p < np * nlive; p += kPT) {
      const uint32_t s = np == 2u ? p >> 1 : p / 3, part = p - np * s;
      const uint32_t gw = rsb[s], g = tbase + (gw & kRgPos), kind = gw >> 14;
      if (kind == kRgValue) {
        if (part == 0) {
          st_meta[g] = rmeta[s];
          st_ab[g] = rab[s];
        }
      } else if (kind >= kRgMap) {
        if (part == 2) continue;
        if (part == 0 && hot_meta && kind == kRgHot) hot_meta[g] = rmeta[s];
        const u64x2 v = part == 0 ? u64x2{rab[s].x, rkey[s]} : u64x2{ridx[s], (uint64_t)rmeta[s] | ((uint64_t)rres[s] << 32)};
        reinterpret_cast<u64x2*>(mrec + g)[part] = v;
      } else {
        u64x2 v;
        if (part == 0) v = rab[s];
        else if (part == 1) v = u64x2{rkey[s], ridx[s]};
        else v = u64x2{(uint64_t)rmeta[s] | ((uint64_t)rres[s] << 32), IDS ? rpad[s] : 0ull};
        reinterpret_cast<u64x2*>(xrec + g)[part] = v;
      }
    }
#if CC_PART_EXT_LATE
    if (more) issue_ids();  // the next chunk's instance ids (its instance column arrived during the write-out)
#endif
    lds_barrier();
    PH(5);
    for (uint32_t k = t; k < sb; k += kPT) trun[k] += ctot[k];
#pragma unroll
    for (int q = 0; q + J < kXQ; ++q) rp[q] = rp[q + J];  // rotate to the next chunk
#pragma unroll
    for (int q = 0; q < kXQ / 4; ++q) tp[q] = (tp[q] >> (8 * J)) | (q + 1 < kXQ / 4 ? tp[q + 1] << (32 - 8 * J) : 0u);
  }
  PH_FLUSH(g_ph_partx);
  if (tbad) atomicOr(err_out, kErrTime);
}

// chunk size of k_part_ext for sb buckets: with maps 2048 while its LDS fits (plus the kernel's static 512 B), else
// 1024; without maps 1024 (no scratch spills at J = 1: c5's partition 4.16 -> 3.98 ms per step; c3's is 1% slower
// at 1024, profiles/r03/ab_chunk); 0: none fits
size_t part_ext_chunk(uint32_t sb, bool maps, bool ids) {
  constexpr size_t kLds = 160u * 1024u - kMaxSb;
  static const bool small = diag_env("CC_PART_EXT_1024");  // A/B: 1024-commit chunks whenever they fit
  if (maps && !small && tile_lds_bytes(sb, true, kChunkMaps, ids) <= kLds) return kChunkMaps;
  if (tile_lds_bytes(sb, true, kPT, ids) <= kLds) return kPT;
  return 0;
}

int launch_part_ext(const PartArgs& a, uint32_t tiles, hipStream_t st) {
  const bool ids = a.inst_id != nullptr, tck = a.time && (a.ext_flags & kExtTimeCheck);
  // (with the clock check, 2048-commit chunks spill at the 128-VGPR cap -- 52-64 B per lane -- and a spill reload waits
  // behind the next chunk's loads: such engines stage 1,024-commit chunks, which need no scratch)
  size_t c = part_ext_chunk(a.sb, a.map_bits != 0, ids);
  if (c == (size_t)kChunkMaps && tck) c = kPT;
  if (c == 0) return -1;
  auto kern = c == (size_t)kChunkMaps
                  ? (ids ? k_part_ext<kChunkMaps, true, false> : k_part_ext<kChunkMaps, false, false>)
                  : (ids ? (tck ? k_part_ext<kPT, true, true> : k_part_ext<kPT, true, false>)
                         : (tck ? k_part_ext<kPT, false, true> : k_part_ext<kPT, false, false>));
  hipLaunchKernelGGL(kern, dim3(tiles), dim3(kPT), tile_lds_bytes(a.sb, true, c, a.inst_id != nullptr), st, a.inst, a.op,
                     a.flags, a.a, a.b, a.key, a.index, a.aux, a.time, a.clock_base, a.ext_flags, a.lo, a.hi, a.inst_id, a.inst_res,
                     a.res_type, a.sb_kind, a.max_inst, a.sb, a.sb_val, a.map_bits, a.sbq_base, a.hot, a.hot_n,
                     a.st_meta, a.st_ab, a.xrec, a.mrec, a.map_bits ? a.hot_meta : nullptr, a.cpos, a.ttab, a.clr, a.err);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace cc
