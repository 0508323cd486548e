// apply_map.hip — MapState apply (DistributedMap key operations) on a GPU open-addressing table.
//
// Table: 2^map_bits regions of 2048 entries in HBM.  A key (map slot, key tag, key payload) lives in the region
// picked by the top bits of map_hash and is found by linear probing from the hash's low 11 bits.  Entry =
// key u64 | word u32 (slot, key tag, USED, PRESENT, value tag) | value u64 | commit index u64 | insert index
// u64 (the commit index that created the HashMap node: Java iteration order within a bucket).
// A removed key keeps its entry (USED, not PRESENT) so that probe chains stay intact; entries of a deleted map
// are marked DEAD.  A region is compacted (live entries re-inserted) when a launch finds it more than 3/4 used.
//
// One 1024-thread workgroup (512 in TTL mode) owns one region for the whole launch: it loads the region into LDS, walks the
// region's staged commits (its run in every partition tile, in log order) in chunks of 1024 (512), and writes the
// region back.  Per chunk:
//   1. binding: commits that can create a node (put, putIfAbsent) find or claim their key's entry — rounds of
//      LDS compare-and-swap; a claim is marked PENDING until the next round so no thread compares against a
//      key that is not yet written;
//   2. lookup: every other key op only finds its entry (a key that is unbound after step 1 is absent at that
//      commit: nothing earlier in the log can have created it);
//   3. a stable counting sort of the chunk by entry (LDS atomics with return, one wave at a time: lane order
//      within a wave, wave order across waves = log order);
//   4. each entry's commits are applied in log order (the reference's single state-machine thread, restricted
//      to one key: different keys of a map are independent, MapState.java:32-289): a segmented scan of the
//      commits' transformers (map_ops.h) gives every commit its pre-state at once; an entry whose run holds a
//      value-comparing op (removeIfPresent/replaceIfPresent) is walked by one thread.
//
// Per-op semantics restate MapState (collections/src/main/java/io/atomix/collections/state/MapState.java):
//   containsKey :38-44, get :65-72, getOrDefault :77-84, put :89-110, putIfAbsent :115-133, remove :138-154,
//   removeIfPresent :159-178, replace :183-202, replaceIfPresent :207-228 (stores `value`, compares `replace`).
// containsValue/size/isEmpty/clear and Delete read or reset a whole map: they are batch barriers applied by
// map_wide.hip.  Not applied on the GPU (the batch fails with CC_ERR_UNSUPPORTED): put/putIfAbsent/replace/
// replaceIfPresent with ttl > 0 before the engine enters TTL mode (k_apply_map<true>: see below).
#include "common.h"
#include "engine_internal.h"
#include "map_ops.h"

namespace cc {

#ifdef CC_PHASE_TIMING
__device__ unsigned long long g_ph_map[kPhases];
int phase_read_map(uint64_t* out) {
  unsigned long long z[kPhases] = {};
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ph_map), sizeof z) != hipSuccess ||
      hipMemcpyToSymbol(HIP_SYMBOL(g_ph_map), z, sizeof z) != hipSuccess)
    return CC_ERR_HIP;
  return CC_OK;
}
#endif

#ifndef CC_MAP_MT
#define CC_MAP_MT 512  // threads of k_apply_map<false>
#endif
#ifndef CC_MAP_CHUNK
#define CC_MAP_CHUNK 2048  // commits per chunk of k_apply_map<false> (CC_MAP_CHUNK / CC_MAP_MT per thread)
#endif
constexpr uint32_t kNoRef = 0xFFFFFFFFu;
constexpr uint32_t kNoEnt = 0xFFFFu;
constexpr uint32_t kEntFull = 0xFFFEu;

__device__ inline uint32_t map_ident_of(uint32_t res, uint32_t flags) { return mw_ident(res, CC_FLAG_KTAG(flags)); }

// The run transformers of map_ops.h (Comp) packed into two words for the chunk scan: per branch (absent / present
// before the run) kind bits 0-1 | value record bits 2-13 | node record bits 14-25 (kPkOrig: the input's node);
// records are chunk slots (< 4095).  A scan step then moves 2 words between lanes instead of 6.
struct PComp {
  uint32_t A, P;
};
constexpr uint32_t kPkOrig = 0xFFFu;
__device__ inline uint32_t pk_kind(uint32_t b) { return b & 3u; }
__device__ inline uint32_t pk_v(uint32_t b) { return (b >> 2) & 0xFFFu; }
__device__ inline uint32_t pk_n(uint32_t b) { return (b >> 14) & 0xFFFu; }
__device__ inline uint32_t pk_br(uint32_t kind, uint32_t v, uint32_t n) { return kind | (v << 2) | (n << 14); }
__device__ inline PComp pc_identity() { return PComp{pk_br(kBrAbsent, 0, 0), pk_br(kBrKeep, 0, 0)}; }
__device__ inline uint32_t pc_apply_present(const PComp& g, uint32_t v, uint32_t n) {  // g on present(v, n)
  const uint32_t k = pk_kind(g.P);
  if (k == kBrKeep) return pk_br(kBrPresent, v, n);
  if (k == kBrPresent) return pk_br(kBrPresent, pk_v(g.P), pk_n(g.P) == kPkOrig ? n : pk_n(g.P));
  return pk_br(kBrAbsent, 0, 0);
}
__device__ inline PComp pc_compose(const PComp& f, const PComp& g) {  // f first, then g
  PComp r;
  r.A = pk_kind(f.A) == kBrAbsent ? g.A : pc_apply_present(g, pk_v(f.A), pk_n(f.A));
  const uint32_t k = pk_kind(f.P);
  r.P = k == kBrKeep ? g.P : (k == kBrPresent ? pc_apply_present(g, pk_v(f.P), pk_n(f.P)) : g.A);
  return r;
}
__device__ inline PComp pc_element(uint32_t m, uint32_t s) {  // element() of map_ops.h, packed
  PComp c = pc_identity();
  if (!map_applied(m)) return c;
  switch (smeta_op(m)) {
    case CC_OP_MAP_PUT:
      c.A = pk_br(kBrPresent, s, s);
      c.P = pk_br(kBrPresent, s, kPkOrig);
      break;
    case CC_OP_MAP_PUTIFABSENT:
      c.A = pk_br(kBrPresent, s, s);
      break;
    case CC_OP_MAP_REMOVE:
      c.P = pk_br(kBrAbsent, 0, 0);
      break;
    case CC_OP_MAP_REPLACE:
      c.P = pk_br(kBrPresent, s, kPkOrig);
      break;
  }
  return c;
}
__device__ inline PComp pc_shfl_up(const PComp& c, int d) {
  return PComp{(uint32_t)__shfl_up((int)c.A, d, 64), (uint32_t)__shfl_up((int)c.P, d, 64)};
}
// materialize_ref of map_ops.h for a packed composite (vref / nref: kOrig when unchanged)
__device__ inline void pc_materialize(const PComp& c, uint32_t w0, uint64_t v0, const uint32_t* rmeta, const u64x2* rab,
                                      uint32_t& w, uint64_t& v, uint32_t& vref, uint32_t& nref) {
  const uint32_t b = (w0 & kMwPresent) ? c.P : c.A;
  vref = nref = kOrig;
  if (pk_kind(b) == kBrKeep) {
    w = w0;
    v = v0;
  } else if (pk_kind(b) == kBrAbsent) {
    w = w0 & ~(kMwPresent | kMwVtagMask);
    v = 0;
  } else {
    const uint32_t rv = pk_v(b), tag = CC_FLAG_TAG_A(smeta_flags(rmeta[rv]));
    w = (w0 & ~(kMwVtagMask | kMwUnseen)) | kMwPresent | (tag << 21);
    v = tag ? rab[rv].x : 0;
    vref = rv;
    nref = pk_n(b) == kPkOrig ? kOrig : pk_n(b);
  }
}

// TTL: the map table has live TTL timers (MapState.java:91-93,119-121,189-192,218-220).  Every entry then carries
// its timer's deadline (tbl_dl, 0 = none) and every run is walked sequentially: before each commit the entry
// expires if its deadline is <= the clock at which the reference last fired timers (module mode: this commit's
// clock; manager mode: the previous commit's, A8), and a commit that stores a value re-arms or cancels the timer.
// The per-record clocks come from the input columns through map_row (staging position -> batch row).
// a node created in entry e by this launch (LDS bitmaps: once -> tc1, twice or more -> tc2 as well)
__device__ inline void claim_mark(uint32_t* tc1, uint32_t* tc2, uint32_t e) {
  const uint32_t bit = 1u << (e & 31);
  if (atomicOr(&tc1[e >> 5], bit) & bit) atomicOr(&tc2[e >> 5], bit);
}

template <bool TTL, bool CLR>
__global__ __launch_bounds__(CC_MAP_MT) void k_apply_map(const MRec* __restrict__ xr, const uint64_t* __restrict__ cb, uint64_t row0,
                                                  const uint16_t* __restrict__ ttab,
                                                  uint32_t tiles, uint32_t sb, uint32_t sb_val, uint64_t* __restrict__ tbl_key,
                                                  uint32_t* __restrict__ tbl_word, uint64_t* __restrict__ tbl_val,
                                                  uint64_t* __restrict__ tbl_ci, uint64_t* __restrict__ tbl_ins,
                                                  uint64_t* __restrict__ tbl_claim, const uint64_t* __restrict__ idx0p,
                                                  unsigned long long* __restrict__ dropped, const uint64_t* __restrict__ cgen,
                                                  CsetEnt* __restrict__ cset, uint64_t cset_mask, uint32_t* __restrict__ cset_full,
                                                  uint64_t* __restrict__ tbl_dl, const uint32_t* __restrict__ map_row,
                                                  const uint64_t* __restrict__ ctime, const uint64_t* __restrict__ caux,
                                                  const uint64_t* __restrict__ clock_base, bool deferred,
                                                  uint8_t* __restrict__ rst_status, uint64_t* __restrict__ rst_value,
                                                  uint32_t* __restrict__ rst_msz, TtlEmit te, CvCtx cv, ClrCtx clr,
                                                  uint32_t* __restrict__ err_out) {
  constexpr int MT = TTL ? 512 : CC_MAP_MT;  // threads (the TTL variant's LDS holds deadlines: 512-commit chunks)
  constexpr int MEPer = kMapRegion / MT;  // table entries per thread
  constexpr int kMPer = TTL ? 1 : CC_MAP_CHUNK / CC_MAP_MT;  // commits per thread per chunk
  constexpr int kMCh = MT * kMPer;
  __shared__ uint64_t tkey[kMapRegion];
  __shared__ uint32_t tword[kMapRegion];
  __shared__ uint64_t tval[kMapRegion];
  // The entry's commit index (MapState.Value.commit) and node-creating index stay in HBM (tbl_ci / tbl_ins): the
  // kernel only records, per entry, the staging position of the commit that last rewrote them (kNoRef: none), and
  // the write-back gathers those commits' log indices.
  __shared__ uint32_t tcr[kMapRegion];
  __shared__ uint32_t tir[kMapRegion];
  // the chunk sorted by entry: rab u64x2 | rmeta u32 | rpos u32 (staging position: the commit index is read from
  // the staging area only for the commits that end up in tbl_ci / tbl_ins); the same bytes hold the per-wave entry
  // counts (u16, 2 per word) during the sort
  constexpr int NW = MT / kWave;
  constexpr int kRb = kMCh * 24 > NW * kMapRegion * 2 ? kMCh * 24 : NW * kMapRegion * 2;
  static_assert(kMPer * kWave < 65536, "per-wave counts are u16");
  __shared__ __align__(16) uint8_t rbuf[kRb];
  u64x2* const rab = reinterpret_cast<u64x2*>(rbuf);
  uint32_t* const rmeta = reinterpret_cast<uint32_t*>(rbuf + kMCh * 16);
  uint32_t* const rpos = reinterpret_cast<uint32_t*>(rbuf + kMCh * 20);
  uint32_t* const wtab = reinterpret_cast<uint32_t*>(rbuf);  // [NW][kMapRegion / 2]
  __shared__ uint16_t rent[kMCh];      // entry
  // results by chunk-list position (the commit's place in this region's list, c - c0): written to the staging
  // result rows at the end of the chunk, run by run (a region's list is contiguous within each partition tile)
  __shared__ uint16_t rci[kMCh];       // chunk-list position of the sorted record
  __shared__ uint64_t resv[kMCh];
  __shared__ uint8_t ress[kMCh];
  __shared__ int8_t resd[kMCh];  // the commit's change of its map's size (launch_map_size)
  __shared__ uint64_t tdl[TTL ? kMapRegion : 1];  // timer deadline of the entry (0: none)
  __shared__ uint64_t rfire[TTL ? kMCh : 1];      // clock of the last timer firing before the commit
  __shared__ uint64_t rdl[TTL ? kMCh : 1];        // deadline the commit arms if it stores (0: none)
  __shared__ uint32_t ecnt[kMapRegion + 1];  // commits per entry in the chunk -> run starts
  __shared__ uint32_t eflag[kMapRegion / 32];  // bit e: the entry's run holds a value-comparing op
  // the entry's claim (tbl_claim, the tree-bin test of map_wide.hip): bound by this launch (free at its load), and
  // how many nodes this launch created in it (one: its claim is that commit's index; more: the sub-batch's first)
  __shared__ uint32_t tnew[kMapRegion / 32], tc1[kMapRegion / 32], tc2[kMapRegion / 32];
  __shared__ uint16_t tmap[kMCh];              // the partition tile of each list position of the next chunk
  __shared__ PComp wcomp[MT / kWave];
  static_assert(kMCh < (int)kPkOrig, "packed composites address chunk slots in 12 bits");
  __shared__ uint32_t whead[MT / kWave];
  __shared__ uint32_t rstart[kMaxTiles];
  __shared__ uint32_t rpre[kMaxTiles + 1];
  __shared__ uint32_t wsum[MT / kWave];
  __shared__ uint32_t flag[3];
  __shared__ uint32_t used_total;
  // the clear epoch each entry's state is at (map_clear.hip: clears in the stream; 0 = the sub-batch start)
  __shared__ uint8_t eep[TTL ? 1 : kMapRegion];

  const uint32_t region = blockIdx.x, k = sb_val + region, t = threadIdx.x, w = t >> 6, l = t & 63;
  constexpr bool clr_live = !TTL && CLR;  // clears in the stream in this batch (map_clear.hip; its own instantiation)
  const uint64_t tb = (uint64_t)region * kMapRegion;
  uint32_t err = 0;
  PH_DECL

  // ---- load the region; compact it when more than 3/4 of its entries are bound ----
  if (t < 3) flag[t] = 0;
  if (t == 0) used_total = 0;
  for (uint32_t q = t; q <= kMapRegion; q += MT) ecnt[q] = 0;
  for (uint32_t q = t; q < kMapRegion / 32; q += MT) eflag[q] = tnew[q] = tc1[q] = tc2[q] = 0;
  {
    uint64_t ek[MEPer], ev[MEPer], edl[MEPer];
    uint32_t ew[MEPer], used = 0;
#pragma unroll
    for (int q = 0; q < MEPer; ++q) {
      const uint32_t e = q * MT + t;
      ek[q] = tbl_key[tb + e];
      ew[q] = tbl_word[tb + e];
      ev[q] = tbl_val[tb + e];
      edl[q] = TTL ? tbl_dl[tb + e] : 0;
      used += (ew[q] & kMwUsed) ? 1 : 0;
    }
    lds_barrier();
    atomicAdd(&used_total, used);
    lds_barrier();
    const bool compact = used_total > kMapRegion * 3 / 4;  // block-uniform
#pragma unroll
    for (int q = 0; q < MEPer; ++q) {
      const uint32_t e = q * MT + t;
      tkey[e] = ek[q];
      tword[e] = compact ? 0u : ew[q];
      tval[e] = ev[q];
      tcr[e] = kNoRef;
      tir[e] = kNoRef;
      if (TTL) tdl[e] = compact ? 0 : edl[q];
      else if (clr_live) eep[e] = compact ? 0 : clr.tbl_ep[tb + e];  // (a hot key's entry: its epoch after k_hot_apply)
    }
    lds_barrier();
    if (compact) {
      // the live entries' indices move with them (read all before any is written: __syncthreads orders HBM too)
      uint64_t eci[MEPer], eins[MEPer], ecl[MEPer];
#pragma unroll
      for (int q = 0; q < MEPer; ++q) {
        eci[q] = tbl_ci[tb + q * MT + t];
        eins[q] = tbl_ins[tb + q * MT + t];
        ecl[q] = tbl_claim[tb + q * MT + t];
      }
      __syncthreads();
      // live keys are distinct: claim the first free slot of each probe chain (no key comparisons needed)
#pragma unroll
      for (int q = 0; q < MEPer; ++q) {
        // a bound key that is absent now is dropped: it still counts toward its map's peak-size bound
        if ((ew[q] & kMwUsed) && !(ew[q] & (kMwPresent | kMwDead | kMwUnseen)) && dropped) {
          atomicAdd(&dropped[ew[q] & kMwSlotMask], 1ull);
          // the key leaves the table: kept in the compacted-key set of its map (the tree-bin test, map_wide.hip)
          const uint32_t ds = ew[q] & kMwSlotMask;
          cset_insert(cset, cset_mask, cset_full, ds, (ew[q] >> 17) & 3u, ek[q], cgen, ecl[q]);
        }
        if ((ew[q] & kMwPresent) && !(ew[q] & kMwDead)) {
          const uint32_t res = ew[q] & kMwSlotMask, kt = (ew[q] >> 17) & 3;
          uint32_t p = (uint32_t)map_hash(res, kt, ek[q]) & (kMapRegion - 1);
          while (atomicCAS(&tword[p], 0u, ew[q]) != 0u) p = (p + 1) & (kMapRegion - 1);
          tkey[p] = ek[q];
          tval[p] = ev[q];
          tbl_ci[tb + p] = eci[q];
          tbl_ins[tb + p] = eins[q];
          tbl_claim[tb + p] = ecl[q];
          if (TTL) tdl[p] = edl[q];
          else if (clr_live) eep[p] = clr.tbl_ep[tb + q * MT + t];  // (written back only at the end of the launch)
        }
      }
      __syncthreads();
    }
#pragma unroll
    for (int q = 0; q < MEPer; ++q) {  // entries free at the load (after compaction): a claim by this launch
      const uint32_t e = q * MT + t;
      if (tword[e] == 0u) atomicOr(&tnew[e >> 5], 1u << (e & 31));
    }
  }

  // ---- this region's list = its run in every partition tile, in tile order ----
  {
    constexpr int PT = kMaxTiles / MT;
    uint32_t len[PT], sum = 0;
#pragma unroll
    for (int q = 0; q < PT; ++q) {
      const uint32_t tt = t * PT + q;
      len[q] = 0;
      if (tt < tiles) {
        const uint16_t* row = ttab + (uint64_t)tt * (sb + 1);
        const uint32_t b0 = row[k], b1 = row[k + 1];
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
    lds_barrier();
    uint32_t run = inc - sum;
    for (uint32_t q = 0; q < w; ++q) run += wsum[q];
#pragma unroll
    for (int q = 0; q < PT; ++q) {
      const uint32_t tt = t * PT + q;
      if (tt < tiles) rpre[tt] = run;
      run += len[q];
    }
    if (t == MT - 1) rpre[tiles] = run;
    lds_barrier();
  }
  const uint32_t cnt = rpre[tiles];
  uint32_t round = 0;  // resolution rounds (continues across chunks: flag[] is a 3-deep ring)
  PH(0);

  // The working registers: the records of chunk c0 (this thread's: chunk order (w, j, l) = log order).  The next
  // chunk's are loaded into the same registers once this chunk's records sit sorted in LDS (after the placement),
  // and land while the chunk is applied.  They are stored as loaded (res = the raw MRec.rr word, ab.y unused) and
  // decoded at the top of their chunk: an op on a loaded value waits for the load right there (one in-order counter).
  uint32_t m[kMPer], res[kMPer], g[kMPer];
  u64x2 ab[kMPer];
  uint64_t key[kMPer];
  // tmap for the chunk at c0: each tile writes its own positions (one search per thread, not one per commit)
  auto build_map = [&](uint32_t c0) {
    const uint32_t cend = c0 + kMCh < cnt ? c0 + kMCh : cnt;
    uint32_t lo = 0, hi = tiles;  // last tile with rpre <= c0
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (rpre[mid] <= c0) lo = mid; else hi = mid;
    }
    for (uint32_t tt = lo + t; tt < tiles && rpre[tt] < cend; tt += MT) {
      const uint32_t a = rpre[tt] > c0 ? rpre[tt] : c0, b = rpre[tt + 1] < cend ? rpre[tt + 1] : cend;
      for (uint32_t c = a; c < b; ++c) tmap[c - c0] = (uint16_t)tt;
    }
  };
  auto load_chunk = [&](uint32_t c0) {
#pragma unroll
    for (int j = 0; j < kMPer; ++j) {
      const uint32_t c = c0 + w * (kWave * kMPer) + j * kWave + l;
      g[j] = 0xFFFFFFFFu;
      if (c < cnt) {
        const uint32_t lo = tmap[c - c0];
        g[j] = rstart[lo] + (c - rpre[lo]);
        const u64x2* rec = reinterpret_cast<const u64x2*>(xr + g[j]);  // (the log index is read at write-back)
        const u64x2 r0 = rec[0], r1 = rec[1];  // (a, key), (idx, meta | rr << 32)
        key[j] = r0.y;
        m[j] = (uint32_t)r1.y;
        res[j] = (uint32_t)(r1.y >> 32);
        ab[j].x = r0.x;
      }
    }
  };
  build_map(0);
  lds_barrier();
  load_chunk(0);
  // every thread has read tmap for chunk 0 before the first chunk's build_map(c0 + kMCh) overwrites it (without
  // this barrier a fast wave could rebuild tmap under a slow wave's chunk-0 lookups: wrong staging positions)
  lds_barrier();
  for (uint32_t c0 = 0; c0 < cnt; c0 += kMCh) {
    uint32_t ent[kMPer], rk[kMPer], ident[kMPer], p[kMPer];
    bool keyop[kMPer];
    const bool more = c0 + kMCh < cnt;  // block-uniform
    // the sort's per-wave counters (wtab aliases the chunk records of rbuf, free since the previous chunk's final
    // barrier); the binding rounds below always pass at least one barrier before the sort's atomics
    for (uint32_t q = t; q < (uint32_t)(NW * kMapRegion / 2); q += MT) wtab[q] = 0;
#pragma unroll
    for (int j = 0; j < kMPer; ++j) {
      ent[j] = kNoEnt;
      keyop[j] = false;
      if (g[j] != 0xFFFFFFFFu) {
        const uint32_t op = smeta_op(m[j]);
        const uint32_t rr = res[j];  // MRec.rr: map slot | row in the tile << 17
        res[j] = rr & kMwSlotMask;
        const uint64_t brow = (uint64_t)(g[j] / kTile) * kTile + (rr >> 17);  // (mrec_ab)
        ab[j].y = 0;
        if (op == CC_OP_MAP_REPLACEIFPRESENT && CC_FLAG_TAG_B(smeta_flags(m[j])) != CC_TAG_NULL) ab[j].y = cb[row0 + brow];
        // (a map cleared in this sub-batch: the commit's clear epoch is in meta bits 25-31, from k_part_ext)
        keyop[j] = map_key_op(op) && (TTL || !(map_reads_ttl(op) && (m[j] & kMetaTtl)));
        ident[j] = map_ident_of(res[j], smeta_flags(m[j]));
        p[j] = (uint32_t)map_hash(res[j], CC_FLAG_KTAG(smeta_flags(m[j])), key[j]) & (kMapRegion - 1);
      }
    }
    PH(1);
    // ---- 1. binding rounds (put / putIfAbsent) ----
    bool pend[kMPer];
#pragma unroll
    for (int j = 0; j < kMPer; ++j) pend[j] = false;
    for (;; ++round) {
      bool again = false;
#pragma unroll
      for (int j = 0; j < kMPer; ++j) {
        if (pend[j]) {  // claimed last round; its key is visible to everyone after that round's barrier
          atomicAnd(&tword[ent[j]], ~kMwPending);
          pend[j] = false;
        }
        if (!keyop[j] || ent[j] != kNoEnt || !map_binds(smeta_op(m[j]))) continue;
        for (uint32_t steps = 0;; ++steps) {
          if (steps == kMapRegion) {
            ent[j] = kEntFull;
            break;
          }
          uint32_t wv = tword[p[j]];
          if (wv == 0u) {
            wv = atomicCAS(&tword[p[j]], 0u, ident[j] | kMwPending);
            if (wv == 0u) {
              tkey[p[j]] = key[j];
              tval[p[j]] = 0;
              ent[j] = p[j];
              pend[j] = true;
              again = true;
              break;
            }
          }
          if (wv & kMwPending) {  // claimed this round by another commit: look again next round
            again = true;
            break;
          }
          if ((wv & kMwIdentMask) == ident[j] && tkey[p[j]] == key[j]) {
            ent[j] = p[j];
            break;
          }
          p[j] = (p[j] + 1) & (kMapRegion - 1);
        }
      }
      if (again) flag[round % 3] = 1;
      lds_barrier();
      const bool go = flag[round % 3] != 0;
      if (t == 0) flag[(round + 2) % 3] = 0;
      if (!go) break;
    }
    ++round;
    PH(2);
    // ---- 2. lookup for the other key ops (nothing is pending now) ----
#pragma unroll
    for (int j = 0; j < kMPer; ++j) {
      if (!keyop[j] || ent[j] != kNoEnt) continue;
      for (uint32_t steps = 0; steps < kMapRegion; ++steps) {
        const uint32_t wv = tword[p[j]];
        if (wv == 0u) break;  // end of chain: absent
        if ((wv & kMwIdentMask) == ident[j] && tkey[p[j]] == key[j]) {
          ent[j] = p[j];
          break;
        }
        p[j] = (p[j] + 1) & (kMapRegion - 1);
      }
    }
    // commits without an entry are resolved now
#pragma unroll
    for (int j = 0; j < kMPer; ++j) {
      if (g[j] == 0xFFFFFFFFu) continue;
      if (ent[j] == kEntFull) {
        err |= kErrCapacity;
        ent[j] = kNoEnt;
      }
      if (ent[j] == kNoEnt || !keyop[j]) {
        ent[j] = kNoEnt;
        uint64_t rv;
        const uint32_t s = map_orphan(smeta_op(m[j]), TTL ? (m[j] & ~kMetaTtl) : m[j], smeta_flags(m[j]), ab[j].x, ab[j].y, rv, err);
        const uint32_t cx = w * (kWave * kMPer) + j * kWave + l;
        ress[cx] = (uint8_t)s;
        resv[cx] = rv;
        resd[cx] = 0;
      }
    }
    PH(3);
    // ---- 3. stable counting sort by entry: per-wave counts (in-wave rank from LDS atomics with return: same-
    //         address lanes of one instruction resolve in lane order, checked at engine start), totals per entry,
    //         then a commit's run position = run start + its entry's count in earlier waves + its in-wave rank ----
    // (wtab was zeroed at the top of the chunk: the binding rounds' barrier orders that before these atomics)
#pragma unroll
    for (int j = 0; j < kMPer; ++j)  // program order over j, lane order inside one instruction = log order
      if (ent[j] != kNoEnt) {
        const uint32_t sh = 16 * (ent[j] & 1);
        rk[j] = (atomicAdd(&wtab[w * (kMapRegion / 2) + (ent[j] >> 1)], 1u << sh) >> sh) & 0xFFFFu;
      }
    lds_barrier();
    for (uint32_t e2 = t; e2 < (uint32_t)(kMapRegion / 2); e2 += MT) {  // totals of 2 entries
      uint32_t s0 = 0, s1 = 0;
#pragma unroll
      for (int q = 0; q < NW; ++q) {
        const uint32_t c = wtab[q * (kMapRegion / 2) + e2];
        s0 += c & 0xFFFF;
        s1 += c >> 16;
      }
      ecnt[2 * e2 + 0] = s0;
      ecnt[2 * e2 + 1] = s1;
    }
#pragma unroll
    for (int j = 0; j < kMPer; ++j)  // + the entry's commits in earlier waves (wave-uniform trip count)
      if (ent[j] != kNoEnt) {
        const uint32_t sh = 16 * (ent[j] & 1);
        for (uint32_t q = 0; q < w; ++q) rk[j] += (wtab[q * (kMapRegion / 2) + (ent[j] >> 1)] >> sh) & 0xFFFFu;
      }
    lds_barrier();
    {
      uint32_t v[MEPer], sum = 0;
#pragma unroll
      for (int q = 0; q < MEPer; ++q) {
        v[q] = ecnt[t * MEPer + q];
        sum += v[q];
      }
      uint32_t inc = sum;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d, 64);
        if (l >= (uint32_t)d) inc += y;
      }
      // (no barrier before this write: wsum's last readers are the previous chunk's, many barriers ago)
      if (l == 63) wsum[w] = inc;
      lds_barrier();
      uint32_t run = inc - sum;
      for (uint32_t q = 0; q < w; ++q) run += wsum[q];
#pragma unroll
      for (int q = 0; q < MEPer; ++q) {
        ecnt[t * MEPer + q] = run;  // run start of entry
        run += v[q];
      }
      if (t == MT - 1) ecnt[kMapRegion] = run;
      lds_barrier();
    }
#pragma unroll
    for (int j = 0; j < kMPer; ++j) {
      if (ent[j] == kNoEnt) continue;
      const uint32_t s = ecnt[ent[j]] + rk[j];
      rab[s] = ab[j];
      rmeta[s] = m[j];
      rpos[s] = g[j];
      rent[s] = (uint16_t)ent[j];
      rci[s] = (uint16_t)(w * (kWave * kMPer) + j * kWave + l);
      if (TTL) {
        const uint64_t cb = clock_base ? *clock_base : 0;
        const uint32_t row = map_row[g[j]];
        const uint64_t ti = ctime ? max(ctime[row], cb) : cb;
        const uint64_t tp = ctime && row > 0 ? max(ctime[row - 1], cb) : cb;
        const uint32_t op = smeta_op(m[j]);
        // the partition marks the rows whose ttl arms a timer (a multimap Put's does not: A18)
        const int64_t ttl = caux && map_reads_ttl(op) && (m[j] & kMetaTtl) ? (int64_t)caux[row] : 0;
        rfire[s] = deferred ? tp : ti;
        rdl[s] = ttl > 0 ? ti + (uint64_t)ttl : 0;
        atomicOr(&eflag[ent[j] >> 5], 1u << (ent[j] & 31));  // every run is walked in order
      } else if (compares_value(m[j])) {
        atomicOr(&eflag[ent[j] >> 5], 1u << (ent[j] & 31));
      }
    }
    lds_barrier();
    PH(4);
    // the chunk's records are in LDS now: the working registers are free for the next chunk (its tmap here, its
    // loads after the scan's first barrier, which orders the tmap writes before them)
    uint32_t gs[kMPer], rs[kMPer];
#pragma unroll
    for (int j = 0; j < kMPer; ++j) {
      gs[j] = g[j];
      rs[j] = res[j];
    }
    if (more) build_map(c0 + kMCh);
    // ---- 4. every run (one entry's commits, log order) at once: a segmented scan of the commits'
    //         transformers gives each commit its entry's state before it (map_ops.h); runs holding a
    //         value-comparing op are walked by one thread instead ----
    {
      const uint32_t total = ecnt[kMapRegion];
      PComp el[kMPer];
      bool hd[kMPer];
      PComp c = pc_identity();
      bool ch = false;
#pragma unroll
      for (int q = 0; q < kMPer; ++q) {
        const uint32_t s = t * kMPer + q;
        el[q] = pc_identity();
        hd[q] = false;
        if (s < total) {
          const uint32_t e = rent[s];
          hd[q] = s == ecnt[e];
          el[q] = pc_element(rmeta[s], s);
          // a clear since the entry's previous commit (or the epoch its state is at): absent first (CLEAR . el)
          if (clr_live && (rmeta[s] >> kMetaEpochShift) != (hd[q] ? (uint32_t)eep[e] : rmeta[s - 1] >> kMetaEpochShift))
            el[q].P = el[q].A;
        }
        c = hd[q] ? el[q] : pc_compose(c, el[q]);
        ch |= hd[q];
      }
      // segmented inclusive scan of the thread aggregates across the wave, then across waves
      PComp inc = c;
      bool ih = ch;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const PComp o = pc_shfl_up(inc, d);
        const bool oh = __shfl_up((int)ih, d, 64) != 0;
        if (l >= (uint32_t)d) {
          if (!ih) inc = pc_compose(o, inc);
          ih |= oh;
        }
      }
      if (l == 63) {
        wcomp[w] = inc;
        whead[w] = ih;
      }
      lds_barrier();
      if (more) load_chunk(c0 + kMCh);
      PComp pre = pc_identity();  // exclusive prefix of this thread (within its run)
      for (uint32_t q = 0; q < w; ++q) {
        if (whead[q]) pre = wcomp[q];
        else pre = pc_compose(pre, wcomp[q]);
      }
      {
        const PComp o = pc_shfl_up(inc, 1);
        const bool oh = __shfl_up((int)ih, 1, 64) != 0;
        if (l > 0) pre = oh ? o : pc_compose(pre, o);
      }
      // walk this thread's commits from its prefix
      uint32_t fe[kMPer], fw[kMPer], fcr[kMPer], fir[kMPer];
      uint64_t fv[kMPer];
      bool fin[kMPer];
      PComp cur = pre;
#pragma unroll
      for (int q = 0; q < kMPer; ++q) {
        const uint32_t s = t * kMPer + q;
        fin[q] = false;
        if (s >= total) continue;
        const uint32_t e = rent[s];
        if (hd[q]) cur = pc_identity();
        if ((eflag[e >> 5] >> (e & 31)) & 1u) continue;
        const uint32_t mm = rmeta[s];
        uint32_t sw, svr, snr;
        uint64_t sv;
        pc_materialize(cur, tword[e], tval[e], rmeta, rab, sw, sv, svr, snr);
        const uint32_t ep = clr_live ? mm >> kMetaEpochShift : 0u;
        if (clr_live && ep != (hd[q] ? (uint32_t)eep[e] : rmeta[s - 1] >> kMetaEpochShift)) {  // cleared before it
          sw &= ~(kMwPresent | kMwVtagMask);
          sv = 0;
        }
        uint64_t rv;
        bool wrote, created;
        const u64x2 x = rab[s];
        const int was = (sw & kMwPresent) != 0;
        const uint32_t sw0 = sw;
        const uint64_t sv0 = sv;
        const uint32_t st = map_apply(smeta_op(mm), smeta_flags(mm), x.x, x.y, sw, sv, rv, wrote, created);
        if (!TTL) cv_change(cv, sw0, sv0, sw, sv, [&]() { return xr[rpos[s]].idx; }, ep, err);
        ress[rci[s]] = (uint8_t)st;
        resv[rci[s]] = rv;
        resd[rci[s]] = (int8_t)(((sw & kMwPresent) != 0) - was);
        if ((sw & kMwPresent) && !was) claim_mark(tc1, tc2, e);
        cur = pc_compose(cur, el[q]);
        if (s + 1 == ecnt[e + 1]) {  // the run's last commit: the entry's new state
          fin[q] = true;
          fe[q] = e;
          uint32_t vr, nr;
          pc_materialize(cur, tword[e], tval[e], rmeta, rab, fw[q], fv[q], vr, nr);
          fcr[q] = vr != kOrig ? rpos[vr] : kNoRef;  // the rewriting commit's staging position
          fir[q] = nr != kOrig ? rpos[nr] : kNoRef;
        }
      }
      lds_barrier();  // every pre-state has been read
#pragma unroll
      for (int q = 0; q < kMPer; ++q) {
        if (!fin[q]) continue;
        tword[fe[q]] = fw[q];
        tval[fe[q]] = fv[q];
        if (fcr[q] != kNoRef) tcr[fe[q]] = fcr[q];
        if (fir[q] != kNoRef) tir[fe[q]] = fir[q];
        if (clr_live) eep[fe[q]] = (uint8_t)(rmeta[ecnt[fe[q] + 1] - 1] >> kMetaEpochShift);  // (its run's last commit)
      }
    }
    PH(5);
    // runs with a value-comparing op: sequentially, by the thread holding the run's first commit
#pragma unroll
    for (int j = 0; j < kMPer; ++j) {
      if (ent[j] == kNoEnt || rk[j] != 0 || !((eflag[ent[j] >> 5] >> (ent[j] & 31)) & 1u)) continue;
      const uint32_t e = ent[j];
      const uint32_t s0 = ecnt[e], s1 = ecnt[e + 1];
      uint32_t wv = tword[e];
      uint64_t vv = tval[e], dl = TTL ? tdl[e] : 0;
      uint32_t ci = 0, ins = 0;
      bool any_w = false, any_c = false;
      for (uint32_t s = s0; s < s1; ++s) {
        const uint32_t mm = rmeta[s];
        const u64x2 x = rab[s];
        uint64_t rv;
        bool wrote, created;
        if (TTL && dl && dl <= rfire[s]) {  // the timer fired: map.remove(key) (MapState.java:91-93)
          // (its size event, if this sub-batch owns the boundary it fired at: common.h TtlEmit)
          if ((wv & kMwPresent) && te.ev_key) ttl_expiry_event(te, clock_base ? *clock_base : 0, wv, tkey[e], dl, err);
          wv &= ~(kMwPresent | kMwVtagMask);
          vv = 0;
          dl = 0;
        }
        const uint32_t ep = clr_live ? mm >> kMetaEpochShift : 0u;
        if (clr_live && ep != (s == s0 ? (uint32_t)eep[e] : rmeta[s - 1] >> kMetaEpochShift)) {  // cleared before it
          wv &= ~(kMwPresent | kMwVtagMask);
          vv = 0;
        }
        const int was = (wv & kMwPresent) != 0;  // (after the expiry: the commit's own change)
        const uint32_t wv0 = wv;
        const uint64_t vv0 = vv;
        const uint32_t st = map_apply(smeta_op(mm), smeta_flags(mm), x.x, x.y, wv, vv, rv, wrote, created);
        if (!TTL) cv_change(cv, wv0, vv0, wv, vv, [&]() { return xr[rpos[s]].idx; }, ep, err);
        if (TTL) {  // a stored commit cancels the old timer and arms its own; a removal cancels it
          if (wrote) dl = rdl[s];
          else if (!(wv & kMwPresent)) dl = 0;
        }
        ress[rci[s]] = (uint8_t)st;
        resv[rci[s]] = rv;
        resd[rci[s]] = (int8_t)(((wv & kMwPresent) != 0) - was);
        if ((wv & kMwPresent) && !was) claim_mark(tc1, tc2, e);
        if (wrote) { ci = rpos[s]; any_w = true; }
        if (created) { ins = rpos[s]; any_c = true; }
      }
      tword[e] = wv;
      tval[e] = vv;
      if (TTL) tdl[e] = dl;
      else if (clr_live) eep[e] = (uint8_t)(rmeta[s1 - 1] >> kMetaEpochShift);
      if (any_w) tcr[e] = ci;
      if (any_c) tir[e] = ins;
    }
    lds_barrier();
#pragma unroll
    for (int j = 0; j < kMPer; ++j)  // this thread's own commits: consecutive lanes -> consecutive staging rows
      if (gs[j] != 0xFFFFFFFFu) {
        const uint32_t cx = w * (kWave * kMPer) + j * kWave + l;
        rst_status[gs[j]] = ress[cx];
        rst_value[gs[j]] = resv[cx];
        rst_msz[gs[j]] = (rs[j] << 2) | (resd[cx] > 0 ? 1u : resd[cx] < 0 ? 2u : 0u);  // (launch_map_size)
      }
    for (uint32_t q = t; q <= kMapRegion; q += MT) ecnt[q] = 0;
    for (uint32_t q = t; q < kMapRegion / 32; q += MT) eflag[q] = 0;
    lds_barrier();
    PH(6);
  }

  // ---- clears in the stream: an entry whose state predates its map's last clear of the sub-batch stays bound but
  //      absent and UNSEEN (no key the map held since the clear: left out of the used count and the tree-bin test,
  //      map_wide.hip), with the clear's index as its claim (a later put makes it seen again, claimed no earlier than
  //      the clear); the keys it held count toward the map's peak-size bound, as at a barrier clear.  (Marking them
  //      DEAD made every later put of the key bind a new slot: regions filled with dead entries, 4x the binding time.)
  constexpr uint8_t kEpKilled = 0xFF;  // eep mark of an entry cleared here (its claim is written back below)
  if (clr_live) {
#pragma unroll
    for (int q = 0; q < MEPer; ++q) {
      const uint32_t e = q * MT + t;
      const uint32_t wv = tword[e];
      if (!(wv & kMwUsed) || (wv & kMwDead)) continue;
      const uint32_t ms = wv & kMwSlotMask;
      if ((clr.mflag[ms] & kMfClr) && eep[e] < clr.eend[ms]) {
        tword[e] = (wv & ~(kMwPresent | kMwVtagMask)) | kMwUnseen;
        if (dropped && !(wv & kMwUnseen)) atomicAdd(&dropped[ms], 1ull);
        eep[e] = kEpKilled;
      }
    }
  }
  // ---- write the region back ----
#pragma unroll
  for (int q = 0; q < MEPer; ++q) {
    const uint32_t e = q * MT + t;
    tbl_key[tb + e] = tkey[e];
    tbl_word[tb + e] = tword[e];
    tbl_val[tb + e] = tval[e];
    if (tcr[e] != kNoRef) tbl_ci[tb + e] = xr[tcr[e]].idx;
    if (tir[e] != kNoRef) tbl_ins[tb + e] = xr[tir[e]].idx;
    if (clr_live && eep[e] == kEpKilled) {  // cleared: claimed again no earlier than its map's last clear
      const uint32_t ms = tword[e] & kMwSlotMask;
      const uint32_t crow = (uint32_t)clr.clr[clr.off[ms] + clr.base[ms] + clr.eend[ms] - 1];
      tbl_claim[tb + e] = idx0p[crow - clr.lo];
    } else if (((tnew[e >> 5] >> (e & 31)) & 1u) && (tword[e] & kMwUsed)) {  // bound by this launch: its claim
      const bool one = ((tc1[e >> 5] >> (e & 31)) & 1u) && !((tc2[e >> 5] >> (e & 31)) & 1u) && tir[e] != kNoRef;
      tbl_claim[tb + e] = one ? xr[tir[e]].idx : *idx0p;
    }
    if (TTL) tbl_dl[tb + e] = tdl[e];
    else if (clr_live) clr.tbl_ep[tb + e] = 0;  // (the next sub-batch's hot keys write theirs before it reads)
  }
  PH(7);
  if (!TTL) PH_FLUSH(g_ph_map);
  if (err) atomicOr(err_out, err);
}

// A deleted / cleared map: its entries become DEAD (never matched; reclaimed by the next compaction of their region),
// and its generation moves on (the keys compacted away before no longer count toward its tree-bin test).
__global__ void k_map_drop(uint32_t* __restrict__ tbl_word, uint64_t entries, uint32_t slot, uint64_t* __restrict__ cgen) {
  const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e == 0 && cgen) ++cgen[slot];
  if (e >= entries) return;
  const uint32_t wv = tbl_word[e];
  if ((wv & kMwUsed) && !(wv & kMwDead) && (wv & kMwSlotMask) == slot) tbl_word[e] = (wv & ~(kMwPresent | kMwVtagMask)) | kMwDead;
}

int launch_apply_map(const MapArgs& a, hipStream_t st) {
  if (a.map_bits == 0 || a.tiles == 0) return 0;
  a.mark(K_APPLY_MAP, 1, st);
  if (a.ttl)
    hipLaunchKernelGGL((k_apply_map<true, false>), dim3(1u << a.map_bits), dim3(512), 0, st, a.mrec, a.cb, a.lo, a.ttab, a.tiles, a.sb, a.sb_val, a.tbl_key, a.tbl_word, a.tbl_val, a.tbl_ci, a.tbl_ins,
                       a.tbl_claim, a.idx0, (unsigned long long*)a.dropped, a.cgen, a.cset, a.cset_mask, a.cset_full, a.tbl_dl, a.map_row, a.time, a.aux, a.clock_base, a.deferred,
                       a.rst_status, a.rst_value, a.rst_msz, a.ttl_emit, CvCtx{}, ClrCtx{}, a.err);
  else if (a.clr.mflag)
    hipLaunchKernelGGL((k_apply_map<false, true>), dim3(1u << a.map_bits), dim3(CC_MAP_MT), 0, st, a.mrec, a.cb, a.lo, a.ttab, a.tiles, a.sb, a.sb_val, a.tbl_key, a.tbl_word, a.tbl_val, a.tbl_ci, a.tbl_ins,
                       a.tbl_claim, a.idx0, (unsigned long long*)a.dropped, a.cgen, a.cset, a.cset_mask, a.cset_full, nullptr, nullptr, nullptr, nullptr, nullptr, false,
                       a.rst_status, a.rst_value, a.rst_msz, TtlEmit{}, a.cv, a.clr, a.err);
  else
    hipLaunchKernelGGL((k_apply_map<false, false>), dim3(1u << a.map_bits), dim3(CC_MAP_MT), 0, st, a.mrec, a.cb, a.lo, a.ttab, a.tiles, a.sb, a.sb_val, a.tbl_key, a.tbl_word, a.tbl_val, a.tbl_ci, a.tbl_ins,
                       a.tbl_claim, a.idx0, (unsigned long long*)a.dropped, a.cgen, a.cset, a.cset_mask, a.cset_full, nullptr, nullptr, nullptr, nullptr, nullptr, false,
                       a.rst_status, a.rst_value, a.rst_msz, TtlEmit{}, a.cv, a.clr, a.err);
  a.mark(K_APPLY_MAP, 0, st);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// staging position -> batch row for the map records of a sub-batch (the TTL variant reads each commit's clock)
__global__ void k_map_rows(const uint16_t* __restrict__ cpos, uint64_t lo, uint64_t hi, uint32_t* __restrict__ map_row) {
  const uint64_t i = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= hi) return;
  const uint16_t c = cpos[i - lo];
  if (c == 0xFFFF) return;
  map_row[((i - lo) / kTile) * kTile + c] = (uint32_t)i;
}

int launch_map_rows(const uint16_t* cpos, uint64_t lo, uint64_t hi, uint32_t* map_row, hipStream_t st) {
  hipLaunchKernelGGL(k_map_rows, dim3((uint32_t)((hi - lo + 255) / 256)), dim3(256), 0, st, cpos, lo, hi, map_row);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_map_drop_resource(uint32_t* tbl_word, uint64_t entries, uint32_t slot, uint64_t* cgen, hipStream_t st) {
  hipLaunchKernelGGL(k_map_drop, dim3((uint32_t)((entries + 255) / 256)), dim3(256), 0, st, tbl_word, entries, slot, cgen);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace cc
