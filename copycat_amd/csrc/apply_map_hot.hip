// apply_map_hot.hip — hot map keys: a key that holds a large share of a batch (Zipf-skewed DistributedMap
// traffic, SURVEY §7 hard part (b)) is applied by a scan over many workgroups instead of one region's chain.
//
// Per sub-batch:
//   k_hot_detect : one workgroup samples 64K commits (64 blocks of 1024 consecutive rows), counts (map, key tag,
//                  key) in an LDS sketch, and takes the (up to) 64 most frequent keys above ~0.1% of the
//                  sample; binds their table entries (apply_map.hip
//                  layout) and publishes the hot set.  The partition routes every commit of a hot key to that
//                  key's own bucket (log order, like any super-bucket).  Hot-ness only steers work: a commit is
//                  applied identically by either path.
//   k_hot_lists  : per hot key: its run in every tile -> list offsets; snapshot of the entry's state.
//   k_hot_agg    : per piece of kHotPiece commits of a key's list: the piece's composite transformer (below).
//   k_hot_carry  : per hot key: the pieces' composites -> their exclusive prefixes (in place).
//   k_hot_apply  : per piece: carry = composite of all earlier pieces applied to the snapshot; the piece's
//                  commits are then applied in log order from that state (results written to staging); the
//                  last piece writes the entry back.
//
// Key ops as transformers of one entry's state (absent | present(value, node)):
//   put(v)          absent -> present(v, new node)     present -> present(v, same node)
//   putIfAbsent(v)  absent -> present(v, new node)     present -> unchanged
//   remove          absent -> absent                   present -> absent
//   replace(v)      absent -> absent                   present -> present(v, same node)
//   containsKey, get, getOrDefault: identity
// This family is closed under composition (each branch ends absent, unchanged, or present with a value and a
// node taken from some commit), so a composite is two branch outcomes that reference staging records: the scan
// is exact.  removeIfPresent/replaceIfPresent compare the stored value (MapState.java:159-178, 207-228) and are
// outside the family: a hot key whose list holds one is applied sequentially (correct, slower).
#include "common.h"
#include "engine_internal.h"
#include "map_ops.h"

namespace cc {

#ifndef CC_HOT_T
#define CC_HOT_T 256
#endif
constexpr int kHT = CC_HOT_T;              // threads per hot-scan workgroup
constexpr int kHPer = kHotPiece / kHT;     // commits per thread per piece (4)
constexpr int kDetT = 1024;
constexpr int kDetSlots = 4096;
constexpr uint32_t kDetSample = 65536;
constexpr uint32_t kDetBlk = 1024;  // consecutive rows per sample block
constexpr int kDetProbe = 8;
constexpr int kDetCand = 1024;      // candidate keys above the sample threshold

// ---------------------------------------------------------------------------------------------------------
// The sample: 64 blocks of 1024 consecutive rows spread evenly over the sub-batch (coalesced column loads; hot-ness
// only steers work, so any sample is correct).  k_hot_sample resolves every sampled row (instance -> resource ->
// type -> map hash) with one thread per row over 64 workgroups, so the dependent gathers overlap across the chip;
// k_hot_detect then only counts the resolved keys (one workgroup, an LDS sketch).
struct HotSamp {
  uint64_t h64;    // map_hash (0: not a keyed commit)
  uint64_t key;
  uint32_t ident;  // mw_ident(slot, key tag)
  uint32_t pad;
};
size_t hot_samp_bytes() { return sizeof(HotSamp) * kDetSample; }

__global__ __launch_bounds__(kDetBlk) void k_hot_sample(const uint32_t* __restrict__ inst, const uint8_t* __restrict__ flags,
                                                       const uint64_t* __restrict__ ckey, uint64_t lo, uint64_t hi,
                                                       const uint32_t* __restrict__ inst_res,
                                                       const uint8_t* __restrict__ res_type, uint32_t max_inst,
                                                       HotSamp* __restrict__ samp) {
  const uint64_t n = hi - lo;
  const uint32_t S = (uint32_t)(n < kDetSample ? n : kDetSample);
  const uint32_t j = blockIdx.x * kDetBlk + threadIdx.x;
  if (j >= S) return;
  const uint64_t spacing = n > kDetSample ? n / (kDetSample / kDetBlk) : kDetBlk;
  const uint64_t i = lo + (uint64_t)(j / kDetBlk) * spacing + (j % kDetBlk);
  const uint32_t sl = inst[i];
  const uint32_t kt = CC_FLAG_KTAG(flags[i]);
  const uint64_t key = ckey[i];
  const uint32_t r = sl < max_inst ? inst_res[sl] : kNoRes;
  HotSamp x{0, key, 0, 0};
  if (r != kNoRes && is_keyed(res_type[r])) {
    x.h64 = map_hash(r, kt, key);
    x.ident = mw_ident(r, kt);
  }
  samp[j] = x;
}

// ---------------------------------------------------------------------------------------------------------
// The hot keys of a batch: counted once per batch (k_hot_count, from k_hot_sample's rows spread over the whole batch:
// correctness never depends on which keys are hot, and one batch's commits share their distribution), bound to their
// table entries before every sub-batch (k_hot_bind: the tables change between sub-batches).  Per-sub-batch counting
// cost ~95 us of one workgroup's LDS atomics each time (c3: 5.6 ms per step).
__global__ __launch_bounds__(kDetT) void k_hot_count(const HotSamp* __restrict__ samp, uint64_t lo, uint64_t hi,
                                                    HotKey* __restrict__ cand_out, uint32_t* __restrict__ cand_n) {
  __shared__ uint64_t th64[kDetSlots];
  __shared__ uint64_t tkey[kDetSlots];
  __shared__ uint32_t tident[kDetSlots];
  __shared__ uint32_t tcnt[kDetSlots];
  __shared__ uint32_t cand[kDetCand];
  __shared__ uint32_t sel[kHotMax];
  __shared__ uint32_t ncand;
  const uint32_t t = threadIdx.x;
  for (uint32_t q = t; q < kDetSlots; q += kDetT) {
    th64[q] = 0;
    tcnt[q] = 0;
  }
  if (t == 0) ncand = 0;
  __syncthreads();
  const uint64_t n = hi - lo;
  const uint32_t S = (uint32_t)(n < kDetSample ? n : kDetSample);
  // the resolved sample (k_hot_sample), 16 rows per thread in flight before their LDS updates
  constexpr int U = 16;
  for (uint32_t j0 = t; j0 < S; j0 += kDetT * U) {
    HotSamp x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t j = j0 + u * kDetT;
      x[u] = j < S ? samp[j] : HotSamp{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t h = x[u].h64;
      if (h == 0) continue;
      // short probes: a Zipf sample holds far more distinct cold keys than the sketch has slots; a hot key shows
      // up early and often, so a sample that finds no slot within kDetProbe steps is dropped
      uint32_t q = (uint32_t)h & (kDetSlots - 1);
      for (int step = 0; step < kDetProbe; ++step, q = (q + 1) & (kDetSlots - 1)) {
        const uint64_t old = atomicCAS((unsigned long long*)&th64[q], 0ull, (unsigned long long)h);
        if (old == 0) {
          tkey[q] = x[u].key;
          tident[q] = x[u].ident;
          atomicAdd(&tcnt[q], 1u);
          break;
        }
        if (old == h) {
          atomicAdd(&tcnt[q], 1u);
          break;
        }
      }
    }
  }
  __syncthreads();
  // hot: >= 1/4096 of the sample (Zipf 0.99 over 1M pairs: the ~280 heaviest keys).  Every key left in the regions
  // then carries < 0.025% of the sub-batch, so no region's chain is more than a few times the average one.
  const uint32_t thresh = S / (16 * kHotMax) > 16 * 256 / kHotMax ? S / (16 * kHotMax) : 16 * 256 / kHotMax;
  for (uint32_t q = t; q < kDetSlots; q += kDetT) {
    if (th64[q] != 0 && tcnt[q] >= thresh) {
      const uint32_t k = atomicAdd(&ncand, 1u);
      if (k < (uint32_t)kDetCand) cand[k] = q;
    }
  }
  __syncthreads();
  const uint32_t nc = ncand < (uint32_t)kDetCand ? ncand : (uint32_t)kDetCand;
  if (t < nc) {  // keep the kHotMax most frequent (ties: lower slot)
    const uint32_t c = cand[t], cc = tcnt[c];
    uint32_t rank = 0;
    for (uint32_t u = 0; u < nc; ++u) {
      const uint32_t o = cand[u], oc = tcnt[o];
      rank += (oc > cc || (oc == cc && o < c)) ? 1 : 0;
    }
    if (rank < (uint32_t)kHotMax) sel[rank] = c;
  }
  __syncthreads();
  const uint32_t nsel = nc < (uint32_t)kHotMax ? nc : (uint32_t)kHotMax;
  if (t < nsel) {
    const uint32_t q = sel[t];
    cand_out[t] = HotKey{th64[q], tkey[q], tident[q], 0u};
  }
  if (t == 0) *cand_n = nsel;
}

__global__ __launch_bounds__(kDetT) void k_hot_bind(const HotKey* __restrict__ cand, const uint32_t* __restrict__ cand_n,
                                                   uint32_t map_bits, uint64_t* tbl_key, uint32_t* tbl_word,
                                                   uint64_t* tbl_val, uint64_t* tbl_ci, uint64_t* tbl_ins,
                                                   uint64_t* tbl_claim, const uint64_t* __restrict__ idx0p,
                                                   HotKey* __restrict__ hot, uint32_t* __restrict__ hot_n,
                                                   const uint8_t* __restrict__ msmall) {
  const uint32_t t = threadIdx.x;
  const uint32_t nc = *cand_n;
  // bind each hot key's table entry (the tables are idle between the sub-batch's kernels): every key looks itself
  // up in parallel (thread = key); the keys not in the table yet are inserted by one wave, one lane at a time, so no
  // two keys race for a slot, as UNSEEN placeholders (a candidate counted over the whole batch may never occur in
  // this sub-batch: such an entry is no key the map held, kMwUnseen); then wave 0 compacts the bound keys in rank order
  const uint32_t nh = nc < (uint32_t)kHotMax ? nc : (uint32_t)kHotMax;
  uint64_t h = 0, key = 0, base = 0;
  uint32_t ident = 0;
  const bool valid = t < nh;
  if (valid) {
    const HotKey c = cand[t];
    h = c.h64;
    key = c.key;
    ident = c.ident;
    base = (h >> (64 - map_bits)) * kMapRegion;
  }
  auto probe = [&](bool insert, uint32_t& pos) -> bool {
    uint32_t p = (uint32_t)h & (kMapRegion - 1);
    for (int step = 0; step < kMapRegion; ++step, p = (p + 1) & (kMapRegion - 1)) {
      const uint32_t w = __hip_atomic_load(&tbl_word[base + p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (w == 0u) {
        if (insert) {
          __hip_atomic_store(&tbl_key[base + p], key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(&tbl_val[base + p], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(&tbl_ci[base + p], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(&tbl_ins[base + p], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          // its claim (the tree-bin test, map_wide.hip): no later than this sub-batch's first commit
          __hip_atomic_store(&tbl_claim[base + p], (uint64_t)*idx0p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(&tbl_word[base + p], ident | kMwUnseen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
          pos = (uint32_t)(base + p);
          return true;
        }
        return false;
      }
      if ((w & kMwIdentMask) == ident &&
          __hip_atomic_load(&tbl_key[base + p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == key) {
        pos = (uint32_t)(base + p);
        return true;
      }
    }
    return false;  // a full region leaves the key cold
  };
  // a map still in its small-table window is followed commit by commit through its regions (map_small.hip)
  auto small_map = [&](uint32_t id) { (void)id; return false; };  // (every map's hot keys: k_hot_apply emits their events)
  uint32_t pos = 0;
  const bool found = valid && !small_map(ident) && probe(false, pos);
  __shared__ uint32_t bpos[kHotMax];
  __shared__ uint8_t bok[kHotMax];
  __shared__ uint32_t nmiss;
  if (t == 0) nmiss = 0;
  __syncthreads();
  if (valid) {
    bpos[t] = pos;
    bok[t] = found ? 1 : 0;
    if (!found) atomicAdd(&nmiss, 1u);
  }
  __syncthreads();
  if (nmiss && t >= kWave && t < 2 * kWave) {  // inserts: wave 1, one key at a time in rank order
    for (uint32_t g0 = 0; g0 < nh; g0 += kWave) {
      const uint32_t gi = g0 + (t - kWave);
      const bool miss = gi < nh && !bok[gi] && !small_map(cand[gi].ident);
      for (uint64_t need = ballot(miss); need; need &= need - 1) {
        const uint32_t leader = (uint32_t)__builtin_ctzll(need);
        if (t - kWave == leader) {
          const HotKey c = cand[gi];
          h = c.h64;
          key = c.key;
          ident = c.ident;
          base = (h >> (64 - map_bits)) * kMapRegion;
          uint32_t ip = 0;
          if (probe(true, ip)) {
            bpos[gi] = ip;
            bok[gi] = 1;
          }
        }
        __threadfence();
      }
    }
  }
  __syncthreads();
  if (t >= kWave) return;
  const uint32_t l = t;
  uint32_t nbound = 0;
  for (uint32_t g0 = 0; g0 < nh; g0 += kWave) {
    const uint32_t gi = g0 + l;
    const bool ok = gi < nh && bok[gi];
    const uint64_t okm = ballot(ok);
    if (ok) {
      const HotKey c = cand[gi];
      const uint32_t k = nbound + (uint32_t)__builtin_popcountll(okm & lanemask_lt());
      hot[k] = HotKey{c.h64, c.key, c.ident, bpos[gi]};
    }
    nbound += (uint32_t)__builtin_popcountll(okm);
  }
  if (l == 0) *hot_n = nbound;
}

// ---------------------------------------------------------------------------------------------------------
struct HotS0 {
  uint64_t v, ci, ins;
  uint32_t w;
  uint32_t pad;
};

__global__ __launch_bounds__(kHT) void k_hot_lists(const uint16_t* __restrict__ ttab, uint32_t tiles, uint32_t sb,
                                                  uint32_t sb_hot, const HotKey* __restrict__ hot,
                                                  const uint32_t* __restrict__ hot_n, const uint64_t* __restrict__ tbl_val,
                                                  const uint32_t* __restrict__ tbl_word, const uint64_t* __restrict__ tbl_ci,
                                                  const uint64_t* __restrict__ tbl_ins, uint32_t* __restrict__ hot_rpre,
                                                  uint32_t* __restrict__ hot_rstart, uint32_t* __restrict__ hot_len,
                                                  uint32_t* __restrict__ hot_cond, HotS0* __restrict__ hot_s0) {
  __shared__ uint32_t wsum[kHT / kWave];
  const uint32_t h = blockIdx.x, t = threadIdx.x, w = t >> 6, l = t & 63;
  if (h >= *hot_n) return;
  const uint32_t k = sb_hot + h;
  constexpr int PT = kMaxTiles / kHT;
  uint32_t len[PT], st[PT], sum = 0;
#pragma unroll
  for (int q = 0; q < PT; ++q) {
    const uint32_t tt = t * PT + q;
    len[q] = 0;
    st[q] = 0;
    if (tt < tiles) {
      const uint16_t* row = ttab + (uint64_t)tt * (sb + 1);
      const uint32_t b0 = row[k], b1 = row[k + 1];
      st[q] = tt * kTile + b0;
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
  uint32_t* rpre = hot_rpre + (uint64_t)h * (kMaxTiles + 1);
  uint32_t* rstart = hot_rstart + (uint64_t)h * kMaxTiles;
#pragma unroll
  for (int q = 0; q < PT; ++q) {
    const uint32_t tt = t * PT + q;
    if (tt < tiles) {
      rpre[tt] = run;
      rstart[tt] = st[q];
    }
    run += len[q];
  }
  if (t == kHT - 1) {
    rpre[tiles] = run;
    hot_len[h] = run;
  }
  if (t == 0) {
    hot_cond[h] = 0;
    const uint32_t p = hot[h].pos;
    hot_s0[h] = HotS0{tbl_val[p], tbl_ci[p], tbl_ins[p], tbl_word[p], 0};
  }
}

// piece enumeration shared by k_hot_agg / k_hot_apply: item -> (hot key, piece)
__device__ inline void hot_items(const uint32_t* __restrict__ hot_n, const uint32_t* __restrict__ hot_len, uint32_t* pfx,
                                 uint32_t& nh) {
  nh = *hot_n;
  hot_piece_prefix(hot_len, nh, pfx);
  __syncthreads();
}

// staging positions of list positions [p0, p0 + cnt): walk the tile runs from the run holding p0.  The key's run
// table is an LDS copy (hot_runs_lds) and the current run's end and base stay in registers: read from HBM, the
// binary search and one dependent load per position made every piece a chain of ~30 global round trips.
struct ListCursor {
  const uint32_t* rpre;    // [tiles + 1] list prefix per tile (LDS)
  const uint32_t* rstart;  // [tiles] staging start of the key's run per tile (LDS)
  uint32_t tiles, tile, pos, nxt, base;
  __device__ void seek(uint32_t p) {
    uint32_t a = 0, b = tiles;  // last tile with rpre <= p
    while (b - a > 1) {
      const uint32_t m = (a + b) >> 1;
      if (rpre[m] <= p) a = m; else b = m;
    }
    tile = a;
    pos = p;
    nxt = rpre[a + 1];
    base = rstart[a] - rpre[a];
  }
  __device__ uint32_t next() {
    while (pos >= nxt) {
      ++tile;
      nxt = rpre[tile + 1];
      base = rstart[tile] - rpre[tile];
    }
    return base + pos++;
  }
};
// the item's key h (binary search over the piece prefix) and its run table copied into LDS (all threads; the
// caller's previous item must be finished with the copy: a barrier at the top)
__device__ inline uint32_t hot_item_key(const uint32_t* pfx, uint32_t nh, uint32_t item) {
  uint32_t a = 0, b = nh;  // last key with pfx <= item
  while (b - a > 1) {
    const uint32_t m = (a + b) >> 1;
    if (pfx[m] <= item) a = m; else b = m;
  }
  return a;
}
__device__ inline void hot_runs_lds(const uint32_t* __restrict__ hot_rpre, const uint32_t* __restrict__ hot_rstart,
                                    uint32_t h, uint32_t tiles, uint32_t* lrpre, uint32_t* lrst,
                                    uint32_t* lflag = nullptr, uint32_t flag = 0) {
  __syncthreads();
  if (lflag && threadIdx.x == 0) *lflag = flag;  // (thread 0's value for the whole workgroup)
  for (uint32_t q = threadIdx.x; q <= tiles; q += blockDim.x) lrpre[q] = hot_rpre[(uint64_t)h * (kMaxTiles + 1) + q];
  for (uint32_t q = threadIdx.x; q < tiles; q += blockDim.x) lrst[q] = hot_rstart[(uint64_t)h * kMaxTiles + q];
  __syncthreads();
}

// (reads each hot commit's meta word from the compact copy k_part_ext writes, hot_meta, not from its 48-byte record)
// A commit's clear epoch (map_clear.hip: the clears of its map in [lo, row)), written into its meta word by k_part_ext.
__device__ inline uint32_t hot_epoch(uint32_t meta) { return meta >> kMetaEpochShift; }
__device__ inline bool hot_cleared(const HotClr& c, uint32_t slot) {
  return c.clr.mflag != nullptr && (c.clr.mflag[slot] & kMfClr) != 0;
}
// an insertion / removal of a map followed by events (a small map's HashMap model, size / isEmpty rows, a cleared
// map's sizes): its event, as k_msize_count emits a region commit's (map_wide.hip map_event)
__device__ inline bool hot_events(const HotClr& c, uint32_t slot) {
  return c.mflag != nullptr && (c.mflag[slot] & (kMfSmall | kMfSize | kMfClr)) != 0;
}
// (at: its slot in the event buffer, reserved by the caller)
__device__ inline void hot_map_event_at(const HotClr& c, uint32_t slot, uint32_t code, const MRec& r, uint32_t at,
                                        uint32_t& err) {
  bool ok;
  const uint32_t kt = CC_FLAG_KTAG(smeta_flags(r.meta));
  const uint32_t jh = java_key_hash(kt, r.key, c.hh_key, c.hh_val, c.hh_n, ok);
  const uint64_t d = r.idx - *c.idx0p;
  if (!ok) err |= kErrHandleHash;
  if (d >> kEvPosBits) err |= kErrSpan;
  if (at < c.ev_cap) {
    c.ev_key[at] = ((uint64_t)slot << kEvMapShift) | ((d & kEvPosMask) << 4) | code;
    c.ev_val[at] = at;
    c.ev_pay[at] = EvPay{r.key, jh, kt};
  }
}
__device__ inline void hot_map_event(const HotClr& c, uint32_t slot, uint32_t code, const MRec& r, uint32_t& err) {
  if (code) hot_map_event_at(c, slot, code, r, wave_append(c.ev_ctl), err);
}

__global__ __launch_bounds__(kHT) void k_hot_agg(const uint32_t* __restrict__ hot_meta, const uint32_t* __restrict__ hot_n,
                                                const uint32_t* __restrict__ hot_len, const uint32_t* __restrict__ hot_rpre,
                                                const uint32_t* __restrict__ hot_rstart, uint32_t tiles,
                                                Comp* __restrict__ agg, uint32_t* __restrict__ hot_cond,
                                                const HotKey* __restrict__ hot, HotClr hc) {
  __shared__ uint32_t pfx[kHotMax + 1];
  __shared__ Comp wtot[kHT / kWave];
  __shared__ uint32_t lrpre[kMaxTiles + 1], lrst[kMaxTiles];
  uint32_t nh;
  hot_items(hot_n, hot_len, pfx, nh);
  const uint32_t t = threadIdx.x, w = t >> 6, l = t & 63;
  for (uint32_t item = blockIdx.x; item < pfx[nh]; item += gridDim.x) {
    const uint32_t h = hot_item_key(pfx, nh, item);
    hot_runs_lds(hot_rpre, hot_rstart, h, tiles, lrpre, lrst);
    const uint32_t p = item - pfx[h], L = hot_len[h];
    const uint32_t p0 = p * kHotPiece + t * kHPer;
    ListCursor cur{lrpre, lrst, tiles, 0, 0, 0, 0};
    Comp c = comp_identity();
    bool cond = false;
    const uint32_t slot = hot[h].ident & kMwSlotMask;
    const bool fl = hot_cleared(hc, slot);  // (item-uniform)
    if (p0 < L) {
      uint32_t pe = 0;  // the epoch of the commit before this thread's first (0: the sub-batch start)
      if (fl && p0 > 0) {
        cur.seek(p0 - 1);
        pe = hot_epoch(hot_meta[cur.next()]);
      }
      cur.seek(p0);
      const uint32_t e = p0 + kHPer < L ? p0 + kHPer : L;
      for (uint32_t q = p0; q < e; ++q) {
        const uint32_t g = cur.next();
        const uint32_t m = hot_meta[g];
        cond |= compares_value(m);
        Comp el = element(m, g);
        if (fl) {  // a clear since the commit before: CLEAR . el (map_clear.hip)
          const uint32_t E = hot_epoch(m);
          if (E != pe) el.P = el.A;
          pe = E;
        }
        c = compose(c, el);
      }
    }
    if (cond) atomicOr(&hot_cond[h], 1u);
    c = wave_scan(c, l);
    if (l == 63) wtot[w] = c;
    __syncthreads();
    if (t == 0) {
      Comp a = wtot[0];
      for (int q = 1; q < kHT / kWave; ++q) a = compose(a, wtot[q]);
      agg[(uint64_t)h * kHotMaxPieces + p] = a;
    }
    __syncthreads();
  }
}

// Each hot key's piece composites -> their exclusive prefixes, in place (one workgroup per key): k_hot_apply then
// reads the composite of pieces [0, p) with one load.  (It folded them itself, wave 0 walking up to p / 64 dependent
// loads per lane for every piece: O(P^2) over a key of P pieces, ~18 loads per lane for the hottest key's last ones.)
__global__ __launch_bounds__(kHT) void k_hot_carry(const uint32_t* __restrict__ hot_n, const uint32_t* __restrict__ hot_len,
                                                  Comp* __restrict__ agg) {
  __shared__ uint32_t pfx[kHotMax + 1];
  __shared__ Comp wtot[kHT / kWave];
  uint32_t nh;
  hot_items(hot_n, hot_len, pfx, nh);
  const uint32_t h = blockIdx.x, t = threadIdx.x, w = t >> 6, l = t & 63;
  if (h >= nh) return;  // block-uniform
  const uint32_t P = pfx[h + 1] - pfx[h];
  Comp* const a = agg + (uint64_t)h * kHotMaxPieces;
  const uint32_t per = (P + kHT - 1) / kHT, q0 = min(t * per, P), q1 = min(q0 + per, P);
  Comp c = comp_identity();
  for (uint32_t q = q0; q < q1; ++q) c = compose(c, a[q]);
  const Comp inc = wave_scan(c, l);
  if (l == 63) wtot[w] = inc;
  __syncthreads();
  Comp run = comp_identity();  // pieces before this thread's: waves before, then lanes before
  for (uint32_t q = 0; q < w; ++q) run = compose(run, wtot[q]);
  {
    const Comp o = comp_shfl_up(inc, 1);
    if (l > 0) run = compose(run, o);
  }
  for (uint32_t q = q0; q < q1; ++q) {
    const Comp x = a[q];
    a[q] = run;
    run = compose(run, x);
  }
}

// materialize a branch outcome applied to the snapshot: map_apply state (word, value) + commit/insert index
// (the snapshot as four words, not a HotS0 reference: the struct was kept in scratch, and its store there waited
// for its load at the top of every item)
__device__ inline void materialize(const Comp& c, const HotS0 s0, const MRec* __restrict__ xr, uint32_t& w,
                                   uint64_t& v, uint64_t& ci, uint64_t& ins) {
  const bool present0 = (s0.w & kMwPresent) != 0;
  Br b;
  b.kind = present0 ? c.P.kind : c.A.kind;
  b.v = present0 ? c.P.v : c.A.v;
  b.n = present0 ? c.P.n : c.A.n;
  const uint32_t base = s0.w & ~(kMwPresent | kMwVtagMask);
  if (b.kind == kBrKeep) {
    w = s0.w;
    v = s0.v;
    ci = s0.ci;
    ins = s0.ins;
  } else if (b.kind == kBrAbsent) {
    w = base;
    v = 0;
    ci = s0.ci;
    ins = s0.ins;
  } else {
    const uint32_t tag = CC_FLAG_TAG_A(smeta_flags(xr[b.v].meta));
    w = (base & ~kMwUnseen) | kMwPresent | (tag << 21);
    v = tag ? xr[b.v].a : 0;
    ci = xr[b.v].idx;
    ins = b.n == kOrig ? s0.ins : xr[b.n].idx;
  }
}

// one commit of a hot key on state (w, v): result -> staging; tracks commit/insert index; returns the commit's
// size change (1 insert, 2 remove, 0 none: the 2-bit codes of hot_msz)
__device__ inline uint32_t hot_step(uint32_t g, uint32_t m, const u64x2& x, uint64_t idx, uint32_t& w, uint64_t& v,
                                    uint64_t& ci, uint64_t& ins, uint8_t* __restrict__ rst_status,
                                    uint64_t* __restrict__ rst_value, const CvCtx& cv, uint32_t ep, uint32_t& err) {
  const uint32_t op = smeta_op(m);
  const int was = (w & kMwPresent) != 0;
  uint64_t rv;
  uint32_t st;
  if (!map_applied(m)) {
    st = map_orphan(op, m, smeta_flags(m), x.x, x.y, rv, err);
  } else {
    bool wrote, created;
    const uint32_t w0 = w;
    const uint64_t v0 = v;
    st = map_apply(op, smeta_flags(m), x.x, x.y, w, v, rv, wrote, created);
    cv_change(cv, w0, v0, w, v, [&]() { return idx; }, ep, err);
    if (wrote) ci = idx;
    if (created) ins = idx;
  }
  rst_status[g] = (uint8_t)st;
  rst_value[g] = rv;
  return msz_word(0, was, (w & kMwPresent) != 0);
}

__global__ __launch_bounds__(kHT) void k_hot_apply(const MRec* __restrict__ xr, const uint64_t* __restrict__ cb, uint64_t row0,
                                                  const uint32_t* __restrict__ hot_n,
                                                  const HotKey* __restrict__ hot, const uint32_t* __restrict__ hot_len,
                                                  const uint32_t* __restrict__ hot_rpre, const uint32_t* __restrict__ hot_rstart,
                                                  uint32_t tiles, const Comp* __restrict__ agg,
                                                  const uint32_t* __restrict__ hot_cond, const HotS0* __restrict__ hot_s0,
                                                  uint64_t* __restrict__ tbl_val, uint32_t* __restrict__ tbl_word,
                                                  uint64_t* __restrict__ tbl_ci, uint64_t* __restrict__ tbl_ins,
                                                  uint8_t* __restrict__ rst_status, uint64_t* __restrict__ rst_value,
                                                  uint32_t* __restrict__ hot_msz, CvCtx cv, HotClr hc,
                                                  uint32_t* __restrict__ err_out) {
  __shared__ uint32_t pfx[kHotMax + 1];
  __shared__ Comp wtot[kHT / kWave];
  __shared__ Comp carry;
  __shared__ uint32_t lrpre[kMaxTiles + 1], lrst[kMaxTiles];
  __shared__ uint32_t evw[kHT / kWave], evbase;  // the item's map events: per-wave counts, the workgroup's reservation
  __shared__ uint32_t iflag;                      // the item's map flags (bit 0 events, bit 1 cleared)
  uint32_t nh;
  hot_items(hot_n, hot_len, pfx, nh);
  const uint32_t t = threadIdx.x, w = t >> 6, l = t & 63;
  uint32_t err = 0;
  for (uint32_t item = blockIdx.x; item < pfx[nh]; item += gridDim.x) {
    const uint32_t h = hot_item_key(pfx, nh, item);
    const uint32_t slot = hot[h].ident & kMwSlotMask;
    // The map's flags are read once, by thread 0, for the whole workgroup (every branch around the event
    // reservation's barriers below is item-uniform).  They do not change while this kernel runs: d_msmall is written
    // on the engine stream only (common.h, the small-map window invariant; a replay on the side stream marks its own
    // buffer, folded in after the engine stream waited for it).
    const uint32_t f0 = t == 0 ? (hot_events(hc, slot) ? 1u : 0u) | (hot_cleared(hc, slot) ? 2u : 0u) : 0u;
    hot_runs_lds(hot_rpre, hot_rstart, h, tiles, lrpre, lrst, &iflag, f0);
    const uint32_t p = item - pfx[h], L = hot_len[h], P = pfx[h + 1] - pfx[h];
    const HotS0 s0 = hot_s0[h];
    const uint32_t pos = hot[h].pos;
    // size-change codes of the key's list (launch_map_size): 2 bits per list position, 16 per word, word
    // pfx[h] * kHotPiece / 16 + position / 16 (a thread's kHPer positions of a piece are whole bytes of one word)
    uint32_t* const msz = hot_msz + (uint64_t)pfx[h] * (kHotPiece / 16);
    ListCursor cur{lrpre, lrst, tiles, 0, 0, 0, 0};
    const bool fl = (iflag & 2u) != 0;   // its map is cleared in this sub-batch (item-uniform)
    const bool evs = (iflag & 1u) != 0;  // its insertions / removals are map events (item-uniform)
    if (hot_cond[h]) {  // value-comparing ops on this key: its whole list, in order, on one thread
      if (p == 0 && t == 0) {
        uint32_t sw = s0.w;
        uint64_t sv = s0.v, ci = s0.ci, ins = s0.ins;
        cur.seek(0);
        uint32_t codes = 0, pe = 0;
        for (uint32_t q = 0; q < L; ++q) {
          const uint32_t g = cur.next();
          uint32_t E = 0;
          if (fl) {
            E = hot_epoch(xr[g].meta);
            if (E != pe) {  // cleared before it
              sw &= ~(kMwPresent | kMwVtagMask);
              sv = 0;
            }
            pe = E;
          }
          const uint32_t code = hot_step(g, xr[g].meta, mrec_ab(xr[g], cb, row0, g), xr[g].idx, sw, sv, ci, ins, rst_status,
                                         rst_value, cv, E, err);
          if (evs) hot_map_event(hc, slot, code, xr[g], err);
          codes |= code << (2 * (q % 16));
          if (q % 16 == 15 || q + 1 == L) {
            msz[q / 16] = codes;
            codes = 0;
          }
        }
        tbl_word[pos] = sw;
        tbl_val[pos] = sv;
        tbl_ci[pos] = ci;
        tbl_ins[pos] = ins;
        if (fl) hc.tbl_ep[pos] = (uint8_t)pe;  // (the region launch drops the entry if it predates the last clear)
      }
      continue;
    }
    // carry: the composite of pieces [0, p) (k_hot_carry's exclusive prefix)
    if (t == 0) carry = agg[(uint64_t)h * kHotMaxPieces + p];
    // this thread's commits and their composite
    const uint32_t p0 = p * kHotPiece + t * kHPer;
    const uint32_t e = p0 < L ? (p0 + kHPer < L ? p0 + kHPer : L) : p0;
    uint32_t gs[kHPer], ms[kHPer], es[kHPer];
    Comp c = comp_identity();
    uint32_t pe0 = 0;  // the epoch of the commit before this thread's first (clears in the stream)
    if (fl && p0 > 0 && p0 < L) {
      cur.seek(p0 - 1);
      pe0 = hot_epoch(xr[cur.next()].meta);
    }
    if (p0 < L) cur.seek(p0);
    uint32_t pe = pe0;
#pragma unroll
    for (int q = 0; q < kHPer; ++q) {
      gs[q] = 0;
      ms[q] = 0;
      es[q] = 0;
      if (p0 + q < e) {
        gs[q] = cur.next();
        ms[q] = xr[gs[q]].meta;
        Comp el = element(ms[q], gs[q]);
        if (fl) {  // a clear since the commit before: CLEAR . el (as k_hot_agg)
          es[q] = hot_epoch(ms[q]);
          if (es[q] != pe) el.P = el.A;
          pe = es[q];
        }
        c = compose(c, el);
      }
    }
    const Comp inc = wave_scan(c, l);
    if (l == 63) wtot[w] = inc;
    __syncthreads();
    // exclusive prefix of this thread = carry . waves before . lanes before
    Comp pre = carry;
    for (uint32_t q = 0; q < w; ++q) pre = compose(pre, wtot[q]);
    Comp lanes = comp_identity();
    {
      Comp o;
      o.A.kind = __shfl_up(inc.A.kind, 1, 64);
      o.A.v = __shfl_up(inc.A.v, 1, 64);
      o.A.n = __shfl_up(inc.A.n, 1, 64);
      o.P.kind = __shfl_up(inc.P.kind, 1, 64);
      o.P.v = __shfl_up(inc.P.v, 1, 64);
      o.P.n = __shfl_up(inc.P.n, 1, 64);
      if (l > 0) lanes = o;
    }
    pre = compose(pre, lanes);
    uint32_t codes = 0;
    if (p0 < L) {
      uint32_t sw;
      uint64_t sv, ci, ins;
      materialize(pre, s0, xr, sw, sv, ci, ins);
      static_assert(kHPer == 16 || kHPer == 8 || kHPer == 4, "size-change codes: whole bytes per thread and piece");
      uint32_t qe = pe0;
#pragma unroll
      for (int q = 0; q < kHPer; ++q)
        if (p0 + q < e) {
          if (fl && es[q] != qe) {  // cleared before it
            sw &= ~(kMwPresent | kMwVtagMask);
            sv = 0;
          }
          qe = es[q];
          const uint32_t code = hot_step(gs[q], ms[q], mrec_ab(xr[gs[q]], cb, row0, gs[q]), xr[gs[q]].idx, sw, sv, ci, ins,
                                         rst_status, rst_value, cv, es[q], err);
          codes |= code << (2 * q);
        }
      // (consecutive threads: consecutive words / halves / bytes of the code words, little-endian)
      if (kHPer == 16) msz[p0 / 16] = codes;
      else if (kHPer == 8) reinterpret_cast<uint16_t*>(msz)[p0 / 8] = (uint16_t)codes;
      else reinterpret_cast<uint8_t*>(msz)[p0 / 4] = (uint8_t)codes;
      if (p == P - 1 && e == L) {  // the key's last commit: write the entry back
        tbl_word[pos] = sw;
        tbl_val[pos] = sv;
        tbl_ci[pos] = ci;
        tbl_ins[pos] = ins;
        if (fl) hc.tbl_ep[pos] = (uint8_t)qe;  // (the region launch drops the entry if it predates the last clear)
      }
    }
    if (evs) {  // (item-uniform) the map events of the item's insertions / removals: one reservation for the
                // workgroup (a wave_append per commit step was ~80K atomics on one counter per c3 sub-batch)
      const uint32_t mine = __popc((codes | (codes >> 1)) & 0x55555555u);
      uint32_t inc = mine;
#pragma unroll
      for (int d = 1; d < kWave; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d, kWave);
        if (l >= (uint32_t)d) inc += y;
      }
      if (l == kWave - 1) evw[w] = inc;
      __syncthreads();
      if (t == 0) {
        uint32_t tot = 0;
        for (int q = 0; q < kHT / kWave; ++q) {
          const uint32_t c = evw[q];
          evw[q] = tot;
          tot += c;
        }
        evbase = tot ? atomicAdd(hc.ev_ctl, tot) : 0u;
      }
      __syncthreads();
      uint32_t at = evbase + evw[w] + inc - mine;
#pragma unroll
      for (int q = 0; q < kHPer; ++q) {
        const uint32_t code = (codes >> (2 * q)) & 3u;
        if (code) hot_map_event_at(hc, slot, code, xr[gs[q]], at++, err);
      }
    }
    __syncthreads();
  }
  if (err) atomicOr(err_out, err);
}

int launch_map_hot_detect(const HotArgs& a, hipStream_t st) {
  if (a.hi <= a.lo) return 0;
  const uint64_t n = a.hi - a.lo;
  const uint32_t S = (uint32_t)(n < kDetSample ? n : kDetSample);
  HotSamp* samp = reinterpret_cast<HotSamp*>(a.hot_samp);
  hipLaunchKernelGGL(k_hot_sample, dim3((S + kDetBlk - 1) / kDetBlk), dim3(kDetBlk), 0, st, a.inst, a.flags, a.key, a.lo, a.hi,
                     a.inst_res, a.res_type, a.max_inst, samp);
  hipLaunchKernelGGL(k_hot_count, dim3(1), dim3(kDetT), 0, st, samp, a.lo, a.hi, a.hot_cand, a.hot_cand_n);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_map_hot_bind(const HotArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(k_hot_bind, dim3(1), dim3(kDetT), 0, st, a.hot_cand, a.hot_cand_n, a.map_bits, a.tbl_key, a.tbl_word,
                     a.tbl_val, a.tbl_ci, a.tbl_ins, a.tbl_claim, a.idx0, a.hot, a.hot_n, a.msmall);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_map_hot_apply(const HotArgs& a, hipStream_t st) {
  if (a.tiles == 0) return 0;
  const uint32_t sb_hot = a.sb_val + (1u << a.map_bits);
  a.mark(K_MAP_HOT, 1, st);
  hipLaunchKernelGGL(k_hot_lists, dim3(kHotMax), dim3(kHT), 0, st, a.ttab, a.tiles, a.sb, sb_hot, a.hot, a.hot_n, a.tbl_val,
                     a.tbl_word, a.tbl_ci, a.tbl_ins, a.hot_rpre, a.hot_rstart, a.hot_len, a.hot_cond,
                     reinterpret_cast<HotS0*>(a.hot_s0));
  hipLaunchKernelGGL(k_hot_agg, dim3(kHotGridAgg), dim3(kHT), 0, st, a.hot_meta, a.hot_n, a.hot_len, a.hot_rpre, a.hot_rstart,
                     a.tiles, reinterpret_cast<Comp*>(a.hot_agg), a.hot_cond, a.hot, a.hc);
  hipLaunchKernelGGL(k_hot_carry, dim3(kHotMax), dim3(kHT), 0, st, a.hot_n, a.hot_len, reinterpret_cast<Comp*>(a.hot_agg));
  hipLaunchKernelGGL(k_hot_apply, dim3(kHotGridApply), dim3(kHT), 0, st, a.mrec, a.cb, a.lo, a.hot_n, a.hot, a.hot_len,
                     a.hot_rpre, a.hot_rstart, a.tiles, reinterpret_cast<const Comp*>(a.hot_agg), a.hot_cond,
                     reinterpret_cast<const HotS0*>(a.hot_s0), a.tbl_val, a.tbl_word, a.tbl_ci, a.tbl_ins, a.rst_status,
                     a.rst_value, a.hot_msz, a.cv, a.hc, a.err);
  a.mark(K_MAP_HOT, 0, st);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

size_t hot_agg_bytes() { return sizeof(Comp) * (size_t)kHotMax * kHotMaxPieces; }
size_t hot_s0_bytes() { return sizeof(HotS0) * (size_t)kHotMax; }

}  // namespace cc
