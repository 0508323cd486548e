// map_small.hip — the java.util.HashMap of a map whose table is still small (capacity <= 64), followed key by key.
//
// MapState keeps its entries in a `new HashMap<>()` (collections/src/main/java/io/atomix/collections/state/
// MapState.java:33), and containsValue (:49-60) walks map.values(): the answer (true, or the NullPointerException of
// a stored null met first) depends on the table's capacity.  The size-driven resizes are tracked by
// launch_map_size (map_wide.hip).  Below capacity 64 there is a second trigger: java.util.HashMap.putVal calls
// treeifyBin when a new key makes its bin's chain 9 long, and treeifyBin RESIZES a table under MIN_TREEIFY_CAPACITY
// (64) instead of treeifying -- at any size.  At capacity 64 the same bin becomes a red-black tree bin, whose
// iteration order (root first, later keys linked after their tree parent) the engine follows here node for node.
//
// Per map in that window the engine keeps the map's HashMap node for node (small_jhm.h: at most 49 nodes) and
// replays its insertions and removals in log order:
//   1. launch_map_size's count kernel (k_msize_count) emits one event per region commit of a small map that inserted
//      or removed a key: key (map << 36 | (log index - the sub-batch's first) << 4 | insert / remove), value = the
//      key's HashMap hash (k_hot_apply emits the same for the map's hot-key commits);
//   2. a radix sort by that key puts each map's events in log order (hipcub);
//   3. alternating remove / put chains of one key are marked for skipping (k_small_chains), then one wave per map
//      stages its events in LDS and lane 0 replays them on an LDS copy of its HashMap: putVal (a chain of 9 calls treeifyBin: a
//      resize below 64, a red-black tree bin at 64), resize, removeNode.  The map leaves the window when its capacity
//      passes 64; a bin that was a tree bin there keeps its mark (tree_bins; see map_wide.hip k_mw_order for the
//      checks above 64).  Inside the window an order-dependent containsValue reads a bin's chain from this model.
// The capacity level reached is merged into the tracked level (mpcap, atomicMax): the true capacity is the larger of
// the size-driven one and the early one (after the window both grow by size alone).
// Cost: nothing once every map has left the window (the host stops looking: no event, no sync); while some are in
// it, one host read of the event count per sub-batch, a sort of the events and one short serial walk per map.
//
// TTL mode (common.h TtlEmit): timers remove keys with no commit, so there every map's commits AND expiries are events
// (an expiry positioned at the boundary where the reference fires the timer, A8), and after the sort k_ttl_replay
// walks each map's run for its size and peak (capacity) while k_small_replay follows the small maps' key sets as
// above: sizes, capacities and small tables stay exact in both modes.
#include <hipcub/hipcub.hpp>

#include "common.h"
#include "engine_internal.h"
#include "small_jhm.h"

namespace cc {

// event runs: the first event of each map's run (the sort put one map's events together, in log order)
__global__ void k_small_seg(const uint64_t* __restrict__ key, const uint32_t* __restrict__ ctl, uint32_t* __restrict__ seg,
                            uint32_t* __restrict__ nseg) {
  const uint32_t E = ctl[0];
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < E; i += gridDim.x * blockDim.x)
    if (i == 0 || (key[i] >> kEvMapShift) != (key[i - 1] >> kEvMapShift)) seg[atomicAdd(nseg, 1u)] = i;
}

// Alternating runs of one key (a hot key of a small map: remove k, put k, remove k, put k, ... with no other event of
// the map between): in a list bin of <= 7 nodes after the removal, the net effect of remove k . put k is k moved to
// its chain's end, with the size back where it was (no resize) and a chain of <= 8 (no treeifyBin), so
// R P R P ... R P == R P and R P ... R == R.  (A list chain of 9 does persist below capacity 64 -- treeifyBin's
// resize keeps it whole when its keys share the new bit -- and a put into it calls treeifyBin again: such a bin, and
// a tree bin, replays every event.)  The maximal alternating chains (commit events only: a clear, a size query or
// another key ends one) are found flat over the sorted events: event i links to i - 1 when both are commits of the
// same map and key with different codes; a max-scan of (i if it does not link) gives every event its chain's start;
// at each chain's end the number of events implied after its first removal is stored there (EvPay.ktag >> 4), and
// k_small_replay checks the bin at that removal.  (It was one wave per map walking 64 events per step: ~5.5 ms per sub-batch for a hot map.)
__device__ inline uint32_t chain_code(uint64_t k) {
  return !(k & 8u) && ((k & 3u) == 1u || (k & 3u) == 2u) ? (uint32_t)(k & 3u) : 0u;
}
struct ChainStart {  // i when event i starts a chain (does not link to i - 1), else 0
  const uint64_t* key;
  const uint32_t* val;
  const EvPay* pay;
  __device__ uint32_t operator()(uint32_t i) const {
    if (i == 0) return 0;
    const uint64_t k = key[i], q = key[i - 1];
    const uint32_t c = chain_code(k), cq = chain_code(q);
    if (!c || !cq || c == cq || (k >> kEvMapShift) != (q >> kEvMapShift)) return i;
    const EvPay x = pay[val[i]], y = pay[val[i - 1]];
    const bool link = x.key == y.key && x.aux == y.aux && (x.ktag & 3u) == (y.ktag & 3u);
    return link ? 0u : i;
  }
};
using ChainIt = hipcub::TransformInputIterator<uint32_t, ChainStart, hipcub::CountingInputIterator<uint32_t>>;
size_t chain_scan_temp_bytes(uint32_t cap) {
  size_t need = 0;
  ChainIt it(hipcub::CountingInputIterator<uint32_t>(0), ChainStart{nullptr, nullptr, nullptr});
  (void)hipcub::DeviceScan::InclusiveScan(nullptr, need, it, (uint32_t*)nullptr, hipcub::Max(), (int)cap, (hipStream_t)0);
  return need;
}
__global__ __launch_bounds__(256) void k_small_chains(const uint64_t* __restrict__ key, const uint32_t* __restrict__ val,
                                                      EvPay* __restrict__ pay, const uint32_t* __restrict__ start, uint32_t E,
                                                      const uint8_t* __restrict__ msmall) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < E; i += gridDim.x * blockDim.x) {
    const uint32_t s0 = start[i];
    if (s0 == i) continue;                               // (a chain of one event)
    if (i + 1 < E && start[i + 1] != i + 1) continue;    // not the chain's end
    const uint64_t k = key[i];
    // (out of the window: not replayed.  The snapshot, not the model's kSmIn: an earlier sub-batch's replay may be
    // writing the model meanwhile; a map the snapshot still shows in the window is skipped by the replay itself)
    if (!(msmall[k >> kEvMapShift] & kMfSmall)) continue;
    const uint32_t r0 = (key[s0] & 3u) == 1u ? s0 + 1 : s0;  // the chain's first removal
    if (i <= r0) continue;
    const uint32_t skip = (k & 3u) == 1u ? i - r0 - 1 : i - r0;
    if (skip) pay[val[r0]].ktag |= skip << kSkipShift;
  }
}
// The events k_small_replay walks: those of maps in the window, less the ones a chain implies (after its first
// removal, all but a final put).  Compacted once (hipcub select), the hot map's ~180K events per c3 sub-batch are
// ~2.5K to replay, read 64 at a time, instead of a fresh dependent read at every chain end.  The replay steps into
// the implied ones only when the chain's bin is a tree bin there (rare: tables of 64 with a bin of 9).
struct ChainKeep {
  const uint64_t* key;
  const uint32_t* start;
  const uint8_t* msmall;  // the engine stream's snapshot (common.h, the small-map window invariant)
  uint32_t E;
  __device__ uint8_t operator()(uint32_t i) const {
    const uint64_t k = key[i];
    if (!(msmall[k >> kEvMapShift] & kMfSmall)) return 0;  // (not replayed)
    const uint32_t s0 = start[i];
    if (s0 == i) return 1;
    const uint32_t r0 = (key[s0] & 3u) == 1u ? s0 + 1 : s0;
    if (i <= r0) return 1;
    const bool end = i + 1 == E || start[i + 1] == i + 1;
    return end && (k & 3u) == 1u ? 1 : 0;
  }
};
using KeepIt = hipcub::TransformInputIterator<uint8_t, ChainKeep, hipcub::CountingInputIterator<uint32_t>>;
size_t keep_select_temp_bytes(uint32_t cap) {
  size_t need = 0;
  KeepIt it(hipcub::CountingInputIterator<uint32_t>(0), ChainKeep{nullptr, nullptr, nullptr, 0});
  (void)hipcub::DeviceSelect::Flagged(nullptr, need, hipcub::CountingInputIterator<uint32_t>(0), it, (uint32_t*)nullptr,
                                      (uint32_t*)nullptr, (int)cap, (hipStream_t)0);
  return need;
}
// the compacted events' runs (one per map)
__global__ void k_small_cseg(const uint64_t* __restrict__ key, const uint32_t* __restrict__ orig, uint32_t* __restrict__ cseg,
                             uint32_t R) {
  const uint32_t n = cseg[R + 1];
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    if (i == 0 || (key[orig[i]] >> kEvMapShift) != (key[orig[i - 1]] >> kEvMapShift)) cseg[atomicAdd(&cseg[R], 1u)] = i;
}

// One wave per run: the map's java.util.HashMap loaded into the wave's registers (small_jhm.h: node i and bin i in
// lane i), its events staged 64 at a time, one per lane (coalesced loads and one gather), then applied in log order
// by the whole wave in lockstep (putVal of a new key, removeNode; every value uniform, each event read from its lane
// with v_readlane), the state written back.  A map whose table passes 64 leaves the window (its later events are not
// followed).  (One thread per run walked the events with three dependent global loads each: ~2.4 ms per c3
// sub-batch for a hot map; an LDS copy walked by one lane still paid ~100 cycles per dependent field access.)
#ifdef CC_PHASE_TIMING  // diagnostics build (CC_SMALL_PHASES=1 cc_debug_phases(K_APPLY_MAP)): the replay's serial work
__device__ unsigned long long g_ph_small[kPhases];  // events applied, max per map, runs, ticks, max ticks, max run length
int phase_read_small(uint64_t* out) {
  unsigned long long z[kPhases] = {};
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ph_small), sizeof z) != hipSuccess ||
      hipMemcpyToSymbol(HIP_SYMBOL(g_ph_small), z, sizeof z) != hipSuccess)
    return CC_ERR_HIP;
  return CC_OK;
}
#endif
constexpr int kSrW = 4;  // runs (waves) per workgroup
__device__ inline uint32_t rlane(uint32_t v, uint32_t i) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)i); }
__device__ inline uint64_t rlane64(uint64_t v, uint32_t i) {
  return (uint64_t)rlane((uint32_t)(v >> 32), i) << 32 | rlane((uint32_t)v, i);
}
__global__ __launch_bounds__(kSrW * kWave) void k_small_replay(const uint64_t* __restrict__ key, const uint32_t* __restrict__ val,
                                                              const EvPay* __restrict__ pay, const uint32_t* __restrict__ orig,
                                                              const uint32_t* __restrict__ ctl,
                                                              const uint32_t* __restrict__ seg, const uint32_t* __restrict__ nseg,
                                                              SmallMap* __restrict__ st, BigMap* __restrict__ big,
                                                              uint8_t* __restrict__ left,
                                                              const uint8_t* __restrict__ msmall,
                                                              uint32_t* __restrict__ mpcap, unsigned long long* __restrict__ lvl_at,
                                                              const uint64_t* __restrict__ idx0, const uint64_t* __restrict__ index,
                                                              uint64_t lo, bool ttl, uint32_t* __restrict__ err) {
  const uint32_t wv = threadIdx.x / kWave, l = __lane_id();
  const uint32_t E = ctl[0], ns = *nseg;
  for (uint32_t r = blockIdx.x * kSrW + wv; r < ns; r += gridDim.x * kSrW) {  // (wave-uniform)
    const uint32_t start = seg[r];
    const uint32_t m = (uint32_t)(key[orig ? orig[start] : start] >> kEvMapShift);
    SmallMap* s = st + m;
    if (!(s->flags & kSmIn)) continue;  // (left the window earlier: its events in a lagging snapshot are skipped)
#ifdef CC_DIAG  // the window invariant: the snapshot keeps every map whose model is in the window (no 0 -> 1 flip)
    if (l == 0 && !(__hip_atomic_load(&msmall[m], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & kMfSmall))
      atomicOr(err, kErrSmallFlag);
#else
    (void)msmall;
    (void)err;
#endif
    SmallJhm j;
    j.load(*s);
#ifdef CC_PHASE_TIMING
    const uint64_t t_run = wall_clock64();
    uint32_t n_app = 0;
#endif
    uint64_t leave_pos = 0;  // the event that grew the table past 64
    // one insertion / removal on the model (the whole wave, uniform arguments); false: the table passed 64
    auto apply = [&](uint64_t kk, uint64_t ykey, uint32_t yh, uint32_t ykt) -> bool {
#ifdef CC_PHASE_TIMING
      ++n_app;
#endif
      if ((kk & 3u) == 1u) {  // a new key: HashMap.putVal
        const uint32_t lv0 = j.lvl;
        const bool stay = j.put(yh, ykt, ykey);
        if (j.lvl > lv0 && lvl_at && l == 0) {  // the table grew at this commit: the capacity-level timeline (common.h)
          const uint64_t d = (kk >> 4) & kEvPosMask;
          // (an index that cannot be known is not recorded: "not left yet" only over-counts, toward refusing)
          if (ttl ? index != nullptr : idx0 != nullptr)
            lvl_reached(lvl_at, m, lv0, j.lvl, ttl ? index[lo + (d - 1) / 2] : *idx0 + d);
        }
        if (!stay) leave_pos = (kk >> 4) & kEvPosMask;
        return stay;
      }
      j.remove(yh, ykt, ykey);  // a key removed: removeNode
      return true;
    };
    uint32_t i = start;
    bool fin = false;
#ifdef CC_PHASE_TIMING
    uint64_t t_stage = 0;
#endif
    while (!fin && i < E) {  // (wave-uniform)
#ifdef CC_PHASE_TIMING
      const uint64_t ts0 = wall_clock64();
#endif
      // lane l stages event i + l: its key (~0: another map's, or past the end), payload, sorted position
      const uint32_t ii = i + l;
      uint64_t k = ~0ull, xkey = 0;
      uint32_t xaux = 0, xkt = 0, o = 0;
      if (ii < E) {
        o = orig ? orig[ii] : ii;
        const uint64_t kk = key[o];
        if ((uint32_t)(kk >> kEvMapShift) == m) {
          k = kk;
          if (!(kk & 8u) && (kk & 3u) != 3u) {  // (a commit: its key; a clear or a query has none)
            const EvPay x = pay[val[o]];
            xkey = x.key;
            xaux = x.aux;
            xkt = x.ktag;
          }
        }
      }
#ifdef CC_PHASE_TIMING
      {  // (the staged values must have landed: a use of each)
        const uint32_t dep = (uint32_t)k ^ (uint32_t)xkey ^ xaux ^ xkt ^ o;
        if (__builtin_amdgcn_readfirstlane((int)dep) == 0x7FFFFFFF) n_app += 0;
        t_stage += wall_clock64() - ts0;
      }
#endif
      uint32_t q = 0;
      for (; q < (uint32_t)kWave; ++q) {
        const uint64_t kk = rlane64(k, q);
        if (kk == ~0ull) {  // the map's run ended
          fin = true;
          break;
        }
        if (kk & 8u) continue;  // a size / isEmpty query (k_size_answer)
        if ((kk & 3u) == 3u) {  // MapState.clear in the stream (map_clear.hip): every key leaves, the table stays
          j.w1 &= ~0xFF0000u;   // (every bin head)
          j.n = 0;
          j.used = 0;
          j.flags &= ~(kSmTree | kSmAmbig);
          j.tree_bins = 0;
          continue;
        }
        const uint64_t ykey = rlane64(xkey, q);
        const uint32_t yh = rlane(xaux, q), ykt = rlane(xkt, q);
        // a removal followed by the put of the same key (a hot key's remove / put, or the two ends of a compacted
        // alternating run): a no-op when the key is the last node of a list bin of <= 8 nodes
        if ((kk & 3u) == 2u && q + 1 < (uint32_t)kWave) {
          const uint64_t kn = rlane64(k, q + 1);
          if (kn != ~0ull && chain_code(kn) == 1u && rlane64(xkey, q + 1) == ykey && rlane(xaux, q + 1) == yh &&
              (rlane(xkt, q + 1) & 3u) == (ykt & 3u) && j.list_tail(yh, ykt & 3u, ykey, 8)) {
            ++q;  // (and every remove / put pair the run implies between them: the key stays the tail)
            continue;
          }
        }
        if (!apply(kk, ykey, yh, ykt & 3u)) {  // the table passed 64: out of the window
          fin = true;
          break;
        }
        // a removal starting an alternating run of its key (k_small_chains): in a list bin of <= 7 nodes after it
        // the run's events after it are implied (the compacted events leave them out; else skipped here); in a tree
        // bin, or a list bin long enough for a put to call treeifyBin, each is applied
        const uint32_t skip = (kk & 3u) == 2u ? ykt >> kSkipShift : 0u;
        if (skip) {
          const bool implied = j.list_len(yh) <= 7u;
          if (!orig) {
            if (implied) q += skip;
          } else if (!implied) {
            const uint32_t o0 = rlane(o, q);
            for (uint32_t u = o0 + 1; u <= o0 + skip && !fin; ++u) {
              const EvPay z = pay[val[u]];
              if (!apply(key[u], z.key, z.aux, z.ktag & 3u)) fin = true;
            }
            if (fin) break;
          }
        }
      }
      i += q;
    }
#ifdef CC_PHASE_TIMING
    if (l == 0) {
      const uint64_t dt = wall_clock64() - t_run;
      atomicAdd(&g_ph_small[0], (unsigned long long)n_app);
      atomicMax(&g_ph_small[1], (unsigned long long)n_app);
      atomicAdd(&g_ph_small[2], 1ull);
      atomicAdd(&g_ph_small[3], (unsigned long long)dt);
      atomicMax(&g_ph_small[4], (unsigned long long)dt);
      atomicMax(&g_ph_small[5], (unsigned long long)(i - start));
      atomicAdd(&g_ph_small[6], (unsigned long long)t_stage);
    }
#endif
    // with a tree bin since the last clear: a big model follows the map from here (map_big.hip k_big_replay takes the
    // model over, right after this kernel; the map keeps its events)
    const bool to_big = !(j.flags & kSmIn) && big && (j.flags & kSmTree);
    if (to_big) j.flags |= kSmBig | kSmBigNew;
    else if (!(j.flags & kSmIn)) {  // only the capacity level and the tree bins matter from here on
      j.n = 0;
      j.used = 0;
    }
    j.store(*s);
    if (l == 0) {  // the map left the window: a mark for the engine stream's fold (d_msmall is not written here)
      if (to_big) s->pad = (uint32_t)leave_pos;
      else if (!(j.flags & kSmIn)) left[m] = 1;
      atomicMax(&mpcap[m], j.lvl);
    }
  }
}

// ---- TTL mode: exact sizes and capacities with timers (common.h TtlEmit) ------------------------------------
// Every table entry whose timer fires at a boundary this sub-batch owns (or, for cc_advance_time, by the new clock)
// and was not seen expiring by a commit of the sub-batch (k_apply_map<true> emits those itself): an expiry event.  An
// entry that expired is still in the table (its key is bound, lazily absent) until a commit or a compaction drops it;
// the boundary ownership keeps every expiry to one event.
__global__ void k_ttl_scan(TtlEmit t, const uint64_t* __restrict__ clock_base, const uint32_t* __restrict__ word,
                           const uint64_t* __restrict__ key, const uint64_t* __restrict__ dl, uint64_t entries,
                           uint32_t* __restrict__ err_out) {
  const uint64_t cb = *clock_base;
  uint32_t err = 0;
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < entries; e += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t d = dl[e];
    if (!d) continue;
    const uint32_t w = word[e];
    if (!(w & kMwUsed) || (w & kMwDead) || !(w & kMwPresent)) continue;
    ttl_expiry_event(t, cb, w, key[e], d, err);
  }
  if (err) atomicOr(err_out, err);
}

// One wave per map run of the sorted events: the size at the run's start (msize), the running size over its commits
// and expiries in log order, its peak -> the capacity level (HashMap.resize never shrinks), the size at the end; a
// size / isEmpty row among them (MapState.size :233-239, isEmpty :244-250) gets the size before it.
__global__ __launch_bounds__(256) void k_ttl_replay(const uint64_t* __restrict__ key, const uint32_t* __restrict__ val,
                                                    const EvPay* __restrict__ pay, const uint32_t* __restrict__ ctl,
                                                    const uint32_t* __restrict__ seg, const uint32_t* __restrict__ nseg,
                                                    uint32_t* __restrict__ msize, uint32_t* __restrict__ mpcap,
                                                    unsigned long long* __restrict__ lvl_at, const uint64_t* __restrict__ index,
                                                    uint64_t lo, uint8_t* __restrict__ out_status, uint64_t* __restrict__ out_value) {
  const uint32_t E = ctl[0], ns = *nseg, l = __lane_id();
  const uint32_t waves = gridDim.x * (blockDim.x / kWave);
  for (uint32_t r = blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave); r < ns; r += waves) {
    const uint32_t start = seg[r];
    const uint32_t m = (uint32_t)(key[start] >> kEvMapShift);
    int64_t size = msize[m], peak = size;
    for (uint32_t b = start;; b += kWave) {
      const uint32_t i = b + l;
      const bool in = i < E && (uint32_t)(key[i] >> kEvMapShift) == m;
      const uint64_t k = in ? key[i] : 0;
      const int32_t dlt = !in || (k & 8u) ? 0 : ((k & 3u) == 1u ? 1 : ((k & 3u) == 2u ? -1 : 0));
      int32_t inc = dlt;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int32_t y = __shfl_up(inc, d, 64);
        if (l >= (uint32_t)d) inc += y;
      }
      if (in && (k & 8u) && out_status) {  // a query: the size before it (its own delta is 0)
        const int64_t at = size + inc;
        const uint32_t row = pay[val[i]].aux;
        if (k & 4u) {  // isEmpty
          out_status[row] = CC_STATUS(CC_ST_OK, CC_TAG_BOOL);
          out_value[row] = at == 0 ? 1ull : 0ull;
        } else {  // size: an int
          out_status[row] = CC_STATUS(CC_ST_OK, CC_TAG_INT);
          out_value[row] = (uint64_t)at;
        }
      }
      int32_t mx = inc;
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) mx = max(mx, __shfl_xor(mx, d, 64));
      if (lvl_at && index && dlt > 0 && size + inc > peak) {  // a commit growing the table (common.h timeline)
        const uint64_t d = (k >> 4) & kEvPosMask;  // (commits sit at odd positions 2 (row - lo) + 1)
        lvl_reached(lvl_at, m, cap_level((uint64_t)max<int64_t>(peak, 0)), cap_level((uint64_t)(size + inc)),
                    index[lo + (d - 1) / 2]);
      }
      peak = max(peak, size + mx);
      size += __shfl(inc, 63, 64);
      if (__ballot(in) != ~0ull) break;
    }
    if (l == 0) {
      msize[m] = (uint32_t)max<int64_t>(size, 0);
      atomicMax(&mpcap[m], cap_level((uint64_t)max<int64_t>(peak, 0)));
    }
  }
}

int launch_ttl_scan(const TtlEmit& t, const uint64_t* clock_base, const uint32_t* word, const uint64_t* key,
                    const uint64_t* dl, uint64_t entries, uint32_t* err, hipStream_t st) {
  if (entries == 0) return 0;
  const uint32_t grid = (uint32_t)std::min<uint64_t>(2048, (entries + 255) / 256);
  hipLaunchKernelGGL(k_ttl_scan, dim3(grid), dim3(256), 0, st, t, clock_base, word, key, dl, entries, err);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// maps still in the window (read by the host with the next sub-batch's event count)
__global__ void k_small_count(const uint8_t* __restrict__ msmall, uint32_t R, uint32_t* __restrict__ ctl) {
  uint32_t c = 0;
  for (uint32_t m = blockIdx.x * blockDim.x + threadIdx.x; m < R; m += gridDim.x * blockDim.x) c += msmall[m] & kMfSmall;
  for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d, 64);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(&ctl[1], c);
}

// MapState.delete (clear / Delete, :255-274): every key leaves; the table keeps its capacity; no tree bin is left
__global__ void k_small_clear(SmallMap* __restrict__ st, uint32_t m) {
  SmallMap& s = st[m];
  const uint32_t t = threadIdx.x;
  s.tab[t] = 0;  // (64 threads: one bin head each)
  if (t == 0) {
    s.n = 0;
    s.used = 0;
    s.flags &= ~(kSmTree | kSmAmbig);
    s.tree_bins = 0;
  }
}

// ---- map size / isEmpty in the stream (MapState.size :233-239, isEmpty :244-250), outside TTL mode ---------------
// The size at a row is the size at the sub-batch's end (the exact tracking, msize) minus the map's net insertions of
// the sub-batch, plus those before the row.  The map's insertions / removals are the events k_msize_count emits for
// flagged maps; the queries join them in the same buffer (key bit 3, after the commit whose index they carry: a
// query takes the index of the command before it), so the radix sort puts each map's events and queries in log order.
// In TTL mode a query sits at its row's position 2 (row - lo) + 1 (common.h TtlEmit): after the timers that fire at
// its boundary, before the commits after it; k_ttl_replay answers it with the running size.
__global__ void k_size_emit(const uint32_t* __restrict__ szq, uint32_t szq_n, uint64_t lo, uint64_t hi,
                            const uint32_t* __restrict__ inst, const uint8_t* __restrict__ op,
                            const uint64_t* __restrict__ index, const uint32_t* __restrict__ inst_res,
                            uint64_t* __restrict__ ev_key, uint32_t* __restrict__ ev_val, EvPay* __restrict__ ev_pay,
                            uint32_t cap, uint32_t* __restrict__ ctl, bool ttl, uint32_t* __restrict__ err) {
  const uint64_t idx0 = ttl ? 0 : index[lo];
  for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < szq_n; q += gridDim.x * blockDim.x) {
    const uint32_t row = szq[q];
    if (row < lo || row >= hi) continue;
    const uint32_t m = inst_res[inst[row]];  // (listed by the barrier scan on a live map: the registry is fixed in a batch)
    const uint64_t d = ttl ? 2 * (row - lo) + 1 : index[row] - idx0;
    if (d >> kEvPosBits) atomicOr(err, kErrSpan);
    const uint32_t at = atomicAdd(ctl, 1u);
    if (at < cap) {
      ev_key[at] = ((uint64_t)m << kEvMapShift) | ((d & kEvPosMask) << 4) | 8u | (op[row] == CC_OP_MAP_ISEMPTY ? 4u : 0u);
      ev_val[at] = at;
      ev_pay[at] = EvPay{0, row, 0};
    }
  }
}

// One wave per map run of the sorted buffer: the run's net change, then a wave-wide running count; each query row
// gets the size before it (events with its index come first: a query follows the command whose index it carries).
__global__ __launch_bounds__(256) void k_size_answer(const uint64_t* __restrict__ key, const uint32_t* __restrict__ val,
                                                     const EvPay* __restrict__ pay, const uint32_t* __restrict__ ctl, const uint32_t* __restrict__ seg,
                                                     const uint32_t* __restrict__ nseg, const uint32_t* __restrict__ msize,
                                                     uint8_t* __restrict__ out_status, uint64_t* __restrict__ out_value) {
  const uint32_t E = ctl[0], ns = *nseg, l = __lane_id();
  const uint32_t waves = gridDim.x * (blockDim.x / kWave);
  for (uint32_t r = blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave); r < ns; r += waves) {
    const uint32_t start = seg[r];
    const uint32_t m = (uint32_t)(key[start] >> kEvMapShift);
    int32_t net = 0;
    bool queries = false;
    uint32_t end = start;
    for (uint32_t b = start;; b += kWave) {  // pass 1: the run's end, net change, and whether it holds a query
      const uint32_t i = b + l;
      const bool in = i < E && (uint32_t)(key[i] >> kEvMapShift) == m;
      const uint64_t k = in ? key[i] : 0;
      const int32_t dlt = !in || (k & 8u) ? 0 : ((k & 3u) == 1u ? 1 : ((k & 3u) == 2u ? -1 : 0));
      int32_t sum = dlt;
      for (int d = 32; d >= 1; d >>= 1) sum += __shfl_xor(sum, d, 64);
      net += sum;
      queries |= __ballot(in && (k & 8u)) != 0;
      const uint64_t inb = __ballot(in);
      end = b + (uint32_t)__builtin_popcountll(inb);
      if (inb != ~0ull) break;
    }
    if (!queries) continue;
    int32_t size = (int32_t)msize[m] - net;  // at the sub-batch's start
    for (uint32_t b = start; b < end; b += kWave) {  // pass 2: running size, answers
      const uint32_t i = b + l;
      const bool in = i < end;
      const uint64_t k = in ? key[i] : 0;
      const int32_t dlt = !in || (k & 8u) ? 0 : ((k & 3u) == 1u ? 1 : ((k & 3u) == 2u ? -1 : 0));
      int32_t inc = dlt;
      for (int d = 1; d < 64; d <<= 1) {
        const int32_t y = __shfl_up(inc, d, 64);
        if (l >= (uint32_t)d) inc += y;
      }
      if (in && (k & 8u)) {
        const int32_t at = size + inc;  // (a query's own delta is 0: inc counts the events before it)
        const uint32_t row = pay[val[i]].aux;
        if (k & 4u) {  // isEmpty
          out_status[row] = CC_STATUS(CC_ST_OK, CC_TAG_BOOL);
          out_value[row] = at == 0 ? 1ull : 0ull;
        } else {  // size: an int
          out_status[row] = CC_STATUS(CC_ST_OK, CC_TAG_INT);
          out_value[row] = (uint64_t)(int64_t)at;
        }
      }
      size += __shfl(inc, 63, 64);
    }
  }
}

__global__ void k_mflag_clear(uint8_t* __restrict__ mflag, uint32_t R) {
  for (uint32_t m = blockIdx.x * blockDim.x + threadIdx.x; m < R; m += gridDim.x * blockDim.x)
    mflag_and(mflag, m, (uint8_t)~(kMfSize | kMfCv | kMfClr));
}

// The fold of a finished replay's exit marks into the engine stream's snapshot (common.h, the small-map window
// invariant): launched on the engine stream right after it waits for that replay; the marks are cleared for the
// set's next replay.  A word of 4 maps per thread (the byte arrays are padded to whole words).
__global__ void k_small_fold(uint8_t* __restrict__ left, uint8_t* __restrict__ msmall, uint32_t R) {
  for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; 4 * q < R; q += gridDim.x * blockDim.x) {
    uint32_t lw = 0;
    for (uint32_t b = 0; b < 4 && 4 * q + b < R; ++b) lw |= (uint32_t)left[4 * q + b] << (8 * b);
    if (!lw) continue;
    uint32_t keep = ~0u;
    for (uint32_t b = 0; b < 4; ++b)
      if ((lw >> (8 * b)) & 0xFFu) keep &= ~((uint32_t)kMfSmall << (8 * b));
    reinterpret_cast<uint32_t*>(msmall)[q] &= keep;
    for (uint32_t b = 0; b < 4 && 4 * q + b < R; ++b) left[4 * q + b] = 0;
  }
}

int launch_small_fold(uint8_t* left, uint8_t* msmall, uint32_t R, hipStream_t st) {
  hipLaunchKernelGGL(k_small_fold, dim3(std::min<uint32_t>(256, (R / 4 + 256) / 256)), dim3(256), 0, st, left, msmall, R);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_size_emit(const SizeArgs& a, hipStream_t st) {
  if (a.szq_n == 0) return 0;
  hipLaunchKernelGGL(k_size_emit, dim3(std::min<uint32_t>(1024, (a.szq_n + 255) / 256)), dim3(256), 0, st, a.szq, a.szq_n,
                     a.lo, a.hi, a.inst, a.op, a.index, a.inst_res, a.ev_key, a.ev_val, a.ev_pay, a.cap, a.ctl, a.ttl, a.err);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_size_answer(const SizeArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(k_size_answer, dim3(256), dim3(256), 0, st, a.sorted_key, a.sorted_val, a.ev_pay, a.ctl, a.seg, a.nseg,
                     a.msize, a.out_status, a.out_value);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// The first row of [lo, hi) whose log index is 2^32 or more past index[lo] (kEvPosBits: a map event's position), by
// binary search over the increasing index column; *out stays ~0 when none is.
__global__ void k_span_cut(const uint64_t* __restrict__ index, uint64_t lo, uint64_t hi, uint64_t* __restrict__ out) {
  if (threadIdx.x != 0) return;
  const uint64_t i0 = index[lo];
  uint64_t a = lo, b = hi;  // the first row in [a, b) past the span
  while (a < b) {
    const uint64_t mid = a + (b - a) / 2;
    if (index[mid] - i0 >= (1ull << kEvPosBits)) b = mid;
    else a = mid + 1;
  }
  if (a < hi) *out = a;
}

int launch_span_cut(const uint64_t* index, uint64_t lo, uint64_t hi, uint64_t* out, hipStream_t st) {
  hipLaunchKernelGGL(k_span_cut, dim3(1), dim3(64), 0, st, index, lo, hi, out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_mflag_clear(uint8_t* mflag, uint32_t R, hipStream_t st) {
  hipLaunchKernelGGL(k_mflag_clear, dim3(std::min<uint32_t>(256, (R + 255) / 256)), dim3(256), 0, st, mflag, R);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_small_replay(const SmallArgs& a, uint32_t E, hipStream_t st, hipStream_t rst) {
  if (E > a.cap) return -2;
  if (E) {
    // the key bits in use: the position and code, then the map slot (< max_resources): 6 digit passes for 4096 maps
    int end_bit = (int)kEvMapShift;
    while (end_bit < 64 && (a.max_resources - 1) >> (end_bit - kEvMapShift)) ++end_bit;
    size_t need = 0;
    if (hipcub::DeviceRadixSort::SortPairs(nullptr, need, a.ev_key, a.ev_key2, a.ev_val, a.ev_val2, (int)E, 0, end_bit,
                                           st) != hipSuccess)
      return -1;
    if (need > a.temp_bytes) return -3;  // (sized for cap events at creation)
    size_t tb = a.temp_bytes;
    if (hipcub::DeviceRadixSort::SortPairs(a.temp, tb, a.ev_key, a.ev_key2, a.ev_val, a.ev_val2, (int)E, 0, end_bit, st) !=
        hipSuccess)
      return -1;
    if (hipMemsetAsync(a.nseg, 0, sizeof(uint32_t), st) != hipSuccess) return -1;
    const uint32_t grid = (uint32_t)std::min<uint64_t>(1024, (E + 255) / 256);
    hipLaunchKernelGGL(k_small_seg, dim3(grid), dim3(256), 0, st, a.ev_key2, a.ctl, a.seg, a.nseg);
    if (!a.msize) {  // (TTL mode replays its runs for sizes as well: every event there)
      // chain starts into the unsorted values' buffer (free after the sort)
      ChainIt it(hipcub::CountingInputIterator<uint32_t>(0), ChainStart{a.ev_key2, a.ev_val2, a.ev_pay});
      size_t tb = a.temp_bytes;
      if (hipcub::DeviceScan::InclusiveScan(a.temp, tb, it, a.ev_val, hipcub::Max(), (int)E, st) != hipSuccess) return -1;
      hipLaunchKernelGGL(k_small_chains, dim3(std::min<uint32_t>(2048, (E + 255) / 256)), dim3(256), 0, st, a.ev_key2,
                         a.ev_val2, const_cast<EvPay*>(a.ev_pay), a.ev_val, E, a.msmall);
    }
    const bool cmp = a.cseg != nullptr && !a.msize;  // the compacted events (outside TTL mode)
    uint32_t* const orig = reinterpret_cast<uint32_t*>(a.ev_key);  // (free after the sort)
    if (cmp) {
      KeepIt it(hipcub::CountingInputIterator<uint32_t>(0), ChainKeep{a.ev_key2, a.ev_val, a.msmall, E});
      size_t tb = a.temp_bytes;
      if (hipMemsetAsync(a.cseg + a.max_resources, 0, sizeof(uint32_t), st) != hipSuccess) return -1;
      if (hipcub::DeviceSelect::Flagged(a.temp, tb, hipcub::CountingInputIterator<uint32_t>(0), it, orig,
                                        a.cseg + a.max_resources + 1, (int)E, st) != hipSuccess)
        return -1;
      hipLaunchKernelGGL(k_small_cseg, dim3(std::min<uint32_t>(1024, (E + 255) / 256)), dim3(256), 0, st, a.ev_key2, orig,
                         a.cseg, a.max_resources);
    }
    if (a.defer && cmp) return hipGetLastError() == hipSuccess ? 0 : -1;  // (launch_small_replay_kernel, later)
    if (rst != st) {  // the replay overlaps what the engine stream does next
      if (hipEventRecord(a.ev_prep, st) != hipSuccess || hipStreamWaitEvent(rst, a.ev_prep, 0) != hipSuccess) return -1;
    }
    hipLaunchKernelGGL(k_small_replay, dim3(1024), dim3(kSrW * kWave), 0, rst, a.ev_key2, a.ev_val2, a.ev_pay,
                       cmp ? orig : nullptr, cmp ? a.cseg + a.max_resources + 1 : a.ctl, cmp ? a.cseg : a.seg,
                       cmp ? a.cseg + a.max_resources : a.nseg, a.state, a.big,
                       a.left, a.msmall, a.mpcap, a.lvl_at, a.idx0, a.index, a.lo, a.msize != nullptr, a.err);
    // (the maps a big model follows, after the small replay on its stream)
    if (launch_big_replay(a, cmp ? orig : nullptr, cmp ? a.cseg + a.max_resources + 1 : a.ctl, cmp ? a.cseg : a.seg,
                          cmp ? a.cseg + a.max_resources : a.nseg, rst))
      return -1;
    // (on this stream: its exit marks fold into the snapshot right after it)
    if (rst == st && launch_small_fold(a.left, a.msmall, a.max_resources, st)) return -1;
    if (a.msize)  // TTL mode: every map's events (commits and expiries) set its size and capacity
      hipLaunchKernelGGL(k_ttl_replay, dim3(256), dim3(256), 0, st, a.ev_key2, a.ev_val2, a.ev_pay, a.ctl, a.seg, a.nseg,
                         a.msize, a.mpcap, a.lvl_at, a.index, a.lo, a.out_status, a.out_value);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// A deferred replay (SmallArgs::defer: its events sorted and compacted by launch_small_replay) on stream rst.
int launch_small_replay_kernel(const SmallArgs& a, hipStream_t rst) {
  uint32_t* const orig = reinterpret_cast<uint32_t*>(a.ev_key);
  hipLaunchKernelGGL(k_small_replay, dim3(1024), dim3(kSrW * kWave), 0, rst, a.ev_key2, a.ev_val2, a.ev_pay, orig,
                     a.cseg + a.max_resources + 1, a.cseg, a.cseg + a.max_resources, a.state, a.big, a.left, a.msmall,
                     a.mpcap, a.lvl_at, a.idx0, a.index, a.lo, false, a.err);
  if (launch_big_replay(a, orig, a.cseg + a.max_resources + 1, a.cseg, a.cseg + a.max_resources, rst)) return -1;
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// the next sub-batch's counters (after the size answers read this one's): events 0, maps still small recounted
int launch_small_finish(const SmallArgs& a, hipStream_t st) {
  if (hipMemsetAsync(a.ctl, 0, 2 * sizeof(uint32_t), st) != hipSuccess) return -1;
  hipLaunchKernelGGL(k_small_count, dim3(std::min<uint32_t>(256, (a.max_resources + 255) / 256)), dim3(256), 0, st, a.msmall,
                     a.max_resources, a.ctl);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

size_t small_sort_temp_bytes(uint32_t cap) {
  size_t need = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, need, (uint64_t*)nullptr, (uint64_t*)nullptr, (uint32_t*)nullptr,
                                           (uint32_t*)nullptr, (int)cap, 0, 64, (hipStream_t)0);
  // (the same scratch serves k_small_chains' scan and the compaction's select)
  return std::max(need, std::max(chain_scan_temp_bytes(cap), keep_select_temp_bytes(cap)));
}

int launch_small_clear(SmallMap* state, uint32_t m, hipStream_t st) {
  hipLaunchKernelGGL(k_small_clear, dim3(1), dim3(64), 0, st, state, m);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}


}  // namespace cc
