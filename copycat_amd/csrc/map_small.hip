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
//      or removed a key: key (map << 44 | (log index - the sub-batch's first) << 4 | insert / remove), value = the
//      key's HashMap hash (hot-key routing is off for small maps, k_hot_bind, so every such commit is a region one);
//   2. a radix sort by that key puts each map's events in log order (hipcub);
//   3. one thread per map replays them on an LDS copy of its HashMap: putVal (a chain of 9 calls treeifyBin: a
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
    if (i == 0 || (key[i] >> 44) != (key[i - 1] >> 44)) seg[atomicAdd(nseg, 1u)] = i;
}

// Alternating runs of one key (a hot key of a small map: remove k, put k, remove k, put k, ... with no other event of
// the map between): in a list bin the net effect of remove k . put k is k moved to its chain's end, with the size
// back where it was (no resize) and a chain no longer than before (no treeifyBin: a list chain of 9 cannot persist
// below capacity 64), so R P R P ... R P == R P and R P ... R == R.  One wave per run of a map still in the window
// finds the maximal alternating chains (commit events only: a clear, a size query or another key ends one) and
// stores, at the chain's first removal, how many events after it are implied (EvPay.ktag >> 4).  k_small_replay
// skips them when the key's bin is a list bin at that removal (a tree bin replays every event).
constexpr uint32_t kSkipShift = 4;
__global__ __launch_bounds__(256) void k_small_chains(const uint64_t* __restrict__ key, const uint32_t* __restrict__ val,
                                                      EvPay* __restrict__ pay, const uint32_t* __restrict__ ctl,
                                                      const uint32_t* __restrict__ seg, const uint32_t* __restrict__ nseg,
                                                      const SmallMap* __restrict__ st) {
  const uint32_t E = ctl[0], ns = *nseg, l = __lane_id();
  const uint32_t waves = gridDim.x * (blockDim.x / kWave);
  for (uint32_t r = blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave); r < ns; r += waves) {
    const uint32_t start = seg[r];
    const uint32_t m = (uint32_t)(key[start] >> 44);
    if (!(st[m].flags & kSmIn)) continue;  // (wave-uniform)
    // the open chain, carried across chunks: its first event, its first removal, the previous event
    uint32_t ca = 0xFFFFFFFFu, cr0 = 0xFFFFFFFFu, cf = 0;
    uint64_t pkey = 0;
    uint32_t pid = 0, pcode = 0;  // previous event's identity hash / code (0: not a commit event)
    for (uint32_t b = start;; b += kWave) {
      const uint32_t i = b + l;
      const bool in = i < E && (uint32_t)(key[i] >> 44) == m;
      const uint64_t k = in ? key[i] : 0;
      const uint32_t code = in && !(k & 8u) && ((k & 3u) == 1u || (k & 3u) == 2u) ? (uint32_t)(k & 3u) : 0u;
      const uint32_t v = in ? val[i] : 0u;
      EvPay x{0, 0, 0};
      if (code) x = pay[v];
      const uint32_t id = x.aux ^ ((x.ktag & 3u) << 30);  // (with the key: the identity)
      // the previous event (lane - 1, or the carried one for lane 0)
      const uint64_t qk = __shfl_up(x.key, 1, 64);
      const uint32_t qi = __shfl_up(id, 1, 64), qc = __shfl_up(code, 1, 64);
      const uint64_t prk = l == 0 ? pkey : qk;
      const uint32_t pri = l == 0 ? pid : qi, prc = l == 0 ? pcode : qc;
      const bool link = code && prc && i > start && prk == x.key && pri == id && prc != code;
      // chain starts: the last start at or before each lane (absolute index; none in the chunk: the carried one)
      int32_t st_l = (in && !link) ? (int32_t)l : -1;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int32_t y = __shfl_up(st_l, d, 64);
        if (l >= (uint32_t)d) st_l = max(st_l, y);
      }
      const uint32_t fcode = __shfl(code, st_l < 0 ? 0 : st_l, 64);  // the chain's first code (if it starts here)
      const uint32_t a = st_l < 0 ? ca : b + (uint32_t)st_l;
      const uint32_t f = st_l < 0 ? cf : fcode;
      const uint32_t r0 = st_l < 0 ? cr0 : (f == 1u ? a + 1 : a);
      // a chain ends at lane i when the next event does not link (lane 63: decided with the next chunk's lane 0)
      const bool nlink = __shfl_down((int)link, 1, 64) != 0;
      const bool end_here = in && l < 63 && !nlink;
      const uint32_t vr0 = __shfl(v, (r0 >= b && r0 < b + 64) ? (int)(r0 - b) : 0, 64);
      const uint32_t cb_code = code;  // the chain's last event's code, at its end lane
      if (end_here && code && r0 != 0xFFFFFFFFu && i > r0) {
        const uint32_t skip = cb_code == 1u ? i - r0 - 1 : i - r0;
        if (skip && r0 >= b) pay[vr0].ktag |= skip << kSkipShift;
        else if (skip) pay[val[r0]].ktag |= skip << kSkipShift;  // (its first removal in an earlier chunk)
      }
      // carry: the chain open at lane 63, the last event
      const uint64_t inb = __ballot(in);
      const bool full = inb == ~0ull;
      ca = (uint32_t)__shfl((int)a, 63, 64);
      cf = (uint32_t)__shfl((int)f, 63, 64);
      cr0 = (uint32_t)__shfl((int)r0, 63, 64);
      pkey = __shfl(x.key, 63, 64);
      pid = (uint32_t)__shfl((int)id, 63, 64);
      pcode = (uint32_t)__shfl((int)code, 63, 64);
      const uint32_t last_code = pcode;
      if (!full) break;
      // lane 63's chain continues only if the next chunk's lane 0 links: checked there (l == 0 uses pkey / pid /
      // pcode); if it does not, the chain ended at lane 63 of this chunk
      const uint32_t i0 = b + kWave;
      bool next_in = i0 < E && (uint32_t)(key[i0] >> 44) == m;
      bool next_link = false;
      if (next_in) {
        const uint64_t k0 = key[i0];
        const uint32_t c0 = !(k0 & 8u) && ((k0 & 3u) == 1u || (k0 & 3u) == 2u) ? (uint32_t)(k0 & 3u) : 0u;
        if (c0 && last_code) {
          const EvPay y = pay[val[i0]];
          next_link = y.key == pkey && (y.aux ^ ((y.ktag & 3u) << 30)) == pid && c0 != last_code;
        }
      }
      if (!next_link && last_code && cr0 != 0xFFFFFFFFu && b + 63 > cr0 && l == 0) {  // the carried chain ended at lane 63
        const uint32_t ib = b + 63;
        const uint32_t skip = last_code == 1u ? ib - cr0 - 1 : ib - cr0;
        if (skip) pay[val[cr0]].ktag |= skip << kSkipShift;
      }
      if (!next_link) {
        ca = cr0 = 0xFFFFFFFFu;
        pcode = 0;  // (lane 0 of the next chunk starts a chain)
      }
      if (!next_in) break;
    }
  }
}

// One thread per run: the map's java.util.HashMap copied into LDS (small_jhm.h: node pool, chains, tree links),
// its events applied in log order (putVal of a new key, removeNode), the state written back.  A map whose table
// passes 64 leaves the window (its later events are not followed).
constexpr int kSrT = 64;                                               // runs per workgroup
constexpr int kSrStride = (int)((kSmHotBytes + 8) / 8) | 1;           // u64 words per run's copy (odd: fewer bank conflicts)
__global__ __launch_bounds__(kSrT) void k_small_replay(const uint64_t* __restrict__ key, const uint32_t* __restrict__ val,
                                                       const EvPay* __restrict__ pay, const uint32_t* __restrict__ ctl, const uint32_t* __restrict__ seg,
                                                       const uint32_t* __restrict__ nseg, SmallMap* __restrict__ st,
                                                       uint8_t* __restrict__ msmall, uint32_t* __restrict__ mpcap,
                                                       unsigned long long* __restrict__ lvl_at, const uint64_t* __restrict__ idx0,
                                                       const uint64_t* __restrict__ index, uint64_t lo, bool ttl) {
  __shared__ uint64_t lds[kSrT * kSrStride];
  static_assert(kSmHotBytes % 8 == 0, "SmallMap copies are u64 words");
  constexpr uint32_t W = kSmHotBytes / 8;  // the hot part; the keys stay in HBM (small_jhm.h)
  SmallMap& lm = *reinterpret_cast<SmallMap*>(lds + threadIdx.x * kSrStride);
  const uint32_t E = ctl[0], ns = *nseg;
  for (uint32_t r = blockIdx.x * kSrT + threadIdx.x; r < ns; r += gridDim.x * kSrT) {
    const uint32_t start = seg[r];
    const uint32_t m = (uint32_t)(key[start] >> 44);
    SmallMap* s = st + m;
    if (!(s->flags & kSmIn)) continue;  // (left the window earlier: no events are emitted for it)
    const uint64_t* src = reinterpret_cast<const uint64_t*>(s);
    uint64_t* dst = reinterpret_cast<uint64_t*>(&lm);
    for (uint32_t q = 0; q < W; ++q) dst[q] = src[q];
    SmallJhm j(lm, *s);
    for (uint32_t i = start; i < E; ++i) {
      const uint64_t k = key[i];
      if ((uint32_t)(k >> 44) != m) break;
      if (k & 8u) continue;  // a size / isEmpty query (k_size_answer)
      if ((k & 3u) == 3u) {  // MapState.clear in the stream (map_clear.hip): every key leaves, the table stays
        for (uint32_t q = 0; q < 64; ++q) lm.tab[q] = 0;
        lm.n = 0;
        lm.used = 0;
        lm.flags &= ~(kSmTree | kSmAmbig);
        lm.tree_bins = 0;
        continue;
      }
      const EvPay x = pay[val[i]];
      if ((k & 3u) == 1u) {  // a new key: HashMap.putVal
        const uint32_t lv0 = lm.lvl;
        const bool stay = j.put(x.aux, x.ktag & 3u, x.key);
        if (lm.lvl > lv0 && lvl_at) {  // the table grew at this commit: the capacity-level timeline (common.h)
          const uint64_t d = (k >> 4) & ((1ull << 40) - 1);
          // (an index that cannot be known is not recorded: "not left yet" only over-counts, toward refusing)
          if (ttl ? index != nullptr : idx0 != nullptr)
            lvl_reached(lvl_at, m, lv0, lm.lvl, ttl ? index[lo + (d - 1) / 2] : *idx0 + d);
        }
        if (!stay) break;  // the table passed 64: out of the window
      } else if ((k & 3u) == 2u) {  // a key removed: removeNode
        j.remove(x.aux, x.ktag & 3u, x.key);
        // an alternating run of this key follows (k_small_chains): implied by this removal and, if the run ends with
        // a put, that put -- in a list bin
        const uint32_t skip = x.ktag >> kSkipShift;
        if (skip && j.list_bin(x.aux)) i += skip;
      }
    }
    if (!(lm.flags & kSmIn)) {  // only the capacity level and the tree bins matter from here on
      lm.n = 0;
      lm.used = 0;
    }
    uint64_t* back = reinterpret_cast<uint64_t*>(s);
    for (uint32_t q = 0; q < W; ++q) back[q] = dst[q];
    msmall[m] = (uint8_t)((msmall[m] & ~kMfSmall) | ((lm.flags & kSmIn) ? kMfSmall : 0u));
    atomicMax(&mpcap[m], lm.lvl);
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
// and expiries in log order, its peak -> the capacity level (HashMap.resize never shrinks), the size at the end.
__global__ __launch_bounds__(256) void k_ttl_replay(const uint64_t* __restrict__ key, const uint32_t* __restrict__ ctl,
                                                    const uint32_t* __restrict__ seg, const uint32_t* __restrict__ nseg,
                                                    uint32_t* __restrict__ msize, uint32_t* __restrict__ mpcap,
                                                    unsigned long long* __restrict__ lvl_at, const uint64_t* __restrict__ index,
                                                    uint64_t lo) {
  const uint32_t E = ctl[0], ns = *nseg, l = __lane_id();
  const uint32_t waves = gridDim.x * (blockDim.x / kWave);
  for (uint32_t r = blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave); r < ns; r += waves) {
    const uint32_t start = seg[r];
    const uint32_t m = (uint32_t)(key[start] >> 44);
    int64_t size = msize[m], peak = size;
    for (uint32_t b = start;; b += kWave) {
      const uint32_t i = b + l;
      const bool in = i < E && (uint32_t)(key[i] >> 44) == m;
      const uint64_t k = in ? key[i] : 0;
      const int32_t dlt = !in || (k & 8u) ? 0 : ((k & 3u) == 1u ? 1 : ((k & 3u) == 2u ? -1 : 0));
      int32_t inc = dlt;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int32_t y = __shfl_up(inc, d, 64);
        if (l >= (uint32_t)d) inc += y;
      }
      int32_t mx = inc;
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) mx = max(mx, __shfl_xor(mx, d, 64));
      if (lvl_at && index && dlt > 0 && size + inc > peak) {  // a commit growing the table (common.h timeline)
        const uint64_t d = (k >> 4) & ((1ull << 40) - 1);  // (commits sit at odd positions 2 (row - lo) + 1)
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
__global__ void k_size_emit(const uint32_t* __restrict__ szq, uint32_t szq_n, uint64_t lo, uint64_t hi,
                            const uint32_t* __restrict__ inst, const uint8_t* __restrict__ op,
                            const uint64_t* __restrict__ index, const uint32_t* __restrict__ inst_res,
                            uint64_t* __restrict__ ev_key, uint32_t* __restrict__ ev_val, EvPay* __restrict__ ev_pay,
                            uint32_t cap, uint32_t* __restrict__ ctl) {
  const uint64_t idx0 = index[lo];
  for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < szq_n; q += gridDim.x * blockDim.x) {
    const uint32_t row = szq[q];
    if (row < lo || row >= hi) continue;
    const uint32_t m = inst_res[inst[row]];  // (listed by the barrier scan on a live map: the registry is fixed in a batch)
    const uint64_t d = (index[row] - idx0) & ((1ull << 40) - 1);
    const uint32_t at = atomicAdd(ctl, 1u);
    if (at < cap) {
      ev_key[at] = ((uint64_t)m << 44) | (d << 4) | 8u | (op[row] == CC_OP_MAP_ISEMPTY ? 4u : 0u);
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
    const uint32_t m = (uint32_t)(key[start] >> 44);
    int32_t net = 0;
    bool queries = false;
    uint32_t end = start;
    for (uint32_t b = start;; b += kWave) {  // pass 1: the run's end, net change, and whether it holds a query
      const uint32_t i = b + l;
      const bool in = i < E && (uint32_t)(key[i] >> 44) == m;
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
    mflag[m] &= (uint8_t)~(kMfSize | kMfCv | kMfClr);
}

int launch_size_emit(const SizeArgs& a, hipStream_t st) {
  if (a.szq_n == 0) return 0;
  hipLaunchKernelGGL(k_size_emit, dim3(std::min<uint32_t>(1024, (a.szq_n + 255) / 256)), dim3(256), 0, st, a.szq, a.szq_n,
                     a.lo, a.hi, a.inst, a.op, a.index, a.inst_res, a.ev_key, a.ev_val, a.ev_pay, a.cap, a.ctl);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_size_answer(const SizeArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(k_size_answer, dim3(256), dim3(256), 0, st, a.sorted_key, a.sorted_val, a.ev_pay, a.ctl, a.seg, a.nseg,
                     a.msize, a.out_status, a.out_value);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_mflag_clear(uint8_t* mflag, uint32_t R, hipStream_t st) {
  hipLaunchKernelGGL(k_mflag_clear, dim3(std::min<uint32_t>(256, (R + 255) / 256)), dim3(256), 0, st, mflag, R);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_small_replay(const SmallArgs& a, uint32_t E, hipStream_t st) {
  if (E > a.cap) return -2;
  if (E) {
    size_t need = 0;
    if (hipcub::DeviceRadixSort::SortPairs(nullptr, need, a.ev_key, a.ev_key2, a.ev_val, a.ev_val2, (int)E, 0, 64, st) !=
        hipSuccess)
      return -1;
    if (need > a.temp_bytes) return -3;  // (sized for cap events at creation)
    size_t tb = a.temp_bytes;
    if (hipcub::DeviceRadixSort::SortPairs(a.temp, tb, a.ev_key, a.ev_key2, a.ev_val, a.ev_val2, (int)E, 0, 64, st) !=
        hipSuccess)
      return -1;
    if (hipMemsetAsync(a.nseg, 0, sizeof(uint32_t), st) != hipSuccess) return -1;
    const uint32_t grid = (uint32_t)std::min<uint64_t>(1024, (E + 255) / 256);
    hipLaunchKernelGGL(k_small_seg, dim3(grid), dim3(256), 0, st, a.ev_key2, a.ctl, a.seg, a.nseg);
    if (!a.msize)  // (TTL mode replays its runs for sizes as well: every event there)
      hipLaunchKernelGGL(k_small_chains, dim3(256), dim3(256), 0, st, a.ev_key2, a.ev_val2, const_cast<EvPay*>(a.ev_pay), a.ctl,
                         a.seg, a.nseg, a.state);
    hipLaunchKernelGGL(k_small_replay, dim3(256), dim3(kSrT), 0, st, a.ev_key2, a.ev_val2, a.ev_pay, a.ctl, a.seg, a.nseg, a.state,
                       a.msmall, a.mpcap, a.lvl_at, a.idx0, a.index, a.lo, a.msize != nullptr);
    if (a.msize)  // TTL mode: every map's events (commits and expiries) set its size and capacity
      hipLaunchKernelGGL(k_ttl_replay, dim3(256), dim3(256), 0, st, a.ev_key2, a.ctl, a.seg, a.nseg, a.msize, a.mpcap,
                         a.lvl_at, a.index, a.lo);
  }
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
  return need;
}

int launch_small_clear(SmallMap* state, uint32_t m, hipStream_t st) {
  hipLaunchKernelGGL(k_small_clear, dim3(1), dim3(64), 0, st, state, m);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}


}  // namespace cc
