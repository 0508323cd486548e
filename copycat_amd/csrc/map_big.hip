// map_big.hip — the java.util.HashMap of a map that left the small window with a tree bin, followed past 64.
//
// MapState.containsValue (collections/src/main/java/io/atomix/collections/state/MapState.java:49-60) answers by the
// first stored null or match in HashMap iteration order.  While the table is small (<= 64) the engine follows the
// map node for node (map_small.hip); a map whose table then grows with a bin that was a red-black tree bin keeps that
// bin's tree-derived chain order through every resize (TreeNode.split), and its later keys follow the tree's order,
// not creation order.  Such a map is handed to a big model (big_jhm.h, common.h BigMap) when its table passes 64:
//   1. k_small_replay keeps the small model at the event that grew the table (kSmBigNew) and k_big_replay copies it
//      into a free big model (kBigResume: the resize to 128 still to do);
//   2. the map stays in the engine's small-map snapshot (kMfSmall), so every insertion / removal of it is still an
//      event, sorted in log order with the others (map_small.hip launch_small_replay);
//   3. k_big_replay, on the small replay's stream right after it, walks each big map's run on one lane: the pending
//      resize to 128 (tree bins split), then putVal / removeNode / clear in log order (the events the small replay
//      already applied are skipped by position).  An alternating remove / put run of one key (k_small_chains) is
//      implied in a list bin of <= 7 nodes and applied event by event otherwise, as in the small replay.
// An order-dependent containsValue then reads the deciding bin's chain from the model (map_wide.hip k_mw_order).  A
// map that outgrows its model (kBigNodes live keys, capacity 16 << kBigMaxLvl) or finds no free one keeps the
// bounds test (which refuses such an answer); it leaves the snapshot through the exit marks as a small map does.
// Cost: nothing for maps without a tree bin (the common case: a tree bin needs 9 keys in one bin of 64); a big map's
// events are walked serially, ~1 us each.
#include "big_jhm.h"
#include "common.h"
#include "engine_internal.h"

namespace cc {

__global__ __launch_bounds__(64) void k_big_replay(const uint64_t* __restrict__ key, const uint32_t* __restrict__ val,
                                                   const EvPay* __restrict__ pay, const uint32_t* __restrict__ orig,
                                                   const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ seg,
                                                   const uint32_t* __restrict__ nseg, SmallMap* __restrict__ st,
                                                   BigMap* __restrict__ big, uint8_t* __restrict__ left,
                                                   uint32_t* __restrict__ mpcap, unsigned long long* __restrict__ lvl_at,
                                                   const uint64_t* __restrict__ idx0, const uint64_t* __restrict__ index,
                                                   uint64_t lo, bool ttl) {
  const uint32_t E = *cnt, ns = *nseg, l = __lane_id();
  for (uint32_t r = blockIdx.x; r < ns; r += gridDim.x) {  // (block-uniform: one wave)
    const uint32_t start = seg[r];
    const uint32_t m = (uint32_t)(key[orig ? orig[start] : start] >> kEvMapShift);
    SmallMap* s = st + m;
    const uint32_t sf = s->flags;
    if (!(sf & kSmBig)) continue;
    if (sf & kSmBigNew) {  // left the window in this sub-batch's small replay: take its model over
      uint32_t slot = 0;
      if (l == 0)
        for (uint32_t b = 0; b < kBigSlots; ++b)
          if (atomicCAS(&big[b].h.owner, 0u, m + 1) == 0u) {
            slot = b + 1;
            break;
          }
      slot = (uint32_t)__builtin_amdgcn_readfirstlane((int)slot);
      if (slot) big_from_small(*s, big + (slot - 1), s->pad);
      __syncthreads();  // (lane 0 reads the copy below)
      if (l == 0) {
        s->flags = slot ? sf & ~kSmBigNew : sf & ~(kSmBig | kSmBigNew);
        s->pad = slot ? slot - 1 : 0u;
        s->n = 0;
        s->used = 0;
        if (!slot) left[m] = 1;  // (none free: the bounds test from here on; the map leaves the snapshot)
      }
      if (!slot) continue;
    }
    if (l != 0) continue;
    BigJhm j;
    j.load(big + s->pad);
    bool ok = true, resume = false;
    uint64_t rpos = 0;
    // one insertion / removal; false: the model cannot hold the map
    auto apply = [&](uint64_t kk, const EvPay& x) -> bool {
      if ((kk & 3u) == 1u) {
        const uint32_t lv0 = j.lvl;
        if (!j.put(x.aux, x.ktag & 3u, x.key)) return false;
        if (j.lvl > lv0 && lvl_at && (ttl ? index != nullptr : idx0 != nullptr)) {  // (common.h timeline)
          const uint64_t d = (kk >> 4) & kEvPosMask;
          lvl_reached(lvl_at, m, lv0, j.lvl, ttl ? index[lo + (d - 1) / 2] : *idx0 + d);
        }
      } else {
        j.remove(x.aux, x.ktag & 3u, x.key);
      }
      return true;
    };
    if (j.flags & kBigResume) {  // converted this sub-batch: the resize to 128 the small model left pending
      resume = true;
      rpos = big[s->pad].h.resume;
      j.flags &= ~kBigResume;
      ok = j.resize();
    }
    for (uint32_t i = start; ok && i < E; ++i) {
      const uint32_t o = orig ? orig[i] : i;
      const uint64_t kk = key[o];
      if ((uint32_t)(kk >> kEvMapShift) != m) break;  // the map's run ended
      if (kk & 8u) continue;                          // a size / isEmpty query
      if (resume && ((kk >> 4) & kEvPosMask) <= rpos) continue;  // (applied by the small replay)
      if ((kk & 3u) == 3u) {  // MapState.clear in the stream (map_clear.hip)
        j.clear();
        continue;
      }
      const EvPay x = pay[val[o]];
      if (!(ok = apply(kk, x))) break;
      // a removal starting an alternating run of its key (k_small_chains): the run's later events are implied in a
      // list bin of <= 7 nodes after it (the compacted events leave them out; else skipped here), else applied
      const uint32_t skip = (kk & 3u) == 2u ? x.ktag >> kSkipShift : 0u;
      if (!skip) continue;
      const bool implied = j.chain_len(x.aux, 8) <= 7u;
      if (!orig) {
        if (implied) i += skip;
      } else if (!implied) {
        for (uint32_t u = o + 1; u <= o + skip && ok; ++u) ok = apply(key[u], pay[val[u]]);
      }
    }
    if (!ok) {  // outgrown: back to the bounds test; the map leaves the snapshot at the next fold
      s->flags &= ~kSmBig;
      big[s->pad].h.owner = 0;
      left[m] = 1;
      continue;
    }
    j.store();
    atomicMax(&mpcap[m], j.lvl);
  }
}

int launch_big_replay(const SmallArgs& a, const uint32_t* orig, const uint32_t* cnt, const uint32_t* seg,
                      const uint32_t* nseg, hipStream_t rst) {
  if (!a.big) return 0;
  hipLaunchKernelGGL(k_big_replay, dim3(256), dim3(64), 0, rst, a.ev_key2, a.ev_val2, a.ev_pay, orig, cnt, seg, nseg,
                     a.state, a.big, a.left, a.mpcap, a.lvl_at, a.idx0, a.index, a.lo, a.msize != nullptr);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// A whole-map barrier's clear / Delete (MapState.clear :255-261, delete :264-274): every key leaves, the table keeps
// its capacity, the model stays the map's (a bin that reaches 9 keys there is a tree bin again, without a resize).
// Before k_small_clear.
__global__ void k_big_clear(BigMap* __restrict__ big, const SmallMap* __restrict__ state, uint32_t m) {
  const SmallMap& s = state[m];
  if (!(s.flags & kSmBig)) return;
  BigMap& B = big[s.pad];
  for (uint32_t t = threadIdx.x; t < kBigTab; t += blockDim.x) B.tab[t] = 0;
  if (threadIdx.x == 0) {
    B.h.n = B.h.top = B.h.free = 0;
    B.h.flags &= ~kSmAmbig;
  }
}

int launch_big_clear(BigMap* big, const SmallMap* state, uint32_t m, hipStream_t st) {
  if (!big) return 0;
  hipLaunchKernelGGL(k_big_clear, dim3(1), dim3(256), 0, st, big, state, m);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

__global__ void k_big_release(BigMap* __restrict__ big, uint32_t first, uint32_t count) {
  const uint32_t b = threadIdx.x;
  if (b >= kBigSlots) return;
  const uint32_t o = big[b].h.owner;
  if (o && o - 1 >= first && o - 1 - first < count) big[b].h.owner = 0;
}

int launch_big_release(BigMap* big, uint32_t first, uint32_t count, hipStream_t st) {
  if (!big) return 0;
  hipLaunchKernelGGL(k_big_release, dim3(1), dim3(64), 0, st, big, first, count);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace cc
