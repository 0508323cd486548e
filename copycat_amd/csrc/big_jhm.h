// big_jhm.h — java.util.HashMap (JDK 8) of a map whose table left the small window (capacity 128 and up) with a tree
// bin, node for node, on the device (common.h BigMap).  MapState keeps its entries in a `new HashMap<>()`
// (collections/src/main/java/io/atomix/collections/state/MapState.java:33) and containsValue (:49-60) walks
// map.values(): when a stored null and a match share a bin, the first of them in the bin's chain decides.  A bin that
// was a red-black tree bin keeps a tree's chain order through every resize: HashMap.resize splits it with
// TreeNode.split (the chain divided in order into the low and high halves; a half of <= 6 nodes untreeified, a half
// of more re-treeified when the other half is not empty, its root moved to the front), and later keys follow
// putTreeVal / removeTreeNode there.  The small model (small_jhm.h) hands its state over when its table passes 64;
// from there this model follows the map's insertions and removals in log order (map_big.hip k_big_replay), one lane.
//
// The structure restates the published JDK 8 algorithm (java.util.HashMap is a JDK class, not part of
// /root/reference; the oracle's JHM, oracle/oracle.cpp, is the CPU restatement it is checked against):
//   put:    putVal — an empty bin takes the node; a tree bin putTreeVal (jhm_tree.h); a list bin appends, and a chain
//           of >= 9 calls treeifyBin (capacity >= 64 here: treeify); then ++size > threshold resizes;
//   remove: removeNode(movable = true);
//   resize: list bins split in order; tree bins TreeNode.split (lc / hc <= UNTREEIFY_THRESHOLD 6: untreeify).
#pragma once
#include "common.h"
#include "jhm_tree.h"

namespace cc {

struct BigJhm : JhmTree<BigJhm> {
  BigMap* b;
  uint32_t n, lvl, flags, top, fr;

  __device__ __forceinline__ void load(BigMap* p) {
    b = p;
    n = p->h.n;
    lvl = p->h.lvl;
    flags = p->h.flags;
    top = p->h.top;
    fr = p->h.free;
  }
  __device__ __forceinline__ void store() const {
    b->h.n = n;
    b->h.lvl = lvl;
    b->h.flags = flags;
    b->h.top = top;
    b->h.free = fr;
  }

  __device__ __forceinline__ uint32_t cap() const { return 16u << lvl; }
  __device__ __forceinline__ BigNode& nd(uint32_t x) const { return b->nd[x - 1]; }
  __device__ __forceinline__ uint32_t nb(uint32_t x) const { return nd(x).nb; }
  __device__ __forceinline__ void set_nb(uint32_t x, uint32_t v) { nd(x).nb = (uint8_t)v; }
  __device__ __forceinline__ uint32_t tab(uint32_t i) const { return b->tab[i]; }
  __device__ __forceinline__ void set_tab(uint32_t i, uint32_t v) { b->tab[i] = (uint16_t)v; }
  __device__ __forceinline__ uint32_t next(uint32_t x) const { return nd(x).nx; }
  __device__ __forceinline__ uint32_t prev(uint32_t x) const { return nd(x).pv; }
  __device__ __forceinline__ uint32_t par(uint32_t x) const { return nd(x).pa; }
  __device__ __forceinline__ uint32_t left(uint32_t x) const { return nd(x).lf; }
  __device__ __forceinline__ uint32_t right(uint32_t x) const { return nd(x).rt; }
  __device__ __forceinline__ void set_next(uint32_t x, uint32_t v) { nd(x).nx = (uint16_t)v; }
  __device__ __forceinline__ void set_prev(uint32_t x, uint32_t v) { nd(x).pv = (uint16_t)v; }
  __device__ __forceinline__ void set_par(uint32_t x, uint32_t v) { nd(x).pa = (uint16_t)v; }
  __device__ __forceinline__ void set_left(uint32_t x, uint32_t v) { nd(x).lf = (uint16_t)v; }
  __device__ __forceinline__ void set_right(uint32_t x, uint32_t v) { nd(x).rt = (uint16_t)v; }
  __device__ __forceinline__ uint32_t hash(uint32_t x) const { return nd(x).jh; }
  __device__ __forceinline__ uint32_t ktv(uint32_t x) const { return nd(x).kt; }
  __device__ __forceinline__ uint64_t keyv(uint32_t x) const { return nd(x).key; }

  // a free node (0: none left -- the map outgrew the model)
  __device__ __forceinline__ uint32_t alloc(uint32_t h, uint32_t kt, uint64_t key) {
    uint32_t x;
    if (fr) {
      x = fr;
      fr = nd(x).nx;
    } else if (top < kBigNodes) {
      x = ++top;
    } else {
      return 0;
    }
    BigNode& z = nd(x);
    z.key = key;
    z.jh = h;
    z.nx = z.pv = z.pa = z.lf = z.rt = 0;
    z.nb = 0;
    z.kt = (uint8_t)kt;
    return x;
  }
  __device__ __forceinline__ void release(uint32_t x) {
    nd(x).nx = (uint16_t)fr;
    fr = x;
  }

  // HashMap.resize to twice the capacity, in place (bins [old, 2 old) are empty at the old capacity and bin j splits
  // into j and j + old only); false: past the model's largest table
  __device__ __forceinline__ bool resize() {
    const uint32_t old = cap();
    if (lvl + 1 > kBigMaxLvl) return false;
    ++lvl;  // (treeify / moveRootToFront below work on the new table)
    for (uint32_t j = 0; j < old; ++j) {
      const uint32_t hd = tab(j);
      if (!hd) continue;
      set_tab(j, 0);
      uint32_t lo = 0, lot = 0, hi = 0, hit = 0, lc = 0, hc = 0;
      const bool tr = tree(hd);
      for (uint32_t q = hd, nxt; q; q = nxt) {
        nxt = next(q);
        set_next(q, 0);
        if ((hash(q) & old) == 0) {
          if (tr) set_prev(q, lot);
          if (lot) set_next(lot, q); else lo = q;
          lot = q, ++lc;
        } else {
          if (tr) set_prev(q, hit);
          if (hit) set_next(hit, q); else hi = q;
          hit = q, ++hc;
        }
      }
      if (!tr) {
        set_tab(j, lo);
        set_tab(j + old, hi);
        continue;
      }
      // TreeNode.split
      if (lo) {
        if (lc <= 6) set_tab(j, untreeify(lo));
        else {
          set_tab(j, lo);
          if (hi) treeify(lo);
        }
      }
      if (hi) {
        if (hc <= 6) set_tab(j + old, untreeify(hi));
        else {
          set_tab(j + old, hi);
          if (lo) treeify(hi);
        }
      }
    }
    return true;
  }
  // putVal of a new key (an existing key's put changes no structure); false: the model cannot hold the map
  __device__ __forceinline__ bool put(uint32_t h, uint32_t kt, uint64_t key) {
    const uint32_t i = (cap() - 1) & h;
    uint32_t p = tab(i);
    if (!p) {
      const uint32_t x = alloc(h, kt, key);
      if (!x) return false;
      set_tab(i, x);
    } else if (tree(p)) {
      if (!put_tree_val(p, h, kt, key)) return false;
    } else {
      uint32_t bin = 0;
      while (next(p)) p = next(p), ++bin;
      const uint32_t x = alloc(h, kt, key);
      if (!x) return false;
      set_next(p, x);
      if (bin >= 7u) treeify_chain(i);  // the chain now holds >= 9 nodes (capacity >= 64: treeifyBin treeifies)
    }
    if (++n > (12u << lvl)) return resize();  // ++size > threshold
    return true;
  }
  // removeNode(movable = true) of the live key (kt, key) with hash h
  __device__ __forceinline__ void remove(uint32_t h, uint32_t kt, uint64_t key) {
    if (!remove_key(h, kt, key, kBigNodes)) flags |= kSmAmbig;  // (a key the model does not hold: order unknown)
  }
  // MapState.clear in the stream: every key leaves, the table keeps its capacity
  __device__ __forceinline__ void clear() {
    for (uint32_t i = 0; i < cap(); ++i) set_tab(i, 0);
    n = top = fr = 0;
    flags &= ~kSmAmbig;
  }
};

// The small model's state at the moment its table passed 64 (small_jhm.h resize: the level already raised, the bins
// still those of 64; map_small.hip kSmBigNew) copied into big model B by the whole wave: node i + 1 from lane i, bin
// heads, the free nodes among the first 64 linked; `pos` is the event that grew the table (k_big_replay resizes to
// 128 and goes on after it).
__device__ inline void big_from_small(const SmallMap& s, BigMap* __restrict__ B, uint64_t pos) {
  const uint32_t l = __lane_id();
  if ((s.used >> l) & 1ull) {
    BigNode& z = B->nd[l];
    z.key = s.key[l];
    z.jh = s.jh[l];
    z.nx = s.nx[l];
    z.pv = s.pv[l];
    z.pa = s.pa[l];
    z.lf = s.lf[l];
    z.rt = s.rt[l];
    z.nb = s.nb[l];
    z.kt = s.kt[l];
  }
  B->tab[l] = s.tab[l];
  for (uint32_t t = kWave + l; t < kBigTab; t += kWave) B->tab[t] = 0;
  if (l == 0) {
    uint32_t fr = 0;
    for (int i = kWave - 1; i >= 0; --i)
      if (!((s.used >> i) & 1ull)) {
        B->nd[i].nx = (uint16_t)fr;
        fr = (uint32_t)i + 1;
      }
    B->h.n = s.n;
    B->h.lvl = s.lvl - 1;  // (64: the pending resize is k_big_replay's)
    B->h.flags = (s.flags & kSmAmbig) | kBigResume;
    B->h.top = kWave;
    B->h.free = fr;
    B->h.resume = pos;
  }
}

// The position of the live key (kt, key) with hash h in its bin's chain; unknown: the model does not hold it.
__device__ inline uint32_t big_chain_pos(const BigMap& B, uint32_t h, uint32_t kt, uint64_t key, bool& unknown) {
  const uint32_t index = ((16u << B.h.lvl) - 1u) & h;
  uint32_t pos = 0, steps = 0;
  for (uint32_t q = B.tab[index]; q && steps < kBigNodes; q = B.nd[q - 1].nx, ++steps, ++pos)
    if (B.nd[q - 1].jh == h && B.nd[q - 1].kt == kt && B.nd[q - 1].key == key) {
      unknown = false;
      return pos;
    }
  unknown = true;
  return ~0u;
}

}  // namespace cc
