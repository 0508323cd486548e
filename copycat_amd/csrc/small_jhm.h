// small_jhm.h — java.util.HashMap (JDK 8) of a map whose table is still small (capacity <= 64), node for node, on
// the device.  MapState keeps its entries in a `new HashMap<>()` (collections/src/main/java/io/atomix/collections/
// state/MapState.java:33) and containsValue (:49-60) walks map.values(): when a stored null and a match share a bin
// the first of them in the bin's chain decides (NullPointerException or true).  A list bin's chain is its
// nodes in creation order, but at capacity 64 a bin whose chain reaches 9 nodes becomes a red-black tree bin
// (HashMap.treeifyBin), whose chain order is the tree's: the root first (moveRootToFront), each later node linked
// after its tree parent (putTreeVal), nodes unlinked by removeTreeNode, the bin turned back into a list (untreeify)
// when a removal leaves the tree too small.  The engine follows all of that here, so an order-dependent
// containsValue on a small map is answered exactly, tree bins included.
//
// The structure restates the published JDK 8 algorithm (java.util.HashMap is a JDK class, not part of
// /root/reference; the oracle's JHM, oracle/oracle.cpp, is the CPU restatement it is checked against):
//   put:    putVal — an empty bin takes the node; a tree bin putTreeVal (by hash as a signed int: the keys' own
//           compareTo is needed only for equal hashes); a list bin appends, and a chain of >= 9 calls treeifyBin
//           (resize() below capacity 64, else treeify); then ++size > threshold resizes;
//   remove: removeNode(movable = true) — MapState.remove / removeIfPresent and the TTL timer call map.remove(key);
//   resize: lists split in order (a tree bin exists only at 64, and a table of 128 leaves this window).
// Nodes carry their keys (tag + value, the events' payload, map_small.hip), so equal hashes are resolved as the JDK
// does: putTreeVal / treeify compare two keys of one class with compareTo (Long, Integer signed; Boolean false <
// true) and keys of different classes by tieBreakOrder (class names: Boolean < Integer < Long < String).  Two String
// keys with one hash in a tree bin would need String.compareTo of texts the engine holds as handles: that order is
// unknown (kSmAmbig; an order-dependent answer then fails with CC_ERR_STATE).  List bins need no comparison.
#pragma once
#include <cstddef>

#include "common.h"
#include "jhm_tree.h"

namespace cc {

// The model lives in the registers of one wave, node i and bin i in lane i (a java.util.HashMap window holds at most
// 64 nodes and 64 bins): every lane runs the same walk, node fields are read with v_readlane (a few cycles) and
// written by the owning lane's select, the scalars (size, level, flags, the node pool) are uniform registers.  (A
// copy in LDS cost a dependent LDS round trip of ~100 cycles per field: ~0.5 us per event of a hot small map.)
// Every method must be called by the whole wave with uniform arguments.
struct SmallJhm : JhmTree<SmallJhm> {
  uint32_t w0;     // lane i: node i + 1's next | prev << 8 | parent << 16 | left << 24
  uint32_t w1;     // lane i: node i + 1's right | flags (bit 0 TreeNode, bit 1 red) << 8 | bin i's head << 16
  uint32_t wjh;    // lane i: node i + 1's hash
  uint32_t wkt;    // lane i: node i + 1's key tag
  uint32_t wklo, wkhi;  // lane i: node i + 1's key
  uint32_t n, lvl, flags;
  uint64_t used, tree_bins;
  uint32_t lane;

  __device__ __forceinline__ void load(const SmallMap& m) {
    lane = __lane_id();
    w0 = m.nx[lane] | (uint32_t)m.pv[lane] << 8 | (uint32_t)m.pa[lane] << 16 | (uint32_t)m.lf[lane] << 24;
    w1 = m.rt[lane] | (uint32_t)m.nb[lane] << 8 | (uint32_t)m.tab[lane] << 16;
    wjh = m.jh[lane];
    wkt = m.kt[lane];
    wklo = (uint32_t)m.key[lane];
    wkhi = (uint32_t)(m.key[lane] >> 32);
    n = m.n;
    lvl = m.lvl;
    flags = m.flags;
    used = m.used;
    tree_bins = m.tree_bins;
  }
  __device__ __forceinline__ void store(SmallMap& m) const {
    m.nx[lane] = (uint8_t)w0;
    m.pv[lane] = (uint8_t)(w0 >> 8);
    m.pa[lane] = (uint8_t)(w0 >> 16);
    m.lf[lane] = (uint8_t)(w0 >> 24);
    m.rt[lane] = (uint8_t)w1;
    m.nb[lane] = (uint8_t)(w1 >> 8);
    m.tab[lane] = (uint8_t)(w1 >> 16);
    m.jh[lane] = wjh;
    m.kt[lane] = (uint8_t)wkt;
    m.key[lane] = (uint64_t)wkhi << 32 | wklo;
    if (lane == 0) {
      m.n = n;
      m.lvl = lvl;
      m.flags = flags;
      m.used = used;
      m.tree_bins = tree_bins;
    }
  }
  __device__ __forceinline__ static uint32_t rl(uint32_t v, uint32_t i) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)i); }
  __device__ __forceinline__ void put8(uint32_t& w, uint32_t i, uint32_t sh, uint32_t v) {
    if (lane == i) w = (w & ~(0xFFu << sh)) | ((v & 0xFFu) << sh);
  }

  __device__ __forceinline__ uint32_t cap() const { return 16u << lvl; }
  __device__ __forceinline__ uint32_t nb(uint32_t x) const { return (rl(w1, x - 1) >> 8) & 0xFFu; }
  __device__ __forceinline__ void set_nb(uint32_t x, uint32_t v) { put8(w1, x - 1, 8, v); }
  __device__ __forceinline__ uint32_t tab(uint32_t b) const { return (rl(w1, b) >> 16) & 0xFFu; }
  __device__ __forceinline__ void set_tab(uint32_t b, uint32_t v) { put8(w1, b, 16, v); }
  // links are node + 1 (0: null)
  __device__ __forceinline__ uint32_t next(uint32_t x) const { return rl(w0, x - 1) & 0xFFu; }
  __device__ __forceinline__ uint32_t prev(uint32_t x) const { return (rl(w0, x - 1) >> 8) & 0xFFu; }
  __device__ __forceinline__ uint32_t par(uint32_t x) const { return (rl(w0, x - 1) >> 16) & 0xFFu; }
  __device__ __forceinline__ uint32_t left(uint32_t x) const { return rl(w0, x - 1) >> 24; }
  __device__ __forceinline__ uint32_t right(uint32_t x) const { return rl(w1, x - 1) & 0xFFu; }
  __device__ __forceinline__ void set_next(uint32_t x, uint32_t v) { put8(w0, x - 1, 0, v); }
  __device__ __forceinline__ void set_prev(uint32_t x, uint32_t v) { put8(w0, x - 1, 8, v); }
  __device__ __forceinline__ void set_par(uint32_t x, uint32_t v) { put8(w0, x - 1, 16, v); }
  __device__ __forceinline__ void set_left(uint32_t x, uint32_t v) { put8(w0, x - 1, 24, v); }
  __device__ __forceinline__ void set_right(uint32_t x, uint32_t v) { put8(w1, x - 1, 0, v); }
  __device__ __forceinline__ uint32_t hash(uint32_t x) const { return rl(wjh, x - 1); }
  __device__ __forceinline__ uint32_t ktv(uint32_t x) const { return rl(wkt, x - 1); }
  __device__ __forceinline__ uint64_t keyv(uint32_t x) const { return (uint64_t)rl(wkhi, x - 1) << 32 | rl(wklo, x - 1); }
  // the bin of hash h is a list bin (or empty) at the current capacity
  __device__ __forceinline__ bool list_bin(uint32_t h) const {
    const uint32_t hd = tab((cap() - 1) & h);
    return hd == 0 || !tree(hd);
  }
  // the chain length of a list bin (a tree bin: kSmNodes + 1)
  __device__ __forceinline__ uint32_t list_len(uint32_t h) const { return chain_len(h, kSmNodes); }
  // the live key (kt, key) with hash h is the last node of a list bin of at most `most` nodes: removeNode then putVal
  // of it changes nothing (it is linked back where it was, no treeifyBin, the size and threshold as before)
  __device__ __forceinline__ bool list_tail(uint32_t h, uint32_t kt, uint64_t key, uint32_t most) const {
    uint32_t q = tab((cap() - 1) & h);
    if (!q || tree(q)) return false;
    for (uint32_t c = 1; c <= most; ++c, q = next(q)) {
      const uint32_t nx = next(q);
      if (hash(q) == h && ktv(q) == kt && keyv(q) == key) return nx == 0;
      if (!nx) return false;
    }
    return false;
  }

  __device__ __forceinline__ uint32_t alloc(uint32_t h, uint32_t kt, uint64_t key) {
    const uint64_t free = ~used;
    if (!free) {
      flags |= kSmAmbig;  // (cannot happen: a table of 64 holds at most 49 nodes for a moment)
      return 0;
    }
    const uint32_t i = (uint32_t)__builtin_ctzll(free);
    used |= 1ull << i;
    if (lane == i) {
      wjh = h;
      wkt = kt;
      wklo = (uint32_t)key;
      wkhi = (uint32_t)(key >> 32);
      w0 = 0;
      w1 &= 0xFF0000u;  // (the lane's bin head stays)
    }
    return i + 1;
  }
  __device__ __forceinline__ void release(uint32_t x) { used &= ~(1ull << (x - 1)); }

  // resize (the window holds list bins only below 64, where nothing is a tree): chains split in order; a table of
  // 128 leaves the window (returns false)
  __device__ __forceinline__ bool resize() {
    const uint32_t old = cap();
    if (lvl + 1 >= 3u) {
      ++lvl;
      flags &= ~kSmIn;
      return false;
    }
    ++lvl;
    // in place: bins [old, 2 old) are unused at the old capacity, and bin j splits into j and j + old only
    for (uint32_t j = 0; j < old; ++j) {
      uint32_t lo = 0, lot = 0, hi = 0, hit = 0;
      for (uint32_t q = tab(j), nxt; q; q = nxt) {
        nxt = next(q);
        set_next(q, 0);
        if ((hash(q) & old) == 0) {
          if (lot) set_next(lot, q); else lo = q;
          lot = q;
        } else {
          if (hit) set_next(hit, q); else hi = q;
          hit = q;
        }
      }
      set_tab(j, lo);
      set_tab(j + old, hi);
    }
    return true;
  }
  __device__ __forceinline__ bool treeify_bin(uint32_t h) {
    if (cap() < 64) return resize();  // MIN_TREEIFY_CAPACITY: resize instead
    const uint32_t index = (cap() - 1) & h;
    treeify_chain(index);
    flags |= kSmTree;
    tree_bins |= 1ull << (index & 63u);
    return true;
  }
  // putVal of a new key (an existing key's put changes no structure); false: the map left the window
  __device__ __forceinline__ bool put(uint32_t h, uint32_t kt, uint64_t key) {
    const uint32_t i = (cap() - 1) & h;
    uint32_t p = tab(i);
    if (!p) {
      const uint32_t x = alloc(h, kt, key);
      set_tab(i, x);
    } else if (tree(p)) {  // putTreeVal: linked after its tree parent, then the root moves to the front
      if (!put_tree_val(p, h, kt, key)) return true;
    } else {
      uint32_t bin = 0;
      while (next(p)) p = next(p), ++bin;
      const uint32_t x = alloc(h, kt, key);
      set_next(p, x);
      if (bin >= 7u && !treeify_bin(h)) return false;  // the chain now holds >= 9 nodes
    }
    if (++n > (12u << lvl)) return resize();  // ++size > threshold
    return true;
  }
  // removeNode(movable = true) of the live key (kt, key) with hash h
  __device__ __forceinline__ void remove(uint32_t h, uint32_t kt, uint64_t key) {
    if (!remove_key(h, kt, key, kSmNodes)) flags |= kSmAmbig;  // (a removal of a key this model does not hold: its order is no longer known)
  }
};

// The position of the live key (kt, key) with hash h in its bin's chain (iteration order inside the bin); unknown:
// the model does not hold it.
__device__ inline uint32_t small_chain_pos(const SmallMap& s, uint32_t h, uint32_t kt, uint64_t key, bool& unknown) {
  const uint32_t index = ((16u << s.lvl) - 1u) & h;
  uint32_t pos = 0, steps = 0;
  for (uint32_t q = s.tab[index]; q && steps < kSmNodes; q = s.nx[q - 1], ++steps, ++pos)
    if (s.jh[q - 1] == h && s.kt[q - 1] == kt && s.key[q - 1] == key) {
      unknown = false;
      return pos;
    }
  unknown = true;
  return ~0u;
}

}  // namespace cc
