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

namespace cc {

// The model lives in the registers of one wave, node i and bin i in lane i (a java.util.HashMap window holds at most
// 64 nodes and 64 bins): every lane runs the same walk, node fields are read with v_readlane (a few cycles) and
// written by the owning lane's select, the scalars (size, level, flags, the node pool) are uniform registers.  (A
// copy in LDS cost a dependent LDS round trip of ~100 cycles per field: ~0.5 us per event of a hot small map.)
// Every method must be called by the whole wave with uniform arguments.
struct SmallJhm {
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
  __device__ __forceinline__ bool tree(uint32_t x) const { return nb(x) & 1u; }
  __device__ __forceinline__ bool red(uint32_t x) const { return x && (nb(x) & 2u); }
  __device__ __forceinline__ void set_red(uint32_t x, bool r) { set_nb(x, (nb(x) & ~2u) | (r ? 2u : 0u)); }
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
  __device__ __forceinline__ uint32_t list_len(uint32_t h) const {
    uint32_t q = tab((cap() - 1) & h), c = 0;
    if (q && tree(q)) return kSmNodes + 1;
    for (; q && c <= kSmNodes; q = next(q)) ++c;
    return c;
  }
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

  // putTreeVal's / treeify's direction for key (kt, key) with hash h at tree node p: the hash as a signed int, then
  // compareComparables (same class), then tieBreakOrder (class names; a new key never equals a live one)
  __device__ __forceinline__ int dir_of(uint32_t h, uint32_t kt, uint64_t key, uint32_t p) {
    const int32_t ph = (int32_t)hash(p), hh = (int32_t)h;
    if (ph > hh) return -1;
    if (ph < hh) return 1;
    const uint32_t pt = ktv(p);
    const uint64_t pk = keyv(p);
    if (kt == pt) {
      switch (kt) {
        case 0: return (int64_t)key < (int64_t)pk ? -1 : 1;  // Long.compareTo
        case 1: return (int32_t)key < (int32_t)pk ? -1 : 1;  // Integer.compareTo
        case 2: return key < pk ? -1 : 1;                    // Boolean.compareTo (false < true)
        default: flags |= kSmAmbig; return 1;              // String.compareTo of texts held as handles
      }
    }
    // tieBreakOrder: getClass().getName() -- java.lang.Boolean < Integer < Long < String (tags 2, 1, 0, 3)
    auto rank = [](uint32_t t) { return (0x3012u >> (4 * t)) & 0xFu; };  // {2, 1, 0, 3} (no indexed array: scratch)
    return rank(kt) < rank(pt) ? -1 : 1;
  }
  __device__ __forceinline__ uint32_t root_of(uint32_t p) const {
    while (par(p)) p = par(p);
    return p;
  }
  __device__ __forceinline__ uint32_t rotate_left(uint32_t root, uint32_t p) {
    uint32_t r, pp, rl;
    if (p && (r = right(p))) {
      rl = left(r);
      set_right(p, rl);
      if (rl) set_par(rl, p);
      pp = par(p);
      set_par(r, pp);
      if (!pp) root = r, set_red(r, false);
      else if (left(pp) == p) set_left(pp, r);
      else set_right(pp, r);
      set_left(r, p);
      set_par(p, r);
    }
    return root;
  }
  __device__ __forceinline__ uint32_t rotate_right(uint32_t root, uint32_t p) {
    uint32_t l, pp, lr;
    if (p && (l = left(p))) {
      lr = right(l);
      set_left(p, lr);
      if (lr) set_par(lr, p);
      pp = par(p);
      set_par(l, pp);
      if (!pp) root = l, set_red(l, false);
      else if (right(pp) == p) set_right(pp, l);
      else set_left(pp, l);
      set_right(l, p);
      set_par(p, l);
    }
    return root;
  }
  __device__ __forceinline__ uint32_t balance_insertion(uint32_t root, uint32_t x) {
    set_red(x, true);
    for (uint32_t xp, xpp, xppl, xppr;;) {
      if (!(xp = par(x))) {
        set_red(x, false);
        return x;
      }
      if (!red(xp) || !(xpp = par(xp))) return root;
      if (xp == (xppl = left(xpp))) {
        if ((xppr = right(xpp)) && red(xppr)) {
          set_red(xppr, false), set_red(xp, false), set_red(xpp, true), x = xpp;
        } else {
          if (x == right(xp)) {
            root = rotate_left(root, x = xp);
            xpp = (xp = par(x)) ? par(xp) : 0;
          }
          if (xp) {
            set_red(xp, false);
            if (xpp) set_red(xpp, true), root = rotate_right(root, xpp);
          }
        }
      } else {
        if (xppl && red(xppl)) {
          set_red(xppl, false), set_red(xp, false), set_red(xpp, true), x = xpp;
        } else {
          if (x == left(xp)) {
            root = rotate_right(root, x = xp);
            xpp = (xp = par(x)) ? par(xp) : 0;
          }
          if (xp) {
            set_red(xp, false);
            if (xpp) set_red(xpp, true), root = rotate_left(root, xpp);
          }
        }
      }
    }
  }
  __device__ __forceinline__ uint32_t balance_deletion(uint32_t root, uint32_t x) {
    for (uint32_t xp, xpl, xpr;;) {
      if (!x || x == root) return root;
      if (!(xp = par(x))) {
        set_red(x, false);
        return x;
      }
      if (red(x)) {
        set_red(x, false);
        return root;
      }
      if ((xpl = left(xp)) == x) {
        if (red(xpr = right(xp))) {
          set_red(xpr, false), set_red(xp, true);
          root = rotate_left(root, xp);
          xpr = (xp = par(x)) ? right(xp) : 0;
        }
        if (!xpr) {
          x = xp;
        } else {
          uint32_t sl = left(xpr), sr = right(xpr);
          if (!red(sr) && !red(sl)) {
            set_red(xpr, true), x = xp;
          } else {
            if (!red(sr)) {
              if (sl) set_red(sl, false);
              set_red(xpr, true);
              root = rotate_right(root, xpr);
              xpr = (xp = par(x)) ? right(xp) : 0;
            }
            if (xpr) {
              set_red(xpr, xp ? red(xp) : false);
              if ((sr = right(xpr))) set_red(sr, false);
            }
            if (xp) set_red(xp, false), root = rotate_left(root, xp);
            x = root;
          }
        }
      } else {
        if (red(xpl)) {
          set_red(xpl, false), set_red(xp, true);
          root = rotate_right(root, xp);
          xpl = (xp = par(x)) ? left(xp) : 0;
        }
        if (!xpl) {
          x = xp;
        } else {
          uint32_t sl = left(xpl), sr = right(xpl);
          if (!red(sl) && !red(sr)) {
            set_red(xpl, true), x = xp;
          } else {
            if (!red(sl)) {
              if (sr) set_red(sr, false);
              set_red(xpl, true);
              root = rotate_left(root, xpl);
              xpl = (xp = par(x)) ? left(xp) : 0;
            }
            if (xpl) {
              set_red(xpl, xp ? red(xp) : false);
              if ((sl = left(xpl))) set_red(sl, false);
            }
            if (xp) set_red(xp, false), root = rotate_right(root, xp);
            x = root;
          }
        }
      }
    }
  }
  __device__ __forceinline__ void to_front(uint32_t root) {  // moveRootToFront
    if (!root) return;
    const uint32_t index = (cap() - 1) & hash(root);
    const uint32_t first = tab(index);
    if (root == first) return;
    set_tab(index, root);
    const uint32_t rp = prev(root), rn = next(root);
    if (rn) set_prev(rn, rp);
    if (rp) set_next(rp, rn);
    if (first) set_prev(first, root);
    set_next(root, first);
    set_prev(root, 0);
  }
  __device__ __forceinline__ void treeify(uint32_t hd) {
    uint32_t root = 0;
    for (uint32_t x = hd, nxt; x; x = nxt) {
      nxt = next(x);
      set_left(x, 0), set_right(x, 0);
      if (!root) {
        set_par(x, 0), set_red(x, false), root = x;
        continue;
      }
      for (uint32_t p = root;;) {
        const int dir = dir_of(hash(x), ktv(x), keyv(x), p);
        const uint32_t xp = p;
        if (!(p = dir <= 0 ? left(p) : right(p))) {
          set_par(x, xp);
          if (dir <= 0) set_left(xp, x);
          else set_right(xp, x);
          root = balance_insertion(root, x);
          break;
        }
      }
    }
    to_front(root);
  }
  __device__ __forceinline__ uint32_t untreeify(uint32_t hd) {
    for (uint32_t q = hd; q; q = next(q)) {
      set_nb(q, 0);
      set_par(q, 0), set_left(q, 0), set_right(q, 0), set_prev(q, 0);
    }
    return hd;
  }
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
    uint32_t tl = 0;
    for (uint32_t q = tab(index); q; q = next(q)) set_nb(q, nb(q) | 1u), set_prev(q, tl), tl = q;
    if (tab(index)) treeify(tab(index));
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
      const uint32_t root = root_of(p);
      for (uint32_t q = root;;) {
        const int dir = dir_of(h, kt, key, q);
        const uint32_t xp = q;
        if (!(q = dir <= 0 ? left(q) : right(q))) {
          const uint32_t xpn = next(xp), x = alloc(h, kt, key);
          if (!x) return true;
          set_nb(x, 1u);
          set_next(x, xpn);
          if (dir <= 0) set_left(xp, x);
          else set_right(xp, x);
          set_next(xp, x);
          set_par(x, xp), set_prev(x, xp);
          if (xpn) set_prev(xpn, x);
          to_front(balance_insertion(root, x));
          break;
        }
      }
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
  __device__ __forceinline__ void remove_tree_node(uint32_t self, uint32_t index) {  // TreeNode.removeTreeNode(map, tab, movable = true)
    uint32_t first = tab(index), root = first, rl;
    const uint32_t succ = next(self), pred = prev(self);
    if (!pred) set_tab(index, first = succ);
    else set_next(pred, succ);
    if (succ) set_prev(succ, pred);
    if (!first) return;
    if (par(root)) root = root_of(root);
    if (!right(root) || !(rl = left(root)) || !left(rl)) {
      set_tab(index, untreeify(first));  // too small
      return;
    }
    const uint32_t p = self, pl = left(p), pr = right(p);
    uint32_t replacement;
    if (pl && pr) {
      uint32_t sx = pr, sl;
      while ((sl = left(sx))) sx = sl;  // successor
      const bool c = red(sx);
      set_red(sx, red(p));
      set_red(p, c);
      const uint32_t sr = right(sx), pp = par(p);
      if (sx == pr) {
        set_par(p, sx);
        set_right(sx, p);
      } else {
        const uint32_t sp = par(sx);
        set_par(p, sp);
        if (sp) {
          if (sx == left(sp)) set_left(sp, p);
          else set_right(sp, p);
        }
        set_right(sx, pr);
        if (pr) set_par(pr, sx);
      }
      set_left(p, 0);
      set_right(p, sr);
      if (sr) set_par(sr, p);
      set_left(sx, pl);
      if (pl) set_par(pl, sx);
      set_par(sx, pp);
      if (!pp) root = sx;
      else if (p == left(pp)) set_left(pp, sx);
      else set_right(pp, sx);
      replacement = sr ? sr : p;
    } else {
      replacement = pl ? pl : (pr ? pr : p);
    }
    if (replacement != p) {
      const uint32_t pp = par(p);
      set_par(replacement, pp);
      if (!pp) root = replacement;
      else if (p == left(pp)) set_left(pp, replacement);
      else set_right(pp, replacement);
      set_left(p, 0), set_right(p, 0), set_par(p, 0);
    }
    const uint32_t r = red(p) ? root : balance_deletion(root, replacement);
    if (replacement == p) {  // detach
      const uint32_t pp = par(p);
      set_par(p, 0);
      if (pp) {
        if (p == left(pp)) set_left(pp, 0);
        else if (p == right(pp)) set_right(pp, 0);
      }
    }
    to_front(r);
  }
  // removeNode(movable = true) of the live key (kt, key) with hash h
  __device__ __forceinline__ void remove(uint32_t h, uint32_t kt, uint64_t key) {
    const uint32_t index = (cap() - 1) & h;
    uint32_t node = 0, prv = 0, pp = 0;
    for (uint32_t q = tab(index), steps = 0; q && steps < kSmNodes; pp = q, q = next(q), ++steps)
      if (hash(q) == h && ktv(q) == kt && keyv(q) == key) {
        node = q, prv = pp;
        break;
      }
    if (!node) {
      flags |= kSmAmbig;  // (a removal of a key this model does not hold: its order is no longer known)
      return;
    }
    if (tree(node)) remove_tree_node(node, index);
    else if (!prv) set_tab(index, next(node));
    else set_next(prv, next(node));
    release(node);
    --n;
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
