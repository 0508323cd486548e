// jhm_tree.h — the red-black tree bins of java.util.HashMap (JDK 8 HashMap.TreeNode), written once over a node
// store: the small-table model (small_jhm.h, one wave's registers) and the model of a map that left the small window
// with a tree bin (big_jhm.h, one workgroup's memory) both derive from it.
//
// The structure restates the published JDK 8 algorithm (java.util.HashMap is a JDK class, not part of
// /root/reference; the oracle's JHM, oracle/oracle.cpp, is the CPU restatement both models are checked against):
//   putTreeVal      a new key walks the tree by hash as a signed int, then compareTo (keys of one class) or
//                   tieBreakOrder (class names); it is linked after its tree parent in the bin's chain, the tree is
//                   rebalanced (balanceInsertion) and the root moves to the chain's front (moveRootToFront);
//   treeify         the bin's chain inserted into a new tree in chain order, the root moved to the front;
//   untreeify       the chain kept in order as plain nodes;
//   removeTreeNode  (movable = true) unlinked from the chain; a tree too small (root, root.right, root.left or
//                   root.left.left missing) turns back into a list, else the red-black delete and moveRootToFront.
//
// D provides the store: links next / prev / par / left / right (node + 1, 0 = null) and their setters, nb / set_nb
// (bit 0 TreeNode, bit 1 red), hash / ktv / keyv, tab / set_tab (bin heads), cap() and a `flags` word (kSmAmbig).
// The small store's methods must be called by the whole wave with uniform arguments; the big store's by one lane.
#pragma once
#include "common.h"

namespace cc {

template <class D>
struct JhmTree {
  __device__ __forceinline__ D& d() { return *static_cast<D*>(this); }
  __device__ __forceinline__ const D& d() const { return *static_cast<const D*>(this); }

  __device__ __forceinline__ bool tree(uint32_t x) const { return d().nb(x) & 1u; }
  __device__ __forceinline__ bool red(uint32_t x) const { return x && (d().nb(x) & 2u); }
  __device__ __forceinline__ void set_red(uint32_t x, bool r) { d().set_nb(x, (d().nb(x) & ~2u) | (r ? 2u : 0u)); }

  // putTreeVal's / treeify's direction for key (kt, key) with hash h at tree node p: the hash as a signed int, then
  // compareComparables (same class), then tieBreakOrder (class names; a new key never equals a live one)
  __device__ __forceinline__ int dir_of(uint32_t h, uint32_t kt, uint64_t key, uint32_t p) {
    D& s = d();
    const int32_t ph = (int32_t)s.hash(p), hh = (int32_t)h;
    if (ph > hh) return -1;
    if (ph < hh) return 1;
    const uint32_t pt = s.ktv(p);
    const uint64_t pk = s.keyv(p);
    if (kt == pt) {
      switch (kt) {
        case 0: return (int64_t)key < (int64_t)pk ? -1 : 1;  // Long.compareTo
        case 1: return (int32_t)key < (int32_t)pk ? -1 : 1;  // Integer.compareTo
        case 2: return key < pk ? -1 : 1;                    // Boolean.compareTo (false < true)
        default: s.flags |= kSmAmbig; return 1;            // String.compareTo of texts held as handles
      }
    }
    // tieBreakOrder: getClass().getName() -- java.lang.Boolean < Integer < Long < String (tags 2, 1, 0, 3)
    auto rank = [](uint32_t t) { return (0x3012u >> (4 * t)) & 0xFu; };  // {2, 1, 0, 3} (no indexed array: scratch)
    return rank(kt) < rank(pt) ? -1 : 1;
  }
  __device__ __forceinline__ uint32_t root_of(uint32_t p) const {
    while (d().par(p)) p = d().par(p);
    return p;
  }
  __device__ __forceinline__ uint32_t rotate_left(uint32_t root, uint32_t p) {
    D& s = d();
    uint32_t r, pp, rl;
    if (p && (r = s.right(p))) {
      rl = s.left(r);
      s.set_right(p, rl);
      if (rl) s.set_par(rl, p);
      pp = s.par(p);
      s.set_par(r, pp);
      if (!pp) root = r, set_red(r, false);
      else if (s.left(pp) == p) s.set_left(pp, r);
      else s.set_right(pp, r);
      s.set_left(r, p);
      s.set_par(p, r);
    }
    return root;
  }
  __device__ __forceinline__ uint32_t rotate_right(uint32_t root, uint32_t p) {
    D& s = d();
    uint32_t l, pp, lr;
    if (p && (l = s.left(p))) {
      lr = s.right(l);
      s.set_left(p, lr);
      if (lr) s.set_par(lr, p);
      pp = s.par(p);
      s.set_par(l, pp);
      if (!pp) root = l, set_red(l, false);
      else if (s.right(pp) == p) s.set_right(pp, l);
      else s.set_left(pp, l);
      s.set_right(l, p);
      s.set_par(p, l);
    }
    return root;
  }
  __device__ __forceinline__ uint32_t balance_insertion(uint32_t root, uint32_t x) {
    D& s = d();
    set_red(x, true);
    for (uint32_t xp, xpp, xppl, xppr;;) {
      if (!(xp = s.par(x))) {
        set_red(x, false);
        return x;
      }
      if (!red(xp) || !(xpp = s.par(xp))) return root;
      if (xp == (xppl = s.left(xpp))) {
        if ((xppr = s.right(xpp)) && red(xppr)) {
          set_red(xppr, false), set_red(xp, false), set_red(xpp, true), x = xpp;
        } else {
          if (x == s.right(xp)) {
            root = rotate_left(root, x = xp);
            xpp = (xp = s.par(x)) ? s.par(xp) : 0;
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
          if (x == s.left(xp)) {
            root = rotate_right(root, x = xp);
            xpp = (xp = s.par(x)) ? s.par(xp) : 0;
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
    D& s = d();
    for (uint32_t xp, xpl, xpr;;) {
      if (!x || x == root) return root;
      if (!(xp = s.par(x))) {
        set_red(x, false);
        return x;
      }
      if (red(x)) {
        set_red(x, false);
        return root;
      }
      if ((xpl = s.left(xp)) == x) {
        if (red(xpr = s.right(xp))) {
          set_red(xpr, false), set_red(xp, true);
          root = rotate_left(root, xp);
          xpr = (xp = s.par(x)) ? s.right(xp) : 0;
        }
        if (!xpr) {
          x = xp;
        } else {
          uint32_t sl = s.left(xpr), sr = s.right(xpr);
          if (!red(sr) && !red(sl)) {
            set_red(xpr, true), x = xp;
          } else {
            if (!red(sr)) {
              if (sl) set_red(sl, false);
              set_red(xpr, true);
              root = rotate_right(root, xpr);
              xpr = (xp = s.par(x)) ? s.right(xp) : 0;
            }
            if (xpr) {
              set_red(xpr, xp ? red(xp) : false);
              if ((sr = s.right(xpr))) set_red(sr, false);
            }
            if (xp) set_red(xp, false), root = rotate_left(root, xp);
            x = root;
          }
        }
      } else {
        if (red(xpl)) {
          set_red(xpl, false), set_red(xp, true);
          root = rotate_right(root, xp);
          xpl = (xp = s.par(x)) ? s.left(xp) : 0;
        }
        if (!xpl) {
          x = xp;
        } else {
          uint32_t sl = s.left(xpl), sr = s.right(xpl);
          if (!red(sl) && !red(sr)) {
            set_red(xpl, true), x = xp;
          } else {
            if (!red(sl)) {
              if (sr) set_red(sr, false);
              set_red(xpl, true);
              root = rotate_left(root, xpl);
              xpl = (xp = s.par(x)) ? s.left(xp) : 0;
            }
            if (xpl) {
              set_red(xpl, xp ? red(xp) : false);
              if ((sl = s.left(xpl))) set_red(sl, false);
            }
            if (xp) set_red(xp, false), root = rotate_right(root, xp);
            x = root;
          }
        }
      }
    }
  }
  __device__ __forceinline__ void to_front(uint32_t root) {  // moveRootToFront
    D& s = d();
    if (!root) return;
    const uint32_t index = (s.cap() - 1) & s.hash(root);
    const uint32_t first = s.tab(index);
    if (root == first) return;
    s.set_tab(index, root);
    const uint32_t rp = s.prev(root), rn = s.next(root);
    if (rn) s.set_prev(rn, rp);
    if (rp) s.set_next(rp, rn);
    if (first) s.set_prev(first, root);
    s.set_next(root, first);
    s.set_prev(root, 0);
  }
  __device__ __forceinline__ void treeify(uint32_t hd) {
    D& s = d();
    uint32_t root = 0;
    for (uint32_t x = hd, nxt; x; x = nxt) {
      nxt = s.next(x);
      s.set_left(x, 0), s.set_right(x, 0);
      if (!root) {
        s.set_par(x, 0), set_red(x, false), root = x;
        continue;
      }
      for (uint32_t p = root;;) {
        const int dir = dir_of(s.hash(x), s.ktv(x), s.keyv(x), p);
        const uint32_t xp = p;
        if (!(p = dir <= 0 ? s.left(p) : s.right(p))) {
          s.set_par(x, xp);
          if (dir <= 0) s.set_left(xp, x);
          else s.set_right(xp, x);
          root = balance_insertion(root, x);
          break;
        }
      }
    }
    to_front(root);
  }
  __device__ __forceinline__ uint32_t untreeify(uint32_t hd) {
    D& s = d();
    for (uint32_t q = hd; q; q = s.next(q)) {
      s.set_nb(q, 0);
      s.set_par(q, 0), s.set_left(q, 0), s.set_right(q, 0), s.set_prev(q, 0);
    }
    return hd;
  }
  // treeifyBin at a capacity >= 64 (MIN_TREEIFY_CAPACITY): the bin's chain becomes TreeNodes (prev links) and a tree
  __device__ __forceinline__ void treeify_chain(uint32_t index) {
    D& s = d();
    uint32_t tl = 0;
    for (uint32_t q = s.tab(index); q; q = s.next(q)) s.set_nb(q, s.nb(q) | 1u), s.set_prev(q, tl), tl = q;
    if (s.tab(index)) treeify(s.tab(index));
  }
  // putTreeVal of a new key into the tree bin whose chain starts at p: linked after its tree parent, then the root
  // moves to the front.  false: the store has no free node.
  __device__ __forceinline__ bool put_tree_val(uint32_t p, uint32_t h, uint32_t kt, uint64_t key) {
    D& s = d();
    const uint32_t root = root_of(p);
    for (uint32_t q = root;;) {
      const int dir = dir_of(h, kt, key, q);
      const uint32_t xp = q;
      if (!(q = dir <= 0 ? s.left(q) : s.right(q))) {
        const uint32_t xpn = s.next(xp), x = s.alloc(h, kt, key);
        if (!x) return false;
        s.set_nb(x, 1u);
        s.set_next(x, xpn);
        if (dir <= 0) s.set_left(xp, x);
        else s.set_right(xp, x);
        s.set_next(xp, x);
        s.set_par(x, xp), s.set_prev(x, xp);
        if (xpn) s.set_prev(xpn, x);
        to_front(balance_insertion(root, x));
        return true;
      }
    }
  }
  __device__ __forceinline__ void remove_tree_node(uint32_t self, uint32_t index) {  // TreeNode.removeTreeNode(map, tab, movable = true)
    D& s = d();
    uint32_t first = s.tab(index), root = first, rl;
    const uint32_t succ = s.next(self), pred = s.prev(self);
    if (!pred) s.set_tab(index, first = succ);
    else s.set_next(pred, succ);
    if (succ) s.set_prev(succ, pred);
    if (!first) return;
    if (s.par(root)) root = root_of(root);
    if (!s.right(root) || !(rl = s.left(root)) || !s.left(rl)) {
      s.set_tab(index, untreeify(first));  // too small
      return;
    }
    const uint32_t p = self, pl = s.left(p), pr = s.right(p);
    uint32_t replacement;
    if (pl && pr) {
      uint32_t sx = pr, sl;
      while ((sl = s.left(sx))) sx = sl;  // successor
      const bool c = red(sx);
      set_red(sx, red(p));
      set_red(p, c);
      const uint32_t sr = s.right(sx), pp = s.par(p);
      if (sx == pr) {
        s.set_par(p, sx);
        s.set_right(sx, p);
      } else {
        const uint32_t sp = s.par(sx);
        s.set_par(p, sp);
        if (sp) {
          if (sx == s.left(sp)) s.set_left(sp, p);
          else s.set_right(sp, p);
        }
        s.set_right(sx, pr);
        if (pr) s.set_par(pr, sx);
      }
      s.set_left(p, 0);
      s.set_right(p, sr);
      if (sr) s.set_par(sr, p);
      s.set_left(sx, pl);
      if (pl) s.set_par(pl, sx);
      s.set_par(sx, pp);
      if (!pp) root = sx;
      else if (p == s.left(pp)) s.set_left(pp, sx);
      else s.set_right(pp, sx);
      replacement = sr ? sr : p;
    } else {
      replacement = pl ? pl : (pr ? pr : p);
    }
    if (replacement != p) {
      const uint32_t pp = s.par(p);
      s.set_par(replacement, pp);
      if (!pp) root = replacement;
      else if (p == s.left(pp)) s.set_left(pp, replacement);
      else s.set_right(pp, replacement);
      s.set_left(p, 0), s.set_right(p, 0), s.set_par(p, 0);
    }
    const uint32_t r = red(p) ? root : balance_deletion(root, replacement);
    if (replacement == p) {  // detach
      const uint32_t pp = s.par(p);
      s.set_par(p, 0);
      if (pp) {
        if (p == s.left(pp)) s.set_left(pp, 0);
        else if (p == s.right(pp)) s.set_right(pp, 0);
      }
    }
    to_front(r);
  }
  // the chain length of a list bin of hash h (a tree bin, or a chain longer than `most`: most + 1)
  __device__ __forceinline__ uint32_t chain_len(uint32_t h, uint32_t most) const {
    const D& s = d();
    uint32_t q = s.tab((s.cap() - 1) & h), c = 0;
    if (q && tree(q)) return most + 1;
    for (; q && c <= most; q = s.next(q)) ++c;
    return c;
  }
  // removeNode(movable = true) of the live key (kt, key) with hash h; false: the store does not hold it
  __device__ __forceinline__ bool remove_key(uint32_t h, uint32_t kt, uint64_t key, uint32_t max_steps) {
    D& s = d();
    const uint32_t index = (s.cap() - 1) & h;
    uint32_t node = 0, prv = 0, pp = 0;
    for (uint32_t q = s.tab(index), steps = 0; q && steps < max_steps; pp = q, q = s.next(q), ++steps)
      if (s.hash(q) == h && s.ktv(q) == kt && s.keyv(q) == key) {
        node = q, prv = pp;
        break;
      }
    if (!node) return false;
    if (tree(node)) remove_tree_node(node, index);
    else if (!prv) s.set_tab(index, s.next(node));
    else s.set_next(prv, s.next(node));
    s.release(node);
    --s.n;
    return true;
  }
};

}  // namespace cc
