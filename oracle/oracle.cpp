// oracle.cpp — CPU restatement of the reference commit-apply path.  TEST INFRASTRUCTURE ONLY (see oracle.h).
//
// Every state-machine method below cites the Java method it restates (paths relative to the reference
// root).  Values are canonical tagged values (tag, payload): Java `equals` on boxed values becomes exact
// (tag, payload) equality.  Commit objects are represented by their log index
// and instance slot; `commit.clean()` matters only where the reference can clean one twice (the
// ResourceManagerCommit assert `Assert.state(open, "commit closed")`, ResourceManagerCommit.java:79-83).
#include "oracle.h"

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <deque>
#include <map>
#include <unordered_map>
#include <utility>
#include <vector>

namespace {

struct TV {
  uint8_t tag = CC_TAG_NULL;
  uint64_t v = 0;
};
inline bool tv_null(const TV& x) { return x.tag == CC_TAG_NULL; }
// x.equals(y) for a non-null receiver x (Long/Integer/Boolean.equals are type-sensitive, A15).
inline bool tv_equals(const TV& x, const TV& y) { return x.tag == y.tag && x.v == y.v; }
inline TV tv(uint8_t tag, uint64_t v) { TV t; t.tag = tag; t.v = tag == CC_TAG_NULL ? 0 : v; return t; }

// Key tags in the flags column map to value tags (keys are never null: MapCommands.java:77).
inline uint8_t ktag_to_tag(uint8_t k) {
  static const uint8_t m[4] = {CC_TAG_LONG, CC_TAG_INT, CC_TAG_BOOL, CC_TAG_HANDLE};
  return m[k & 3];
}

struct MapKey {
  uint8_t tag;
  uint64_t k;
  bool operator==(const MapKey& o) const { return tag == o.tag && k == o.k; }
};
struct MapKeyHash {
  size_t operator()(const MapKey& x) const { return (size_t)(x.k * 0x9E3779B97F4A7C15ull) ^ x.tag; }
};
// ---- java.util.HashMap, JDK 8 (the reference's CI JDK, .travis.yml: oraclejdk8) -------------------------------
// java.util.HashMap is not in /root/reference (a JDK class).  Its published JDK 8 algorithm is restated here for the
// outputs that depend on iteration order (MapState.containsValue :49-60 walks map.values(); ResourceManager.close
// :250-264 walks sessions.values()): the bins, each bin's `next` chain, and the red-black tree bins --
//   hash(key) = h ^ (h >>> 16), h = key.hashCode()  (Long: (int)(v ^ (v >>> 32)); Integer: v; Boolean: 1231 / 1237;
//     String: s[0]*31^(n-1) + ... over its UTF-16 units -- a HANDLE key is a String registered with orc_handle_string);
//   putVal: a new key is appended to its bin's chain; when the chain it joined then holds >= 9 nodes
//     (binCount >= TREEIFY_THRESHOLD - 1), treeifyBin: capacity < 64 (MIN_TREEIFY_CAPACITY) -> resize(), else the
//     bin becomes a tree (treeify, root moved to the front); a tree bin takes a new key through putTreeVal (linked
//     after its tree parent in the chain, root moved to the front); then ++size > threshold -> resize();
//   resize: capacity 16 (threshold 12) at the first put, then doubled; chains split into lo / hi keeping their order;
//     tree bins split the same way and untreeify at <= 6 nodes (UNTREEIFY_THRESHOLD) or are re-treeified;
//   removeNode(movable = true): chains unlink; tree bins unlink from the chain, untreeify when the tree is too small
//     (root.right / root.left / root.left.left null), else the red-black delete, root moved to the front;
//   iteration: bins in index order, each along `next`.
// Tree order: hash (signed int compare), then compareTo for keys of one class, else the class names (tieBreakOrder:
// java.lang.Boolean < Integer < Long < String).  Distinct keys of one class never compare equal, so
// System.identityHashCode is never reached.
struct JCtx {  // String contents of HANDLE keys (handle -> UTF-16 units), registered by the test harness
  std::unordered_map<uint64_t, std::vector<uint16_t>> str;
};
inline int32_t java_hashcode(const JCtx& cx, uint8_t tag, uint64_t v) {
  switch (tag) {
    case CC_TAG_INT: return (int32_t)(uint32_t)v;
    case CC_TAG_BOOL: return v ? 1231 : 1237;
    case CC_TAG_HANDLE: {
      auto it = cx.str.find(v);
      if (it != cx.str.end()) {
        uint32_t h = 0;  // String.hashCode
        for (uint16_t u : it->second) h = 31u * h + u;
        return (int32_t)h;
      }
      break;  // an unregistered handle: hashed as a Long (the engine refuses to guess: CC_ERR_STATE)
    }
    default: break;
  }
  return (int32_t)(uint32_t)(v ^ (v >> 32));
}
inline uint32_t java_spread(int32_t h) { return (uint32_t)h ^ ((uint32_t)h >> 16); }
inline uint32_t java_hash(const JCtx& cx, uint8_t tag, uint64_t v) { return java_spread(java_hashcode(cx, tag, v)); }

struct JHM {
  static constexpr int kNil = -1;
  struct Node {
    uint32_t hash = 0;
    MapKey key{};
    int next = kNil, prev = kNil, parent = kNil, left = kNil, right = kNil;
    bool tree = false, red = false;
  };
  std::vector<Node> nd;
  std::vector<int> free_;
  std::vector<int> tab;  // empty until the first put (HashMap() allocates lazily)
  uint32_t size = 0, threshold = 0;
  std::unordered_map<MapKey, int, MapKeyHash> where;  // key -> node (a lookup shortcut; order lives in nd / tab)

  uint32_t capacity() const { return (uint32_t)tab.size(); }
  static int cls_rank(uint8_t tag) {  // getClass().getName() order
    return tag == CC_TAG_BOOL ? 0 : tag == CC_TAG_INT ? 1 : tag == CC_TAG_LONG ? 2 : 3;
  }
  // dir of key k (hash h) against node p, as treeify / putTreeVal compute it for a key not in the tree
  static int dir_of(const JCtx& cx, uint32_t h, const MapKey& k, const Node& p) {
    const int32_t ph = (int32_t)p.hash, hh = (int32_t)h;
    if (ph > hh) return -1;
    if (ph < hh) return 1;
    const MapKey& pk = p.key;
    if (k.tag == pk.tag) {  // compareComparables: same class
      int c = 0;
      switch (k.tag) {
        case CC_TAG_LONG: c = (int64_t)k.k < (int64_t)pk.k ? -1 : ((int64_t)k.k > (int64_t)pk.k ? 1 : 0); break;
        case CC_TAG_INT: c = (int32_t)k.k < (int32_t)pk.k ? -1 : ((int32_t)k.k > (int32_t)pk.k ? 1 : 0); break;
        case CC_TAG_BOOL: c = (k.k != 0) == (pk.k != 0) ? 0 : (k.k ? 1 : -1); break;
        default: {  // String.compareTo (unregistered handles: by handle number)
          auto a = cx.str.find(k.k), b = cx.str.find(pk.k);
          if (a != cx.str.end() && b != cx.str.end()) {
            const auto &x = a->second, &y = b->second;
            const size_t n = std::min(x.size(), y.size());
            for (size_t i = 0; i < n && !c; ++i) c = x[i] < y[i] ? -1 : (x[i] > y[i] ? 1 : 0);
            if (!c) c = x.size() < y.size() ? -1 : (x.size() > y.size() ? 1 : 0);
          } else {
            c = k.k < pk.k ? -1 : (k.k > pk.k ? 1 : 0);
          }
        }
      }
      if (c) return c;
    }
    // tieBreakOrder: class names (equal keys of one class never get here)
    return cls_rank(k.tag) <= cls_rank(pk.tag) ? -1 : 1;
  }

  int new_node(uint32_t h, const MapKey& k) {
    int x;
    if (!free_.empty()) { x = free_.back(); free_.pop_back(); nd[x] = Node(); }
    else { x = (int)nd.size(); nd.emplace_back(); }
    nd[x].hash = h;
    nd[x].key = k;
    return x;
  }

  // ---- red-black tree bins (HashMap.TreeNode) ----
  int rotate_left(int root, int p) {
    int r, pp, rl;
    if (p != kNil && (r = nd[p].right) != kNil) {
      if ((rl = nd[p].right = nd[r].left) != kNil) nd[rl].parent = p;
      if ((pp = nd[r].parent = nd[p].parent) == kNil) { root = r; nd[r].red = false; }
      else if (nd[pp].left == p) nd[pp].left = r;
      else nd[pp].right = r;
      nd[r].left = p;
      nd[p].parent = r;
    }
    return root;
  }
  int rotate_right(int root, int p) {
    int l, pp, lr;
    if (p != kNil && (l = nd[p].left) != kNil) {
      if ((lr = nd[p].left = nd[l].right) != kNil) nd[lr].parent = p;
      if ((pp = nd[l].parent = nd[p].parent) == kNil) { root = l; nd[l].red = false; }
      else if (nd[pp].right == p) nd[pp].right = l;
      else nd[pp].left = l;
      nd[l].right = p;
      nd[p].parent = l;
    }
    return root;
  }
  int balance_insertion(int root, int x) {
    nd[x].red = true;
    for (int xp, xpp, xppl, xppr;;) {
      if ((xp = nd[x].parent) == kNil) { nd[x].red = false; return x; }
      else if (!nd[xp].red || (xpp = nd[xp].parent) == kNil) return root;
      if (xp == (xppl = nd[xpp].left)) {
        if ((xppr = nd[xpp].right) != kNil && nd[xppr].red) {
          nd[xppr].red = false; nd[xp].red = false; nd[xpp].red = true; x = xpp;
        } else {
          if (x == nd[xp].right) {
            root = rotate_left(root, x = xp);
            xpp = (xp = nd[x].parent) == kNil ? kNil : nd[xp].parent;
          }
          if (xp != kNil) {
            nd[xp].red = false;
            if (xpp != kNil) { nd[xpp].red = true; root = rotate_right(root, xpp); }
          }
        }
      } else {
        if (xppl != kNil && nd[xppl].red) {
          nd[xppl].red = false; nd[xp].red = false; nd[xpp].red = true; x = xpp;
        } else {
          if (x == nd[xp].left) {
            root = rotate_right(root, x = xp);
            xpp = (xp = nd[x].parent) == kNil ? kNil : nd[xp].parent;
          }
          if (xp != kNil) {
            nd[xp].red = false;
            if (xpp != kNil) { nd[xpp].red = true; root = rotate_left(root, xpp); }
          }
        }
      }
    }
  }
  int balance_deletion(int root, int x) {
    for (int xp, xpl, xpr;;) {
      if (x == kNil || x == root) return root;
      else if ((xp = nd[x].parent) == kNil) { nd[x].red = false; return x; }
      else if (nd[x].red) { nd[x].red = false; return root; }
      else if ((xpl = nd[xp].left) == x) {
        if ((xpr = nd[xp].right) != kNil && nd[xpr].red) {
          nd[xpr].red = false; nd[xp].red = true;
          root = rotate_left(root, xp);
          xpr = (xp = nd[x].parent) == kNil ? kNil : nd[xp].right;
        }
        if (xpr == kNil) x = xp;
        else {
          int sl = nd[xpr].left, sr = nd[xpr].right;
          if ((sr == kNil || !nd[sr].red) && (sl == kNil || !nd[sl].red)) {
            nd[xpr].red = true; x = xp;
          } else {
            if (sr == kNil || !nd[sr].red) {
              if (sl != kNil) nd[sl].red = false;
              nd[xpr].red = true;
              root = rotate_right(root, xpr);
              xpr = (xp = nd[x].parent) == kNil ? kNil : nd[xp].right;
            }
            if (xpr != kNil) {
              nd[xpr].red = (xp == kNil) ? false : nd[xp].red;
              if ((sr = nd[xpr].right) != kNil) nd[sr].red = false;
            }
            if (xp != kNil) { nd[xp].red = false; root = rotate_left(root, xp); }
            x = root;
          }
        }
      } else {  // symmetric
        if (xpl != kNil && nd[xpl].red) {
          nd[xpl].red = false; nd[xp].red = true;
          root = rotate_right(root, xp);
          xpl = (xp = nd[x].parent) == kNil ? kNil : nd[xp].left;
        }
        if (xpl == kNil) x = xp;
        else {
          int sl = nd[xpl].left, sr = nd[xpl].right;
          if ((sl == kNil || !nd[sl].red) && (sr == kNil || !nd[sr].red)) {
            nd[xpl].red = true; x = xp;
          } else {
            if (sl == kNil || !nd[sl].red) {
              if (sr != kNil) nd[sr].red = false;
              nd[xpl].red = true;
              root = rotate_left(root, xpl);
              xpl = (xp = nd[x].parent) == kNil ? kNil : nd[xp].left;
            }
            if (xpl != kNil) {
              nd[xpl].red = (xp == kNil) ? false : nd[xp].red;
              if ((sl = nd[xpl].left) != kNil) nd[sl].red = false;
            }
            if (xp != kNil) { nd[xp].red = false; root = rotate_right(root, xp); }
            x = root;
          }
        }
      }
    }
  }
  void move_root_to_front(int root) {
    if (root == kNil || tab.empty()) return;
    const uint32_t index = (capacity() - 1) & nd[root].hash;
    const int first = tab[index];
    if (root != first) {
      int rn;
      tab[index] = root;
      const int rp = nd[root].prev;
      if ((rn = nd[root].next) != kNil) nd[rn].prev = rp;
      if (rp != kNil) nd[rp].next = rn;
      if (first != kNil) nd[first].prev = root;
      nd[root].next = first;
      nd[root].prev = kNil;
    }
  }
  int root_of(int p) const {
    while (nd[p].parent != kNil) p = nd[p].parent;
    return p;
  }
  // TreeNode.treeify from chain head `hd` (every node already a tree node, linked by next / prev)
  void treeify(const JCtx& cx, int hd) {
    int root = kNil;
    for (int x = hd, next; x != kNil; x = next) {
      next = nd[x].next;
      nd[x].left = nd[x].right = kNil;
      if (root == kNil) {
        nd[x].parent = kNil;
        nd[x].red = false;
        root = x;
      } else {
        for (int p = root;;) {
          const int dir = dir_of(cx, nd[x].hash, nd[x].key, nd[p]);
          const int xp = p;
          if ((p = (dir <= 0) ? nd[p].left : nd[p].right) == kNil) {
            nd[x].parent = xp;
            if (dir <= 0) nd[xp].left = x;
            else nd[xp].right = x;
            root = balance_insertion(root, x);
            break;
          }
        }
      }
    }
    move_root_to_front(root);
  }
  // TreeNode.untreeify: plain nodes, same chain order
  int untreeify(int hd) {
    for (int q = hd; q != kNil; q = nd[q].next) {
      nd[q].tree = false;
      nd[q].red = false;
      nd[q].parent = nd[q].left = nd[q].right = nd[q].prev = kNil;
    }
    return hd;
  }
  void treeify_bin(const JCtx& cx, uint32_t h) {
    const uint32_t n = capacity();
    if (n < 64) {  // MIN_TREEIFY_CAPACITY
      resize(cx);
      return;
    }
    const uint32_t index = (n - 1) & h;
    int e = tab[index];
    if (e == kNil) return;
    int tl = kNil;
    for (; e != kNil; e = nd[e].next) {  // replacementTreeNode: chain order kept, prev links added
      nd[e].tree = true;
      nd[e].prev = tl;
      tl = e;
    }
    treeify(cx, tab[index]);
  }
  // TreeNode.split on resize
  void split(const JCtx& cx, std::vector<int>& ntab, int b, uint32_t index, uint32_t bit) {
    int loHead = kNil, loTail = kNil, hiHead = kNil, hiTail = kNil;
    int lc = 0, hc = 0;
    for (int e = b, next; e != kNil; e = next) {
      next = nd[e].next;
      nd[e].next = kNil;
      if ((nd[e].hash & bit) == 0) {
        if ((nd[e].prev = loTail) == kNil) loHead = e;
        else nd[loTail].next = e;
        loTail = e;
        ++lc;
      } else {
        if ((nd[e].prev = hiTail) == kNil) hiHead = e;
        else nd[hiTail].next = e;
        hiTail = e;
        ++hc;
      }
    }
    std::vector<int> saved;
    saved.swap(tab);  // treeify / moveRootToFront work on the NEW table
    tab.swap(ntab);
    if (loHead != kNil) {
      if (lc <= 6) tab[index] = untreeify(loHead);
      else {
        tab[index] = loHead;
        if (hiHead != kNil) treeify(cx, loHead);
      }
    }
    if (hiHead != kNil) {
      if (hc <= 6) tab[index + bit] = untreeify(hiHead);
      else {
        tab[index + bit] = hiHead;
        if (loHead != kNil) treeify(cx, hiHead);
      }
    }
    tab.swap(ntab);
    saved.swap(tab);
  }
  void resize(const JCtx& cx) {
    const uint32_t oldCap = capacity();
    uint32_t newCap, newThr;
    if (oldCap > 0) { newCap = oldCap << 1; newThr = threshold << 1; }
    else { newCap = 16; newThr = 12; }
    threshold = newThr;
    std::vector<int> ntab(newCap, kNil);
    for (uint32_t j = 0; j < oldCap; ++j) {
      const int e = tab[j];
      if (e == kNil) continue;
      if (nd[e].next == kNil) ntab[nd[e].hash & (newCap - 1)] = e;
      else if (nd[e].tree) split(cx, ntab, e, j, oldCap);
      else {  // preserve order
        int loHead = kNil, loTail = kNil, hiHead = kNil, hiTail = kNil;
        for (int q = e, next; q != kNil; q = next) {
          next = nd[q].next;
          if ((nd[q].hash & oldCap) == 0) {
            if (loTail == kNil) loHead = q; else nd[loTail].next = q;
            loTail = q;
          } else {
            if (hiTail == kNil) hiHead = q; else nd[hiTail].next = q;
            hiTail = q;
          }
        }
        if (loTail != kNil) { nd[loTail].next = kNil; ntab[j] = loHead; }
        if (hiTail != kNil) { nd[hiTail].next = kNil; ntab[j + oldCap] = hiHead; }
      }
    }
    tab.swap(ntab);
  }
  // putVal for a key NOT in the map (an existing key's put changes no structure)
  void put_new(const JCtx& cx, const MapKey& k) {
    if (where.count(k)) return;
    const uint32_t h = java_hash(cx, k.tag, k.k);
    if (tab.empty()) resize(cx);
    const uint32_t i = (capacity() - 1) & h;
    int p = tab[i];
    if (p == kNil) {
      tab[i] = where[k] = new_node(h, k);
    } else if (nd[p].tree) {  // putTreeVal
      const int root = nd[p].parent != kNil ? root_of(p) : p;
      for (int q = root;;) {
        const int dir = dir_of(cx, h, k, nd[q]);
        const int xp = q;
        if ((q = (dir <= 0) ? nd[q].left : nd[q].right) == kNil) {
          const int xpn = nd[xp].next;
          const int x = new_node(h, k);
          where[k] = x;
          nd[x].tree = true;
          nd[x].next = xpn;
          if (dir <= 0) nd[xp].left = x; else nd[xp].right = x;
          nd[xp].next = x;
          nd[x].parent = nd[x].prev = xp;
          if (xpn != kNil) nd[xpn].prev = x;
          move_root_to_front(balance_insertion(root, x));
          break;
        }
      }
    } else {
      int binCount = 0;
      while (nd[p].next != kNil) { p = nd[p].next; ++binCount; }
      const int x = new_node(h, k);
      where[k] = x;
      nd[p].next = x;
      if (binCount >= 7) treeify_bin(cx, h);  // TREEIFY_THRESHOLD - 1: the chain now holds >= 9 nodes
    }
    if (++size > threshold) resize(cx);
  }
  // removeNode(hash, key, null, false, movable) for a key in the map: map.remove(key) passes movable = true,
  // an iterator's remove() movable = false (no untreeify when small, no moveRootToFront)
  void remove(const JCtx& cx, const MapKey& k, bool movable = true) {
    auto it = where.find(k);
    if (it == where.end()) return;
    const int node = it->second;
    where.erase(it);
    const uint32_t n = capacity();
    const uint32_t index = (n - 1) & nd[node].hash;
    if (nd[node].tree) {
      remove_tree_node(node, index, movable);
    } else {
      int p = tab[index];
      if (p == node) tab[index] = nd[node].next;
      else {
        while (nd[p].next != node) p = nd[p].next;
        nd[p].next = nd[node].next;
      }
    }
    --size;
    free_.push_back(node);
  }
  void remove_tree_node(int self, uint32_t index, bool movable) {  // TreeNode.removeTreeNode(map, tab, movable)
    int first = tab[index], root = first, rl;
    const int succ = nd[self].next, pred = nd[self].prev;
    if (pred == kNil) tab[index] = first = succ;
    else nd[pred].next = succ;
    if (succ != kNil) nd[succ].prev = pred;
    if (first == kNil) return;
    if (nd[root].parent != kNil) root = root_of(root);
    if (root == kNil || (movable && (nd[root].right == kNil || (rl = nd[root].left) == kNil || nd[rl].left == kNil))) {
      tab[index] = untreeify(first);  // too small
      return;
    }
    int p = self, pl = nd[self].left, pr = nd[self].right, replacement;
    if (pl != kNil && pr != kNil) {
      int s = pr, sl;
      while ((sl = nd[s].left) != kNil) s = sl;  // successor
      const bool c = nd[s].red;
      nd[s].red = nd[p].red;
      nd[p].red = c;  // swap colors
      const int sr = nd[s].right;
      const int pp = nd[p].parent;
      if (s == pr) {  // p was s's direct parent
        nd[p].parent = s;
        nd[s].right = p;
      } else {
        const int sp = nd[s].parent;
        if ((nd[p].parent = sp) != kNil) {
          if (s == nd[sp].left) nd[sp].left = p;
          else nd[sp].right = p;
        }
        if ((nd[s].right = pr) != kNil) nd[pr].parent = s;
      }
      nd[p].left = kNil;
      if ((nd[p].right = sr) != kNil) nd[sr].parent = p;
      if ((nd[s].left = pl) != kNil) nd[pl].parent = s;
      if ((nd[s].parent = pp) == kNil) root = s;
      else if (p == nd[pp].left) nd[pp].left = s;
      else nd[pp].right = s;
      replacement = sr != kNil ? sr : p;
    } else if (pl != kNil) replacement = pl;
    else if (pr != kNil) replacement = pr;
    else replacement = p;
    if (replacement != p) {
      const int pp = nd[replacement].parent = nd[p].parent;
      if (pp == kNil) root = replacement;
      else if (p == nd[pp].left) nd[pp].left = replacement;
      else nd[pp].right = replacement;
      nd[p].left = nd[p].right = nd[p].parent = kNil;
    }
    const int r = nd[p].red ? root : balance_deletion(root, replacement);
    if (replacement == p) {  // detach
      const int pp = nd[p].parent;
      nd[p].parent = kNil;
      if (pp != kNil) {
        if (p == nd[pp].left) nd[pp].left = kNil;
        else if (p == nd[pp].right) nd[pp].right = kNil;
      }
    }
    if (movable) move_root_to_front(r);
  }
  // MapState.delete (iterator.remove() on every entry): every bin empties, the table keeps its capacity
  void clear() {
    std::fill(tab.begin(), tab.end(), kNil);
    nd.clear();
    free_.clear();
    where.clear();
    size = 0;
  }
  // map.values() / keySet() iteration order
  template <class F>
  void for_each(F f) const {
    for (int b : tab)
      for (int q = b; q != kNil; q = nd[q].next) f(nd[q].key);
  }
};

struct Commit {  // a retained commit: index + instance-session slot
  uint64_t index = 0;
  uint32_t inst = 0;
  bool cleaned = false;
};

// AtomicValueState.java:32-36
struct ValueSM {
  TV value;
  bool has_current = false;
  Commit current;
  std::vector<std::pair<uint32_t, uint64_t>> listeners;  // (instance slot, listen index); insertion order
};

// MapState.Value{commit, timer} MapState.java:279-287
struct MapEntry {
  TV value;
  uint64_t commit_index = 0;
  uint64_t timer = 0;  // 0 = none
};
struct MapSM {
  std::unordered_map<MapKey, MapEntry, MapKeyHash> m;
  JHM order;  // the java.util.HashMap structure (iteration order)
};

// LockState.java:33-36
struct LockSM {
  bool held = false;
  Commit lock;
  std::deque<Commit> queue;
  std::unordered_map<uint64_t, uint64_t> timers;  // commit index -> timer id
};

// LeaderElectionState.java:31-33 (LinkedHashMap<Long, Commit> = insertion-ordered vector)
struct ElectionSM {
  bool has_leader = false;
  Commit leader;
  std::vector<std::pair<uint64_t, Commit>> listeners;  // (instance id, listen commit)
};

// MembershipGroupState.java:33-34 (HashMap<Long, Commit>)
struct GroupSM {
  std::unordered_map<uint64_t, Commit> members;  // instance id -> join commit
};

struct Resource {
  bool exists = false;
  uint32_t type = CC_RES_NONE;
  uint64_t id = 0;   // resource id (= creating commit index under the manager)
  uint64_t key = 0;  // interned key handle
  bool has_key = false;
  // removed from ResourceManager.resources by a deleteResource whose delete() threw (:214-220): the instances that
  // still name its id find `resources.get(id) == null` forever, so the slot is never handed out again
  bool zombie = false;
  std::unordered_map<uint64_t, uint64_t> sessions;  // ResourceHolder.sessions: client session -> instance id
  ValueSM v;
  MapSM m;
  LockSM l;
  ElectionSM e;
  GroupSM g;
  // QueueState.queue: ArrayDeque of commits (QueueState.java:33): value, index, and whether element() already
  // clean()ed the head commit it did not remove (:111-124)
  struct QEnt {
    TV v;
    uint64_t idx = 0;
    bool cleaned = false;
  };
  std::deque<QEnt> q;
  // commits dropped without clean(): retained by the log for good (AtomicValueState.listen re-put :42,
  // MembershipGroupState.close :37-38)
  std::vector<uint64_t> leaked;
};

struct Inst {  // ResourceManager.SessionHolder + ManagedResourceSession
  bool open = false;
  uint32_t res = 0;
  uint64_t id = 0;      // instance id (ManagedResourceSession.id())
  uint64_t client = 0;  // parent client session id
};

enum TimerKind : uint8_t { T_MAP_TTL = 1, T_MAP_REPLACE_TTL = 2, T_LOCK_TIMEOUT = 3, T_GROUP_SCHEDULE = 4 };
struct Timer {
  uint64_t id = 0, deadline = 0;
  uint32_t res = 0;
  uint8_t kind = 0;
  MapKey key{0, 0};
  uint64_t commit_index = 0;
  uint64_t member = 0;
  TV callback;
};

struct Event {
  uint32_t pos, target;
  uint8_t code, src, tag;
  uint64_t payload;
};

}  // namespace

struct orc {
  uint32_t max_res, max_inst, flags;
  std::vector<Resource> res;
  std::vector<Inst> inst;
  std::unordered_map<uint64_t, uint32_t> inst_by_id;  // ResourceManager.sessions key -> slot
  JHM sessions_order;                                  // ResourceManager.sessions (HashMap<Long, ...>) structure
  JCtx cx;                                             // String contents of HANDLE keys (java hashCode / compareTo)
  std::unordered_map<uint64_t, uint64_t> keys;         // ResourceManager.keys: key -> resource id
  std::unordered_map<uint64_t, uint32_t> res_by_id;    // ResourceManager.resources: id -> slot
  std::map<std::pair<uint64_t, uint64_t>, Timer> timers;  // (deadline, id) -> timer
  std::unordered_map<uint64_t, uint64_t> timer_deadline;  // id -> deadline
  uint64_t next_timer = 1;
  uint64_t clock = 0;
  uint64_t applied = 0;
  std::vector<Event> events;
  std::vector<std::pair<uint32_t, uint64_t>> aux;
  uint32_t cur_pos = 0;
  uint8_t cur_src = CC_EVSRC_COMMIT;

  void publish(uint32_t target, uint8_t code, TV payload) {
    events.push_back(Event{cur_pos, target, code, cur_src, payload.tag, payload.v});
  }

  // ---- timers: deterministic executor clock (Copycat ServerStateMachineExecutor, not vendored) ------
  uint64_t schedule(uint64_t delay, Timer t) {
    t.id = next_timer++;
    t.deadline = clock + delay;
    timers.emplace(std::make_pair(t.deadline, t.id), t);
    timer_deadline[t.id] = t.deadline;
    return t.id;
  }
  void cancel(uint64_t id) {
    auto it = timer_deadline.find(id);
    if (it == timer_deadline.end()) return;
    timers.erase(std::make_pair(it->second, id));
    timer_deadline.erase(it);
  }
  void fire_due() {
    uint8_t saved = cur_src;
    cur_src = CC_EVSRC_TIMER;
    while (!timers.empty() && timers.begin()->first.first <= clock) {
      Timer t = timers.begin()->second;
      timers.erase(timers.begin());
      timer_deadline.erase(t.id);
      run_timer(t);
    }
    cur_src = saved;
  }
  void run_timer(const Timer& t) {
    Resource& r = res[t.res];
    if (!r.exists) return;
    switch (t.kind) {
      case T_MAP_TTL:          // MapState.java:91-93,119-121,218-220: map.remove(key).commit.clean()
      case T_MAP_REPLACE_TTL: {  // MapState.java:189-192: map.remove(key); commit.clean()
        auto it = r.m.m.find(t.key);
        if (it != r.m.m.end()) { r.m.m.erase(it); r.m.order.remove(cx, t.key); }
        break;
      }
      case T_LOCK_TIMEOUT: {   // LockState.java:54-58 (silent, A7)
        r.l.timers.erase(t.commit_index);
        for (auto it = r.l.queue.begin(); it != r.l.queue.end(); ++it)
          if (it->index == t.commit_index) { r.l.queue.erase(it); break; }
        break;
      }
      case T_GROUP_SCHEDULE: {  // MembershipGroupState.java:92-98
        auto it = r.g.members.find(t.member);
        if (it != r.g.members.end()) publish(it->second.inst, CC_EV_EXECUTE, t.callback);
        break;
      }
    }
  }
  void cancel_resource_timers(uint32_t slot) {  // ResourceManagerStateMachineExecutor.close :137-140
    std::vector<uint64_t> ids;
    for (auto& kv : timers) if (kv.second.res == slot) ids.push_back(kv.second.id);
    for (uint64_t id : ids) cancel(id);
  }

  // ---- registry ------------------------------------------------------------------------------------
  void register_instance(uint32_t slot, uint32_t rslot, uint64_t id, uint64_t client) {
    Inst& in = inst[slot];
    in.open = true; in.res = rslot; in.id = id; in.client = client;
    inst_by_id[id] = slot;
    sessions_order.put_new(cx, MapKey{CC_TAG_LONG, id});
  }
  void unregister_instance(uint32_t slot) {
    Inst& in = inst[slot];
    if (!in.open) return;
    in.open = false;
    inst_by_id.erase(in.id);
    // ResourceManager removes holders only through sessions.entrySet().iterator().remove() (:227, :261)
    sessions_order.remove(cx, MapKey{CC_TAG_LONG, in.id}, /*movable=*/false);
  }
  int alloc_res_slot() {
    for (uint32_t s = 0; s < max_res; ++s) if (!res[s].exists && !res[s].zombie) return (int)s;
    return -1;
  }
  int alloc_inst_slot() {
    for (uint32_t s = 0; s < max_inst; ++s) if (!inst[s].open) return (int)s;
    return -1;
  }
  void init_resource(uint32_t slot, uint32_t type, uint64_t id) {
    Resource fresh;
    res[slot] = std::move(fresh);
    res[slot].exists = true;
    res[slot].type = type;
    res[slot].id = id;
    res_by_id[id] = slot;
  }

  // ---- state machine delete() overrides ----------------------------------------------------------------
  // returns a status code (the reference can throw "commit closed" from a double clean)
  uint8_t sm_delete(uint32_t slot) {
    Resource& r = res[slot];
    switch (r.type) {
      case CC_RES_VALUE:  // AtomicValueState.delete :146-157 (timer is always null, A2)
        if (r.v.has_current) { r.v.has_current = false; r.v.value = TV(); }
        return CC_ST_OK;
      case CC_RES_QUEUE:  // QueueState.delete :191-199
        r.q.clear();
        return CC_ST_OK;
      case CC_RES_MULTIMAP:  // MultiMapState.delete :209-222 (its value maps are always empty: A18)
      case CC_RES_SET:  // SetState.delete :123-134 (same shape: cancel timers, clean, clear)
      case CC_RES_MAP: {  // MapState.delete :264-274
        for (auto& kv : r.m.m) if (kv.second.timer) cancel(kv.second.timer);
        r.m.order.clear();
        r.m.m.clear();
        return CC_ST_OK;
      }
      case CC_RES_LOCK: {  // LockState.delete :87-98 — `lock` is cleaned but NOT nulled
        uint8_t st = CC_ST_OK;
        if (r.l.held) {
          if (r.l.lock.cleaned) return CC_ST_ILLEGAL_STATE;  // ResourceManagerCommit.clean: "commit closed"
          r.l.lock.cleaned = true;
        }
        r.l.queue.clear();
        for (auto& kv : r.l.timers) cancel(kv.second);
        r.l.timers.clear();
        return st;
      }
      case CC_RES_ELECTION: {  // LeaderElectionState.delete :100-108 — `leader` cleaned, NOT nulled
        if (r.e.has_leader) {
          if (r.e.leader.cleaned) return CC_ST_ILLEGAL_STATE;
          r.e.leader.cleaned = true;
        }
        r.e.listeners.clear();
        return CC_ST_OK;
      }
      case CC_RES_GROUP:  // MembershipGroupState.delete :121-125
        r.g.members.clear();
        return CC_ST_OK;
    }
    return CC_ST_OK;
  }

  // ---- StateMachine.close(Session) overrides (ResourceManager.close fan-out) ---------------------------
  // returns false if the close threw (aborts the ResourceManager.close loop; unpinned)
  bool sm_close(uint32_t islot) {
    Inst& in = inst[islot];
    Resource& r = res[in.res];
    switch (r.type) {
      case CC_RES_VALUE: {  // AtomicValueState.listen onClose hook :43-48 (parent session closed)
        auto& L = r.v.listeners;
        L.erase(std::remove_if(L.begin(), L.end(), [&](const std::pair<uint32_t, uint64_t>& p) { return p.first == islot; }),
                L.end());
        return true;
      }
      case CC_RES_ELECTION: {  // LeaderElectionState.close :35-52
        ElectionSM& e = r.e;
        if (e.has_leader && e.leader.inst == islot) {
          if (e.leader.cleaned) return false;  // leader.clean() throws "commit closed"
          e.has_leader = false;
          if (!e.listeners.empty()) {
            e.leader = e.listeners.front().second;
            e.has_leader = true;
            e.listeners.erase(e.listeners.begin());
            publish(e.leader.inst, CC_EV_ELECT, tv(CC_TAG_LONG, e.leader.index));
          }
        } else {
          for (auto it = e.listeners.begin(); it != e.listeners.end(); ++it)
            if (it->first == in.id) { e.listeners.erase(it); break; }
        }
        return true;
      }
      case CC_RES_GROUP: {  // MembershipGroupState.close :36-42 — publishes leave even for non-members (A10)
        auto mit = r.g.members.find(in.id);  // members.remove without clean(): the join commit is never released
        if (mit != r.g.members.end()) {
          r.leaked.push_back(mit->second.index);
          r.g.members.erase(mit);
        }
        for (auto& kv : r.g.members) publish(kv.second.inst, CC_EV_LEAVE, tv(CC_TAG_LONG, in.id));
        return true;
      }
      default:
        return true;  // MapState / LockState have no close handler (A11)
    }
  }

  // ---- one commit ------------------------------------------------------------------------------------
  struct Row {
    uint64_t index, time, key, a, b, aux;
    uint32_t inst;
    uint8_t op, flags;
  };

  // ResourceManager.operateResource :56-72 -> executors :90-102 / :73-91 -> state machine method
  void apply_one(const Row& c, uint8_t& status, uint64_t& value) {
    status = CC_STATUS(CC_ST_OK, CC_TAG_NULL);
    value = 0;
    if (c.inst >= max_inst || !inst[c.inst].open) {  // sessions.get(instanceId) == null
      status = CC_STATUS(CC_ST_UNKNOWN_SESSION, CC_TAG_NULL);
      return;
    }
    const Inst& in = inst[c.inst];
    Resource& r = res[in.res];
    if (!r.exists) {  // holder left behind by a failed deleteResource: resource.executor NPE (:71)
      status = CC_STATUS(CC_ST_NULL_POINTER, CC_TAG_NULL);
      return;
    }
    TV a = tv(CC_FLAG_TAG_A(c.flags), c.a);
    TV b = tv(CC_FLAG_TAG_B(c.flags), c.b);
    auto ret = [&](uint8_t code, TV v) { status = CC_STATUS(code, v.tag); value = v.v; };

    if (c.op == CC_OP_DELETE) {  // ResourceStateMachine.init DeleteCommand :34-40
      ret(sm_delete(in.res), TV());
      return;
    }
    switch (r.type) {
      case CC_RES_VALUE: {
        ValueSM& s = r.v;
        switch (c.op) {
          case CC_OP_VALUE_GET:  // AtomicValueState.get :77-83
            ret(CC_ST_OK, s.has_current ? s.value : TV());
            return;
          case CC_OP_VALUE_SET:  // set :114-118 (cleanCurrent; value = v; setCurrent)
            s.value = a;
            s.has_current = true;
            s.current = Commit{c.index, c.inst, false};
            value_change(s);
            ret(CC_ST_OK, TV());
            return;
          case CC_OP_VALUE_CAS: {  // compareAndSet :123-133
            bool eq = (tv_null(s.value) && tv_null(a)) || (!tv_null(s.value) && !tv_null(a) && tv_equals(s.value, a));
            if (eq) {
              s.value = b;
              s.has_current = true;
              s.current = Commit{c.index, c.inst, false};
              value_change(s);
            }
            ret(CC_ST_OK, tv(CC_TAG_BOOL, eq ? 1 : 0));
            return;
          }
          case CC_OP_VALUE_GETANDSET: {  // getAndSet :138-144
            TV prev = s.value;
            s.value = a;
            s.has_current = true;
            s.current = Commit{c.index, c.inst, false};
            value_change(s);
            ret(CC_ST_OK, prev);
            return;
          }
          case CC_OP_VALUE_LISTEN: {  // listen :41-49 (listeners.put(session, commit))
            bool found = false;
            for (auto& p : s.listeners)
              if (p.first == c.inst) {  // listeners.put replaces the session's commit without clean()ing it
                r.leaked.push_back(p.second);
                p.second = c.index;
                found = true;
              }
            if (!found) s.listeners.emplace_back(c.inst, c.index);
            ret(CC_ST_OK, TV());
            return;
          }
          case CC_OP_VALUE_UNLISTEN: {  // unlisten :54-63
            for (auto it = s.listeners.begin(); it != s.listeners.end(); ++it)
              if (it->first == c.inst) { s.listeners.erase(it); break; }
            ret(CC_ST_OK, TV());
            return;
          }
        }
        break;
      }
      case CC_RES_MAP: {
        MapSM& s = r.m;
        MapKey k{ktag_to_tag(CC_FLAG_KTAG(c.flags)), c.key};
        int64_t ttl = (int64_t)c.aux;
        switch (c.op) {
          case CC_OP_MAP_CONTAINSKEY:  // containsKey :38-44
            ret(CC_ST_OK, tv(CC_TAG_BOOL, s.m.count(k) ? 1 : 0));
            return;
          case CC_OP_MAP_CONTAINSVALUE: {  // containsValue :49-60 — iterates in HashMap order; a stored
            // null value NPEs on `.equals` before a later match is reached (A5).
            bool done = false;
            s.order.for_each([&](const MapKey& key) {
              if (done) return;
              const MapEntry& e = s.m.at(key);
              if (tv_null(e.value)) { ret(CC_ST_NULL_POINTER, TV()); done = true; }
              else if (tv_equals(e.value, a)) { ret(CC_ST_OK, tv(CC_TAG_BOOL, 1)); done = true; }
            });
            if (done) return;
            ret(CC_ST_OK, tv(CC_TAG_BOOL, 0));
            return;
          }
          case CC_OP_MAP_GET: {  // get :65-72 (a key mapped to null is present, A6)
            auto it = s.m.find(k);
            ret(CC_ST_OK, it != s.m.end() ? it->second.value : TV());
            return;
          }
          case CC_OP_MAP_GETORDEFAULT: {  // getOrDefault :77-84 (default = operand a)
            auto it = s.m.find(k);
            ret(CC_ST_OK, it != s.m.end() ? it->second.value : a);
            return;
          }
          case CC_OP_MAP_PUT: {  // put :89-110
            uint64_t timer = 0;
            if (ttl > 0) { Timer t; t.res = in.res; t.kind = T_MAP_TTL; t.key = k; t.commit_index = c.index; timer = schedule((uint64_t)ttl, t); }
            auto it = s.m.find(k);
            if (it != s.m.end()) {
              if (it->second.timer) cancel(it->second.timer);
              TV prev = it->second.value;
              it->second.value = a; it->second.commit_index = c.index; it->second.timer = timer;
              ret(CC_ST_OK, prev);
            } else {
              MapEntry e; e.value = a; e.commit_index = c.index; e.timer = timer; s.order.put_new(cx, k);
              s.m.emplace(k, e);
              ret(CC_ST_OK, TV());
            }
            return;
          }
          case CC_OP_MAP_PUTIFABSENT: {  // putIfAbsent :115-133
            auto it = s.m.find(k);
            if (it == s.m.end()) {
              uint64_t timer = 0;
              if (ttl > 0) { Timer t; t.res = in.res; t.kind = T_MAP_TTL; t.key = k; t.commit_index = c.index; timer = schedule((uint64_t)ttl, t); }
              MapEntry e; e.value = a; e.commit_index = c.index; e.timer = timer; s.order.put_new(cx, k);
              s.m.emplace(k, e);
              ret(CC_ST_OK, TV());
            } else {
              ret(CC_ST_OK, it->second.value);
            }
            return;
          }
          case CC_OP_MAP_REMOVE: {  // remove :138-154
            auto it = s.m.find(k);
            if (it != s.m.end()) {
              if (it->second.timer) cancel(it->second.timer);
              TV prev = it->second.value;
              s.m.erase(it); s.order.remove(cx, k);
              ret(CC_ST_OK, prev);
            } else {
              ret(CC_ST_OK, TV());
            }
            return;
          }
          case CC_OP_MAP_REMOVEIFPRESENT: {  // removeIfPresent :159-178
            auto it = s.m.find(k);
            bool fail = it == s.m.end() || (tv_null(it->second.value) && !tv_null(a)) ||
                        (!tv_null(it->second.value) && !tv_equals(it->second.value, a));
            if (fail) { ret(CC_ST_OK, tv(CC_TAG_BOOL, 0)); return; }
            if (it->second.timer) cancel(it->second.timer);
            s.m.erase(it); s.order.remove(cx, k);
            ret(CC_ST_OK, tv(CC_TAG_BOOL, 1));
            return;
          }
          case CC_OP_MAP_REPLACE: {  // replace :183-202
            auto it = s.m.find(k);
            if (it != s.m.end()) {
              if (it->second.timer) cancel(it->second.timer);
              uint64_t timer = 0;
              if (ttl > 0) { Timer t; t.res = in.res; t.kind = T_MAP_REPLACE_TTL; t.key = k; t.commit_index = c.index; timer = schedule((uint64_t)ttl, t); }
              TV prev = it->second.value;
              it->second.value = a; it->second.commit_index = c.index; it->second.timer = timer;
              ret(CC_ST_OK, prev);
            } else {
              ret(CC_ST_OK, TV());
            }
            return;
          }
          case CC_OP_MAP_REPLACEIFPRESENT: {  // replaceIfPresent :207-228 (stores `value`=a, compares `replace`=b, A1)
            auto it = s.m.find(k);
            if (it == s.m.end()) { ret(CC_ST_OK, tv(CC_TAG_BOOL, 0)); return; }
            const TV& cur = it->second.value;
            bool ok = (tv_null(cur) && tv_null(b)) || (!tv_null(cur) && tv_equals(cur, b));
            if (ok) {
              if (it->second.timer) cancel(it->second.timer);
              uint64_t timer = 0;
              if (ttl > 0) { Timer t; t.res = in.res; t.kind = T_MAP_TTL; t.key = k; t.commit_index = c.index; timer = schedule((uint64_t)ttl, t); }
              it->second.value = a; it->second.commit_index = c.index; it->second.timer = timer;
              ret(CC_ST_OK, tv(CC_TAG_BOOL, 1));
            } else {
              ret(CC_ST_OK, tv(CC_TAG_BOOL, 0));
            }
            return;
          }
          case CC_OP_MAP_ISEMPTY:  // isEmpty :244-250
            ret(CC_ST_OK, tv(CC_TAG_BOOL, s.m.empty() ? 1 : 0));
            return;
          case CC_OP_MAP_SIZE:  // size :233-239 (int)
            ret(CC_ST_OK, tv(CC_TAG_INT, (uint64_t)(int64_t)(int32_t)s.m.size()));
            return;
          case CC_OP_MAP_CLEAR:  // clear :255-261 -> delete()
            sm_delete(in.res);
            ret(CC_ST_OK, TV());
            return;
        }
        break;
      }
      case CC_RES_QUEUE: {  // QueueState (collections/src/main/java/io/atomix/collections/state/QueueState.java)
        auto& q = r.q;
        auto first_match = [&](size_t& at) -> int {  // 1 match, 0 none, -1 NPE (a stored null's equals)
          for (size_t i = 0; i < q.size(); ++i) {
            if (tv_null(q[i].v)) return -1;
            if (tv_equals(q[i].v, a)) { at = i; return 1; }
          }
          return 0;
        };
        switch (c.op) {
          case CC_OP_QUEUE_CONTAINS: {  // contains :36-46
            size_t at = 0;
            int m = first_match(at);
            if (m < 0) ret(CC_ST_NULL_POINTER, TV());
            else ret(CC_ST_OK, tv(CC_TAG_BOOL, m ? 1 : 0));
            return;
          }
          case CC_OP_QUEUE_ADD:    // add :51-59 (returns false)
          case CC_OP_QUEUE_OFFER:  // offer :64-72 (returns false)
            q.push_back(Resource::QEnt{a, c.index, false});
            ret(CC_ST_OK, tv(CC_TAG_BOOL, 0));
            return;
          case CC_OP_QUEUE_PEEK:  // peek :77-87
            ret(CC_ST_OK, q.empty() ? TV() : q.front().v);
            return;
          case CC_OP_QUEUE_POLL:  // poll :92-105
            if (q.empty()) { ret(CC_ST_OK, TV()); return; }
            ret(CC_ST_OK, q.front().v);
            q.pop_front();
            return;
          case CC_OP_QUEUE_ELEMENT:  // element :111-124 — ArrayDeque.element throws when empty; does not remove
            if (q.empty()) { ret(CC_ST_NO_SUCH_ELEMENT, TV()); return; }
            ret(CC_ST_OK, q.front().v);
            q.front().cleaned = true;  // value.clean() on the head it leaves in place
            return;
          case CC_OP_QUEUE_REMOVE: {  // remove :130-157
            if (!tv_null(a)) {
              size_t at = 0;
              int m = first_match(at);
              if (m < 0) { ret(CC_ST_NULL_POINTER, TV()); return; }
              if (m) q.erase(q.begin() + (std::ptrdiff_t)at);
              ret(CC_ST_OK, tv(CC_TAG_BOOL, m ? 1 : 0));
              return;
            }
            if (q.empty()) { ret(CC_ST_NO_SUCH_ELEMENT, TV()); return; }  // ArrayDeque.remove()
            ret(CC_ST_OK, q.front().v);
            q.pop_front();
            return;
          }
          case CC_OP_QUEUE_SIZE:  // size :162-168 (int)
            ret(CC_ST_OK, tv(CC_TAG_INT, (uint64_t)(int64_t)(int32_t)q.size()));
            return;
          case CC_OP_QUEUE_ISEMPTY:  // isEmpty :173-179
            ret(CC_ST_OK, tv(CC_TAG_BOOL, q.empty() ? 1 : 0));
            return;
          case CC_OP_QUEUE_CLEAR:  // clear :184-190 -> delete()
            q.clear();
            ret(CC_ST_OK, TV());
            return;
        }
        break;
      }
      case CC_RES_SET: {  // SetState (collections/src/main/java/io/atomix/collections/state/SetState.java)
        MapSM& s = r.m;  // element -> Value{commit, timer}; the stored value is a Boolean TRUE marker
        MapKey k{ktag_to_tag(CC_FLAG_KTAG(c.flags)), c.key};
        int64_t ttl = (int64_t)c.aux;
        switch (c.op) {
          case CC_OP_SET_CONTAINS:  // contains :38-44
            ret(CC_ST_OK, tv(CC_TAG_BOOL, s.m.count(k) ? 1 : 0));
            return;
          case CC_OP_SET_ADD: {  // add :49-66 — returns false whether or not the element was added
            if (!s.m.count(k)) {
              uint64_t timer = 0;
              if (ttl > 0) { Timer t; t.res = in.res; t.kind = T_MAP_TTL; t.key = k; t.commit_index = c.index; timer = schedule((uint64_t)ttl, t); }
              MapEntry e; e.value = tv(CC_TAG_BOOL, 1); e.commit_index = c.index; e.timer = timer; s.order.put_new(cx, k);
              s.m.emplace(k, e);
            }
            ret(CC_ST_OK, tv(CC_TAG_BOOL, 0));
            return;
          }
          case CC_OP_SET_REMOVE: {  // remove :70-87
            auto it = s.m.find(k);
            if (it == s.m.end()) { ret(CC_ST_OK, tv(CC_TAG_BOOL, 0)); return; }
            if (it->second.timer) cancel(it->second.timer);
            s.m.erase(it); s.order.remove(cx, k);
            ret(CC_ST_OK, tv(CC_TAG_BOOL, 1));
            return;
          }
          case CC_OP_SET_SIZE:  // size :92-98 (int)
            ret(CC_ST_OK, tv(CC_TAG_INT, (uint64_t)(int64_t)(int32_t)s.m.size()));
            return;
          case CC_OP_SET_ISEMPTY:  // isEmpty :103-109
            ret(CC_ST_OK, tv(CC_TAG_BOOL, s.m.empty() ? 1 : 0));
            return;
          case CC_OP_SET_CLEAR:  // clear :114-120 -> delete()
            sm_delete(in.res);
            ret(CC_ST_OK, TV());
            return;
        }
        break;
      }
      case CC_RES_MULTIMAP: {  // MultiMapState (collections/src/main/java/io/atomix/collections/state/MultiMapState.java)
        // map: key -> LinkedHashMap<value, commit>; put registers the key's map but never stores the value into it
        // (:70-82), so every value map stays empty and the state is the set of keys (A18).  Entries of r.m are those
        // keys (value Boolean TRUE as a marker).
        MapSM& s = r.m;
        MapKey k{ktag_to_tag(CC_FLAG_KTAG(c.flags)), c.key};
        switch (c.op) {
          case CC_OP_MMAP_CONTAINSKEY:  // containsKey :37-43
            ret(CC_ST_OK, tv(CC_TAG_BOOL, s.m.count(k) ? 1 : 0));
            return;
          case CC_OP_MMAP_GET:  // get :48-63 — the key's (empty) value map -> an empty collection
            ret(CC_ST_OK, tv(CC_TAG_LIST, 0));
            return;
          case CC_OP_MMAP_PUT: {  // put :68-91 — !values.containsKey(value) always holds: true, commit never cleaned;
            // a ttl > 0 schedules keyValues.remove(value).clean(), which throws (remove returns null) and changes
            // nothing (A18)
            if (!s.m.count(k)) {
              MapEntry e; e.value = tv(CC_TAG_BOOL, 1); e.commit_index = c.index; s.order.put_new(cx, k);
              s.m.emplace(k, e);
            }
            r.leaked.push_back(c.index);
            ret(CC_ST_OK, tv(CC_TAG_BOOL, 1));
            return;
          }
          case CC_OP_MMAP_REMOVE:  // remove :96-135
            if (!tv_null(a)) {  // values.remove(value) finds nothing: false, the key stays
              ret(CC_ST_OK, tv(CC_TAG_BOOL, 0));
              return;
            }
            if (s.m.erase(k)) s.order.remove(cx, k);  // map.remove(key): its (empty) values as a collection
            ret(CC_ST_OK, tv(CC_TAG_LIST, 0));
            return;
          case CC_OP_MMAP_REMOVEVALUE:  // removeValue :140-165 — no entry matches; every (empty) value map goes
          case CC_OP_MMAP_CLEAR:        // clear :201-207 -> delete()
            sm_delete(in.res);
            ret(CC_ST_OK, TV());
            return;
          case CC_OP_MMAP_SIZE:  // size :170-185 — sums of empty value maps
            ret(CC_ST_OK, tv(CC_TAG_INT, 0));
            return;
          case CC_OP_MMAP_ISEMPTY:  // isEmpty :190-196 — keys with empty value maps still count
            ret(CC_ST_OK, tv(CC_TAG_BOOL, s.m.empty() ? 1 : 0));
            return;
        }
        break;  // ContainsEntry / ContainsValue: no handler
      }
      case CC_RES_LOCK: {
        LockSM& s = r.l;
        switch (c.op) {
          case CC_OP_LOCK_LOCK: {  // LockState.lock :41-61 (timeout: -1 forever, 0 try, >0 ms)
            int64_t timeout = (int64_t)c.aux;
            if (!s.held) {
              s.held = true;
              s.lock = Commit{c.index, c.inst, false};
              publish(c.inst, CC_EV_LOCK, tv(CC_TAG_BOOL, 1));
            } else if (timeout == 0) {
              publish(c.inst, CC_EV_LOCK, tv(CC_TAG_BOOL, 0));
            } else {
              s.queue.push_back(Commit{c.index, c.inst, false});
              if (timeout > 0) {
                Timer t; t.res = in.res; t.kind = T_LOCK_TIMEOUT; t.commit_index = c.index;
                s.timers[c.index] = schedule((uint64_t)timeout, t);
              }
            }
            ret(CC_ST_OK, TV());
            return;
          }
          case CC_OP_LOCK_UNLOCK: {  // LockState.unlock :66-85
            if (s.held) {
              if (s.lock.inst != c.inst) { ret(CC_ST_ILLEGAL_STATE, TV()); return; }  // "not the lock holder"
              if (s.lock.cleaned) { ret(CC_ST_ILLEGAL_STATE, TV()); return; }        // "commit closed" (after delete)
              if (s.queue.empty()) {
                s.held = false;
              } else {
                s.lock = s.queue.front();
                s.queue.pop_front();
                auto t = s.timers.find(s.lock.index);
                if (t != s.timers.end()) { cancel(t->second); s.timers.erase(t); }
                publish(s.lock.inst, CC_EV_LOCK, tv(CC_TAG_BOOL, 1));
              }
            }
            ret(CC_ST_OK, TV());
            return;
          }
        }
        break;
      }
      case CC_RES_ELECTION: {
        ElectionSM& s = r.e;
        switch (c.op) {
          case CC_OP_ELECT_LISTEN: {  // listen :57-66
            if (!s.has_leader) {
              s.has_leader = true;
              s.leader = Commit{c.index, c.inst, false};
              publish(c.inst, CC_EV_ELECT, tv(CC_TAG_LONG, c.index));
            } else {
              bool found = false;
              for (auto& p : s.listeners) if (p.first == in.id) { found = true; break; }
              if (!found) s.listeners.emplace_back(in.id, Commit{c.index, c.inst, false});  // may be the leader's own session (A9)
            }
            ret(CC_ST_OK, TV());
            return;
          }
          case CC_OP_ELECT_UNLISTEN: {  // unlisten :71-91
            if (s.has_leader && s.leader.inst == c.inst) {
              if (s.leader.cleaned) { ret(CC_ST_ILLEGAL_STATE, TV()); return; }  // "commit closed"
              s.has_leader = false;
              if (!s.listeners.empty()) {
                s.leader = s.listeners.front().second;
                s.has_leader = true;
                s.listeners.erase(s.listeners.begin());
                publish(s.leader.inst, CC_EV_ELECT, tv(CC_TAG_LONG, s.leader.index));
              }
            } else {
              for (auto it = s.listeners.begin(); it != s.listeners.end(); ++it)
                if (it->first == in.id) { s.listeners.erase(it); break; }
            }
            ret(CC_ST_OK, TV());
            return;
          }
          case CC_OP_ELECT_ISLEADER: {  // isLeader :96-98 — epoch is not serialized, so 0 (A3)
            bool r2 = s.has_leader && s.leader.inst == c.inst && s.leader.index == 0;
            ret(CC_ST_OK, tv(CC_TAG_BOOL, r2 ? 1 : 0));
            return;
          }
        }
        break;
      }
      case CC_RES_GROUP: {
        GroupSM& s = r.g;
        switch (c.op) {
          case CC_OP_GROUP_JOIN: {  // join :47-64
            uint64_t sid = in.id;
            auto it = s.members.find(sid);
            if (it != s.members.end()) {
              it->second = Commit{c.index, c.inst, false};  // previous.clean()
            } else {
              s.members.emplace(sid, Commit{c.index, c.inst, false});
              for (auto& kv : s.members)
                if (kv.second.index != c.index) publish(kv.second.inst, CC_EV_JOIN, tv(CC_TAG_LONG, sid));
            }
            std::vector<uint64_t> ids;
            ids.reserve(s.members.size());
            for (auto& kv : s.members) ids.push_back(kv.first);
            std::sort(ids.begin(), ids.end());
            for (uint64_t id : ids) aux.emplace_back(cur_pos, id);
            ret(CC_ST_OK, tv(CC_TAG_SET, ids.size()));
            return;
          }
          case CC_OP_GROUP_LEAVE: {  // leave :69-81
            uint64_t sid = in.id;
            auto it = s.members.find(sid);
            if (it != s.members.end()) {
              s.members.erase(it);
              for (auto& kv : s.members) publish(kv.second.inst, CC_EV_LEAVE, tv(CC_TAG_LONG, sid));
            }
            ret(CC_ST_OK, TV());
            return;
          }
          case CC_OP_GROUP_SCHEDULE: {  // schedule :86-103 (member = key, callback = a, delay = aux)
            if (!s.members.count(c.key)) { ret(CC_ST_ILLEGAL_ARGUMENT, TV()); return; }
            Timer t; t.res = in.res; t.kind = T_GROUP_SCHEDULE; t.member = c.key; t.callback = a; t.commit_index = c.index;
            int64_t delay = (int64_t)c.aux;
            schedule(delay > 0 ? (uint64_t)delay : 0, t);
            ret(CC_ST_OK, TV());
            return;
          }
          case CC_OP_GROUP_EXECUTE: {  // execute :108-119
            auto it = s.members.find(c.key);
            if (it == s.members.end()) { ret(CC_ST_ILLEGAL_ARGUMENT, TV()); return; }
            publish(it->second.inst, CC_EV_EXECUTE, a);
            ret(CC_ST_OK, TV());
            return;
          }
        }
        break;
      }
    }
    // ResourceStateMachineExecutor.executeCommand :78 / ResourceManagerStateMachineExecutor.execute :96
    ret(CC_ST_UNKNOWN_OP, TV());
  }

  // AtomicValueState.change :68-72 (HashMap<Session> order is identity-hash based: compare per target)
  void value_change(ValueSM& s) {
    for (auto& p : s.listeners) publish(p.first, CC_EV_CHANGE, s.value);
  }
};

extern "C" {

orc* orc_create(uint32_t max_resources, uint32_t max_instances, uint32_t flags) {
  orc* o = new orc();
  o->max_res = max_resources;
  o->max_inst = max_instances;
  o->flags = flags;
  o->res.resize(max_resources);
  o->inst.resize(max_instances);
  return o;
}
void orc_destroy(orc* o) { delete o; }

int orc_resource_create(orc* o, uint32_t slot, uint32_t type) {
  if (!o || slot >= o->max_res || type < CC_RES_VALUE || type > CC_RES_MULTIMAP || o->res[slot].exists || o->res[slot].zombie)
    return CC_ERR_INVALID;
  o->init_resource(slot, type, slot);
  return CC_OK;
}

int orc_resource_delete(orc* o, uint32_t slot) {
  if (!o || slot >= o->max_res || !o->res[slot].exists) return CC_ERR_INVALID;
  uint8_t st;
  uint64_t id = o->res[slot].id;
  return orc_delete_resource(o, id, &st) == CC_OK && CC_STATUS_CODE(st) == CC_ST_OK ? CC_OK : CC_ERR_INVALID;
}

int orc_instance_open(orc* o, uint32_t inst, uint32_t res, uint64_t instance_id, uint64_t client_session) {
  if (!o || inst >= o->max_inst || res >= o->max_res || !o->res[res].exists || o->inst[inst].open) return CC_ERR_INVALID;
  if (o->inst_by_id.count(instance_id)) return CC_ERR_INVALID;
  o->register_instance(inst, res, instance_id, client_session);
  return CC_OK;
}

// ResourceManager.getResource :77-143
int orc_get_resource(orc* o, uint64_t key, uint32_t type, uint64_t client, uint64_t index, uint64_t* instance_id,
                     uint32_t* inst_slot, uint8_t* status) {
  *status = CC_STATUS(CC_ST_OK, CC_TAG_LONG);
  auto kit = o->keys.find(key);
  if (kit == o->keys.end()) {
    int rs = o->alloc_res_slot(), is = o->alloc_inst_slot();
    if (rs < 0 || is < 0) return CC_ERR_CAPACITY;
    uint64_t rid = index;  // resource id = index of the creating commit (:87)
    o->keys[key] = rid;
    o->init_resource((uint32_t)rs, type, rid);
    o->res[rs].key = key; o->res[rs].has_key = true;
    o->register_instance((uint32_t)is, (uint32_t)rs, index, client);  // instance id = commit index (:103)
    o->res[rs].sessions[client] = index;
    *instance_id = index; *inst_slot = (uint32_t)is;
    return CC_OK;
  }
  auto rit = o->res_by_id.find(kit->second);
  if (rit == o->res_by_id.end() || o->res[rit->second].type != type) {  // :119-121
    *status = CC_STATUS(CC_ST_TYPE_MISMATCH, CC_TAG_NULL);
    return CC_OK;
  }
  Resource& r = o->res[rit->second];
  auto hit = r.sessions.find(client);
  if (hit == r.sessions.end()) {  // :126-136
    int is = o->alloc_inst_slot();
    if (is < 0) return CC_ERR_CAPACITY;
    o->register_instance((uint32_t)is, rit->second, index, client);
    r.sessions[client] = index;
    *instance_id = index; *inst_slot = (uint32_t)is;
  } else {  // :137-141
    *instance_id = hit->second;
    *inst_slot = o->inst_by_id[hit->second];
  }
  return CC_OK;
}

// ResourceManager.createResource :148-196 (a new instance every time, not added to resource.sessions)
int orc_create_resource(orc* o, uint64_t key, uint32_t type, uint64_t client, uint64_t index, uint64_t* instance_id,
                        uint32_t* inst_slot, uint8_t* status) {
  *status = CC_STATUS(CC_ST_OK, CC_TAG_LONG);
  uint32_t rslot;
  auto kit = o->keys.find(key);
  if (kit == o->keys.end()) {
    int rs = o->alloc_res_slot();
    if (rs < 0) return CC_ERR_CAPACITY;
    o->keys[key] = index;
    o->init_resource((uint32_t)rs, type, index);
    o->res[rs].key = key; o->res[rs].has_key = true;
    rslot = (uint32_t)rs;
  } else {
    auto rit = o->res_by_id.find(kit->second);
    if (rit == o->res_by_id.end() || o->res[rit->second].type != type) {
      *status = CC_STATUS(CC_ST_TYPE_MISMATCH, CC_TAG_NULL);
      return CC_OK;
    }
    rslot = rit->second;
  }
  int is = o->alloc_inst_slot();
  if (is < 0) return CC_ERR_CAPACITY;
  o->register_instance((uint32_t)is, rslot, index, client);
  *instance_id = index; *inst_slot = (uint32_t)is;
  return CC_OK;
}

// ResourceManager.deleteResource :212-235 (looked up as a RESOURCE id although clients send the instance id, A13)
int orc_delete_resource(orc* o, uint64_t resource_id, uint8_t* status) {
  auto rit = o->res_by_id.find(resource_id);
  if (rit == o->res_by_id.end()) { *status = CC_STATUS(CC_ST_UNKNOWN_RESOURCE, CC_TAG_NULL); return CC_OK; }
  uint32_t slot = rit->second;
  o->res_by_id.erase(rit);
  Resource& r = o->res[slot];
  uint8_t st = o->sm_delete(slot);   // resource.stateMachine.delete()
  if (CC_STATUS_CODE(st) != CC_ST_OK) {
    // delete() threw after resources.remove(): keys, timers and instance holders are left behind; a later
    // commit on such an instance hits `resources.get(...) == null` -> NullPointerException (:62,71).
    r.exists = false;
    r.zombie = true;
    *status = st;
    return CC_OK;
  }
  o->cancel_resource_timers(slot);   // resource.executor.close()
  if (r.has_key) o->keys.erase(r.key);
  // :223-229: every holder of the resource, iterator.remove()d in sessions' HashMap iteration order
  std::vector<uint32_t> gone;
  o->sessions_order.for_each([&](const MapKey& id) {
    const uint32_t i = o->inst_by_id.at(id.k);
    if (o->inst[i].open && o->inst[i].res == slot) gone.push_back(i);
  });
  for (uint32_t i : gone) o->unregister_instance(i);
  r.exists = false;
  *status = CC_STATUS_CODE(st) == CC_ST_OK ? CC_STATUS(CC_ST_OK, CC_TAG_BOOL) : st;
  return CC_OK;
}

int orc_resource_exists(orc* o, uint64_t key) { return o->keys.count(key) ? 1 : 0; }  // :201-207
int orc_inst_slot_of(orc* o, uint64_t id) { auto it = o->inst_by_id.find(id); return it == o->inst_by_id.end() ? -1 : (int)it->second; }
int orc_res_slot_of(orc* o, uint64_t id) { auto it = o->res_by_id.find(id); return it == o->res_by_id.end() ? -1 : (int)it->second; }

int orc_apply(orc* o, const cc_batch* cols, uint64_t n, uint8_t* status, uint64_t* value) {
  if (!o || !cols || !cols->inst || !cols->op) return CC_ERR_INVALID;
  const bool deferred = (o->flags & ORC_TIMERS_DEFERRED) != 0;
  for (uint64_t i = 0; i < n; ++i) {
    orc::Row r;
    r.index = cols->index ? cols->index[i] : 0;
    r.time = cols->time ? cols->time[i] : 0;
    r.inst = cols->inst[i];
    r.op = cols->op[i];
    r.flags = cols->flags ? cols->flags[i] : 0;
    r.key = cols->key ? cols->key[i] : 0;
    r.a = cols->a ? cols->a[i] : 0;
    r.b = cols->b ? cols->b[i] : 0;
    r.aux = cols->aux ? cols->aux[i] : 0;
    o->cur_pos = (uint32_t)i;
    if (r.time > o->clock) o->clock = r.time;
    if (!deferred && !o->timers.empty()) o->fire_due();
    o->cur_src = CC_EVSRC_COMMIT;
    o->apply_one(r, status[i], value[i]);
    if (deferred && !o->timers.empty()) o->fire_due();
    if (r.index > o->applied) o->applied = r.index;
  }
  return CC_OK;
}

// A HANDLE key's String (UTF-16 units): its java hashCode and compareTo (java.util.HashMap bins and tree bins).
int orc_handle_string(orc* o, uint64_t handle, const uint16_t* units, uint64_t n) {
  o->cx.str[handle] = std::vector<uint16_t>(units, units + n);
  return CC_OK;
}

int orc_advance_time(orc* o, uint64_t now) {
  if (now > o->clock) o->clock = now;
  o->cur_pos = UINT32_MAX;
  o->fire_due();
  return CC_OK;
}

// ResourceManager.close :250-264 — iterates ResourceManager.sessions in HashMap order
int orc_session_close(orc* o, uint64_t client) {
  std::vector<std::pair<uint64_t, uint32_t>> ord;  // sessions.values() in HashMap iteration order
  o->sessions_order.for_each([&](const MapKey& id) {
    const uint32_t slot = o->inst_by_id.at(id.k);
    if (o->inst[slot].client == client) ord.emplace_back(ord.size(), slot);
  });
  uint8_t saved = o->cur_src;
  o->cur_src = CC_EVSRC_CLOSE;
  o->cur_pos = UINT32_MAX;
  for (auto& p : ord) {
    uint32_t islot = p.second;
    Inst& in = o->inst[islot];
    Resource& r = o->res[in.res];
    if (r.exists) {
      r.sessions.erase(in.client);
      if (!o->sm_close(islot)) break;  // an exception aborts the fan-out (unpinned)
    }
    o->unregister_instance(islot);
  }
  o->cur_src = saved;
  return CC_OK;
}

// ResourceManager.expire :238-247 calls StateMachine.expire, which none of the covered state machines
// override; Copycat then closes the session [not vendored] -> close fan-out.
int orc_session_expire(orc* o, uint64_t client) { return orc_session_close(o, client); }

uint64_t orc_applied_index(orc* o) { return o->applied; }

uint64_t orc_event_count(orc* o) { return o->events.size(); }
void orc_events_read(orc* o, uint32_t* pos, uint32_t* target, uint8_t* code, uint8_t* src, uint8_t* tag, uint64_t* payload) {
  for (size_t i = 0; i < o->events.size(); ++i) {
    const Event& e = o->events[i];
    pos[i] = e.pos; target[i] = e.target; code[i] = e.code; src[i] = e.src; tag[i] = e.tag; payload[i] = e.payload;
  }
}
void orc_events_clear(orc* o) { o->events.clear(); }
uint64_t orc_aux_count(orc* o) { return o->aux.size(); }
void orc_aux_read(orc* o, uint32_t* pos, uint64_t* member) {
  for (size_t i = 0; i < o->aux.size(); ++i) { pos[i] = o->aux[i].first; member[i] = o->aux[i].second; }
}
void orc_aux_clear(orc* o) { o->aux.clear(); }

int orc_read_value_state(orc* o, uint32_t first, uint32_t count, uint8_t* tag, uint64_t* value, uint8_t* has_current) {
  if ((uint64_t)first + count > o->max_res) return CC_ERR_INVALID;
  for (uint32_t i = 0; i < count; ++i) {
    const Resource& r = o->res[first + i];
    bool live = r.exists && r.type == CC_RES_VALUE;
    tag[i] = live ? r.v.value.tag : 0;
    value[i] = live ? r.v.value.v : 0;
    has_current[i] = live && r.v.has_current ? 1 : 0;
  }
  return CC_OK;
}

// retained value commit (AtomicValueState.current, never clean()ed: :88-157), 0 if none
int orc_read_value_retained(orc* o, uint32_t first, uint32_t count, uint64_t* index) {
  if ((uint64_t)first + count > o->max_res) return CC_ERR_INVALID;
  for (uint32_t i = 0; i < count; ++i) {
    const Resource& r = o->res[first + i];
    index[i] = r.exists && r.type == CC_RES_VALUE && r.v.has_current ? r.v.current.index : 0;
  }
  return CC_OK;
}

// Every commit the resource's state machine holds without having clean()ed it (the log cannot compact them), as
// ascending log indices; -1: no resource in the slot.  AtomicValueState current :88-109 + listeners :41-63 (+ re-put
// leaks); MapState / SetState entries' commits; LockState holder (unless delete() cleaned it) + waiters :41-98;
// LeaderElectionState leader + listeners :35-108; MembershipGroupState members + close leaks :36-42 + pending
// schedule commits :86-103; QueueState elements not clean()ed by element() :51-199.
int64_t orc_read_retained(orc* o, uint32_t slot, uint64_t cap, uint64_t* out) {
  if (slot >= o->max_res || !o->res[slot].exists) return -1;
  const Resource& r = o->res[slot];
  std::vector<uint64_t> v(r.leaked.begin(), r.leaked.end());
  switch (r.type) {
    case CC_RES_VALUE:
      if (r.v.has_current) v.push_back(r.v.current.index);
      for (auto& p : r.v.listeners) v.push_back(p.second);
      break;
    case CC_RES_MAP:
    case CC_RES_SET:
      for (auto& kv : r.m.m) v.push_back(kv.second.commit_index);
      break;
    case CC_RES_LOCK:
      if (r.l.held && !r.l.lock.cleaned) v.push_back(r.l.lock.index);
      for (auto& c : r.l.queue) v.push_back(c.index);
      break;
    case CC_RES_ELECTION:
      if (r.e.has_leader && !r.e.leader.cleaned) v.push_back(r.e.leader.index);
      for (auto& p : r.e.listeners) v.push_back(p.second.index);
      break;
    case CC_RES_GROUP:
      for (auto& kv : r.g.members) v.push_back(kv.second.index);
      for (auto& kv : o->timers)
        if (kv.second.res == slot && kv.second.kind == T_GROUP_SCHEDULE) v.push_back(kv.second.commit_index);
      break;
    case CC_RES_QUEUE:
      for (auto& e : r.q) if (!e.cleaned) v.push_back(e.idx);
      break;
    case CC_RES_MULTIMAP:  // every Put (in `leaked`)
      break;
  }
  std::sort(v.begin(), v.end());
  for (uint64_t i = 0; i < v.size() && i < cap; ++i) out[i] = v[i];
  return (int64_t)v.size();
}

int64_t orc_map_size(orc* o, uint32_t res) {
  if (res >= o->max_res || !o->res[res].exists || (o->res[res].type != CC_RES_MAP && o->res[res].type != CC_RES_SET && o->res[res].type != CC_RES_MULTIMAP)) return -1;
  return (int64_t)o->res[res].m.m.size();
}

int64_t orc_map_entries(orc* o, uint32_t res, uint64_t cap, uint8_t* ktag, uint64_t* key, uint8_t* vtag, uint64_t* val,
                        uint64_t* commit_index) {
  if (res >= o->max_res || !o->res[res].exists || (o->res[res].type != CC_RES_MAP && o->res[res].type != CC_RES_SET && o->res[res].type != CC_RES_MULTIMAP)) return -1;
  std::vector<std::pair<MapKey, MapEntry>> v(o->res[res].m.m.begin(), o->res[res].m.m.end());
  std::sort(v.begin(), v.end(), [](const std::pair<MapKey, MapEntry>& x, const std::pair<MapKey, MapEntry>& y) {
    return x.first.tag != y.first.tag ? x.first.tag < y.first.tag : x.first.k < y.first.k;
  });
  uint64_t n = std::min<uint64_t>(cap, v.size());
  for (uint64_t i = 0; i < n; ++i) {
    ktag[i] = v[i].first.tag; key[i] = v[i].first.k; vtag[i] = v[i].second.value.tag; val[i] = v[i].second.value.v;
    if (commit_index) commit_index[i] = v[i].second.commit_index;
  }
  return (int64_t)n;
}

int64_t orc_lock_state(orc* o, uint32_t res, int64_t* holder, uint64_t* holder_index, uint8_t* holder_cleaned, uint64_t cap,
                       uint32_t* queue_inst, uint64_t* queue_index) {
  if (res >= o->max_res || !o->res[res].exists || o->res[res].type != CC_RES_LOCK) return -1;
  const LockSM& l = o->res[res].l;
  *holder = l.held ? (int64_t)l.lock.inst : -1;
  *holder_index = l.held ? l.lock.index : 0;
  *holder_cleaned = l.held && l.lock.cleaned ? 1 : 0;
  uint64_t n = std::min<uint64_t>(cap, l.queue.size());
  for (uint64_t i = 0; i < n; ++i) { queue_inst[i] = l.queue[i].inst; queue_index[i] = l.queue[i].index; }
  return (int64_t)l.queue.size();
}

int64_t orc_election_state(orc* o, uint32_t res, int64_t* leader, uint64_t* leader_index, uint64_t cap,
                           uint32_t* listener_inst, uint64_t* listener_index) {
  if (res >= o->max_res || !o->res[res].exists || o->res[res].type != CC_RES_ELECTION) return -1;
  const ElectionSM& e = o->res[res].e;
  *leader = e.has_leader ? (int64_t)e.leader.inst : -1;
  *leader_index = e.has_leader ? e.leader.index : 0;
  uint64_t n = std::min<uint64_t>(cap, e.listeners.size());
  for (uint64_t i = 0; i < n; ++i) { listener_inst[i] = e.listeners[i].second.inst; listener_index[i] = e.listeners[i].second.index; }
  return (int64_t)e.listeners.size();
}

int64_t orc_group_members(orc* o, uint32_t res, uint64_t cap, uint64_t* ids) {
  if (res >= o->max_res || !o->res[res].exists || o->res[res].type != CC_RES_GROUP) return -1;
  std::vector<uint64_t> v;
  for (auto& kv : o->res[res].g.members) v.push_back(kv.first);
  std::sort(v.begin(), v.end());
  uint64_t n = std::min<uint64_t>(cap, v.size());
  for (uint64_t i = 0; i < n; ++i) ids[i] = v[i];
  return (int64_t)v.size();
}

uint64_t orc_pending_timers(orc* o) { return o->timers.size(); }

// a14 — leader commit index: the quorum-th largest match index, gated by the current-term start and
// monotonicity (Raft §5.3/§5.4.2; Copycat's LeaderState is not vendored: rule defined by this build).
void orc_quorum_commit(const uint64_t* match, uint32_t replicas, uint64_t groups, const uint64_t* term_start,
                       const uint64_t* commit_in, uint64_t* commit_out) {
  const uint32_t quorum = replicas / 2 + 1;
  std::vector<uint64_t> m(replicas);
  for (uint64_t g = 0; g < groups; ++g) {
    for (uint32_t r = 0; r < replicas; ++r) m[r] = match[(uint64_t)r * groups + g];
    std::sort(m.begin(), m.end(), [](uint64_t x, uint64_t y) { return x > y; });
    uint64_t n = m[quorum - 1];
    commit_out[g] = (n >= term_start[g] && n > commit_in[g]) ? n : commit_in[g];
  }
}

// a15 — expired iff now - last > timeout (signed difference)
void orc_expire_sweep(const uint64_t* last, uint64_t sessions, uint64_t now, uint64_t timeout, uint64_t* bitmap,
                      uint64_t* count) {
  uint64_t words = (sessions + 63) / 64, c = 0;
  for (uint64_t w = 0; w < words; ++w) bitmap[w] = 0;
  for (uint64_t s = 0; s < sessions; ++s) {
    int64_t d = (int64_t)(now - last[s]);
    if (d > (int64_t)timeout) { bitmap[s / 64] |= 1ull << (s % 64); ++c; }
  }
  *count += c;
}

}  // extern "C"
