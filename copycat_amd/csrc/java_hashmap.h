// java_hashmap.h — java.util.HashMap<Long, V> (JDK 8) as a host-side structure: the iteration order of
// ResourceManager.sessions (manager/src/main/java/io/atomix/manager/ResourceManager.java:37, a HashMap<Long,
// SessionHolder>), which orders the close / expire fan-out (ResourceManager.close :250-264, expire :238-247).  Host
// code only (the control plane).
//
// java.util.HashMap is a JDK class, not part of /root/reference; this restates the published JDK 8 algorithm for Long
// keys: hash = h ^ (h >>> 16) with h = (int)(v ^ (v >>> 32)); a new key is appended to its bin's chain, and a chain
// that reaches 9 nodes calls treeifyBin -- a resize below capacity 64, else a red-black tree bin whose root is moved to
// the chain's front (new keys then link after their tree parent); ++size > threshold resizes (16 at the first put,
// then doubling; chains and trees split in order, trees untreeify at <= 6 nodes); removeNode unlinks, untreeifies a
// tree that became too small or runs the red-black delete.  Tree order: the spread hash as a signed int, then
// Long.compareTo.  Iteration: bins in index order, each bin's `next` chain.
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <unordered_map>
#include <vector>

namespace cc {

class JavaLongHashMap {
 public:
  static constexpr int kNil = -1;
  struct Node {  // no implicit padding: snapshots of equal states are equal byte for byte
    uint32_t hash;
    uint32_t pad0;
    int64_t key;
    int32_t next, prev, parent, left, right;
    uint8_t tree, red, pad[2];
  };
  static_assert(sizeof(Node) == 40, "Node must have no implicit padding");

  static uint32_t spread(int64_t v) {
    const uint32_t h = (uint32_t)((uint64_t)v ^ ((uint64_t)v >> 32));
    return h ^ (h >> 16);
  }
  uint32_t size() const { return size_; }
  uint32_t capacity() const { return (uint32_t)tab_.size(); }
  bool contains(int64_t k) const { return where_.count(k) != 0; }

  void put(int64_t k) {  // HashMap.put of a key (an existing key changes no structure)
    if (where_.count(k)) return;
    const uint32_t h = spread(k);
    if (tab_.empty()) resize();
    const uint32_t i = (capacity() - 1) & h;
    int p = tab_[i];
    if (p == kNil) {
      tab_[i] = where_[k] = alloc(h, k);
    } else if (nd_[p].tree) {  // putTreeVal: linked after its tree parent, root to the front
      const int root = root_of(p);
      for (int q = root;;) {
        const int dir = dir_of(h, k, nd_[q]);
        const int xp = q;
        if ((q = dir <= 0 ? nd_[q].left : nd_[q].right) == kNil) {
          const int xpn = nd_[xp].next, x = alloc(h, k);
          where_[k] = x;
          nd_[x].tree = 1;
          nd_[x].next = xpn;
          (dir <= 0 ? nd_[xp].left : nd_[xp].right) = x;
          nd_[xp].next = x;
          nd_[x].parent = nd_[x].prev = xp;
          if (xpn != kNil) nd_[xpn].prev = x;
          to_front(balance_insertion(root, x));
          break;
        }
      }
    } else {
      int bin = 0;
      while (nd_[p].next != kNil) p = nd_[p].next, ++bin;
      const int x = alloc(h, k);
      where_[k] = x;
      nd_[p].next = x;
      if (bin >= 7) treeify_bin(h);  // the chain now holds >= 9 nodes (TREEIFY_THRESHOLD - 1)
    }
    if (++size_ > threshold_) resize();
  }

  // removeNode(hash, key, null, false, movable).  ResourceManager only ever removes through its entry-set iterator
  // (deleteResource :223-229, close :251-263), and HashIterator.remove calls removeNode(..., movable = false): a tree
  // bin then loses the node from its chain and its red-black links, but is neither untreeified when small nor has its
  // root moved to the front.
  void remove(int64_t k, bool movable) {
    auto it = where_.find(k);
    if (it == where_.end()) return;
    const int node = it->second;
    where_.erase(it);
    const uint32_t index = (capacity() - 1) & nd_[node].hash;
    if (nd_[node].tree) {
      remove_tree_node(node, index, movable);
    } else {
      int p = tab_[index];
      if (p == node) tab_[index] = nd_[node].next;
      else {
        while (nd_[p].next != node) p = nd_[p].next;
        nd_[p].next = nd_[node].next;
      }
    }
    --size_;
    free_.push_back(node);
  }

  template <class F>
  void for_each(F f) const {  // values() / keySet() iteration order
    for (int b : tab_)
      for (int q = b; q != kNil; q = nd_[q].next) f(nd_[q].key);
  }

  // snapshot form: size, threshold, table, node pool (the lookup index is rebuilt)
  void save(std::vector<uint8_t>& out) const {
    auto put_u32 = [&](uint32_t x) { out.insert(out.end(), (const uint8_t*)&x, (const uint8_t*)&x + 4); };
    put_u32(size_);
    put_u32(threshold_);
    put_u32((uint32_t)tab_.size());
    put_u32((uint32_t)nd_.size());
    put_u32((uint32_t)free_.size());
    const uint8_t* t = (const uint8_t*)tab_.data();
    out.insert(out.end(), t, t + 4 * tab_.size());
    const uint8_t* n = (const uint8_t*)nd_.data();
    out.insert(out.end(), n, n + sizeof(Node) * nd_.size());
    const uint8_t* f = (const uint8_t*)free_.data();
    out.insert(out.end(), f, f + 4 * free_.size());
  }
  // returns the bytes consumed, 0 on a malformed blob
  size_t load(const uint8_t* p, size_t len) {
    if (len < 20) return 0;
    uint32_t hd[5];
    std::memcpy(hd, p, 20);
    const size_t need = 20 + 4ull * hd[2] + sizeof(Node) * (size_t)hd[3] + 4ull * hd[4];
    if (len < need) return 0;
    size_ = hd[0];
    threshold_ = hd[1];
    tab_.resize(hd[2]);
    nd_.resize(hd[3]);
    free_.resize(hd[4]);
    std::memcpy(tab_.data(), p + 20, 4ull * hd[2]);
    std::memcpy(nd_.data(), p + 20 + 4ull * hd[2], sizeof(Node) * (size_t)hd[3]);
    std::memcpy(free_.data(), p + 20 + 4ull * hd[2] + sizeof(Node) * hd[3], 4ull * hd[4]);
    // the blob is untrusted: every table slot and node link must name a node (or kNil), the table must be a power
    // of two, and no chain may be longer than the pool (a cycle would loop the rebuild below forever)
    const int64_t nn = (int64_t)nd_.size();
    auto ok = [nn](int32_t x) { return x == kNil || (x >= 0 && x < nn); };
    if (!tab_.empty() && (tab_.size() & (tab_.size() - 1))) return 0;
    for (int b : tab_)
      if (!ok(b)) return 0;
    for (const Node& q : nd_)
      if (!ok(q.next) || !ok(q.prev) || !ok(q.parent) || !ok(q.left) || !ok(q.right)) return 0;
    for (int f : free_)
      if (f < 0 || f >= nn) return 0;
    where_.clear();
    size_t walked = 0;
    for (int b : tab_)
      for (int q = b; q != kNil; q = nd_[q].next) {
        if (++walked > nd_.size()) return 0;
        where_[nd_[q].key] = q;
      }
    return where_.size() == size_ && walked == size_ ? need : 0;
  }

 private:
  std::vector<Node> nd_;
  std::vector<int> free_;
  std::vector<int> tab_;  // allocated at the first put
  uint32_t size_ = 0, threshold_ = 0;
  std::unordered_map<int64_t, int> where_;

  int alloc(uint32_t h, int64_t k) {
    int x;
    if (!free_.empty()) x = free_.back(), free_.pop_back();
    else x = (int)nd_.size(), nd_.emplace_back();
    nd_[x] = Node{h, 0, k, kNil, kNil, kNil, kNil, kNil, 0, 0, {0, 0}};
    return x;
  }
  static int dir_of(uint32_t h, int64_t k, const Node& p) {  // hash (signed), then Long.compareTo
    if ((int32_t)p.hash > (int32_t)h) return -1;
    if ((int32_t)p.hash < (int32_t)h) return 1;
    return k < p.key ? -1 : 1;  // distinct Longs never compare equal
  }
  int root_of(int p) const {
    while (nd_[p].parent != kNil) p = nd_[p].parent;
    return p;
  }
  int rotate_left(int root, int p) {
    int r, pp, rl;
    if (p != kNil && (r = nd_[p].right) != kNil) {
      if ((rl = nd_[p].right = nd_[r].left) != kNil) nd_[rl].parent = p;
      if ((pp = nd_[r].parent = nd_[p].parent) == kNil) root = r, nd_[r].red = 0;
      else if (nd_[pp].left == p) nd_[pp].left = r;
      else nd_[pp].right = r;
      nd_[r].left = p;
      nd_[p].parent = r;
    }
    return root;
  }
  int rotate_right(int root, int p) {
    int l, pp, lr;
    if (p != kNil && (l = nd_[p].left) != kNil) {
      if ((lr = nd_[p].left = nd_[l].right) != kNil) nd_[lr].parent = p;
      if ((pp = nd_[l].parent = nd_[p].parent) == kNil) root = l, nd_[l].red = 0;
      else if (nd_[pp].right == p) nd_[pp].right = l;
      else nd_[pp].left = l;
      nd_[l].right = p;
      nd_[p].parent = l;
    }
    return root;
  }
  bool red(int x) const { return x != kNil && nd_[x].red; }
  int balance_insertion(int root, int x) {
    nd_[x].red = 1;
    for (int xp, xpp, xppl, xppr;;) {
      if ((xp = nd_[x].parent) == kNil) {
        nd_[x].red = 0;
        return x;
      }
      if (!nd_[xp].red || (xpp = nd_[xp].parent) == kNil) return root;
      if (xp == (xppl = nd_[xpp].left)) {
        if ((xppr = nd_[xpp].right) != kNil && nd_[xppr].red) {
          nd_[xppr].red = nd_[xp].red = 0, nd_[xpp].red = 1, x = xpp;
        } else {
          if (x == nd_[xp].right) {
            root = rotate_left(root, x = xp);
            xpp = (xp = nd_[x].parent) == kNil ? kNil : nd_[xp].parent;
          }
          if (xp != kNil) {
            nd_[xp].red = 0;
            if (xpp != kNil) nd_[xpp].red = 1, root = rotate_right(root, xpp);
          }
        }
      } else {
        if (xppl != kNil && nd_[xppl].red) {
          nd_[xppl].red = nd_[xp].red = 0, nd_[xpp].red = 1, x = xpp;
        } else {
          if (x == nd_[xp].left) {
            root = rotate_right(root, x = xp);
            xpp = (xp = nd_[x].parent) == kNil ? kNil : nd_[xp].parent;
          }
          if (xp != kNil) {
            nd_[xp].red = 0;
            if (xpp != kNil) nd_[xpp].red = 1, root = rotate_left(root, xpp);
          }
        }
      }
    }
  }
  int balance_deletion(int root, int x) {
    for (int xp, xpl, xpr;;) {
      if (x == kNil || x == root) return root;
      if ((xp = nd_[x].parent) == kNil) {
        nd_[x].red = 0;
        return x;
      }
      if (nd_[x].red) {
        nd_[x].red = 0;
        return root;
      }
      if ((xpl = nd_[xp].left) == x) {
        if (red(xpr = nd_[xp].right)) {
          nd_[xpr].red = 0, nd_[xp].red = 1;
          root = rotate_left(root, xp);
          xpr = (xp = nd_[x].parent) == kNil ? kNil : nd_[xp].right;
        }
        if (xpr == kNil) {
          x = xp;
        } else {
          int sl = nd_[xpr].left, sr = nd_[xpr].right;
          if (!red(sr) && !red(sl)) {
            nd_[xpr].red = 1, x = xp;
          } else {
            if (!red(sr)) {
              if (sl != kNil) nd_[sl].red = 0;
              nd_[xpr].red = 1;
              root = rotate_right(root, xpr);
              xpr = (xp = nd_[x].parent) == kNil ? kNil : nd_[xp].right;
            }
            if (xpr != kNil) {
              nd_[xpr].red = xp == kNil ? 0 : nd_[xp].red;
              if ((sr = nd_[xpr].right) != kNil) nd_[sr].red = 0;
            }
            if (xp != kNil) nd_[xp].red = 0, root = rotate_left(root, xp);
            x = root;
          }
        }
      } else {
        if (red(xpl)) {
          nd_[xpl].red = 0, nd_[xp].red = 1;
          root = rotate_right(root, xp);
          xpl = (xp = nd_[x].parent) == kNil ? kNil : nd_[xp].left;
        }
        if (xpl == kNil) {
          x = xp;
        } else {
          int sl = nd_[xpl].left, sr = nd_[xpl].right;
          if (!red(sl) && !red(sr)) {
            nd_[xpl].red = 1, x = xp;
          } else {
            if (!red(sl)) {
              if (sr != kNil) nd_[sr].red = 0;
              nd_[xpl].red = 1;
              root = rotate_left(root, xpl);
              xpl = (xp = nd_[x].parent) == kNil ? kNil : nd_[xp].left;
            }
            if (xpl != kNil) {
              nd_[xpl].red = xp == kNil ? 0 : nd_[xp].red;
              if ((sl = nd_[xpl].left) != kNil) nd_[sl].red = 0;
            }
            if (xp != kNil) nd_[xp].red = 0, root = rotate_right(root, xp);
            x = root;
          }
        }
      }
    }
  }
  void to_front(int root) {  // moveRootToFront
    if (root == kNil || tab_.empty()) return;
    const uint32_t index = (capacity() - 1) & nd_[root].hash;
    const int first = tab_[index];
    if (root == first) return;
    tab_[index] = root;
    const int rp = nd_[root].prev, rn = nd_[root].next;
    if (rn != kNil) nd_[rn].prev = rp;
    if (rp != kNil) nd_[rp].next = rn;
    if (first != kNil) nd_[first].prev = root;
    nd_[root].next = first;
    nd_[root].prev = kNil;
  }
  void treeify(int hd) {
    int root = kNil;
    for (int x = hd, next; x != kNil; x = next) {
      next = nd_[x].next;
      nd_[x].left = nd_[x].right = kNil;
      if (root == kNil) {
        nd_[x].parent = kNil, nd_[x].red = 0, root = x;
        continue;
      }
      for (int p = root;;) {
        const int dir = dir_of(nd_[x].hash, nd_[x].key, nd_[p]);
        const int xp = p;
        if ((p = dir <= 0 ? nd_[p].left : nd_[p].right) == kNil) {
          nd_[x].parent = xp;
          (dir <= 0 ? nd_[xp].left : nd_[xp].right) = x;
          root = balance_insertion(root, x);
          break;
        }
      }
    }
    to_front(root);
  }
  int untreeify(int hd) {
    for (int q = hd; q != kNil; q = nd_[q].next)
      nd_[q].tree = nd_[q].red = 0, nd_[q].parent = nd_[q].left = nd_[q].right = nd_[q].prev = kNil;
    return hd;
  }
  void treeify_bin(uint32_t h) {
    if (capacity() < 64) {  // MIN_TREEIFY_CAPACITY
      resize();
      return;
    }
    const uint32_t index = (capacity() - 1) & h;
    int tl = kNil;
    for (int e = tab_[index]; e != kNil; e = nd_[e].next) nd_[e].tree = 1, nd_[e].prev = tl, tl = e;
    if (tab_[index] != kNil) treeify(tab_[index]);
  }
  void split(std::vector<int>& ntab, int b, uint32_t index, uint32_t bit) {
    int lo = kNil, lot = kNil, hi = kNil, hit = kNil, lc = 0, hc = 0;
    for (int e = b, next; e != kNil; e = next) {
      next = nd_[e].next;
      nd_[e].next = kNil;
      if ((nd_[e].hash & bit) == 0) {
        if ((nd_[e].prev = lot) == kNil) lo = e;
        else nd_[lot].next = e;
        lot = e, ++lc;
      } else {
        if ((nd_[e].prev = hit) == kNil) hi = e;
        else nd_[hit].next = e;
        hit = e, ++hc;
      }
    }
    tab_.swap(ntab);  // treeify / moveRootToFront work on the new table
    if (lo != kNil) {
      if (lc <= 6) tab_[index] = untreeify(lo);
      else {
        tab_[index] = lo;
        if (hi != kNil) treeify(lo);
      }
    }
    if (hi != kNil) {
      if (hc <= 6) tab_[index + bit] = untreeify(hi);
      else {
        tab_[index + bit] = hi;
        if (lo != kNil) treeify(hi);
      }
    }
    tab_.swap(ntab);
  }
  void resize() {
    const uint32_t old = capacity();
    const uint32_t cap = old ? old << 1 : 16;
    threshold_ = old ? threshold_ << 1 : 12;
    std::vector<int> ntab(cap, kNil);
    for (uint32_t j = 0; j < old; ++j) {
      const int e = tab_[j];
      if (e == kNil) continue;
      if (nd_[e].next == kNil) {
        ntab[nd_[e].hash & (cap - 1)] = e;
      } else if (nd_[e].tree) {
        split(ntab, e, j, old);
      } else {  // chains keep their order
        int lo = kNil, lot = kNil, hi = kNil, hit = kNil;
        for (int q = e, next; q != kNil; q = next) {
          next = nd_[q].next;
          if ((nd_[q].hash & old) == 0) (lot == kNil ? lo : nd_[lot].next) = q, lot = q;
          else (hit == kNil ? hi : nd_[hit].next) = q, hit = q;
        }
        if (lot != kNil) nd_[lot].next = kNil, ntab[j] = lo;
        if (hit != kNil) nd_[hit].next = kNil, ntab[j + old] = hi;
      }
    }
    tab_.swap(ntab);
  }
  void remove_tree_node(int self, uint32_t index, bool movable) {  // TreeNode.removeTreeNode(map, tab, movable)
    int first = tab_[index], root = first, rl;
    const int succ = nd_[self].next, pred = nd_[self].prev;
    if (pred == kNil) tab_[index] = first = succ;
    else nd_[pred].next = succ;
    if (succ != kNil) nd_[succ].prev = pred;
    if (first == kNil) return;
    if (nd_[root].parent != kNil) root = root_of(root);
    if (movable && (nd_[root].right == kNil || (rl = nd_[root].left) == kNil || nd_[rl].left == kNil)) {
      tab_[index] = untreeify(first);  // too small
      return;
    }
    const int p = self, pl = nd_[p].left, pr = nd_[p].right;
    int replacement;
    if (pl != kNil && pr != kNil) {
      int s = pr, sl;
      while ((sl = nd_[s].left) != kNil) s = sl;  // successor
      std::swap(nd_[s].red, nd_[p].red);
      const int sr = nd_[s].right, pp = nd_[p].parent;
      if (s == pr) {
        nd_[p].parent = s;
        nd_[s].right = p;
      } else {
        const int sp = nd_[s].parent;
        if ((nd_[p].parent = sp) != kNil) (s == nd_[sp].left ? nd_[sp].left : nd_[sp].right) = p;
        if ((nd_[s].right = pr) != kNil) nd_[pr].parent = s;
      }
      nd_[p].left = kNil;
      if ((nd_[p].right = sr) != kNil) nd_[sr].parent = p;
      if ((nd_[s].left = pl) != kNil) nd_[pl].parent = s;
      if ((nd_[s].parent = pp) == kNil) root = s;
      else (p == nd_[pp].left ? nd_[pp].left : nd_[pp].right) = s;
      replacement = sr != kNil ? sr : p;
    } else {
      replacement = pl != kNil ? pl : (pr != kNil ? pr : p);
    }
    if (replacement != p) {
      const int pp = nd_[replacement].parent = nd_[p].parent;
      if (pp == kNil) root = replacement;
      else (p == nd_[pp].left ? nd_[pp].left : nd_[pp].right) = replacement;
      nd_[p].left = nd_[p].right = nd_[p].parent = kNil;
    }
    const int r = nd_[p].red ? root : balance_deletion(root, replacement);
    if (replacement == p) {  // detach
      const int pp = nd_[p].parent;
      nd_[p].parent = kNil;
      if (pp != kNil) {
        if (p == nd_[pp].left) nd_[pp].left = kNil;
        else if (p == nd_[pp].right) nd_[pp].right = kNil;
      }
    }
    if (movable) to_front(r);
  }
};

}  // namespace cc
