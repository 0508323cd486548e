"""java.util.HashMap (JDK 8) in pure Python, written from the published JDK 8 algorithm as an independent check
of the oracle's C++ restatement (oracle/oracle.cpp JHM).  Test infrastructure only.

The reference's MapState (collections/src/main/java/io/atomix/collections/state/MapState.java:33) keeps its entries
in a `new HashMap<>()`; containsValue (:49-60) walks map.values(), so its answer (true vs NullPointerException when a
stored value is null) depends on HashMap's iteration order: bins in index order, each bin's `next` chain.
Keys are canonical (tag, payload) pairs: tag 1 Long, 2 Integer, 3 Boolean, 4 String (payload = the str itself).
"""

TREEIFY_THRESHOLD, UNTREEIFY_THRESHOLD, MIN_TREEIFY_CAPACITY = 8, 6, 64
LONG, INT, BOOL, STR = 1, 2, 3, 4
CLASS_NAME = {LONG: "java.lang.Long", INT: "java.lang.Integer", BOOL: "java.lang.Boolean", STR: "java.lang.String"}


def _i32(x):
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >> 31 else x


def hash_code(key):
    tag, v = key
    if tag == LONG:
        v &= 0xFFFFFFFFFFFFFFFF
        return _i32(v ^ (v >> 32))
    if tag == INT:
        return _i32(v)
    if tag == BOOL:
        return 1231 if v else 1237
    h = 0
    for u in _utf16(v):
        h = (31 * h + u) & 0xFFFFFFFF
    return _i32(h)


def _utf16(s):
    b = s.encode("utf-16-le")
    return [b[i] | (b[i + 1] << 8) for i in range(0, len(b), 2)]


def spread(h):  # HashMap.hash: (h = key.hashCode()) ^ (h >>> 16), as a Java int
    u = h & 0xFFFFFFFF
    return _i32(u ^ (u >> 16))


def compare_to(a, b):  # Comparable.compareTo for two keys of one class
    (ta, va), (_, vb) = a, b
    if ta == LONG:
        va, vb = _i64(va), _i64(vb)
    elif ta == INT:
        va, vb = _i32(va), _i32(vb)
    elif ta == BOOL:
        va, vb = bool(va), bool(vb)
    elif ta == STR:
        va, vb = _utf16(va), _utf16(vb)
    return (va > vb) - (va < vb)


def _i64(x):
    x &= 0xFFFFFFFFFFFFFFFF
    return x - (1 << 64) if x >> 63 else x


def tie_break_order(a, b):
    ca, cb = CLASS_NAME[a[0]], CLASS_NAME[b[0]]
    d = (ca > cb) - (ca < cb)
    if d == 0:
        raise AssertionError("identityHashCode tie: equal keys of one class")
    return -1 if d <= 0 else 1


class Node:
    __slots__ = ("hash", "key", "next")

    def __init__(self, h, key, nxt):
        self.hash, self.key, self.next = h, key, nxt


class TreeNode(Node):
    __slots__ = ("parent", "left", "right", "prev", "red")

    def __init__(self, h, key, nxt):
        super().__init__(h, key, nxt)
        self.parent = self.left = self.right = self.prev = None
        self.red = False

    def root(self):
        r = self
        while r.parent is not None:
            r = r.parent
        return r


def _dir(h, k, p):
    """treeify / putTreeVal direction of key k (hash h) at node p (k not in the tree)."""
    if p.hash > h:
        return -1
    if p.hash < h:
        return 1
    if k[0] == p.key[0]:
        d = compare_to(k, p.key)
        if d != 0:
            return d
    return tie_break_order(k, p.key)


def rotate_left(root, p):
    if p is not None and p.right is not None:
        r = p.right
        rl = p.right = r.left
        if rl is not None:
            rl.parent = p
        pp = r.parent = p.parent
        if pp is None:
            root = r
            r.red = False
        elif pp.left is p:
            pp.left = r
        else:
            pp.right = r
        r.left = p
        p.parent = r
    return root


def rotate_right(root, p):
    if p is not None and p.left is not None:
        l_ = p.left
        lr = p.left = l_.right
        if lr is not None:
            lr.parent = p
        pp = l_.parent = p.parent
        if pp is None:
            root = l_
            l_.red = False
        elif pp.right is p:
            pp.right = l_
        else:
            pp.left = l_
        l_.right = p
        p.parent = l_
    return root


def balance_insertion(root, x):
    x.red = True
    while True:
        xp = x.parent
        if xp is None:
            x.red = False
            return x
        xpp = xp.parent
        if not xp.red or xpp is None:
            return root
        xppl = xpp.left
        if xp is xppl:
            xppr = xpp.right
            if xppr is not None and xppr.red:
                xppr.red = False
                xp.red = False
                xpp.red = True
                x = xpp
            else:
                if x is xp.right:
                    x = xp
                    root = rotate_left(root, x)
                    xp = x.parent
                    xpp = None if xp is None else xp.parent
                if xp is not None:
                    xp.red = False
                    if xpp is not None:
                        xpp.red = True
                        root = rotate_right(root, xpp)
        else:
            if xppl is not None and xppl.red:
                xppl.red = False
                xp.red = False
                xpp.red = True
                x = xpp
            else:
                if x is xp.left:
                    x = xp
                    root = rotate_right(root, x)
                    xp = x.parent
                    xpp = None if xp is None else xp.parent
                if xp is not None:
                    xp.red = False
                    if xpp is not None:
                        xpp.red = True
                        root = rotate_left(root, xpp)


def _red(n):
    return n is not None and n.red


def balance_deletion(root, x):
    while True:
        if x is None or x is root:
            return root
        xp = x.parent
        if xp is None:
            x.red = False
            return x
        if x.red:
            x.red = False
            return root
        xpl = xp.left
        if xpl is x:
            xpr = xp.right
            if _red(xpr):
                xpr.red = False
                xp.red = True
                root = rotate_left(root, xp)
                xp = x.parent
                xpr = None if xp is None else xp.right
            if xpr is None:
                x = xp
            else:
                sl, sr = xpr.left, xpr.right
                if not _red(sr) and not _red(sl):
                    xpr.red = True
                    x = xp
                else:
                    if not _red(sr):
                        if sl is not None:
                            sl.red = False
                        xpr.red = True
                        root = rotate_right(root, xpr)
                        xp = x.parent
                        xpr = None if xp is None else xp.right
                    if xpr is not None:
                        xpr.red = False if xp is None else xp.red
                        sr = xpr.right
                        if sr is not None:
                            sr.red = False
                    if xp is not None:
                        xp.red = False
                        root = rotate_left(root, xp)
                    x = root
        else:
            if _red(xpl):
                xpl.red = False
                xp.red = True
                root = rotate_right(root, xp)
                xp = x.parent
                xpl = None if xp is None else xp.left
            if xpl is None:
                x = xp
            else:
                sl, sr = xpl.left, xpl.right
                if not _red(sl) and not _red(sr):
                    xpl.red = True
                    x = xp
                else:
                    if not _red(sl):
                        if sr is not None:
                            sr.red = False
                        xpl.red = True
                        root = rotate_left(root, xpl)
                        xp = x.parent
                        xpl = None if xp is None else xp.left
                    if xpl is not None:
                        xpl.red = False if xp is None else xp.red
                        sl = xpl.left
                        if sl is not None:
                            sl.red = False
                    if xp is not None:
                        xp.red = False
                        root = rotate_right(root, xp)
                    x = root


class HashMap:
    def __init__(self):
        self.table = None
        self.size = 0
        self.threshold = 0

    # ---- lookups ----
    def _find(self, key):
        if self.table is None:
            return None
        h = spread(hash_code(key))
        e = self.table[(len(self.table) - 1) & h]
        while e is not None:
            if e.hash == h and e.key == key:
                return e
            e = e.next
        return None

    def __contains__(self, key):
        return self._find(key) is not None

    def keys(self):  # iteration order (HashIterator)
        out = []
        if self.table is not None:
            for b in self.table:
                e = b
                while e is not None:
                    out.append(e.key)
                    e = e.next
        return out

    def capacity(self):
        return 0 if self.table is None else len(self.table)

    # ---- structure ----
    def move_root_to_front(self, tab, root):
        if root is None or tab is None or len(tab) == 0:
            return
        index = (len(tab) - 1) & root.hash
        first = tab[index]
        if root is not first:
            tab[index] = root
            rp = root.prev
            rn = root.next
            if rn is not None:
                rn.prev = rp
            if rp is not None:
                rp.next = rn
            if first is not None:
                first.prev = root
            root.next = first
            root.prev = None

    def treeify(self, hd, tab):
        root = None
        x = hd
        while x is not None:
            nxt = x.next
            x.left = x.right = None
            if root is None:
                x.parent = None
                x.red = False
                root = x
            else:
                p = root
                while True:
                    d = _dir(x.hash, x.key, p)
                    xp = p
                    p = p.left if d <= 0 else p.right
                    if p is None:
                        x.parent = xp
                        if d <= 0:
                            xp.left = x
                        else:
                            xp.right = x
                        root = balance_insertion(root, x)
                        break
            x = nxt
        self.move_root_to_front(tab, root)

    @staticmethod
    def untreeify(hd):
        head = tail = None
        q = hd
        while q is not None:
            p = Node(q.hash, q.key, None)
            if tail is None:
                head = p
            else:
                tail.next = p
            tail = p
            q = q.next
        return head

    def treeify_bin(self, tab, h):
        if tab is None or len(tab) < MIN_TREEIFY_CAPACITY:
            self.resize()
            return
        index = (len(tab) - 1) & h
        e = tab[index]
        if e is None:
            return
        hd = tl = None
        while e is not None:
            p = TreeNode(e.hash, e.key, None)
            if tl is None:
                hd = p
            else:
                p.prev = tl
                tl.next = p
            tl = p
            e = e.next
        tab[index] = hd
        self.treeify(hd, tab)

    def split(self, b, tab, index, bit):
        lo_h = lo_t = hi_h = hi_t = None
        lc = hc = 0
        e = b
        while e is not None:
            nxt = e.next
            e.next = None
            if (e.hash & bit) == 0:
                e.prev = lo_t
                if lo_t is None:
                    lo_h = e
                else:
                    lo_t.next = e
                lo_t = e
                lc += 1
            else:
                e.prev = hi_t
                if hi_t is None:
                    hi_h = e
                else:
                    hi_t.next = e
                hi_t = e
                hc += 1
            e = nxt
        if lo_h is not None:
            if lc <= UNTREEIFY_THRESHOLD:
                tab[index] = self.untreeify(lo_h)
            else:
                tab[index] = lo_h
                if hi_h is not None:
                    self.treeify(lo_h, tab)
        if hi_h is not None:
            if hc <= UNTREEIFY_THRESHOLD:
                tab[index + bit] = self.untreeify(hi_h)
            else:
                tab[index + bit] = hi_h
                if lo_h is not None:
                    self.treeify(hi_h, tab)

    def resize(self):
        old = self.table
        old_cap = 0 if old is None else len(old)
        if old_cap > 0:
            new_cap, new_thr = old_cap << 1, self.threshold << 1
        else:
            new_cap, new_thr = 16, 12
        self.threshold = new_thr
        tab = [None] * new_cap
        self.table = tab
        for j in range(old_cap):
            e = old[j]
            if e is None:
                continue
            old[j] = None
            if e.next is None:
                tab[e.hash & (new_cap - 1)] = e
            elif isinstance(e, TreeNode):
                self.split(e, tab, j, old_cap)
            else:
                lo_h = lo_t = hi_h = hi_t = None
                while e is not None:
                    nxt = e.next
                    if (e.hash & old_cap) == 0:
                        if lo_t is None:
                            lo_h = e
                        else:
                            lo_t.next = e
                        lo_t = e
                    else:
                        if hi_t is None:
                            hi_h = e
                        else:
                            hi_t.next = e
                        hi_t = e
                    e = nxt
                if lo_t is not None:
                    lo_t.next = None
                    tab[j] = lo_h
                if hi_t is not None:
                    hi_t.next = None
                    tab[j + old_cap] = hi_h
        return tab

    def put(self, key):
        """putVal for the structure: returns True if the key was new."""
        h = spread(hash_code(key))
        tab = self.table
        if tab is None or len(tab) == 0:
            tab = self.resize()
        n = len(tab)
        i = (n - 1) & h
        p = tab[i]
        if p is None:
            tab[i] = Node(h, key, None)
        elif p.hash == h and p.key == key:
            return False
        elif isinstance(p, TreeNode):
            if not self.put_tree_val(p, tab, h, key):
                return False
        else:
            bin_count = 0
            while True:
                e = p.next
                if e is None:
                    p.next = Node(h, key, None)
                    if bin_count >= TREEIFY_THRESHOLD - 1:
                        self.treeify_bin(tab, h)
                    break
                if e.hash == h and e.key == key:
                    return False
                p = e
                bin_count += 1
        self.size += 1
        if self.size > self.threshold:
            self.resize()
        return True

    def put_tree_val(self, first, tab, h, k):
        root = first.root() if first.parent is not None else first
        searched = False
        p = root
        while True:
            if p.hash > h:
                d = -1
            elif p.hash < h:
                d = 1
            elif p.key == k:
                return False
            else:
                d = compare_to(k, p.key) if k[0] == p.key[0] else 0
                if d == 0:
                    if not searched:
                        searched = True
                        for ch in (p.left, p.right):
                            if ch is not None and self._tree_find(ch, h, k) is not None:
                                return False
                    d = tie_break_order(k, p.key)
            xp = p
            p = p.left if d <= 0 else p.right
            if p is None:
                xpn = xp.next
                x = TreeNode(h, k, xpn)
                if d <= 0:
                    xp.left = x
                else:
                    xp.right = x
                xp.next = x
                x.parent = x.prev = xp
                if xpn is not None:
                    xpn.prev = x
                self.move_root_to_front(tab, balance_insertion(root, x))
                return True

    @staticmethod
    def _tree_find(p, h, k):  # an exhaustive subtree search (only its result matters here)
        stack = [p]
        while stack:
            q = stack.pop()
            if q is None:
                continue
            if q.hash == h and q.key == k:
                return q
            stack.append(q.left)
            stack.append(q.right)
        return None

    def remove(self, key, movable=True):
        tab = self.table
        if tab is None:
            return False
        h = spread(hash_code(key))
        index = (len(tab) - 1) & h
        p = tab[index]
        node = None
        if p is None:
            return False
        if p.hash == h and p.key == key:
            node = p
        else:
            e = p.next
            if e is not None:
                if isinstance(p, TreeNode):
                    node = self._tree_find(p.root(), h, key)
                else:
                    while e is not None:
                        if e.hash == h and e.key == key:
                            node = e
                            break
                        p = e
                        e = e.next
        if node is None:
            return False
        if isinstance(node, TreeNode):
            self.remove_tree_node(node, tab, movable)
        elif node is p:
            tab[index] = node.next
        else:
            p.next = node.next
        self.size -= 1
        return True

    def remove_tree_node(self, this, tab, movable):
        n = len(tab)
        index = (n - 1) & this.hash
        first = tab[index]
        root = first
        succ, pred = this.next, this.prev
        if pred is None:
            tab[index] = first = succ
        else:
            pred.next = succ
        if succ is not None:
            succ.prev = pred
        if first is None:
            return
        if root.parent is not None:
            root = root.root()
        if root is None or (movable and (root.right is None or root.left is None or root.left.left is None)):
            tab[index] = self.untreeify(first)
            return
        p, pl, pr = this, this.left, this.right
        if pl is not None and pr is not None:
            s = pr
            while s.left is not None:
                s = s.left
            s.red, p.red = p.red, s.red
            sr = s.right
            pp = p.parent
            if s is pr:
                p.parent = s
                s.right = p
            else:
                sp = s.parent
                p.parent = sp
                if sp is not None:
                    if s is sp.left:
                        sp.left = p
                    else:
                        sp.right = p
                s.right = pr
                if pr is not None:
                    pr.parent = s
            p.left = None
            p.right = sr
            if sr is not None:
                sr.parent = p
            s.left = pl
            if pl is not None:
                pl.parent = s
            s.parent = pp
            if pp is None:
                root = s
            elif p is pp.left:
                pp.left = s
            else:
                pp.right = s
            replacement = sr if sr is not None else p
        elif pl is not None:
            replacement = pl
        elif pr is not None:
            replacement = pr
        else:
            replacement = p
        if replacement is not p:
            pp = replacement.parent = p.parent
            if pp is None:
                root = replacement
            elif p is pp.left:
                pp.left = replacement
            else:
                pp.right = replacement
            p.left = p.right = p.parent = None
        r = root if p.red else balance_deletion(root, replacement)
        if replacement is p:
            pp = p.parent
            p.parent = None
            if pp is not None:
                if p is pp.left:
                    pp.left = None
                elif p is pp.right:
                    pp.right = None
        if movable:
            self.move_root_to_front(tab, r)

    def clear_by_iterator(self):
        """MapState.delete (:264-274): iterator.remove() on every entry, i.e. removeNode(..., movable=false)."""
        for k in self.keys():
            self.remove(k, movable=False)
        assert self.size == 0


class MapStateModel:
    """MapState's map: values by key plus the HashMap structure; containsValue as :49-60 (None = null)."""

    def __init__(self):
        self.hm = HashMap()
        self.vals = {}

    def put(self, k, v):
        prev = self.vals.get(k)
        self.hm.put(k)
        self.vals[k] = v
        return prev

    def remove(self, k):
        if k in self.vals:
            self.hm.remove(k)
            return self.vals.pop(k)
        return None

    def clear(self):
        self.hm.clear_by_iterator()
        self.vals.clear()

    def contains_value(self, v):
        """'NPE', True or False."""
        for k in self.hm.keys():
            s = self.vals[k]
            if s is None:
                return "NPE"
            if s == v:
                return True
        return False
