#!/usr/bin/env python3
"""Writes tests/golden/kats.json: known-answer tests for the commit-apply path.

Two kinds of KAT, each citing where its expected answers come from:
  * "reference": the assertions of the reference's own tests (TestNG, run against a real Copycat cluster),
    transcribed as (committed command, expected result / event) sequences.  The client-side API call is
    mapped to the command(s) it submits (e.g. DistributedAtomicLong.incrementAndGet -> Get + CompareAndSet,
    DistributedAtomicLong.java:117-146).  Strings are interned to HANDLE ids (see "strings").
  * "quirk": hand-derived from the reference source for behaviour SURVEY Appendix A lists (A1..A15).
  * "defined": rules that live in the un-vendored Copycat jar (timer order, quorum, expiry) — the answer
    is this engine's documented rule, i.e. "parity unpinned".

Value encoding: ["NULL"] | ["LONG", n] | ["INT", n] | ["BOOL", b] | ["H", handle] | ["SET", [ids...]]
| ["LIST", [values...]].
Run: python tests/golden/make_kats.py  (deterministic; the JSON is committed)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from java_hashmap import MapStateModel  # noqa: E402  (tests/java_hashmap.py)

STRINGS = {}


def S(s):
    """Interned String handle."""
    if s not in STRINGS:
        STRINGS[s] = len(STRINGS) + 1
    return ["H", STRINGS[s]]


NULL = ["NULL"]


def L(n):
    return ["LONG", n]


def I(n):
    return ["INT", n]


def B(b):
    return ["BOOL", bool(b)]


def SET(*ids):
    return ["SET", sorted(ids)]


def LIST(*vals):
    return ["LIST", list(vals)]


class K:
    def __init__(self, name, kind, source, mode="deferred"):
        self.d = {"name": name, "kind": kind, "source": source, "timer_mode": mode,
                  "resources": [], "instances": [], "steps": []}

    def res(self, slot, rtype):
        self.d["resources"].append([slot, rtype])
        return self

    def inst(self, slot, res, iid, client):
        self.d["instances"].append([slot, res, iid, client])
        return self

    def c(self, inst, op, key=None, a=None, b=None, aux=0, expect=None, status="OK", events=(), time=None):
        step = {"commit": {"inst": inst, "op": op}}
        cm = step["commit"]
        if key is not None:
            cm["key"] = key
        if a is not None:
            cm["a"] = a
        if b is not None:
            cm["b"] = b
        if aux:
            cm["aux"] = aux
        if time is not None:
            cm["time"] = time
        step["expect"] = {"status": status, "result": expect if expect is not None else NULL}
        if events:
            step["events"] = [list(e) for e in events]
        self.d["steps"].append(step)
        return self

    def advance(self, now, events=()):
        step = {"advance": now}
        if events:
            step["events"] = [list(e) for e in events]
        self.d["steps"].append(step)
        return self

    def close(self, client, events=()):
        step = {"close": client}
        if events:
            step["events"] = [list(e) for e in events]
        self.d["steps"].append(step)
        return self

    def ctl(self, what, expect_status="OK", **kw):
        step = {"control": dict(what=what, **kw), "expect": {"status": expect_status}}
        self.d["steps"].append(step)
        return self

    def state(self, **kw):
        self.d["steps"].append({"state": kw})
        return self


def kats():
    out = []
    MAPT = "collections/src/test/java/io/atomix/collections/DistributedMapTest.java"

    def map_kat(name, lines):
        return K(name, "reference", f"{MAPT}:{lines}").res(0, "MAP").inst(0, 0, 100, 1)

    hw, hwa = S("Hello world!"), S("Hello world again!")
    foo, bar = S("foo"), S("bar")
    out.append(map_kat("map_put_get_remove", "41-66")
               .c(0, "MAP_PUT", key=foo, a=hw)
               .c(0, "MAP_GET", key=foo, expect=hw)
               .c(0, "MAP_REMOVE", key=foo, expect=hw)
               .c(0, "MAP_GET", key=foo, expect=NULL))
    out.append(map_kat("map_put_if_absent", "72-90")
               .c(0, "MAP_PUT", key=foo, a=hw)
               .c(0, "MAP_PUTIFABSENT", key=foo, a=S("something else"), expect=hw)
               .c(0, "MAP_PUTIFABSENT", key=bar, a=S("something"), expect=NULL))
    # putIfAbsent(foo, v, 100 ms) at t=0; Thread.sleep(1000) (session keep-alives tick the log clock);
    # put(bar) at t=1000; containsKey(foo) == false
    out.append(map_kat("map_put_if_absent_ttl", "96-111")
               .c(0, "MAP_PUTIFABSENT", key=foo, a=hw, aux=100, time=0)
               .advance(1000)
               .c(0, "MAP_PUT", key=bar, a=hwa, time=1000)
               .c(0, "MAP_CONTAINSKEY", key=foo, expect=B(False), time=1000))
    out.append(map_kat("map_get_or_default", "117-136")
               .c(0, "MAP_PUT", key=foo, a=hw)
               .c(0, "MAP_GETORDEFAULT", key=foo, a=S("something else"), expect=hw)
               .c(0, "MAP_GETORDEFAULT", key=bar, a=S("something"), expect=S("something")))
    out.append(map_kat("map_contains_key", "142-161")
               .c(0, "MAP_CONTAINSKEY", key=foo, expect=B(False))
               .c(0, "MAP_PUT", key=foo, a=hw, expect=NULL)
               .c(0, "MAP_CONTAINSKEY", key=foo, expect=B(True)))
    out.append(map_kat("map_contains_value", "167-186")
               .c(0, "MAP_CONTAINSVALUE", a=hw, expect=B(False))
               .c(0, "MAP_PUT", key=foo, a=hw, expect=NULL)
               .c(0, "MAP_CONTAINSVALUE", a=hw, expect=B(True)))
    out.append(map_kat("map_size", "192-220")
               .c(0, "MAP_SIZE", expect=I(0))
               .c(0, "MAP_PUT", key=foo, a=hw)
               .c(0, "MAP_SIZE", expect=I(1))
               .c(0, "MAP_PUT", key=bar, a=hwa)
               .c(0, "MAP_SIZE", expect=I(2)))
    out.append(map_kat("map_put_ttl", "226-253")
               .c(0, "MAP_PUT", key=foo, a=hw, aux=1000, time=0)
               .c(0, "MAP_GET", key=foo, expect=hw, time=0)
               .advance(3000)
               .c(0, "MAP_GET", key=foo, expect=NULL, time=3000)
               .c(0, "MAP_SIZE", expect=I(0), time=3000))
    out.append(map_kat("map_clear", "258-286")
               .c(0, "MAP_PUT", key=foo, a=hw)
               .c(0, "MAP_PUT", key=bar, a=hwa)
               .c(0, "MAP_SIZE", expect=I(2))
               .c(0, "MAP_ISEMPTY", expect=B(False))
               .c(0, "MAP_CLEAR")
               .c(0, "MAP_SIZE", expect=I(0))
               .c(0, "MAP_ISEMPTY", expect=B(True)))

    AV = "atomic/src/test/java/io/atomix/atomic/DistributedAtomicValueTest.java"
    out.append(K("atomic_value_set_get", "reference", f"{AV}:40-51").res(0, "VALUE").inst(0, 0, 100, 1)
               .c(0, "VALUE_SET", a=hw)
               .c(0, "VALUE_GET", expect=hw)
               .state(value=[0, hw, True]))

    # DistributedAtomicLongTest: a.get() then op; the op is the client CAS loop (DistributedAtomicLong.java:117-146):
    # getValue() -> Get (cache empty) -> null -> E' = 0; CompareAndSet(null, 0 + delta) succeeds (A4).
    # The test never awaits (A17): these are its intended answers.
    AL = "atomic/src/test/java/io/atomix/atomic/DistributedAtomicLongTest.java"
    for name, lines, delta in [("increment_and_get", "44-46", 1), ("decrement_and_get", "51-53", -1),
                               ("get_and_increment", "58-60", 1), ("get_and_decrement", "65-67", -1),
                               ("add_and_get", "72-74", 10), ("get_and_add", "79-81", 10)]:
        out.append(K(f"atomic_long_{name}", "reference", f"{AL}:{lines},84-105").res(0, "VALUE").inst(0, 0, 100, 1)
                   .c(0, "VALUE_GET", expect=NULL)             # a.get() (null -> 0 on the client)
                   .c(0, "VALUE_GET", expect=NULL)             # updateValue: getValue() with an empty cache
                   .c(0, "VALUE_CAS", a=NULL, b=L(delta), expect=B(True))
                   .state(value=[0, L(delta), True]))

    LK = "coordination/src/test/java/io/atomix/coordination/DistributedLockTest.java"
    # lock() submits Lock(-1) (DistributedLock.java:107-117); the grant is the "lock"(true) event
    out.append(K("lock_unlock", "reference", f"{LK}:38-48").res(0, "LOCK").inst(0, 0, 100, 1)
               .c(0, "LOCK_LOCK", aux=-1, events=[(0, "LOCK", B(True))])
               .c(0, "LOCK_UNLOCK")
               .state(lock=[0, None, []]))

    EL = "coordination/src/test/java/io/atomix/coordination/DistributedLeaderElectionTest.java"
    out.append(K("election_elect", "reference", f"{EL}:41-48").res(0, "ELECTION").inst(0, 0, 100, 1)
               .c(0, "ELECT_LISTEN", events=[(0, "ELECT", L(1))]))  # epoch = index of the Listen commit
    # two clients; client1 closes -> client2 elected with a strictly larger epoch
    out.append(K("election_next_on_close", "reference", f"{EL}:53-80").res(0, "ELECTION")
               .inst(0, 0, 100, 1).inst(1, 0, 101, 2)
               .c(0, "ELECT_LISTEN", events=[(0, "ELECT", L(1))])
               .c(1, "ELECT_LISTEN")
               .close(1, events=[(1, "ELECT", L(2))]))

    # ResourceManager.sessions is a java.util.HashMap<Long, SessionHolder> (ResourceManager.java:37); close() walks it
    # (:250-264), so the instances of a closing client close in HashMap order.  Instance ids 5 + 16 i (i = 0..9) all
    # hash to bin 5 at capacity 16 (Long.hashCode = the id; spread leaves ids < 2^16 alone); the 9th put makes the bin
    # 9 long and treeifyBin resizes to 32 (capacity < 64): even i stay in bin 5, odd i move to bin 21, so the client's
    # instances close in the order 0 2 4 6 8 1 3 5 7 9.  Instance 1 leads the election; 0, 2..9 and then instance 10
    # (another client, id 1000) listen.  Closing 0 2 4 6 8 removes them as listeners (no event); closing 1 hands the
    # lead to the first listener left, 3 (its listen is commit 4), then 3 -> 5 -> 7 -> 9 -> 10
    # (LeaderElectionState.close :35-52).  (Insertion order would close 0 1 2 3 ...: 2, 3, .. 10 elected in turn.)
    kat = K("A12_close_order_treeify_resize", "quirk", "manager/src/main/java/io/atomix/manager/ResourceManager.java:37,250-264")
    kat.res(0, "ELECTION")
    for i in range(10):
        kat.inst(i, 0, 5 + 16 * i, 7)
    kat.inst(10, 0, 1000, 8)
    kat.c(1, "ELECT_LISTEN", events=[(1, "ELECT", L(1))])
    for i in [0, 2, 3, 4, 5, 6, 7, 8, 9, 10]:
        kat.c(i, "ELECT_LISTEN")
    kat.close(7, events=[(3, "ELECT", L(4)), (5, "ELECT", L(6)), (7, "ELECT", L(8)), (9, "ELECT", L(10)),
                         (10, "ELECT", L(11))])
    out.append(kat)

    # ResourceManager removes holders only through sessions.entrySet().iterator().remove() (deleteResource :223-229,
    # close :251-263), and JDK 8's HashIterator.remove calls removeNode(..., movable = false): a tree bin loses the node
    # but is neither untreeified when small nor has its root moved to the bin's front.  Instance ids 5 + 64 i
    # (i = 0..10) share bin 5: the 9th and 10th puts resize 16 -> 32 -> 64 (treeifyBin below capacity 64), the 11th
    # treeifies the bin.  Closing client 7 (8 of the 11) leaves a 3-node tree {261, 389, 517} whose chain order is
    # 389, 261, 517 (movable = true would untreeify it, or move its root 261 to the front).  709 then joins the bin.
    # Listens are commits 646..656 (ids in order) and 710 (709).  Close 7 walks 197 5 69 133 325 453 581 645: the lead
    # goes 5 -> 69 (647) -> 133 (648) -> 261 (650).  Close 8 walks 389 then 261: 389 leaves the listeners, 261 hands
    # the lead to 517 (654) (261 first would elect 389 (652) and then 517).  Close 9 walks 517 709: 709 (710) leads.
    kat = K("A12_close_after_tree_bin_removal", "quirk",
            "manager/src/main/java/io/atomix/manager/ResourceManager.java:37,223-229,250-264")
    tree_el = S("tree-bin-election")
    ph1 = [(5, 7), (69, 7), (133, 7), (197, 7), (261, 8), (325, 7), (389, 8), (453, 7), (517, 9), (581, 7), (645, 7)]
    for iid, client in ph1:
        kat.ctl("create", key=tree_el, type="ELECTION", client=client, index=iid, expect_instance=iid)
    kat.c("@5", "ELECT_LISTEN", events=[("@5", "ELECT", L(646))])
    for iid, _ in ph1[1:]:
        kat.c(f"@{iid}", "ELECT_LISTEN")
    kat.close(7, events=[("@69", "ELECT", L(647)), ("@133", "ELECT", L(648)), ("@261", "ELECT", L(650))])
    kat.ctl("create", key=tree_el, type="ELECTION", client=9, index=709, expect_instance=709)
    kat.c("@709", "ELECT_LISTEN")
    kat.close(8, events=[("@517", "ELECT", L(654))])
    kat.close(9, events=[("@709", "ELECT", L(710))])
    out.append(kat)

    GR = "coordination/src/test/java/io/atomix/coordination/DistributedMembershipGroupTest.java"
    out.append(K("group_join", "reference", f"{GR}:42-65").res(0, "GROUP").inst(0, 0, 100, 1).inst(1, 0, 101, 2)
               .c(1, "GROUP_JOIN", expect=SET(101))
               .c(0, "GROUP_JOIN", expect=SET(100, 101), events=[(1, "JOIN", L(100))]))
    out.append(K("group_leave", "reference", f"{GR}:70-91").res(0, "GROUP").inst(0, 0, 100, 1).inst(1, 0, 101, 2)
               .c(1, "GROUP_JOIN", expect=SET(101))
               .c(0, "GROUP_JOIN", expect=SET(100, 101), events=[(1, "JOIN", L(100))])
               .c(1, "GROUP_LEAVE", events=[(0, "LEAVE", L(101))])
               .state(members=[0, [100]]))
    cb = S("counter::incrementAndGet")
    out.append(K("group_remote_execute", "reference", f"{GR}:96-117").res(0, "GROUP").inst(0, 0, 100, 1)
               .inst(1, 0, 101, 2)
               .c(1, "GROUP_JOIN", expect=SET(101))
               .c(0, "GROUP_JOIN", expect=SET(100, 101), events=[(1, "JOIN", L(100))])
               .c(0, "GROUP_EXECUTE", key=L(100), a=cb, events=[(0, "EXECUTE", cb)])
               .c(0, "GROUP_EXECUTE", key=L(101), a=cb, events=[(1, "EXECUTE", cb)]))

    RT = "manager/src/test/java/io/atomix/AtomixReplicaTest.java"
    test = S("test")
    out.append(K("manager_create_concurrency", "reference", f"{RT}:154-168")
               .ctl("create", key=test, type="VALUE", client=1, index=10, expect_instance=10)
               .ctl("create", key=test, type="VALUE", client=2, index=11, expect_instance=11)
               .c("@10", "VALUE_SET", a=hw)
               .c("@11", "VALUE_GET", expect=hw))
    out.append(K("manager_get_create_concurrency", "reference", f"{RT}:173-189")
               .ctl("get", key=test, type="VALUE", client=1, index=10, expect_instance=10)
               .ctl("create", key=test, type="VALUE", client=2, index=11, expect_instance=11)
               .c("@10", "VALUE_SET", a=hw)
               .c("@11", "VALUE_GET", expect=hw))
    t1, t2 = S("test1"), S("test2")
    out.append(K("manager_operate_many", "reference", f"{RT}:194-215")
               .ctl("get", key=t1, type="VALUE", client=1, index=10, expect_instance=10)
               .ctl("create", key=t1, type="VALUE", client=2, index=11, expect_instance=11)
               .ctl("get", key=t2, type="VALUE", client=1, index=12, expect_instance=12)
               .ctl("create", key=t2, type="VALUE", client=2, index=13, expect_instance=13)
               .c("@10", "VALUE_SET", a=foo)
               .c("@11", "VALUE_GET", expect=foo)
               .c("@12", "VALUE_SET", a=bar)
               .c("@13", "VALUE_GET", expect=bar)
               .c("@10", "VALUE_GET", expect=foo)
               .c("@12", "VALUE_GET", expect=bar))
    out.append(K("manager_get_reuses_instance", "quirk", "manager/src/main/java/io/atomix/manager/ResourceManager.java:125-141")
               .ctl("get", key=test, type="VALUE", client=1, index=10, expect_instance=10)
               .ctl("get", key=test, type="VALUE", client=1, index=11, expect_instance=10)
               .ctl("get", key=test, type="MAP", client=3, index=12, expect_status="TYPE_MISMATCH")
               .ctl("exists", key=test, expect_bool=True)
               .ctl("exists", key=S("nope"), expect_bool=False))

    # ---- quirk KATs, hand-derived from the cited source lines ------------------------
    MS = "collections/src/main/java/io/atomix/collections/state/MapState.java"
    out.append(K("A1_replace_if_present_inverts_args", "quirk", f"{MS}:207-228; DistributedMap.java:653-654")
               .res(0, "MAP").inst(0, 0, 100, 1)
               .c(0, "MAP_PUT", key=foo, a=S("old"))
               # client replace(foo, "old", "new") -> ReplaceIfPresent(value="old", replace="new"): compares "new"
               .c(0, "MAP_REPLACEIFPRESENT", key=foo, a=S("old"), b=S("new"), expect=B(False))
               .c(0, "MAP_REPLACEIFPRESENT", key=foo, a=S("X"), b=S("old"), expect=B(True))
               .c(0, "MAP_GET", key=foo, expect=S("X")))
    AVS = "atomic/src/main/java/io/atomix/atomic/state/AtomicValueState.java"
    out.append(K("A2_atomic_ttl_not_serialized", "quirk", "atomic/.../AtomicValueCommands.java:125-133,181-191")
               .res(0, "VALUE").inst(0, 0, 100, 1)
               .c(0, "VALUE_SET", a=L(5), aux=100, time=0)
               .advance(10_000)
               .c(0, "VALUE_GET", expect=L(5), time=10_000))
    ES = "coordination/src/main/java/io/atomix/coordination/state/LeaderElectionState.java"
    out.append(K("A3_is_leader_epoch_zero", "quirk", f"{ES}:96-98; LeaderElectionCommands.java:99-123")
               .res(0, "ELECTION").inst(0, 0, 100, 1)
               .c(0, "ELECT_LISTEN", events=[(0, "ELECT", L(1))])
               .c(0, "ELECT_ISLEADER", aux=1, expect=B(False)))
    out.append(K("A4_first_cas_null_expect", "quirk", f"{AVS}:124")
               .res(0, "VALUE").inst(0, 0, 100, 1)
               .c(0, "VALUE_CAS", a=L(0), b=L(7), expect=B(False))
               .c(0, "VALUE_CAS", a=NULL, b=L(7), expect=B(True))
               .c(0, "VALUE_CAS", a=NULL, b=L(8), expect=B(False))
               .c(0, "VALUE_GETANDSET", a=NULL, expect=L(7))
               .c(0, "VALUE_GET", expect=NULL)
               .state(value=[0, NULL, True]))
    # A5: HashMap order: Long key 1 -> bucket 1, key 2 -> bucket 2 (cap 16)
    out.append(K("A5_contains_value_npe_order", "quirk", f"{MS}:49-60")
               .res(0, "MAP").inst(0, 0, 100, 1).res(64, "MAP").inst(1, 64, 101, 1)
               .c(0, "MAP_PUT", key=L(1), a=S("x"))
               .c(0, "MAP_PUT", key=L(2), a=NULL)
               .c(0, "MAP_CONTAINSVALUE", a=S("x"), expect=B(True))
               .c(0, "MAP_CONTAINSVALUE", a=S("y"), status="NULL_POINTER")
               .c(1, "MAP_PUT", key=L(1), a=NULL)
               .c(1, "MAP_PUT", key=L(2), a=S("x"))
               .c(1, "MAP_CONTAINSVALUE", a=S("x"), status="NULL_POINTER"))
    # java.util.HashMap (JDK 8, the reference CI's JDK) iteration order, hand-derived from putVal / treeifyBin /
    # resize / treeify / moveRootToFront.  Long.hashCode(k) = (int)(k ^ k >>> 32); HashMap.hash spreads it as
    # h ^ (h >>> 16).  Keys k_i = i * 2^20 + 5: h = i * 2^20 + 5, spread = h ^ (i * 2^4), so at capacity 16 every k_i
    # is in bin 5; at capacity 32 the even i stay in bin 5 and the odd i go to bin 21.  The 9th put appends the bin's
    # 9th node (binCount 7 >= TREEIFY_THRESHOLD - 1) and treeifyBin RESIZES (capacity 16 < MIN_TREEIFY_CAPACITY 64),
    # although size 9 <= threshold 12: iteration is then k0 k2 k4 k6 k8 | k1 k3 k5 k7.  With k1 -> null and
    # k2 -> 7, containsValue(7) meets k2 first: true (a model that resizes on size alone stays at 16 and NPEs on k1).
    kA = [L(i * (1 << 20) + 5) for i in range(9)]
    kat = K("A5_contains_value_treeify_resize", "quirk", f"{MS}:49-60").res(0, "MAP").inst(0, 0, 100, 1)
    for i, k in enumerate(kA):
        kat.c(0, "MAP_PUT", key=k, a=NULL if i == 1 else L(7) if i == 2 else L(100 + i))
    kat.c(0, "MAP_CONTAINSVALUE", a=L(7), expect=B(True))
    kat.c(0, "MAP_CONTAINSVALUE", a=L(8), status="NULL_POINTER")  # bin 5 holds no 8: bin 21's k1 (null) NPEs
    kat.c(0, "MAP_CONTAINSVALUE", a=L(107), status="NULL_POINTER")  # k7 (107) is in bin 21 after k1 (null)
    kat.c(0, "MAP_CONTAINSVALUE", a=L(106), expect=B(True))         # k6 (106) is in bin 5, before bin 21
    out.append(kat)
    # String keys hash by String.hashCode ("a" 97 -> bin 1, "b" 98 -> bin 2), not by their interned handle: "b" is
    # interned first (handle order b < a), yet "a" comes first in iteration.
    sb, sa = S("b"), S("a")
    out.append(K("A5_contains_value_string_hash_order", "quirk", f"{MS}:49-60").res(0, "MAP").inst(0, 0, 100, 1)
               .c(0, "MAP_PUT", key=sb, a=NULL)
               .c(0, "MAP_PUT", key=sa, a=L(7))
               .c(0, "MAP_CONTAINSVALUE", a=L(7), expect=B(True))
               .c(0, "MAP_CONTAINSVALUE", a=L(8), status="NULL_POINTER"))
    # A tree bin: keys k_i = i * 2^22 + 5 (spread = h ^ (i * 2^6): bin 5 at every capacity <= 64).  The 9th put
    # resizes 16 -> 32, the 10th 32 -> 64 (treeifyBin below 64), the 11th treeifies bin 5 (capacity 64): treeify
    # inserts k0..k10 into a red-black tree in chain order (ascending hash), whose root is k3, and moveRootToFront
    # links k3 first: iteration k3 k0 k1 k2 k4 .. k10.  With k0 -> null and k3 -> 7: containsValue(7) is true.
    kT = [L(i * (1 << 22) + 5) for i in range(11)]
    kat = K("A5_contains_value_tree_bin_order", "quirk", f"{MS}:49-60").res(0, "MAP").inst(0, 0, 100, 1)
    for i, k in enumerate(kT):
        kat.c(0, "MAP_PUT", key=k, a=NULL if i == 0 else L(7) if i == 3 else L(100 + i))
    kat.c(0, "MAP_CONTAINSVALUE", a=L(7), expect=B(True))
    kat.c(0, "MAP_CONTAINSVALUE", a=L(8), status="NULL_POINTER")
    out.append(kat)

    # More tree bins, with the expected answers computed by tests/java_hashmap.py (an independent Python restatement of
    # the JDK 8 HashMap, cross-checked against the oracle's JHM by tests/test_oracle_hashmap.py): every value is
    # queried, so each answer pins the chain order of its key against the null's.
    def tree_kat(name, ops, refuses=False):
        kat = K(name, "quirk", f"{MS}:49-60,89-110,138-154").res(0, "MAP").inst(0, 0, 100, 1)
        model = MapStateModel()
        for op in ops:
            if op[0] == "put":
                prev = model.put((1, op[1]), op[2])
                kat.c(0, "MAP_PUT", key=L(op[1]), a=NULL if op[2] is None else L(op[2]),
                      expect=NULL if prev is None else L(prev))
            elif op[0] == "remove":
                prev = model.remove((1, op[1]))
                kat.c(0, "MAP_REMOVE", key=L(op[1]), expect=NULL if prev is None else L(prev))
            else:  # query every stored value and one absent value
                for v in sorted({x for x in model.vals.values() if x is not None}) + [999_999]:
                    r = model.contains_value(v)
                    if r == "NPE":
                        kat.c(0, "MAP_CONTAINSVALUE", a=L(v), status="NULL_POINTER")
                    else:
                        kat.c(0, "MAP_CONTAINSVALUE", a=L(v), expect=B(r))
        if refuses:
            kat.d["gpu"] = "refuses"
        out.append(kat)

    kt = [i * (1 << 22) + 5 for i in range(16)]  # one bin (5) at every capacity <= 64
    # putTreeVal after the treeify (keys 11..13 linked after their tree parents), the null in the middle
    tree_kat("A5_tree_bin_put_after_treeify",
             [("put", k, None if i == 5 else 200 + i) for i, k in enumerate(kt[:14])] + [("query",)])
    # removeTreeNode (the root among them), then removals until the tree is too small and turns back into a list
    tree_kat("A5_tree_bin_remove_and_untreeify",
             [("put", k, None if i == 9 else 300 + i) for i, k in enumerate(kt[:13])] + [("query",)] +
             [("remove", kt[i]) for i in (3, 0, 7)] + [("query",)] +
             [("remove", kt[i]) for i in (1, 2, 4, 5, 6, 8)] + [("query",)] +
             [("put", kt[13], 413), ("put", kt[3], 403)] + [("query",)])
    # the tree bin's table grows past 64 (51 keys): its halves split off the tree order at 128 (TreeNode.split), which
    # the engine follows with the map's big model (map_big.hip)
    others = [k for k in range(3000, 3200) if k % 64 != 5][:40]
    tree_kat("A5_tree_bin_leaves_small_window",
             [("put", k, None if i == 0 else 500 + i) for i, k in enumerate(kt[:11])] +
             [("put", k, 600 + j) for j, k in enumerate(others)] + [("query",)])
    out.append(K("A6_null_value_is_present", "quirk", f"{MS}:115-133,38-44,65-72")
               .res(0, "MAP").inst(0, 0, 100, 1)
               .c(0, "MAP_PUT", key=foo, a=NULL)
               .c(0, "MAP_PUTIFABSENT", key=foo, a=S("v"), expect=NULL)
               .c(0, "MAP_CONTAINSKEY", key=foo, expect=B(True))
               .c(0, "MAP_GET", key=foo, expect=NULL)
               .c(0, "MAP_GETORDEFAULT", key=foo, a=S("d"), expect=NULL)
               .c(0, "MAP_REMOVEIFPRESENT", key=foo, a=S("v"), expect=B(False))
               .c(0, "MAP_REMOVEIFPRESENT", key=foo, a=NULL, expect=B(True))
               .c(0, "MAP_SIZE", expect=I(0)))
    LS = "coordination/src/main/java/io/atomix/coordination/state/LockState.java"
    out.append(K("A7_trylock_timeout_is_silent", "quirk", f"{LS}:41-61")
               .res(0, "LOCK").inst(0, 0, 100, 1).inst(1, 0, 101, 2)
               .c(0, "LOCK_LOCK", aux=-1, events=[(0, "LOCK", B(True))], time=0)
               .c(1, "LOCK_LOCK", aux=100, time=0)     # tryLock(100 ms): queued, timer armed
               .c(1, "LOCK_LOCK", aux=0, events=[(1, "LOCK", B(False))], time=10)  # tryLock(): fails now
               .advance(200)                              # the waiter's timer fires: no event
               .c(0, "LOCK_UNLOCK", time=200)             # nobody queued: lock becomes free
               .state(lock=[0, None, []]))
    out.append(K("lock_fifo_handoff_and_not_holder", "quirk", f"{LS}:66-85")
               .res(0, "LOCK").inst(0, 0, 100, 1).inst(1, 0, 101, 2).inst(2, 0, 102, 3)
               .c(0, "LOCK_LOCK", aux=-1, events=[(0, "LOCK", B(True))])
               .c(1, "LOCK_LOCK", aux=-1)
               .c(2, "LOCK_LOCK", aux=5000)
               .c(2, "LOCK_UNLOCK", status="ILLEGAL_STATE")
               .c(0, "LOCK_UNLOCK", events=[(1, "LOCK", B(True))])
               .c(1, "LOCK_UNLOCK", events=[(2, "LOCK", B(True))])
               .state(lock=[0, 2, []]))
    out.append(K("A9_leader_relisten_appended", "quirk", f"{ES}:57-66,71-91")
               .res(0, "ELECTION").inst(0, 0, 100, 1)
               .c(0, "ELECT_LISTEN", events=[(0, "ELECT", L(1))])
               .c(0, "ELECT_LISTEN")
               .c(0, "ELECT_UNLISTEN", events=[(0, "ELECT", L(2))]))
    GS = "coordination/src/main/java/io/atomix/coordination/state/MembershipGroupState.java"
    out.append(K("A10_close_publishes_leave_for_non_member", "quirk", f"{GS}:36-42")
               .res(0, "GROUP").inst(0, 0, 100, 1).inst(1, 0, 101, 2)
               .c(0, "GROUP_JOIN", expect=SET(100))
               .close(2, events=[(0, "LEAVE", L(101))]))
    out.append(K("A11_lock_survives_holder_close", "quirk", f"{LS}:33-100")
               .res(0, "LOCK").inst(0, 0, 100, 1).inst(1, 0, 101, 2)
               .c(0, "LOCK_LOCK", aux=-1, events=[(0, "LOCK", B(True))])
               .c(1, "LOCK_LOCK", aux=-1)
               .close(1)
               .state(lock=[0, 0, [1]]))
    out.append(K("A13_delete_resource_by_instance_id", "quirk", "manager/.../ResourceManager.java:212-235; InstanceClient.java:73-74")
               .ctl("get", key=test, type="VALUE", client=1, index=10, expect_instance=10)
               .ctl("get", key=test, type="VALUE", client=2, index=11, expect_instance=11)
               .ctl("delete", resource=11, expect_status="UNKNOWN_RESOURCE")
               .ctl("delete", resource=10, expect_status="OK")
               .c("#0", "VALUE_GET", status="UNKNOWN_SESSION"))
    out.append(K("A15_long_is_not_integer", "quirk", f"{AVS}:124")
               .res(0, "VALUE").inst(0, 0, 100, 1)
               .c(0, "VALUE_SET", a=L(1))
               .c(0, "VALUE_CAS", a=I(1), b=L(2), expect=B(False))
               .c(0, "VALUE_CAS", a=L(1), b=I(2), expect=B(True))
               .c(0, "VALUE_CAS", a=I(2), b=B(True), expect=B(True))
               .c(0, "VALUE_GET", expect=B(True)))
    out.append(K("lock_delete_then_unlock_commit_closed", "quirk", f"{LS}:87-98; ResourceManagerCommit.java:79-83")
               .res(0, "LOCK").inst(0, 0, 100, 1)
               .c(0, "LOCK_LOCK", aux=-1, events=[(0, "LOCK", B(True))])
               .c(0, "DELETE")
               .c(0, "LOCK_UNLOCK", status="ILLEGAL_STATE")
               .c(0, "DELETE", status="ILLEGAL_STATE"))
    out.append(K("dispatch_errors", "quirk", "manager/.../ResourceManager.java:60-69; ResourceStateMachineExecutor.java:78")
               .res(0, "VALUE").inst(0, 0, 100, 1).res(64, "GROUP").inst(1, 64, 101, 1)
               .c(5, "VALUE_GET", status="UNKNOWN_SESSION")
               .c(0, "MAP_PUT", key=foo, a=hw, status="UNKNOWN_OP")
               .c(1, "GROUP_EXECUTE", key=L(999), a=cb, status="ILLEGAL_ARGUMENT")
               .c(1, "GROUP_SCHEDULE", key=L(999), a=cb, aux=10, status="ILLEGAL_ARGUMENT"))
    out.append(K("group_schedule_fires_on_clock", "defined", f"{GS}:86-103 (timer order: Copycat, unpinned)")
               .res(0, "GROUP").inst(0, 0, 100, 1)
               .c(0, "GROUP_JOIN", expect=SET(100), time=0)
               .c(0, "GROUP_SCHEDULE", key=L(100), a=cb, aux=50, time=0)
               .advance(49)
               .advance(50, events=[(0, "EXECUTE", cb)]))
    # timer order rule (A8): manager mode defers due timers to after the commit that advanced the clock
    out.append(K("A8_timer_deferred_after_commit", "defined", "ResourceManagerStateMachineExecutor.java:104-109")
               .res(0, "MAP").inst(0, 0, 100, 1)
               .c(0, "MAP_PUT", key=foo, a=hw, aux=100, time=0)
               .c(0, "MAP_GET", key=foo, expect=hw, time=100)
               .c(0, "MAP_GET", key=foo, expect=NULL, time=100))
    QT = "collections/src/test/java/io/atomix/collections/DistributedQueueTest.java"

    def queue_kat(name, lines):
        return K(name, "reference", f"{QT}:{lines}").res(0, "QUEUE").inst(0, 0, 100, 1).inst(1, 0, 101, 2)

    out.append(queue_kat("queue_offer_poll", "41-65")
               .c(0, "QUEUE_OFFER", a=hw, expect=B(False))
               .c(1, "QUEUE_SIZE", expect=I(1))
               .c(1, "QUEUE_POLL", expect=hw)
               .c(1, "QUEUE_ISEMPTY", expect=B(True)))
    out.append(queue_kat("queue_offer_remove", "70-94")
               .c(0, "QUEUE_OFFER", a=hw, expect=B(False))
               .c(1, "QUEUE_SIZE", expect=I(1))
               .c(1, "QUEUE_REMOVE", expect=hw)  # remove() with no element: the head (QueueState.java:143-152)
               .c(1, "QUEUE_ISEMPTY", expect=B(True)))
    out.append(queue_kat("queue_offer_peek", "99-123")
               .c(0, "QUEUE_OFFER", a=hw, expect=B(False))
               .c(1, "QUEUE_SIZE", expect=I(1))
               .c(1, "QUEUE_PEEK", expect=hw)
               .c(1, "QUEUE_ISEMPTY", expect=B(False)))
    out.append(queue_kat("queue_offer_element", "128-152")
               .c(0, "QUEUE_OFFER", a=hw, expect=B(False))
               .c(1, "QUEUE_SIZE", expect=I(1))
               .c(1, "QUEUE_ELEMENT", expect=hw)
               .c(1, "QUEUE_ISEMPTY", expect=B(False)))
    out.append(queue_kat("queue_add_remove", "158-176")
               .c(0, "QUEUE_CONTAINS", a=hw, expect=B(False))
               .c(1, "QUEUE_CONTAINS", a=hw, expect=B(False))
               .c(0, "QUEUE_ADD", a=hw, expect=B(False))
               .c(0, "QUEUE_CONTAINS", a=hw, expect=B(True))
               .c(1, "QUEUE_CONTAINS", a=hw, expect=B(True))
               .c(1, "QUEUE_REMOVE", a=hw, expect=B(True))
               .c(0, "QUEUE_CONTAINS", a=hw, expect=B(False))
               .c(1, "QUEUE_CONTAINS", a=hw, expect=B(False)))
    k = K("queue_null_and_empty_quirks", "defined", "collections/src/main/java/io/atomix/collections/state/QueueState.java:36-157")
    out.append(k.res(0, "QUEUE").inst(0, 0, 100, 1)
               .c(0, "QUEUE_ELEMENT", status="NO_SUCH_ELEMENT")   # ArrayDeque.element on empty throws
               .c(0, "QUEUE_REMOVE", status="NO_SUCH_ELEMENT")    # ArrayDeque.remove() on empty throws
               .c(0, "QUEUE_POLL", expect=NULL)
               .c(0, "QUEUE_ADD", a=NULL, expect=B(False))       # a null value is stored (the commit is the element)
               .c(0, "QUEUE_ADD", a=foo, expect=B(False))
               .c(0, "QUEUE_CONTAINS", a=foo, status="NULL_POINTER")  # the stored null's equals NPEs first
               .c(0, "QUEUE_POLL", expect=NULL)
               .c(0, "QUEUE_CONTAINS", a=foo, expect=B(True))
               .c(0, "QUEUE_SIZE", expect=I(1)))
    SETT = "collections/src/test/java/io/atomix/collections/DistributedSetTest.java"
    # two clients, one set: contains false, add, contains true (both), remove, contains false (both)
    out.append(K("set_add_remove", "reference", f"{SETT}:42-58").res(0, "SET").inst(0, 0, 100, 1).inst(1, 0, 101, 2)
               .c(0, "SET_CONTAINS", key=hw, expect=B(False))
               .c(1, "SET_CONTAINS", key=hw, expect=B(False))
               .c(0, "SET_ADD", key=hw, expect=B(False))  # SetState.add returns false even when it adds (:65)
               .c(0, "SET_CONTAINS", key=hw, expect=B(True))
               .c(1, "SET_CONTAINS", key=hw, expect=B(True))
               .c(1, "SET_REMOVE", key=hw, expect=B(True))
               .c(0, "SET_CONTAINS", key=hw, expect=B(False))
               .c(1, "SET_CONTAINS", key=hw, expect=B(False)))
    k = K("set_ttl_size_clear", "defined", "collections/src/main/java/io/atomix/collections/state/SetState.java:49-134")
    out.append(k.res(0, "SET").inst(0, 0, 100, 1)
               .c(0, "SET_ADD", key=foo, aux=100, expect=B(False), time=0)
               .c(0, "SET_ADD", key=bar, expect=B(False), time=0)
               .c(0, "SET_ADD", key=bar, expect=B(False), time=0)
               .c(0, "SET_SIZE", expect=I(2), time=0)
               .c(0, "SET_SIZE", expect=I(2), time=150)  # manager mode: the due timer fires after this commit (A8)
               .c(0, "SET_CONTAINS", key=foo, expect=B(False), time=150)
               .c(0, "SET_SIZE", expect=I(1), time=150)
               .c(0, "SET_REMOVE", key=foo, expect=B(False), time=150)
               .c(0, "SET_CLEAR", time=150)
               .c(0, "SET_ISEMPTY", expect=B(True), time=150))
    k = K("A8_timer_immediate_module_mode", "defined", "ResourceStateMachineExecutor.java:109-117", mode="immediate")
    out.append(k.res(0, "MAP").inst(0, 0, 100, 1)
               .c(0, "MAP_PUT", key=foo, a=hw, aux=100, time=0)
               .c(0, "MAP_GET", key=foo, expect=NULL, time=100))
    # MultiMapState.put registers the key's value map but never stores the value (MultiMapState.java:70-82): every
    # put answers true, get and size see empty value maps, remove(key, value) finds nothing, removeValue drops every
    # key (all value maps are empty, :140-165), and a put's TTL timer throws before it changes anything (A18).
    k = K("A18_multimap_put_never_stores", "quirk", "collections/src/main/java/io/atomix/collections/state/MultiMapState.java:37-222")
    out.append(k.res(0, "MULTIMAP").inst(0, 0, 100, 1).inst(1, 0, 101, 2)
               .c(0, "MMAP_ISEMPTY", expect=B(True), time=0)
               .c(0, "MMAP_PUT", key=foo, a=hw, expect=B(True), time=0)
               .c(1, "MMAP_PUT", key=foo, a=hw, expect=B(True), time=0)   # the value is still not "contained"
               .c(1, "MMAP_CONTAINSKEY", key=foo, expect=B(True), time=0)
               .c(0, "MMAP_GET", key=foo, expect=LIST(), time=0)
               .c(0, "MMAP_SIZE", key=foo, expect=I(0), time=0)
               .c(0, "MMAP_ISEMPTY", expect=B(False), time=0)
               .c(0, "MMAP_REMOVE", key=foo, a=hw, expect=B(False), time=0)
               .c(0, "MMAP_CONTAINSKEY", key=foo, expect=B(True), time=0)
               .c(0, "MMAP_CONTAINSENTRY", key=foo, a=hw, status="UNKNOWN_OP", time=0)  # no handler
               .c(0, "MMAP_CONTAINSVALUE", a=hw, status="UNKNOWN_OP", time=0)
               .c(1, "MMAP_REMOVE", key=foo, expect=LIST(), time=0)
               .c(0, "MMAP_CONTAINSKEY", key=foo, expect=B(False), time=0)
               .c(0, "MMAP_REMOVE", key=foo, expect=LIST(), time=0)          # absent key: EMPTY_LIST
               .c(0, "MMAP_PUT", key=bar, a=hw, aux=50, expect=B(True), time=0)
               .c(0, "MMAP_PUT", key=foo, a=NULL, expect=B(True), time=0)
               .c(0, "MMAP_CONTAINSKEY", key=bar, expect=B(True), time=100)  # the TTL timer changed nothing
               .c(0, "MMAP_CONTAINSKEY", key=bar, expect=B(True), time=100)
               .c(1, "MMAP_REMOVEVALUE", a=foo, time=100)                     # drops every (empty) key
               .c(0, "MMAP_ISEMPTY", expect=B(True), time=100)
               .c(0, "MMAP_PUT", key=foo, a=bar, expect=B(True), time=100)
               .c(0, "MMAP_CLEAR", time=100)
               .c(0, "MMAP_CONTAINSKEY", key=foo, expect=B(False), time=100))
    return out


def main():
    data = {"comment": __doc__.strip().splitlines()[0], "strings": None, "kats": [k.d for k in kats()]}
    data["strings"] = STRINGS
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kats.json")
    with open(path, "w") as f:
        json.dump(data, f, indent=1, sort_keys=False)
        f.write("\n")
    print(f"wrote {len(data['kats'])} KATs to {path}")


if __name__ == "__main__":
    main()
