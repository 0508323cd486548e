"""GPU parity of the session close / expire fan-out (close.hip, cc_sessions_close / cc_sessions_expire) vs the oracle.

Reference: ResourceManager.close(Session) :250-264 and expire :238-247 (manager/src/main/java/io/atomix/manager/
ResourceManager.java) over the state machines' close overrides: LeaderElectionState.close :35-52 (hand-over to the first
listener, "elect"), MembershipGroupState.close :36-42 ("leave" to every remaining member, even for a non-member, A10),
the AtomicValueState listener drop (:43-48); locks and maps have none (A11).

Bar: the events of each close, per target session in publish order (A12: only per-target order is fixed across
sessions); every instance the closed clients owned leaves the dispatch table (later commits on it get
CC_ST_UNKNOWN_SESSION, bit-exact vs the oracle); final lock / election / group / value state."""
import numpy as np
import pytest

from copycat_amd import abi
from tests.test_gpu_coord import FLAGS, E_, G, L, V, _check_batch, _check_state, _setup

pytestmark = pytest.mark.gpu

CLOSE_POS = 0xFFFFFFFF


def _per_target(target, code, tag, payload):
    out = {}
    for t, c, g, p in zip(target.tolist(), code.tolist(), tag.tolist(), payload.tolist()):
        out.setdefault(t, []).append((c, g, p))
    return out


def _check_close(E, O, clients):
    closed, ev = E.sessions_close(clients, capacity=1 << 18)
    for c in clients:
        O.session_close(int(c))
    oe = O.take_events()
    assert (ev["pos"] == CLOSE_POS).all() and (ev["src"] == abi.CC_EVSRC_CLOSE).all()
    assert (oe["src"] == abi.CC_EVSRC_CLOSE).all()
    got = _per_target(ev["target"], ev["code"], ev["tag"], ev["payload"])
    want = _per_target(oe["target"], oe["code"], oe["tag"], oe["payload"])
    assert got == want
    return closed, ev


def _open_slots(E, O, R, K):
    """Instance slots still registered, checked equal on both sides (a close that throws ends its client's loop)."""
    ids = [1000 + i for i in range(R * K)]
    e = np.array([E.instance_slot(i) >= 0 for i in ids])
    o = np.array([O.inst_slot_of(i) >= 0 for i in ids])
    assert np.array_equal(e, o), np.nonzero(e != o)[0][:10]
    return np.nonzero(e)[0].astype(np.uint32)


def _follow_up(b, types, K, max_inst, open_inst):
    """A batch on the same instances whose lock rows on still-open instances become isLeader (UNKNOWN_OP on a lock):
    the generator's lock client model does not know about the closes."""
    res = np.where(b.inst < len(types) * K, b.inst // K, 0)
    is_lock = (types[np.minimum(res, len(types) - 1)] == L) & (b.inst < len(types) * K)
    live = np.isin(b.inst, open_inst)
    b.op[is_lock & live] = abi.CC_OP_ELECT_ISLEADER
    return b


@pytest.mark.parametrize("R,K,n,seed", [(8, 3, 500, 1), (64, 5, 20_000, 2), (1200, 4, 200_000, 3)])
def test_close_fanout_random(R, K, n, seed):
    """Random coordination state, then clients closed one and two at a time; value listeners, election hand-overs
    and group leaves are compared per target; later commits on closed instances are UNKNOWN_SESSION."""
    from copycat_amd.workload import coord_random_stream

    types = np.array([L, E_, G, V] * ((R + 3) // 4), np.uint8)[:R]
    E, O, max_inst = _setup(types, K, FLAGS)
    b = coord_random_stream(n, types, K, max_inst, seed=seed)
    _check_batch(E, O, b)
    clients = [7 + k for k in range(K)]  # _setup: instance r*K+k belongs to client 7+k
    rng = np.random.default_rng(seed)
    rng.shuffle(clients)
    to_close = [clients[:1], clients[1:3]]
    before = len(_open_slots(E, O, R, K))
    total = 0
    for group in to_close:
        closed, _ = _check_close(E, O, group)
        total += closed
    open_inst = _open_slots(E, O, R, K)
    assert total == before - len(open_inst) and total > 0  # (Delete rows leave cleaned leaders: their close throws)
    _check_state(E, O, types)
    closed_inst = np.setdiff1d(np.arange(R * K, dtype=np.uint32), open_inst)
    b2 = coord_random_stream(max(n // 2, 200), types, K, max_inst, seed=seed + 100, index0=n + 1)
    b2.time[:] = np.maximum(b2.time, b.time[-1])
    b2 = _follow_up(b2, types, K, max_inst, open_inst)
    s, _, _ = _check_batch(E, O, b2)
    on_closed = np.isin(b2.inst, closed_inst)
    assert on_closed.any() and (abi.status_code(s[on_closed]) == abi.CC_ST_UNKNOWN_SESSION).all()
    _check_state(E, O, types)
    # a client with no open instance closes nothing
    closed, ev = _check_close(E, O, [to_close[0][0], 999])
    assert closed == 0 and len(ev["pos"]) == 0


def test_close_unknown_session_after_close():
    from copycat_amd.batch import Batch

    types = np.array([V, E_, G], np.uint8)
    K = 2
    E, O, max_inst = _setup(types, K, FLAGS)
    n = 6
    b = Batch.from_columns(index=np.arange(1, n + 1), time=np.ones(n), inst=np.arange(n),
                           op=np.array([abi.CC_OP_VALUE_LISTEN, abi.CC_OP_VALUE_SET, abi.CC_OP_ELECT_LISTEN,
                                        abi.CC_OP_ELECT_LISTEN, abi.CC_OP_GROUP_JOIN, abi.CC_OP_GROUP_JOIN], np.uint8),
                           flags=np.full(n, abi.cc_flags(abi.CC_TAG_LONG, 0, 0), np.uint8), a=np.full(n, 5))
    _check_batch(E, O, b)
    _check_close(E, O, [7])  # instances 0, 2, 4 (k = 0)
    b2 = Batch.from_columns(index=np.arange(n + 1, 2 * n + 1), time=np.ones(n), inst=np.arange(n),
                            op=np.array([abi.CC_OP_VALUE_GET, abi.CC_OP_VALUE_GET, abi.CC_OP_ELECT_ISLEADER,
                                         abi.CC_OP_ELECT_ISLEADER, abi.CC_OP_GROUP_LEAVE, abi.CC_OP_GROUP_LEAVE], np.uint8))
    s, v, _ = E.apply_host_events(b2)
    assert [abi.status_code(x) for x in s] == [abi.CC_ST_UNKNOWN_SESSION, abi.CC_ST_OK] * 3
    s2, v2 = O.apply(b2)
    assert np.array_equal(s, s2) and np.array_equal(v, v2)
    O.take_events()
    _check_state(E, O, types)


@pytest.mark.parametrize("S,seed", [(64, 1), (5000, 2)])
def test_expire_sweep_then_fanout(S, seed):
    """cc_expire_sweep's bitmap over client sessions -> cc_sessions_expire closes the expired clients in ascending
    id order (ResourceManager.expire :238-247, then Copycat's close); the oracle closes the same ids one by one."""
    import torch

    from copycat_amd.engine import expire_sweep
    from copycat_amd.workload import coord_random_stream

    R, K = 40, 6
    types = np.array([L, E_, G, V] * (R // 4), np.uint8)
    E, O, max_inst = _setup(types, K, FLAGS)
    _check_batch(E, O, coord_random_stream(30_000, types, K, max_inst, seed=seed))
    rng = np.random.default_rng(seed)
    now, timeout = 1_000_000, 5000
    last = (now - rng.integers(0, 2 * timeout, S)).astype(np.uint64)
    last[7:7 + K] = now - np.array([10, 9000, 6000, 1, 7000, 2], np.uint64)  # clients 8, 9, 11 expire
    d_last = torch.from_numpy(last.view(np.int64)).cuda()
    d_bm = torch.zeros((S + 63) // 64, dtype=torch.int64, device="cuda")
    d_cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    expire_sweep(d_last, now, timeout, d_bm, d_cnt)
    torch.cuda.synchronize()
    closed, ev = E.sessions_expire(d_bm, S, capacity=1 << 16)
    expired = [s for s in range(S) if now - int(last[s]) > timeout]
    for s in expired:
        O.session_expire(s)
    oe = O.take_events()
    open_inst = _open_slots(E, O, R, K)
    assert closed == R * K - len(open_inst) and closed > 0
    got = _per_target(ev["target"], ev["code"], ev["tag"], ev["payload"])
    want = _per_target(oe["target"], oe["code"], oe["tag"], oe["payload"])
    assert got == want
    _check_state(E, O, types)
