"""Config 1 (BASELINE.json configs[0]) restated: examples/atomic-value (AtomicValueExample.java:38-69) against three
in-process replicas.  The client creates "atomic" (ResourceManager.createResource, ResourceManager.java:148-196) and
loops set(random UUID) -> get() -> schedule 1 s (AtomicValueExample.java:62-69).  Raft hands every replica the same
committed log, so the three replicas' state machines must produce identical results and state; here each replica is
one CPU oracle (and, on the GPU box, the engine is a fourth replica fed the same log).

The Java example cannot run here (no JVM); this is the plumbing check §8(d) c1 asks for."""
import uuid

import numpy as np
import pytest

from copycat_amd import abi
from copycat_amd.batch import Batch, Interner

KEY = "atomic"
CLIENT = 1
ITERS = 200


def committed_log(seed=1):
    """The example's committed entries: (CreateResource at index 1) then per iteration Set(UUID) and Get, 1 s apart."""
    rnd = np.random.default_rng(seed)
    intern = Interner()
    key = intern(KEY)
    values = [str(uuid.UUID(bytes=rnd.bytes(16), version=4)) for _ in range(ITERS)]
    b = Batch(2 * ITERS)
    for i, v in enumerate(values):
        for j, (op, a) in enumerate(((abi.CC_OP_VALUE_SET, intern(v)), (abi.CC_OP_VALUE_GET, None))):
            r = 2 * i + j
            b.index[r] = 2 + r
            b.time[r] = 1000 * i
            b.op[r] = op
            b.flags[r] = abi.cc_flags(abi.CC_TAG_HANDLE if a is not None else abi.CC_TAG_NULL, 0, 0)
            b.a[r] = a.h if a is not None else 0
    return key.h, b, [intern(v).h for v in values]


class OracleReplica:
    def __init__(self):
        from oracle.oracle_py import Oracle

        self.O = Oracle(16, 16)

    def create(self, key, index):
        st, iid, slot = self.O.create_resource(key, abi.CC_RES_VALUE, CLIENT, index)
        return st, iid, slot

    def apply(self, b):
        return self.O.apply(b)

    def state(self, iid):
        return tuple(int(x[0]) for x in self.O.value_state(self.O.L.orc_res_slot_of(self.O.h, iid), 1))


def _run(replicas):
    key, log, handles = committed_log()
    outs = []
    for rep in replicas:
        st, iid, slot = rep.create(key, 1)
        assert abi.status_code(st) == abi.CC_ST_OK and iid == 1  # instance id = the CreateResource commit's index
        b = Batch.from_columns(**log.columns())
        b.inst[:] = slot
        s, v = rep.apply(b)
        outs.append((s, v, rep.state(iid)))
    for s, v, state in outs[1:]:
        assert np.array_equal(s, outs[0][0]) and np.array_equal(v, outs[0][1]) and state == outs[0][2]
    s, v, state = outs[0]
    gets = slice(1, None, 2)
    # every get returns the value the example's preceding set wrote (AtomicValueState.get :77-83)
    assert (abi.status_tag(s[gets]) == abi.CC_TAG_HANDLE).all() and v[gets].tolist() == handles
    assert state == (abi.CC_TAG_HANDLE, handles[-1], 1)


def test_three_oracle_replicas_agree(oracle_lib):
    _run([OracleReplica() for _ in range(3)])


class EngineReplica:
    def __init__(self):
        from copycat_amd.engine import Engine

        self.E = Engine(16, 16, 1 << 12)

    def create(self, key, index):
        return self.E.create_resource(key, abi.CC_RES_VALUE, CLIENT, index)

    def apply(self, b):
        return self.E.apply_host(b)

    def state(self, iid):
        return tuple(int(x[0]) for x in self.E.value_state(self.E.resource_slot(iid), 1))


@pytest.mark.gpu
def test_engine_is_a_fourth_replica():
    _run([OracleReplica(), OracleReplica(), OracleReplica(), EngineReplica()])
