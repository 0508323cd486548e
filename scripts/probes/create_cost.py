"""Control-plane cost probe: wall time of 32,768 cc_create_resource calls (lock / election / group in turn) on a
coordination engine, then one tiny batch (the queued registry writes are applied before it)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from copycat_amd import abi  # noqa: E402
from copycat_amd.engine import Engine  # noqa: E402

R = 32768
kinds = [abi.CC_RES_LOCK, abi.CC_RES_ELECTION, abi.CC_RES_GROUP]
E = Engine(R + 256, R + 1024, 1 << 20, flags=abi.CC_CFG_TIMERS_DEFERRED, max_events=1 << 20)
t0 = time.perf_counter()
for r in range(R):
    st, iid, islot = E.create_resource(r + 1, kinds[r % 3], 1, 1000 + r)
    assert abi.status_code(st) == abi.CC_ST_OK
t1 = time.perf_counter()
E.sync()
t2 = time.perf_counter()
print(f"{R} creates: {(t1 - t0) * 1e6 / R:.2f} us each, flush+sync {(t2 - t1) * 1e3:.2f} ms")
