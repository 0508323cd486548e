"""Diagnostics: the first row where test_map_contains_value_in_stream_parity[302] differs, with its context."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from copycat_amd import abi  # noqa: E402
from copycat_amd.batch import Batch  # noqa: E402
from copycat_amd.workload import map_random_stream  # noqa: E402
from tests.test_gpu_map import _cv_rows, _engines  # noqa: E402

n, maps, keys, sub_batch, hot, p_hot, seed = 100_000, 16, 64, 8192, 2, 0.3, 302
max_inst = maps + 8
b = map_random_stream(n, maps, max_inst, keys=keys, seed=seed, hot=hot, p_hot=p_hot)
even = (b.inst % 2) == 0
f = b.flags
ta, tb = f & 7, (f >> 3) & 7
f[even & (ta == abi.CC_TAG_NULL)] |= np.uint8(abi.CC_TAG_LONG)
f[even & (tb == abi.CC_TAG_NULL)] |= np.uint8(abi.CC_TAG_LONG << 3)
rows = _cv_rows(b, 0.02, seed, clear_rate=0.0005)
mid = n // 2
b.op[mid], b.inst[mid], b.flags[mid] = abi.CC_OP_MAP_PUT, 0, np.uint8(abi.CC_TAG_NULL)
E, O = _engines(maps, max_inst, n, 65536, sub_batch=sub_batch)
gs, gv = E.apply_host(b)
os_, ov = O.apply(b)
bad = np.nonzero((gs != os_) | (gv != ov))[0]
print("bad rows", bad[:10], "counters", E.counters())
for r in bad[:3]:
    m = int(b.inst[r])
    print("row", r, "op", b.op[r], "map", m, "tag", b.flags[r] & 7, "a", b.a[r], "gpu", gs[r], gv[r], "oracle", os_[r], ov[r])
    cl = np.nonzero((b.op == abi.CC_OP_MAP_CLEAR) & (b.inst == m))[0]
    print("  clears of the map", cl, "sub-batch", r // sub_batch, "sub-batch start", (r // sub_batch) * sub_batch)
    nul = np.nonzero((b.inst == m) & np.isin(b.op, [62, 63, 68, 69]) & ((b.flags & 7) == 0))[0]
    print("  null stores of the map", nul[:10])
    # the writes of value a on this map before r (last 3000 rows)
    w = np.nonzero((b.inst[:r] == m) & (b.a[:r] == b.a[r]) & np.isin(b.op[:r], [62, 63, 68, 69]) & ((b.flags[:r] & 7) == (b.flags[r] & 7)))[0]
    print("  writes of the operand on the map", w[-8:], "keys", b.key[w[-8:]], "ktags", (b.flags[w[-8:]] >> 6) & 3, "ops", b.op[w[-8:]])
    for k in set(b.key[w[-4:]].tolist()):
        kr = np.nonzero((b.inst[:r + 1] == m) & (b.key[:r + 1] == k))[0]
        print("   key", k, "rows", kr[-10:], "ops", b.op[kr[-10:]], "a", b.a[kr[-10:]], "kt", (b.flags[kr[-10:]] >> 6) & 3)
r = int(bad[0])
m = int(b.inst[r])
seg = np.nonzero((b.inst[44000:r + 1] == m))[0] + 44000
for i in seg:
    if i >= 44400:
        print(" ", i, "op", b.op[i], "key", np.int64(b.key[i]), "kt", (b.flags[i] >> 6) & 3, "ta", b.flags[i] & 7, "a", np.int64(b.a[i]), "gpu", gs[i], np.int64(gv[i]), "orc", os_[i], np.int64(ov[i]))
