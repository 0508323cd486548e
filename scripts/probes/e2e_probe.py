"""Where does a PCIe-inclusive c2 step spend its time?  Each stage synchronized and timed on the host."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from copycat_amd import abi  # noqa: E402
from copycat_amd.batch import Batch  # noqa: E402
from copycat_amd.engine import DeviceBatch, Engine  # noqa: E402
from copycat_amd.workload import AtomicLongClients  # noqa: E402

n, R = 100_000_000, 65536
dev = torch.device("cuda", 0)
E = Engine(R, R, n)
E.resource_create_range(0, R, abi.CC_RES_VALUE)
E.instance_open_range(0, R, 0, 1, 1)
host = AtomicLongClients(R).next(n, out=Batch(n))
names = ("index", "inst", "op", "flags", "a", "b")
tdt = {"index": torch.int64, "inst": torch.int32, "op": torch.uint8, "flags": torch.uint8, "a": torch.int64, "b": torch.int64}
for rep in range(3):
    t = time.perf_counter()
    pinned = {k: torch.from_numpy(getattr(host, k).view(np.dtype(str(tdt[k]).replace("torch.", "")))).pin_memory() for k in names}
    print("pin", time.perf_counter() - t)
    dcols = {k: torch.empty(n, dtype=tdt[k], device=dev) for k in names}
    st, va = torch.empty(n, dtype=torch.uint8, device=dev), torch.empty(n, dtype=torch.int64, device=dev)
    hs, hv = torch.empty(n, dtype=torch.uint8).pin_memory(), torch.empty(n, dtype=torch.int64).pin_memory()
    torch.cuda.synchronize()
    cs = torch.cuda.current_stream()
    t0 = time.perf_counter()
    for k in names:
        dcols[k].copy_(pinned[k], non_blocking=True)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    E.apply(DeviceBatch(dcols, n), st, va, stream=cs)
    t2 = time.perf_counter()
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    hs.copy_(st, non_blocking=True)
    hv.copy_(va, non_blocking=True)
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    print(f"h2d {1e3*(t1-t0):.1f} ms, apply enqueue {1e3*(t2-t1):.1f} ms, apply run {1e3*(t3-t2):.1f} ms, d2h {1e3*(t4-t3):.1f} ms")
