"""copycat_amd — MI355X-native batched commit-apply engine for the Atomix/Copycat state-machine hot path.

The product is `libcopycat_apply.so` (hand-written gfx950 HIP kernels behind the C-ABI of
include/copycat_apply.h).  This package holds the host half of the boundary: the column encoder
(`batch`), the ctypes binding of the C-ABI (`engine`), and the synthetic workload generators (`workload`).
"""
from . import abi  # noqa: F401
from .batch import Batch, Encoder, Handle, Int, Interner, tagged, untagged  # noqa: F401
