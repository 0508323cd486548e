"""GPU parity of the quorum commit-index kernel and the session expiry sweep vs the oracle (bit-exact)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _t(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).cuda().view(torch.uint64)


def _h(t):
    import torch

    return t.view(torch.int64).cpu().numpy().view(np.uint64)


@pytest.mark.parametrize("groups,replicas", [(1, 5), (2, 5), (1001, 5), (1 << 20, 5), (4096, 3), (4097, 7), (999, 4), (64, 1)])
def test_quorum_parity(groups, replicas):
    import torch

    from copycat_amd.engine import quorum_commit
    from copycat_amd.workload import quorum_groups
    from oracle.oracle_py import quorum_commit as oq

    match, ts, ci = quorum_groups(groups, replicas=replicas, seed=groups + replicas)
    out = torch.zeros(groups, dtype=torch.int64, device="cuda")
    quorum_commit(_t(match), _t(ts), _t(ci), out)
    torch.cuda.synchronize()
    assert np.array_equal(_h(out), oq(match, ts, ci))


@pytest.mark.parametrize("sessions", [1, 63, 64, 127, 128, 129, 100_000, 1 << 20])
def test_expiry_parity(sessions):
    import torch

    from copycat_amd.engine import expire_sweep
    from copycat_amd.workload import expiry_sessions
    from oracle.oracle_py import expire_sweep as oe

    last, now, timeout = expiry_sessions(sessions, seed=sessions)
    last[: min(3, sessions)] = now + 5  # keep-alive stamped in the future never expires
    words = (sessions + 63) // 64
    bm = torch.zeros(words, dtype=torch.int64, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    expire_sweep(_t(last), now, timeout, bm, cnt)
    torch.cuda.synchronize()
    ebm, ec = oe(last, now, timeout)
    assert np.array_equal(_h(bm), ebm)
    assert int(_h(cnt)[0]) == ec
