"""The host-memory boundary a JVM binds, exercised in a fresh interpreter without torch.

tests/host_boundary_check.py binds libcopycat_apply.so with bare ctypes and runs a lock / election / group / value
listener stream through cc_apply_batch_host_events, then the session close / expire fan-out, the schedule timers and
the compaction bitmap through their *_host forms, and a quorum commit through the plain device-memory API, comparing
every result and every event per target session with the oracle (Session.publish -> InstanceEvent,
ManagedResourceSession.java:64-71, InstanceEvent.java:29-80)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_host_event_path_without_torch():
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "host_boundary_check.py")], cwd=ROOT,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "host boundary ok" in r.stdout
