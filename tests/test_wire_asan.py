"""cc_wire_decode (copycat_amd/csrc/wire.cpp) under AddressSanitizer + UndefinedBehaviorSanitizer, host only.

The decoder parses committed log bytes (InstanceOperation.writeObject/readObject,
manager/src/main/java/io/atomix/resource/InstanceOperation.java:59-69), i.e. untrusted input.  tests/fuzz/wire_fuzz.cpp
decodes the committed fixture, every truncation of every fixture entry and 200,000 random mutations (byte flips,
splices, garbage, 0xFF length runs, random codec parameters), each from an exact-size heap copy: any overread, leak or
undefined behaviour aborts the run; every input must come back CC_OK or CC_ERR_INVALID."""
import json
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_wire_decode_asan_ubsan_fuzz(tmp_path):
    exe = tmp_path / "wire_fuzz"
    cmd = [HIPCC, "-std=c++17", "-g", "-O1", "-fsanitize=address,undefined", "-fno-gpu-sanitize",
           "-fno-sanitize-recover=all", f"-I{ROOT}/copycat_amd/csrc", f"-I{ROOT}/include",
           f"{ROOT}/copycat_amd/csrc/wire.cpp", f"{HERE}/fuzz/wire_fuzz.cpp", "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    with open(os.path.join(HERE, "golden", "wire_fixture.json")) as f:
        offs = json.load(f)["offsets"]
    (tmp_path / "offs.txt").write_text(" ".join(map(str, offs)))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe), os.path.join(HERE, "golden", "wire_fixture.bin"), str(tmp_path / "offs.txt"),
                        "200000"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr
    assert "decoded" in r.stdout
    shutil.rmtree(tmp_path, ignore_errors=True)
