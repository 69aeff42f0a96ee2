"""Host-side sanitizer runs of the native runtime (race detection / sanitizers).

The clip reader's thread pool + pread core (csrc/runtime/clip_reader_core.h) is compiled standalone with
ThreadSanitizer and with AddressSanitizer+UBSan and stress-tested with random job mixes.  GPU sanitizers
are not available on the MI355X pool; device code is covered by numerics tests instead."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "clip_reader_test.cpp")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_clip_reader_under_sanitizer(tmp_path, san):
    exe = tmp_path / "clip_reader_test"
    cmd = ["g++", "-std=c++17", "-O1", "-g", f"-fsanitize={san}", "-fno-omit-frame-pointer", SRC, "-o", str(exe),
           "-pthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="detect_leaks=1:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([str(exe), str(tmp_path)], capture_output=True, text=True, env=env, timeout=300)
    if san == "thread" and "unexpected memory mapping" in r.stderr:
        pytest.skip("ThreadSanitizer cannot map shadow memory in this kernel configuration")
    assert r.returncode == 0 and "clip_reader_test ok" in r.stdout, r.stdout + r.stderr
