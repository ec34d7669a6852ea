"""Host runtime under sanitizers: the native self-test
(csrc/host/tests/selftest.cpp) statically links every host source and is run
once under AddressSanitizer + UndefinedBehaviorSanitizer and once under
ThreadSanitizer (the persistent thread pool and every parallel_for user).
GPU sanitizers are not available on this pool; the HIP kernels are covered by
the numerics tests in test_gpu_kernels.py instead."""
import glob
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "build", "sanitize")
SRCS = sorted(glob.glob(os.path.join(ROOT, "csrc", "host", "*.cpp"))) + [
    os.path.join(ROOT, "csrc", "host", "tests", "selftest.cpp")]
DEPS = SRCS + glob.glob(os.path.join(ROOT, "csrc", "host", "*.h"))
FLAVOURS = {
    "asan_ubsan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"],
    "tsan": ["-fsanitize=thread"],
}

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")


def _build(name: str) -> str:
    os.makedirs(BUILD, exist_ok=True)
    exe = os.path.join(BUILD, f"selftest_{name}")
    if not os.path.exists(exe) or any(os.path.getmtime(s) > os.path.getmtime(exe) for s in DEPS):
        cmd = ["g++", "-O1", "-g", "-std=c++17", "-pthread", "-mpopcnt", "-fno-omit-frame-pointer",
               *FLAVOURS[name], "-I", os.path.join(ROOT, "csrc", "host"), *SRCS, "-o", exe + ".tmp"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        assert r.returncode == 0, r.stderr[-4000:]
        os.replace(exe + ".tmp", exe)
    return exe


@pytest.mark.parametrize("name", sorted(FLAVOURS))
def test_host_runtime_under_sanitizer(name):
    exe = _build(name)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe, "8"], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0 and "selftest ok" in r.stdout, (r.stdout[-2000:], r.stderr[-6000:])
