"""Sanitizer runs of the native host runtime (race detection / sanitizers).

The reference has no sanitizers or determinism checks.  The threaded CIFAR-10 decoder and the
sampler index math (csrc/runtime/core.cpp) are compiled standalone, with the self-test driver
csrc/selftest/runtime_selftest.cpp, under AddressSanitizer + UndefinedBehaviorSanitizer and
under ThreadSanitizer, and executed on the CPU.  (GPU sanitizers are not available on the
MI355X pool; device-side determinism is covered by the GPU tests.)
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = [d for d in os.listdir(ROOT) if d.endswith("_amd") and os.path.isdir(os.path.join(ROOT, d))][0]
CSRC = os.path.join(ROOT, PKG, "csrc")
CXX = shutil.which("g++") or shutil.which("clang++")


@pytest.mark.skipif(CXX is None, reason="no host C++ compiler")
@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_runtime_under_sanitizer(tmp_path, san):
    exe = tmp_path / "selftest"
    cmd = [CXX, "-std=c++17", "-O1", "-g", f"-fsanitize={san}", "-fno-omit-frame-pointer", "-pthread",
           os.path.join(CSRC, "runtime", "core.cpp"), os.path.join(CSRC, "selftest", "runtime_selftest.cpp"),
           "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0 and "sanitize" in (r.stderr or ""):
        pytest.skip(f"toolchain lacks -fsanitize={san}: {r.stderr[-300:]}")
    assert r.returncode == 0, r.stderr
    data = tmp_path / "data"
    data.mkdir()
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", TSAN_OPTIONS="halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([str(exe), str(data)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0 and "selftest ok" in r.stdout, (r.returncode, r.stdout, r.stderr[-2000:])
