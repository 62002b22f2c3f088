"""Race detection / memory checking of the native host runtime: the runtime sources and a
multi-threaded stress driver are compiled with ThreadSanitizer and AddressSanitizer (host code only — GPU
sanitizers are not available on this pool) and must run clean."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _build(tmp_path, san):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("g++ not available")
    rt = os.path.join(ROOT, "csrc", "runtime")
    srcs = [os.path.join(rt, f) for f in sorted(os.listdir(rt)) if f.endswith(".cpp")]
    out = str(tmp_path / f"runtime_stress_{san}")
    cmd = [cxx, "-std=c++17", "-O1", "-g", f"-fsanitize={san}", "-fno-omit-frame-pointer", "-pthread",
           f"-I{rt}", os.path.join(ROOT, "csrc", "tools", "runtime_stress.cpp"), *srcs, "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    return out


@pytest.mark.parametrize("san", ["thread", "address"])
def test_runtime_stress_under_sanitizer(tmp_path, san):
    exe = _build(tmp_path, san)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1",
               ASAN_OPTIONS="detect_leaks=1:halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0 and "0 error(s)" in r.stdout, (r.stdout + r.stderr)[-4000:]
    assert "WARNING: ThreadSanitizer" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr
