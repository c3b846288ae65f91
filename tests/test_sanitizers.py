"""Host sanitizers over the CPU code: csrc/cpu/*.cpp + csrc/tests/sanitize_main.cpp
built with -fsanitize=address,undefined and run; any report fails the test. GPU sanitizers are
not available on the target pool (see README)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_asan_ubsan_cpu_paths(tmp_path):
    exe = tmp_path / "sanitize"
    srcs = [os.path.join(ROOT, "csrc", "cpu", f) for f in ("generator.cpp", "cpu_tree.cpp")]
    srcs.append(os.path.join(ROOT, "csrc", "tests", "sanitize_main.cpp"))
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-I", os.path.join(ROOT, "csrc", "include"), *srcs, "-o", str(exe),
           "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "sanitize ok" in r.stdout
