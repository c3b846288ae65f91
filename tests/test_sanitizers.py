"""Host sanitizers over the CPU code:
* AddressSanitizer + UndefinedBehaviorSanitizer over the generator, the CPU builders and NN
  searches, and the global decomposition's planner (csrc/cpu/global_plan.cpp: segment,
  make_layout, share_blocks, make_plan swept over P = 1..64, k = -1..6, n up to 2^32 - 1 with
  random per-leaf counts; csrc/tests/sanitize_main.cpp);
* ThreadSanitizer over the loopback communicator's thread hand-offs (pkdtree/loopback.hpp,
  csrc/tests/tsan_loopback.cpp).
Any report fails the test. GPU sanitizers are not available on the target pool (see README)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_asan_ubsan_cpu_paths(tmp_path):
    exe = tmp_path / "sanitize"
    srcs = [os.path.join(ROOT, "csrc", "cpu", f) for f in ("generator.cpp", "cpu_tree.cpp", "global_plan.cpp")]
    srcs.append(os.path.join(ROOT, "csrc", "tests", "sanitize_main.cpp"))
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-I", os.path.join(ROOT, "csrc", "include"), *srcs, "-o", str(exe),
           "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "sanitize ok" in r.stdout and "layouts ok" in r.stdout


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_tsan_loopback_communicator(tmp_path):
    exe = tmp_path / "tsan_loopback"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-I", os.path.join(ROOT, "csrc", "include"),
           os.path.join(ROOT, "csrc", "tests", "tsan_loopback.cpp"), "-o", str(exe), "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1:exitcode=66")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "tsan loopback ok" in r.stdout and "ThreadSanitizer" not in r.stderr
