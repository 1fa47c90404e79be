"""Host runtime under ThreadSanitizer and AddressSanitizer/UBSan: the HTTP server and
client pool, gateway failover, batcher, LRU cache, ring, breaker and JSON codec hammered from many
threads (csrc/tests/stress_main.cpp).  A sanitizer report or a failed check fails the test."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "distributed-inference-engine-cpp_amd", "bin")


@pytest.mark.slow
@pytest.mark.parametrize("kind", ["tsan", "asan"])
def test_stress_under_sanitizer(kind):
    subprocess.run(["make", "stress-" + kind], cwd=REPO, check=True, stdout=subprocess.DEVNULL,
                   stderr=subprocess.STDOUT, timeout=900)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1",
               ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([os.path.join(BIN, "die_stress_" + kind), "1"], stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, timeout=600, env=env)
    out = r.stdout.decode(errors="replace")
    assert r.returncode == 0, out[-4000:]
    for bad in ("ThreadSanitizer", "AddressSanitizer", "runtime error:", "LeakSanitizer"):
        assert bad not in out, out[-4000:]
    assert "stress done: 0 check failures" in out
