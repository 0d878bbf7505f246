"""The CPU oracle under AddressSanitizer + UBSan (SURVEY §5's sanitizer
auxiliary): oracle/san_driver.cpp drives every matcher entry point the parity
tests use -- all three sim-YAML levels, the beam-subsampling edges, beams off
the grid on every side, FAST, std::sort over heavy ties -- and any invalid
access or undefined behaviour aborts it. Host code only: GPU sanitizers are not
available on this pool."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_oracle_clean_under_asan_ubsan():
    b = subprocess.run(["make", "-C", ORACLE, "san"], capture_output=True, text=True, timeout=300)
    if b.returncode != 0 and "sanitize" in b.stderr and "cannot find" in b.stderr:
        pytest.skip("sanitizer runtime not installed")
    assert b.returncode == 0, b.stderr[-2000:]
    env = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:detect_leaks=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", OMP_NUM_THREADS="1")
    r = subprocess.run([os.path.join(ORACLE, "build", "san_driver")], capture_output=True, text=True,
                       timeout=600, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "san_driver ok" in r.stdout
