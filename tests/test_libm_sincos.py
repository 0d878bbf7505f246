"""glibc 2.35's sincos restated (roborts-edu-slam_amd/csrc/libm_sincos.hpp,
the code the device's angle rows run) against this machine's ::sincos on the
CPU: tools/ubench/sincos_check.cpp compiled with the library's host flags
(-O2 -ffp-contract=off), the table located in the process's libm as the
library does, 8 M seeded arguments over every branch plus each branch
threshold's neighbours; tolerance 0 (bit-equal sin and cos). The GPU side of
the same code is tests/test_gpu_sincos.py.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("sincos") / "sincos_check")
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-fno-fast-math", "-std=c++17", "-pthread",
                    "-I", os.path.join(ROOT, "roborts-edu-slam_amd", "csrc"),
                    os.path.join(ROOT, "tools", "ubench", "sincos_check.cpp"), "-o", exe, "-ldl"], check=True)
    return exe


def test_restated_sincos_equals_host_libm(checker):
    r = subprocess.run([checker, "2000000", "4"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout


def test_restated_sincos_detects_a_wrong_constant(checker, tmp_path):
    """The check has teeth: the restatement with pi/2's low word off by one
    unit differs from the host's sincos."""
    src = os.path.join(ROOT, "roborts-edu-slam_amd", "csrc")
    for f in ("libm_sincos.hpp", "libm_sincos_table.hpp"):
        text = open(os.path.join(src, f)).read()
        if f == "libm_sincos.hpp":
            assert "0x3c91a62633145c07ull" in text
            text = text.replace("0x3c91a62633145c07ull", "0x3c91a62633145c06ull")
        (tmp_path / f).write_text(text)
    exe = str(tmp_path / "mutant")
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-std=c++17", "-pthread", "-I", str(tmp_path),
                    os.path.join(ROOT, "tools", "ubench", "sincos_check.cpp"), "-o", exe, "-ldl"], check=True)
    r = subprocess.run([exe, "500000", "2"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 1 and "mismatches 0" not in r.stdout
