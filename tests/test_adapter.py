"""The reference-side C++ adapter (include/csm_reference_adapter.hpp).

CPU: it compiles against types shaped like the reference's, and it runs its
error path (no usable device): logs, returns 0.0 (kMinResponse), pose and
covariance untouched, no exception (correlate_scan_matcher.h:790-795).
GPU: tests/cpp/adapter_run drives it like ScanMatchers::ScanMatch
(scan_matchers.h:238,249,256) over a map mutated between scans (cell updates,
resets, ExtendSize), and every level is compared with the oracle bit for bit.
"""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "build", "adapter_run")


def test_adapter_compiles(tmp_path):
    src = os.path.join(ROOT, "tests", "cpp", "adapter_compile.cpp")
    out = tmp_path / "adapter.o"
    r = subprocess.run(["g++", "-std=c++14", "-Wall", "-Werror", "-c", src, "-o", str(out),
                        "-I", os.path.join(ROOT, "include")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def _binary():
    if not os.path.exists(BIN):
        pytest.skip("tests/cpp/build/adapter_run not built (__graft_entry__.build() builds it)")
    return BIN


def test_adapter_error_path_runs_without_throwing():
    r = subprocess.run([_binary(), "nodevice"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out == {"response": 0, "logged": 1, "ok": 1}


@pytest.mark.gpu
def test_adapter_three_levels_bit_exact_on_device():
    r = subprocess.run([_binary(), "check", "24"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["mismatches"] == 0 and out["incremental_refreshes"] > 0 and out["whole_uploads"] > 1
