"""CPU: the reference-side C++ adapter compiles against types shaped like the
reference's (map, range data, param, Eigen vectors)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_adapter_compiles(tmp_path):
    src = os.path.join(ROOT, "tests", "cpp", "adapter_compile.cpp")
    out = tmp_path / "adapter.o"
    r = subprocess.run(["g++", "-std=c++14", "-Wall", "-Werror", "-c", src, "-o", str(out),
                        "-I", os.path.join(ROOT, "include")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
