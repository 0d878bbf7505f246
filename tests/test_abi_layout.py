"""The ctypes structures of the Python binding against the C headers they
mirror (include/*.h): every struct's size and every field's offset, from a
small C program gcc compiles against the headers. A field the binding moved or
resized would otherwise only show up as wrong numbers on the GPU. No GPU."""
import ctypes as C
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "roborts-edu-slam_amd"))


def _structs():
    from roborts_csm import _abi, backend, frontend
    return [
        ("csm.h", "csm_param", _abi.CsmParam),
        ("csm.h", "csm_map_info", _abi.CsmMapInfo),
        ("csm.h", "csm_best", _abi.CsmBest),
        ("csm.h", "csm_kernel_stat", _abi.CsmKernelStat),
        ("csm.h", "csm_optimize_param", _abi.CsmOptimizeParam),
        ("csm.h", "csm_search_options", _abi.CsmSearchOptions),
        ("csm.h", "csm_search_stats", _abi.CsmSearchStats),
        ("csm_gridmap.h", "csm_gridmap_state", _abi.CsmGridmapState),
        ("csm_loop_closure.h", "csm_loop_closure_result", _abi.CsmLoopClosureResult),
        ("csm_backend.h", "csm_backend_param", backend.CsmBackendParam),
        ("csm_backend.h", "csm_backend_job", backend.CsmBackendJob),
        ("csm_frontend.h", "csm_frontend_param", frontend.CsmFrontendParam),
        ("csm_frontend.h", "csm_frontend_result", frontend.CsmFrontendResult),
    ]


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc")
def test_ctypes_layout_matches_headers(tmp_path):
    structs = _structs()
    headers = sorted({h for h, _, _ in structs})
    lines = ["#include <stdio.h>", "#include <stddef.h>"] + [f'#include "{h}"' for h in headers]
    lines.append("int main(void) {")
    for _, cname, cls in structs:
        lines.append(f'  printf("{cname} size %zu\\n", sizeof({cname}));')
        for fname, _ in cls._fields_:
            lines.append(f'  printf("{cname} {fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("  return 0;\n}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines) + "\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = {}
    for line in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.splitlines():
        cname, key, val = line.split()
        got[(cname, key)] = int(val)
    for _, cname, cls in structs:
        assert got[(cname, "size")] == C.sizeof(cls), cname
        for fname, _ in cls._fields_:
            assert got[(cname, fname)] == getattr(cls, fname).offset, (cname, fname)
