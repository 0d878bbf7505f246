"""CPU: the C-ABI library loads, exports every symbol include/*.h declare,
and its host-only entry points behave (no compute calls without a GPU)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from roborts_csm import _abi
from roborts_csm.params import (CONFIG1_PARAM, FAST_PARAM, IN_CLASS_LEVELS, PARAM_CONFIG_LEVELS,
                                SIM_YAML_LEVELS)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    names = set()
    for h in sorted(f for f in os.listdir(os.path.join(ROOT, "include")) if f.endswith(".h")):
        txt = open(os.path.join(ROOT, "include", h)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        names |= set(re.findall(r"\b(csm_[a-z_0-9]+)\s*\(", txt))
    return sorted(names)


def test_library_exports_every_declared_symbol():
    lib = C.CDLL(_abi.LIB_PATH)
    declared = _declared()
    assert declared, "no declarations parsed"
    for name in declared:
        assert hasattr(lib, name), name
    assert sorted(_abi.EXPORTED) == declared


def test_abi_version_and_struct_sizes():
    lib = _abi.load_library()
    assert lib.csm_abi_version() == 1
    assert C.sizeof(_abi.CsmParam) == 5 * 8 + 4 * 4
    assert C.sizeof(_abi.CsmMapInfo) == 3 * 8 + 4 * 4
    assert C.sizeof(_abi.CsmBest) == 5 * 8


@pytest.mark.parametrize("p,expect", [
    (CONFIG1_PARAM, (16, 21)),                                  # BASELINE config 1
    (SIM_YAML_LEVELS[0], (30, 13)),
    (SIM_YAML_LEVELS[1], (11, 11)),
    (SIM_YAML_LEVELS[2], (21, 3)),
    (PARAM_CONFIG_LEVELS[0], (101, 9)),
    (IN_CLASS_LEVELS[0], (81, 9)),
    (FAST_PARAM, (300, 81)),
])
def test_window_dims(p, expect):
    import roborts_csm
    assert roborts_csm.window_dims(p) == expect


def test_window_dims_rejects_bad_params():
    lib = _abi.load_library()
    p = CONFIG1_PARAM.with_(search_angle_resolution=0.0).to_c()
    a, b = C.c_int32(), C.c_int32()
    assert lib.csm_window_dims(C.byref(p), C.byref(a), C.byref(b)) == _abi.CSM_ERR_INVALID_ARG


def test_create_without_gpu_fails_cleanly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    lib = _abi.load_library()
    h = C.c_void_p()
    assert lib.csm_create(0, C.byref(h)) == _abi.CSM_ERR_HIP
    assert not h.value
    assert lib.csm_last_error(None) == b"null context"


def test_package_import_is_loud_about_missing_library(tmp_path):
    with pytest.raises(OSError):
        _abi.load_library(str(tmp_path / "nope.so"))


def test_loop_closure_create_without_gpu_fails_cleanly():
    """csm_loop_closure_create loads RCCL privately, then fails on the
    missing device with a message (no crash, no partial handle leak)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from roborts_csm import CsmError
    from roborts_csm.loop_closure import DeviceLoopClosure
    with pytest.raises(CsmError):
        DeviceLoopClosure([0])
