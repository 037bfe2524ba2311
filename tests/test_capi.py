"""The C-ABI library builds for gfx950, loads, and exports every entry point include/whisper_mi355.h declares
(no compute calls: there is no GPU in the CPU test environment)."""
import os
import re
import subprocess

import pytest

from vlog_amd import _capi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    text = open(os.path.join(ROOT, "include", "whisper_mi355.h")).read()
    return sorted(set(re.findall(r"\b(wm_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_header_symbols():
    if not os.path.isfile(_capi.LIB_PATH):
        subprocess.run(["make", "-C", os.path.join(ROOT, "vlog_amd", "csrc"), "-j8"], check=True)
    out = subprocess.run(["nm", "-D", "--defined-only", _capi.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (wm_\w+)", out))
    declared = _header_symbols()
    assert declared and set(declared) <= exported, set(declared) - exported
    assert set(declared) == set(_capi.SYMBOLS)


def test_library_loads_and_reports_abi():
    lib = _capi.load()
    assert lib.wm_abi_version() == _capi.ABI_VERSION
    assert lib.wm_profile_classes() > 5
    assert lib.wm_profile_name(0) == b"logmel"


def test_errors_are_reported_not_raised():
    import ctypes as C
    lib = _capi.load()
    dims = _capi.ModelDimsC(80, 100, 3, 1, 1, 51865, 1500, 448, 0, 0, 0, 0, 0, 0)   # head_dim != 64
    h = C.c_void_p()
    assert lib.wm_create(C.byref(dims), 0, C.byref(h)) == -1
    assert b"head_dim" in lib.wm_last_error()
    with pytest.raises(RuntimeError):
        _capi.check(-1, "wm_create")
