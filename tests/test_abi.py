"""The C-ABI library loads on a host without a GPU and exports every entry point include/hipgle.h
declares; calls that need a device fail loudly with an error code and message (no CPU fallback)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT


def header_symbols():
    src = open(os.path.join(ROOT, "include", "hipgle.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(gle_\w+)\s*\(", src, re.M)))


def test_header_and_binding_agree():
    from sclmd_amd import _native

    assert header_symbols() == sorted(_native.EXPORTS)


def test_library_exports_every_symbol():
    from sclmd_amd import _native

    lib = _native.load()
    for s in header_symbols():
        assert hasattr(lib, s), s
    assert lib.gle_abi_version() == 1


def test_create_without_device_fails_loudly():
    from sclmd_amd import _native

    if _native.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(_native.GLEError) as e:
        _native.Stepper(12, 1, 16, 0.38)
    assert "gle_create failed" in str(e.value)


def test_bad_config_rejected():
    from sclmd_amd import _native

    lib = _native.load()
    cfg = _native.gle_config(12, 1, 15, 0.38, 0, 0, 0, 0)  # odd nmd (fields: ..., far_mode, max_block)
    h = ctypes.c_void_p()
    assert lib.gle_create(ctypes.byref(cfg), ctypes.byref(h)) == -1
    assert b"even" in lib.gle_last_error(None)


def test_missing_library_message(monkeypatch, tmp_path):
    from sclmd_amd import _native

    monkeypatch.setattr(_native, "_lib", None)
    monkeypatch.setattr(_native, "LIB_PATH", str(tmp_path / "nope.so"))
    with pytest.raises(_native.GLEError, match="not found"):
        _native.load()


def test_header_constants_match_binding():
    """Every #define of include/hipgle.h that the ctypes binding mirrors has the same value."""
    from sclmd_amd import _native

    src = open(os.path.join(ROOT, "include", "hipgle.h")).read()
    defs = {k: int(v) for k, v in re.findall(r"^#define\s+(GLE_\w+)\s+\(?(-?\d+)\)?", src, re.M)}
    mirror = {"GLE_REC_P": _native.REC_P, "GLE_REC_Q": _native.REC_Q, "GLE_REC_F": _native.REC_F,
              "GLE_REC_HIST": _native.REC_HIST, "GLE_PROFILE_EVENTS": _native.PROFILE_EVENTS,
              "GLE_PROFILE_COUNT": _native.PROFILE_COUNT, "GLE_COMM_ID_BYTES": _native.COMM_ID_BYTES,
              "GLE_PLAN_AUTO": _native.PLAN_AUTO, "GLE_PLAN_SMALL_BATHS": _native.PLAN_SMALL_BATHS,
              "GLE_PLAN_LARGE_BATHS": _native.PLAN_LARGE_BATHS}
    for k, v in mirror.items():
        assert defs.get(k) == v, (k, defs.get(k), v)
