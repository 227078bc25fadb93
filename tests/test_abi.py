"""C-ABI boundary checks that need no GPU: the library loads, exports every entry point that
include/svo_c.h declares, the ctypes table matches, and errors come back as codes (no exceptions,
no silent CPU fallback)."""
import ctypes
import os
import re

import pytest

import svo_amd
from svo_amd import _capi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "svo_c.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\*\s]+?\b(svo_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_entry_points():
    names = header_functions()
    assert "svo_image_align" not in names
    for must in ("svo_ctx_create", "svo_pyramid_set_build", "svo_align_batch_run", "svo_feature_align"):
        assert must in names


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(_capi.lib_path())
    for name in header_functions():
        assert hasattr(lib, name), name


def test_ctypes_table_matches_header():
    assert sorted(_capi.EXPORTED) == header_functions()


def test_errors_are_codes():
    L = _capi.lib()
    assert L.svo_abi_version() == 2
    h = ctypes.c_void_p()
    assert L.svo_pyramid_set_create(None, 1, 64, 64, 3, ctypes.byref(h)) == _capi.SVO_ERR_ARG
    assert b"null" in L.svo_last_error()
    assert L.svo_align_batch_run(None) == _capi.SVO_ERR_ARG
    assert L.svo_ctx_create(0, None) == _capi.SVO_ERR_ARG


def test_no_gpu_fails_loudly():
    n = ctypes.c_int32(-1)
    assert _capi.lib().svo_device_count(ctypes.byref(n)) == 0
    if n.value > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(svo_amd.SvoError) as e:
        svo_amd.Context(0)
    assert e.value.code == _capi.SVO_ERR_NODEV
