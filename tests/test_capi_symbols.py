"""The C-ABI library loads and exports every symbol include/lodestar_bls.h declares.

CPU only: no compute calls without a GPU.
"""
import ctypes
import os
import re

from lodestar_amd import native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "lodestar_bls.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(lb_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_expected_entry_points():
    fns = declared_functions()
    assert set(native.EXPORTED_SYMBOLS) == set(fns), set(native.EXPORTED_SYMBOLS) ^ set(fns)


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(native.library_path())
    for name in declared_functions():
        assert hasattr(lib, name), name


def test_no_device_is_reported_cleanly_without_gpu():
    lib = native.load_library()
    n = lib.lb_device_count()
    if n == 0:
        h = ctypes.c_void_p()
        assert lib.lb_create(0, ctypes.byref(h)) == native.LB_ERR_NO_DEVICE
        assert lib.lb_destroy(None) == native.LB_OK


def test_library_is_gfx950_code_object():
    blob = open(native.library_path(), "rb").read()
    assert b"gfx950" in blob
