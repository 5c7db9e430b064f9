"""The C-ABI library loads and exports every symbol include/psgd.h declares (no compute calls
without a GPU); error paths that need no device behave."""
import ctypes
import os
import re

import pytest

from conftest import ROOT, has_gpu


def header_functions():
    src = open(os.path.join(ROOT, "include", "psgd.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int32_t|void|const char\*)\s+(psgd_\w+)\s*\(", src, re.M)))


def test_header_matches_binding_table(pkg):
    assert header_functions() == sorted(pkg._native.EXPORTED)


def test_library_exports_every_declared_symbol(pkg):
    path = pkg._native.LIB_PATH
    assert os.path.exists(path), "libpsgd.so not built (run __graft_entry__.build())"
    lib = ctypes.CDLL(path)
    for name in header_functions():
        assert hasattr(lib, name), name


def test_abi_version_and_no_device_error(pkg):
    L = pkg._native.lib()
    assert L.psgd_abi_version() == 1
    if has_gpu():
        pytest.skip("device present")
    h = ctypes.c_void_p()
    rc = L.psgd_ctx_create(0, ctypes.byref(h))
    assert rc == pkg._native.PSGD_EDEVICE
    assert b"no HIP device" in L.psgd_last_error()
    assert L.psgd_ctx_destroy(None) == 0
    # null-context calls fail cleanly
    assert L.psgd_clear_partitions(None) == pkg._native.PSGD_EINVAL


def test_kernels_are_gfx950_code_objects(pkg):
    data = open(pkg._native.LIB_PATH, "rb").read()
    assert b"gfx950" in data
    assert b"chain_dense" in data and b"chain_general" in data and b"fold_kernel" in data
