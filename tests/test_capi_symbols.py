"""The C-ABI library loads and exports every symbol include/psgd.h declares (no compute calls
without a GPU); error paths that need no device behave."""
import ctypes
import os
import re

import pytest

from conftest import ROOT, has_gpu


def header_functions():
    src = open(os.path.join(ROOT, "include", "psgd.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int32_t|int64_t|void|const char\*)\s+(psgd_\w+)\s*\(", src, re.M)))


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


def test_kernel_selection_limits_on_the_host(pkg):
    """The dispatch predicates are host code (no device needed). chain_sparse_lds (fp32 and fp64)
    counts a chain's rows in 32 bits, so a partition of more than INT32_MAX rows must not select
    it (such partitions fit in HBM as 16-byte CSR rows); chain_sparse64 takes fp64 CSR
    with Simple, or SquaredL2 while alpha stays in range, with or without the per-sample break
    (variants 420/421, 460/461)."""
    lib = ctypes.CDLL(pkg._native.LIB_PATH)
    lds = lib._ZN4psgd18sparse_lds_appliesElll
    lds.restype, lds.argtypes = ctypes.c_bool, [ctypes.c_int64] * 3
    lds64 = lib._ZN4psgd20sparse_lds64_appliesEllibbl
    lds64.restype = ctypes.c_bool
    lds64.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_bool, ctypes.c_bool, ctypes.c_int64]
    s64 = lib._ZN4psgd21sparse64_path_appliesEiiibb
    s64.restype = ctypes.c_bool
    s64.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_bool, ctypes.c_bool]
    big = 2**31 - 1
    assert lds(47236, 94, big) and not lds(47236, 94, big + 1)
    assert lds64(47236, 94, 0, False, True, big) and not lds64(47236, 94, 0, False, True, big + 1)
    assert not lds(47236, 129, 100)              # rows of more than 128 entries
    CSR, DENSE, F64, F32 = 1, 0, 0, 1
    SIMPLE, L2, L1 = 0, 1, 2
    assert s64(CSR, F64, SIMPLE, False, False) and s64(CSR, F64, L2, False, True)
    assert not s64(CSR, F64, L2, False, False)   # alpha out of range: chain_general renormalises
    assert s64(CSR, F64, SIMPLE, True, True)      # the per-sample break runs in chain_sparse64 too
    assert lds64(47236, 94, 0, True, True, 1000)   # ... and in chain_sparse_lds
    assert not s64(CSR, F32, SIMPLE, False, True) and not s64(DENSE, F64, SIMPLE, False, True)
    assert not s64(CSR, F64, L1, False, True)
