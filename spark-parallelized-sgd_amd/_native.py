"""ctypes binding of libpsgd.so -- the C ABI declared in include/psgd.h.

The shared library holds the gfx950 HIP kernels; there is no CPU implementation behind this
module. If the library is missing or no gfx950 device is present, every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
# PSGD_LIB: another build of the same library (diagnostics, e.g. `make -C csrc stamps`)
LIB_PATH = os.environ.get("PSGD_LIB") or os.path.join(HERE, "libpsgd.so")
CSRC = os.path.join(HERE, "csrc")

PSGD_OK, PSGD_EINVAL, PSGD_EUNSUPPORTED, PSGD_EDEVICE, PSGD_ENOMEM, PSGD_ESTATE = 0, -1, -2, -3, -4, -5
F64, F32 = 0, 1

# Symbols include/psgd.h declares (checked by tests/test_capi_symbols.py).
EXPORTED = (
    "psgd_abi_version", "psgd_last_error", "psgd_ctx_create", "psgd_ctx_destroy",
    "psgd_register_dense", "psgd_register_csr", "psgd_register_dense_device", "psgd_register_csr_device",
    "psgd_clear_partitions", "psgd_num_partitions", "psgd_run_epoch", "psgd_run_epoch_device",
    "psgd_fold_partials_device", "psgd_run_epoch_device_mirror", "psgd_fold_partials_device_mirror",
    "psgd_convergence_terms_device", "psgd_initial_regval",
    "psgd_ctx_last_kernel", "psgd_ctx_last_chain_ms", "psgd_ctx_chain_launches", "psgd_ctx_chain_ms",
    "psgd_vmm_stats", "psgd_reroll_stats", "psgd_libsvm_read", "psgd_libsvm_free",
    "psgd_sample_partition", "psgd_host_alloc", "psgd_host_free", "psgd_register_wait",
)


class psgd_libsvm(C.Structure):
    _fields_ = [("n_rows", C.c_int64), ("d", C.c_int32), ("n_parts", C.c_int32),
                ("part_offsets", C.POINTER(C.c_int64)), ("labels", C.POINTER(C.c_double)),
                ("row_ptr", C.POINTER(C.c_int64)), ("col", C.POINTER(C.c_int32)),
                ("val", C.POINTER(C.c_double))]


class IllegalArgumentException(ValueError):
    """The reference's `require` failures (java.lang.IllegalArgumentException)."""


class UnsupportedOperationException(NotImplementedError):
    """Valid in the reference but not built here yet."""


class DeviceError(RuntimeError):
    """HIP runtime failure inside libpsgd."""


class psgd_params(C.Structure):
    _fields_ = [
        ("gradient", C.c_int32), ("updater", C.c_int32), ("compute_dtype", C.c_int32),
        ("iteration", C.c_int32), ("step_size", C.c_double), ("reg_param", C.c_double),
        ("mini_batch_fraction", C.c_double), ("convergence_tol", C.c_double),
        ("adam_beta", C.c_double), ("adam_gamma", C.c_double), ("adam_eps", C.c_double),
        ("num_classes", C.c_int32),
    ]


def build(force: bool = False) -> str:
    """Compile libpsgd.so in-tree (hipcc --offload-arch=gfx950)."""
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-s", "-C", CSRC, "-j2"], check=True)
    return LIB_PATH


_lib = None
_lock = threading.Lock()


def lib():
    """Load libpsgd.so (after torch, so both share one HIP runtime)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        try:  # torch bundles libamdhip64.so.7; load it first so there is one HIP runtime
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise DeviceError(
                f"{LIB_PATH} is missing: build it with `make -C {CSRC}` (hipcc, gfx950)")
        L = C.CDLL(LIB_PATH)
        vp, dp, i64p, i32p = C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_int64), C.POINTER(C.c_int32)
        P = C.POINTER(psgd_params)
        sig = {
            "psgd_abi_version": ([], C.c_int32),
            "psgd_last_error": ([], C.c_char_p),
            "psgd_ctx_create": ([C.c_int32, C.POINTER(vp)], C.c_int32),
            "psgd_ctx_destroy": ([vp], C.c_int32),
            "psgd_register_dense": ([vp, C.c_int64, C.c_int64, C.c_int32, vp, vp, C.c_int32], C.c_int32),
            "psgd_register_csr": ([vp, C.c_int64, C.c_int64, C.c_int32, vp, vp, vp, vp, C.c_int32], C.c_int32),
            "psgd_register_dense_device": ([vp, C.c_int64, C.c_int64, C.c_int32, C.c_int64, vp, vp, C.c_int32], C.c_int32),
            "psgd_register_csr_device": ([vp, C.c_int64, C.c_int64, C.c_int32, vp, vp, vp, vp, C.c_int32], C.c_int32),
            "psgd_clear_partitions": ([vp], C.c_int32),
            "psgd_num_partitions": ([vp, i64p, i64p], C.c_int32),
            "psgd_run_epoch": ([vp, P, vp, vp, dp, dp, i64p, vp], C.c_int32),
            "psgd_run_epoch_device": ([vp, P, vp, vp, vp, vp], C.c_int32),
            "psgd_fold_partials_device": ([vp, C.c_int32, C.c_int32, vp, vp, vp], C.c_int32),
            "psgd_run_epoch_device_mirror": ([vp, P, vp, vp, vp, vp, vp], C.c_int32),
            "psgd_fold_partials_device_mirror": ([vp, C.c_int32, C.c_int32, vp, vp, vp, vp], C.c_int32),
            "psgd_convergence_terms_device": ([vp, C.c_int32, vp, vp, dp, vp], C.c_int32),
            "psgd_initial_regval": ([vp, P, C.c_int32, vp, dp], C.c_int32),
            "psgd_ctx_last_kernel": ([vp], C.c_int32),
            "psgd_ctx_last_chain_ms": ([vp, dp], C.c_int32),
            "psgd_ctx_chain_launches": ([vp], C.c_int64),
            "psgd_ctx_chain_ms": ([vp, C.c_int64, dp], C.c_int32),
            "psgd_vmm_stats": ([i64p], C.c_int32),
            "psgd_reroll_stats": ([i64p], C.c_int32),
            "psgd_libsvm_read": ([C.c_char_p, C.c_int32, C.c_int32, C.POINTER(C.POINTER(psgd_libsvm))], C.c_int32),
            "psgd_libsvm_free": ([C.POINTER(psgd_libsvm)], None),
            "psgd_sample_partition": ([C.c_int32, C.c_int64, C.c_int64, C.c_double, vp, i64p], C.c_int32),
            "psgd_host_alloc": ([vp, C.c_int64, C.POINTER(vp)], C.c_int32),
            "psgd_host_free": ([vp, vp], C.c_int32),
            "psgd_register_wait": ([vp], C.c_int32),
        }
        for name, (args, res) in sig.items():
            f = getattr(L, name)
            f.argtypes = args
            f.restype = res
        _lib = L
        return L


def check(rc: int) -> None:
    if rc == PSGD_OK:
        return
    msg = lib().psgd_last_error().decode(errors="replace")
    if rc == PSGD_EINVAL:
        raise IllegalArgumentException(msg)
    if rc == PSGD_EUNSUPPORTED:
        raise UnsupportedOperationException(msg)
    raise DeviceError(f"libpsgd error {rc}: {msg}")


def vmm_stats() -> dict:
    """Process-wide counters of the CSR weight vectors' virtual-memory mappings (psgd_vmm_stats)."""
    out = (C.c_int64 * 4)()
    check(lib().psgd_vmm_stats(out))
    return {"mapped": out[0], "unmapped": out[1], "live_bytes": out[2], "failures": out[3]}


def reroll_stats() -> dict:
    """Process-wide counters of the CSR vector sets' placement re-roll (psgd_reroll_stats)."""
    out = (C.c_int64 * 2)()
    check(lib().psgd_reroll_stats(out))
    return {"sets": out[0], "swaps": out[1]}


def sample_partition(seed: int, n: int, fraction: float, device: int = 0):
    """Row indices RDD.sample(false, fraction, .) keeps from an n-row partition whose sampler
    seed is `seed`, selected on the device (psgd_sample_partition)."""
    import numpy as np
    rows = np.empty(max(int(n), 1), dtype=np.int32)
    m = C.c_int64()
    check(lib().psgd_sample_partition(device, int(seed), int(n), float(fraction), rows.ctypes.data,
                                      C.byref(m)))
    return rows[: m.value].copy()


class _PinnedBuffer:
    """Page-locked host memory from psgd_host_alloc; freed when the last numpy view of it goes
    (the context must outlive it)."""

    def __init__(self, ctx, addr, nbytes):
        self._ctx, self._addr = ctx, addr
        self.view = (C.c_char * nbytes).from_address(addr)
        self.view.owner = self      # numpy views keep the ctypes array, which keeps this

    def __del__(self):
        try:
            if self._ctx.handle and self._addr:
                self._ctx._L.psgd_host_free(self._ctx.handle, self._addr)
        except Exception:
            pass
        self._addr = None


class Context:
    """Owns one psgd_ctx (one device, its stream, registry and buffers)."""

    def __init__(self, device: int = 0):
        self._L = lib()
        h = C.c_void_p()
        check(self._L.psgd_ctx_create(device, C.byref(h)))
        self.handle = h
        self.device = device

    def close(self):
        if self.handle:
            self._L.psgd_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # registry -------------------------------------------------------------------------------
    def register_dense(self, part, labels, x):
        import numpy as np
        labels = np.ascontiguousarray(labels, dtype=np.float64)
        if x.dtype not in (np.float32, np.float64):
            x = x.astype(np.float64)
        x = np.ascontiguousarray(x)
        n, d = x.shape
        dt = F32 if x.dtype == np.float32 else F64
        check(self._L.psgd_register_dense(self.handle, part, n, d, labels.ctypes.data,
                                          x.ctypes.data, dt))

    def register_csr(self, part, labels, row_ptr, col, val, d):
        import numpy as np
        labels = np.ascontiguousarray(labels, dtype=np.float64)
        row_ptr = np.ascontiguousarray(row_ptr, dtype=np.int64)
        col = np.ascontiguousarray(col, dtype=np.int32)
        if val.dtype not in (np.float32, np.float64):
            val = val.astype(np.float64)
        val = np.ascontiguousarray(val)
        dt = F32 if val.dtype == np.float32 else F64
        check(self._L.psgd_register_csr(self.handle, part, len(labels), d, labels.ctypes.data,
                                        row_ptr.ctypes.data, col.ctypes.data, val.ctypes.data, dt))

    def register_dense_device(self, part, n_rows, d, ld, labels_ptr, x_ptr, dtype):
        check(self._L.psgd_register_dense_device(self.handle, part, n_rows, d, ld, labels_ptr,
                                                 x_ptr, dtype))

    def register_csr_device(self, part, n_rows, d, labels_ptr, row_ptr_ptr, col_ptr, val_ptr, dtype):
        check(self._L.psgd_register_csr_device(self.handle, part, n_rows, d, labels_ptr, row_ptr_ptr,
                                               col_ptr, val_ptr, dtype))

    def register_wait(self):
        """Block until every registration copy has landed in HBM (psgd_register_wait)."""
        check(self._L.psgd_register_wait(self.handle))

    def host_array(self, shape, dtype):
        """A numpy array over page-locked host memory (psgd_host_alloc): registration from it is
        one direct DMA, no staging copy. Freed with the returned array's owner (`.base`)."""
        import numpy as np
        dt = np.dtype(dtype)
        n = int(np.prod(shape)) * dt.itemsize
        p = C.c_void_p()
        check(self._L.psgd_host_alloc(self.handle, max(n, 1), C.byref(p)))
        buf = _PinnedBuffer(self, p.value, max(n, 1))
        return np.frombuffer(buf.view, dtype=dt, count=int(np.prod(shape))).reshape(shape)

    def clear(self):
        check(self._L.psgd_clear_partitions(self.handle))

    def num_partitions(self):
        a, b = C.c_int64(), C.c_int64()
        check(self._L.psgd_num_partitions(self.handle, C.byref(a), C.byref(b)))
        return a.value, b.value

    def last_kernel(self) -> int:
        return int(self._L.psgd_ctx_last_kernel(self.handle))

    def last_chain_ms(self) -> float:
        """Device time of the last chain-kernel launch (HIP events on its stream)."""
        ms = C.c_double()
        check(self._L.psgd_ctx_last_chain_ms(self.handle, C.byref(ms)))
        return ms.value

    def chain_launches(self) -> int:
        """Chain-kernel launches this context has made (the index of the next one)."""
        return int(self._L.psgd_ctx_chain_launches(self.handle))

    def chain_ms(self, launch: int) -> float:
        """Device time of chain-kernel launch `launch` (0-based; one of the last 64)."""
        ms = C.c_double()
        check(self._L.psgd_ctx_chain_ms(self.handle, C.c_int64(launch), C.byref(ms)))
        return ms.value

    # epochs ---------------------------------------------------------------------------------
    def run_epoch_device(self, params, w_ptr, partial_ptr, counts_ptr=None, stream=None):
        check(self._L.psgd_run_epoch_device(self.handle, C.byref(params), w_ptr, partial_ptr,
                                            counts_ptr, stream))

    def fold_partials_device(self, n, d, partials_ptr, out_ptr, stream=None):
        check(self._L.psgd_fold_partials_device(self.handle, n, d, partials_ptr, out_ptr, stream))

    def run_epoch_device_mirror(self, params, w_ptr, partial_ptr, counts_ptr, stream, h_ptr):
        """run_epoch_device whose fold also writes {regVal, lossSum, count} to h_ptr[3]
        (page-locked host memory, host_array)."""
        check(self._L.psgd_run_epoch_device_mirror(self.handle, C.byref(params), w_ptr, partial_ptr,
                                                   counts_ptr, stream, h_ptr))

    def fold_partials_device_mirror(self, n, d, partials_ptr, out_ptr, stream, h_ptr):
        check(self._L.psgd_fold_partials_device_mirror(self.handle, n, d, partials_ptr, out_ptr, stream,
                                                       h_ptr))

    def convergence_terms_device(self, d, prev_ptr, cur_ptr, stream=None):
        out = (C.c_double * 2)()
        check(self._L.psgd_convergence_terms_device(self.handle, d, prev_ptr, cur_ptr, out, stream))
        return out[0], out[1]

    def initial_regval(self, params, w):
        import numpy as np
        w = np.ascontiguousarray(w, dtype=np.float64)
        out = C.c_double()
        check(self._L.psgd_initial_regval(self.handle, C.byref(params), len(w), w.ctypes.data,
                                          C.byref(out)))
        return out.value

    def run_epoch(self, params, w_in):
        """Host-pointer form (the JNI-shaped call): returns (w, regVal, lossSum, count, counts)."""
        import numpy as np
        w_in = np.ascontiguousarray(w_in, dtype=np.float64)
        nparts, _ = self.num_partitions()
        w_out = np.zeros_like(w_in)
        rv, loss = C.c_double(), C.c_double()
        cnt = C.c_int64()
        counts = np.zeros(max(nparts, 1), dtype=np.int64)
        check(self._L.psgd_run_epoch(self.handle, C.byref(params), w_in.ctypes.data,
                                     w_out.ctypes.data, C.byref(rv), C.byref(loss), C.byref(cnt),
                                     counts.ctypes.data))
        return w_out, rv.value, loss.value, cnt.value, counts[:nparts]
