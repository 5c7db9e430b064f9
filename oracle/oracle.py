"""ctypes wrapper over the C oracle (oracle/libpsgd_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() (as the checker) and
bench.py's cpu_baseline leg. The product path (spark-parallelized-sgd_amd/) never imports it.

Parity status: PARTIALLY PINNED (see psgd_oracle.h / DESIGN.md §Oracle).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libpsgd_oracle.so")

GRAD = {"logistic": 0, "least_squares": 1, "hinge": 2}
UPD = {"simple": 0, "squared_l2": 1, "l1": 2, "adagrad": 3, "adam": 4}


class _Matrix(C.Structure):
    _fields_ = [
        ("n_total", C.c_int64), ("d", C.c_int32), ("is_csr", C.c_int32),
        ("labels", C.POINTER(C.c_double)), ("X", C.POINTER(C.c_double)), ("ld", C.c_int64),
        ("row_ptr", C.POINTER(C.c_int64)), ("col", C.POINTER(C.c_int32)),
        ("val", C.POINTER(C.c_double)),
    ]


class _Params(C.Structure):
    _fields_ = [
        ("gradient", C.c_int32), ("updater", C.c_int32), ("step_size", C.c_double),
        ("reg_param", C.c_double), ("convergence_tol", C.c_double),
        ("adam_beta", C.c_double), ("adam_gamma", C.c_double), ("adam_eps", C.c_double),
        ("mini_batch_fraction", C.c_double), ("num_classes", C.c_int32),
    ]


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        dp, i64p, i32p = C.POINTER(C.c_double), C.POINTER(C.c_int64), C.POINTER(C.c_int32)
        L.or_run.argtypes = [C.POINTER(_Matrix), C.c_int32, i64p, i32p, C.c_int32,
                             C.POINTER(_Params), C.c_int32, dp, dp, dp, i32p, i64p, C.c_int32]
        L.or_run_chains.argtypes = [C.POINTER(_Matrix), C.c_int32, i64p, i64p,
                                    C.POINTER(_Params), dp, dp, dp, dp, i64p, C.c_int32]
        L.or_chain.argtypes = [C.POINTER(_Matrix), C.c_int64, C.c_int64, C.POINTER(_Params),
                               dp, dp, dp, dp, i64p]
        L.or_set_margin_probe.argtypes = [dp, C.c_int32, C.c_int32]
        L.or_set_ratio_trace.argtypes = [C.c_int32, dp, C.c_int64]
        L.or_ratio_trace_len.restype = C.c_int64
        L.or_fdlibm_log.argtypes = [C.c_double]
        L.or_fdlibm_log.restype = C.c_double
        L.or_generate_gd_input.argtypes = [C.c_double, C.c_double, C.c_int32, C.c_int32, dp, dp]
        L.or_jrandom_doubles.argtypes = [C.c_int64, C.c_int32, dp]
        L.or_jrandom_gaussians.argtypes = [C.c_int64, C.c_int32, dp]
        L.or_initial_regval.argtypes = [C.c_int32, dp, C.POINTER(_Params)]
        L.or_initial_regval.restype = C.c_double
        L.or_partition_seeds.argtypes = [C.c_int64, C.c_int32, i64p]
        L.or_xorshift_hash_seed.argtypes = [C.c_int64]
        L.or_xorshift_hash_seed.restype = C.c_int64
        L.or_sample_partition.argtypes = [C.c_int64, C.c_int64, C.c_double, i32p]
        L.or_sample_partition.restype = C.c_int64
        L.or_set_f32_chain.argtypes = [C.c_int32, C.c_int32]
        _lib = L
    return _lib


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


class Matrix:
    """Keeps numpy buffers alive behind an or_matrix."""

    def __init__(self, labels, X=None, row_ptr=None, col=None, val=None, d=None):
        self.labels = np.ascontiguousarray(labels, dtype=np.float64)
        m = _Matrix()
        m.n_total = len(self.labels)
        m.labels = _dp(self.labels)
        if X is not None:
            self.X = np.ascontiguousarray(X, dtype=np.float64)
            m.d = self.X.shape[1]
            m.ld = self.X.shape[1]
            m.is_csr = 0
            m.X = _dp(self.X)
        else:
            self.row_ptr = np.ascontiguousarray(row_ptr, dtype=np.int64)
            self.col = np.ascontiguousarray(col, dtype=np.int32)
            self.val = np.ascontiguousarray(val, dtype=np.float64)
            m.d = int(d)
            m.is_csr = 1
            m.row_ptr = self.row_ptr.ctypes.data_as(C.POINTER(C.c_int64))
            m.col = self.col.ctypes.data_as(C.POINTER(C.c_int32))
            m.val = _dp(self.val)
        self.m = m
        self.d = m.d


def params(gradient, updater, step, reg=0.0, tol=0.001, beta=0.9, gamma=0.999, eps=1e-8,
           fraction=1.0, num_classes=2):
    p = _Params()
    p.mini_batch_fraction = fraction
    p.num_classes = num_classes
    p.gradient = GRAD[gradient] if isinstance(gradient, str) else int(gradient)
    p.updater = UPD[updater] if isinstance(updater, str) else int(updater)
    p.step_size, p.reg_param, p.convergence_tol = step, reg, tol
    p.adam_beta, p.adam_gamma, p.adam_eps = beta, gamma, eps
    return p


def weight_dim(d, gradient, num_classes=2):
    g = GRAD[gradient] if isinstance(gradient, str) else int(gradient)
    return (num_classes - 1) * d if g == GRAD["logistic"] and num_classes > 2 else d


def run(mat: Matrix, part_offsets, gradient, updater, step, iters, reg, w0, tol=0.001,
        groups=None, n_threads=1, **kw):
    """ParallelizedSGD.runParallelizedSGD restated (fraction=... sets miniBatchFraction).
    Returns (weights, loss_history, chain_counts[iters_run, P]). num_classes=K > 2 selects the
    multinomial LogisticGradient (weights of (K - 1) * d)."""
    L = lib()
    offs = np.ascontiguousarray(part_offsets, dtype=np.int64)
    P = len(offs) - 1
    w0 = np.ascontiguousarray(w0, dtype=np.float64)
    w_out = np.zeros(weight_dim(mat.d, gradient, kw.get("num_classes", 2)), dtype=np.float64)
    assert w0.size == w_out.size, (w0.size, w_out.size)
    hist = np.zeros(max(iters, 1), dtype=np.float64)
    nh = C.c_int32(0)
    counts = np.zeros((max(iters, 1), max(P, 1)), dtype=np.int64)
    if groups is not None:
        g = np.ascontiguousarray(groups, dtype=np.int32)
        gp, ng = g.ctypes.data_as(C.POINTER(C.c_int32)), len(g) - 1
    else:
        gp, ng = None, 0
    prm = params(gradient, updater, step, reg, tol, **kw)
    rc = L.or_run(C.byref(mat.m), P, offs.ctypes.data_as(C.POINTER(C.c_int64)), gp, ng,
                  C.byref(prm), iters, _dp(w0), _dp(w_out), _dp(hist), C.byref(nh),
                  counts.ctypes.data_as(C.POINTER(C.c_int64)), n_threads)
    if rc != 0:
        raise RuntimeError("oracle or_run failed")
    n = nh.value
    return w_out, hist[:n].copy(), counts[:iters].copy()


# Break margins: the kernels decide isConverged with other (reassociated,
# recurrence-carried) arithmetic than the reference's sums, so an exact per-chain count is a
# guarantee only where the oracle's decision is far from flipping. Not thread-safe (one global
# probe in the C library); test infrastructure only.
BREAK_MARGIN_F64 = 1e-11   # the fp64 kernels' stated bound on the relative error of diff / rhs


def run_with_margins(mat: Matrix, part_offsets, gradient, updater, step, iters, reg, w0, tol=0.001,
                     **kw):
    """run() plus margins[iters_run, P]: per outer iteration and chain, the smallest
    |diff / (tol max(norm, 1)) - 1| over the chain's per-sample isConverged tests
    (ParallelizedSGD.scala:262, :324-336) -- how far the closest decision was from flipping
    (+inf for a chain that tested nothing)."""
    P = len(part_offsets) - 1
    buf = np.full((max(iters, 1), max(P, 1)), np.inf)
    lib().or_set_margin_probe(_dp(buf), max(iters, 1), max(P, 1))
    try:
        w, h, counts = run(mat, part_offsets, gradient, updater, step, iters, reg, w0, tol=tol, **kw)
    finally:
        lib().or_set_margin_probe(None, 0, 0)
    return w, h, counts, buf[: len(counts)].copy()


def ratio_trace(mat: Matrix, part_offsets, chain, gradient, updater, step, reg, w0, **kw):
    """r_k = diff_k / max(norm_k, 1) of every sample k of `chain` in the first outer iteration at
    tol = 0 (no break): sample k passes isConverged iff r_k < tol, so tol = r_k (1 +- e) puts a
    decision e from flipping (the adversarial break cases)."""
    n = int(part_offsets[chain + 1] - part_offsets[chain])
    buf = np.zeros(max(n, 1))
    lib().or_set_ratio_trace(chain, _dp(buf), n)
    try:
        run(mat, part_offsets, gradient, updater, step, 1, reg, w0, tol=0.0, **kw)
        m = lib().or_ratio_trace_len()
    finally:
        lib().or_set_ratio_trace(-1, None, 0)
    return buf[:m].copy()


def run_f32(mat: Matrix, part_offsets, gradient, updater, step, iters, reg, w0, order=0, **kw):
    """run() with every dense Simple / SquaredL2 chain evaluated in IEEE single precision
    (or_set_f32_chain: the sequential fp32 restatement; order 0 = left-fold dots, 1 = 64 strided
    partials + pairwise tree, 2 = only the weights float, the dot and multiplier in double, tol = 0).
    The driver and the combine stay in double, as on the device."""
    lib().or_set_f32_chain(1, int(order))
    try:
        return run(mat, part_offsets, gradient, updater, step, iters, reg, w0, **kw)
    finally:
        lib().or_set_f32_chain(0, 0)


def run_chains(mat: Matrix, part_offsets, gradient, updater, step, reg, w_in, tol=0.0,
               limits=None, n_threads=1, **kw):
    """One epoch of chains (no combine): (w[P,d], rv[P], loss[P], count[P])."""
    L = lib()
    offs = np.ascontiguousarray(part_offsets, dtype=np.int64)
    P = len(offs) - 1
    w_in = np.ascontiguousarray(w_in, dtype=np.float64)
    w = np.zeros((P, weight_dim(mat.d, gradient, kw.get("num_classes", 2))), dtype=np.float64)
    assert w_in.size == w.shape[1], (w_in.size, w.shape)
    rv = np.zeros(P)
    loss = np.zeros(P)
    cnt = np.zeros(P, dtype=np.int64)
    lim = None
    if limits is not None:
        lim_arr = np.ascontiguousarray(limits, dtype=np.int64)
        lim = lim_arr.ctypes.data_as(C.POINTER(C.c_int64))
    prm = params(gradient, updater, step, reg, tol, **kw)
    rc = L.or_run_chains(C.byref(mat.m), P, offs.ctypes.data_as(C.POINTER(C.c_int64)), lim,
                         C.byref(prm), _dp(w_in), _dp(w), _dp(rv), _dp(loss),
                         cnt.ctypes.data_as(C.POINTER(C.c_int64)), n_threads)
    if rc != 0:
        raise RuntimeError("oracle or_run_chains failed")
    return w, rv, loss, cnt


def partition_seeds(seed, P):
    """PartitionwiseSampledRDD.getPartitions: java.util.Random(seed).nextLong() per partition."""
    out = np.zeros(P, dtype=np.int64)
    lib().or_partition_seeds(seed, P, out.ctypes.data_as(C.POINTER(C.c_int64)))
    return out


def xorshift_hash_seed(s):
    return int(lib().or_xorshift_hash_seed(int(s)))


def sample_partition(seed, n, fraction):
    """BernoulliSampler(fraction) with setSeed(seed) over n rows: the selected row offsets."""
    out = np.zeros(max(n, 1), dtype=np.int32)
    m = lib().or_sample_partition(int(seed), int(n), float(fraction),
                                  out.ctypes.data_as(C.POINTER(C.c_int32)))
    return out[:m].copy()


def generate_gd_input(offset, scale, n, seed):
    x = np.zeros(n)
    y = np.zeros(n)
    lib().or_generate_gd_input(offset, scale, n, seed, _dp(x), _dp(y))
    return x, y


def fdlibm_log(x: float) -> float:
    return lib().or_fdlibm_log(x)


def jrandom_doubles(seed, n):
    out = np.zeros(n)
    lib().or_jrandom_doubles(seed, n, _dp(out))
    return out


def jrandom_gaussians(seed, n):
    out = np.zeros(n)
    lib().or_jrandom_gaussians(seed, n, _dp(out))
    return out
