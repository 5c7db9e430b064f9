"""The fp32 restatements of the chain (oracle.run_f32, psgd_oracle.c chain_rows_f32): the evidence
behind the fp32 mode's stated tolerance at BASELINE config 3 (DESIGN.md §4,
tests/test_gpu_fp32_c3.py). CPU only.

At C3's hyper-parameters (Logistic, d = 1,024, step 1.0; ParallelizedSGD.scala:253-268) and
thousands of rows per chain, a plain fp32 evaluation of the reference's own loop already sits
1e-3 .. 3e-2 x max|w| from the fp64 reference (swept in DESIGN.md §4). It is the trajectory's, not
a kernel's: even with every dot and multiplier in double and only the weights stored as float
(order 2), the error stays above 2e-4, so no kernel with fp32 weights can meet the 2e-4 bound that
holds on the other configs. At short chains and small steps the restatements stay inside 2e-4.
"""
import numpy as np
import pytest


def c3_prefix(P, per, d=1024, seed=44):
    rng = np.random.default_rng(seed)
    n = P * per
    X = rng.standard_normal((n, d), dtype=np.float32)
    w = rng.standard_normal(d) / np.sqrt(d)
    y = ((X.astype(np.float64) @ w + rng.logistic(size=n)) > 0).astype(np.float64)
    return X, y, [i * n // P for i in range(P)] + [n]


def errors(oracle, P, per, grad="logistic", upd="simple", step=1.0, reg=0.0):
    """(errors of the three fp32 restatements -- left fold, tree, weights-only -- relative to
    max|w| of the fp64 oracle, the left fold's loss error, its chain counts)."""
    X, y, offs = c3_prefix(P, per)
    if grad == "least_squares":
        y = X.astype(np.float64) @ (np.arange(X.shape[1]) % 7 - 3.0) / 64.0
    mat = oracle.Matrix(y, X.astype(np.float64))
    a = (mat, offs, grad, upd, step, 3, reg, np.zeros(X.shape[1]))
    wr, hr, _ = oracle.run(*a, tol=0.0, n_threads=8)
    s = np.max(np.abs(wr))
    errs, h0, c0 = [], None, None
    for order in (0, 1, 2):
        w, h, c = oracle.run_f32(*a, order=order, tol=0.0, n_threads=8)
        errs.append(np.max(np.abs(w - wr)) / s)
        if order == 0:
            h0, c0 = h, c
    return errs, np.max(np.abs(h0 - hr) / np.abs(hr)), c0


@pytest.mark.parametrize("P,per", [(64, 2000), (8, 4000)])
def test_f32_weights_alone_leave_2e4_at_c3(oracle, P, per):
    (seq, tree, wonly), loss, counts = errors(oracle, P, per)
    print(f"\nC3 {P} x {per}: fp32 left fold {seq:.3g}, tree {tree:.3g}, weights-only {wonly:.3g}, "
          f"loss {loss:.3g}")
    assert (counts == per).all()
    assert min(seq, tree, wonly) > 2e-4, (seq, tree, wonly)
    # ... and inside the C3 fp32 weight tolerance (tests/test_gpu_fp32_c3.py FP32_C3_W_REL)
    assert max(seq, tree, wonly) < 5e-2
    assert loss < 1e-3


@pytest.mark.parametrize("P,per", [(256, 40), (256, 200)])
def test_f32_restatements_short_chains_inside_2e4(oracle, P, per):
    (seq, tree, wonly), loss, _ = errors(oracle, P, per)
    assert max(seq, tree, wonly) < 2e-4, (seq, tree, wonly)
    assert loss < 1e-4


@pytest.mark.parametrize("grad,upd,step,reg", [("least_squares", "simple", 1e-4, 0.0),
                                               ("hinge", "squared_l2", 0.01, 0.1),
                                               ("logistic", "squared_l2", 0.05, 0.01)])
def test_f32_restatements_small_steps(oracle, grad, upd, step, reg):
    """Away from C3's step 1.0 the fp32 restatements sit at fp32 rounding of the fp64 chain."""
    (seq, tree, wonly), loss, _ = errors(oracle, 32, 200, grad, upd, step, reg)
    assert max(seq, tree, wonly) < 2e-4, (seq, tree, wonly)
    assert loss < 1e-4
