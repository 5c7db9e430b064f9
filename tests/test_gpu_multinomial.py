"""The multinomial LogisticGradient(numClasses > 2) chain (csrc/psgd_multinomial.hip) against the
CPU oracle (oracle/psgd_oracle.c multinomial_compute, restating MLlib 1.6.1's LogisticGradient).

fp64 compute: weights and loss history within 1e-9 relative (the parity bar of
test_gpu_parity.py), chain counts exact (per-sample convergence breaks included). The golden
cases with num_classes run in test_gpu_parity.py::test_golden_cases_fp64; here: wider rows,
more classes, every updater on dense and CSR rows, fp32 storage, sampled batches.
"""
import numpy as np
import pytest

from conftest import has_gpu
from test_gpu_parity import U, assert_close

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not has_gpu():
        pytest.skip("no GPU")


def dense_case(rng, n, d, K):
    X = rng.standard_normal((n, d)) / np.sqrt(d)
    X[rng.uniform(size=(n, d)) < 0.1] = 0.0
    W = 2.0 * rng.standard_normal((K, d))
    y = np.argmax(X @ W.T + rng.gumbel(size=(n, K)), 1).astype(np.float64)
    return X, y


def csr_case(rng, n, d, K, kmax):
    rp, col, val = [0], [], []
    for _ in range(n):
        k = int(rng.integers(0, kmax + 1))
        col += sorted(rng.choice(d, size=k, replace=False).tolist())
        val += rng.uniform(-1, 1, size=k).tolist()
        rp.append(len(col))
    rp, col, val = np.array(rp, np.int64), np.array(col, np.int32), np.array(val)
    y = rng.integers(0, K, size=n).astype(np.float64)
    return rp, col, val, y


def run_both(pkg, oracle, parts, mat, offs, K, upd, d, step=0.2, iters=3, reg=0.01, tol=0.0, frac=1.0,
             w0=None):
    data = pkg.PartitionedData(parts)
    w0 = np.zeros((K - 1) * d) if w0 is None else w0
    w, h, counts = pkg.runParallelizedSGD(data, pkg.LogisticGradient(K), getattr(pkg, U[upd])(), step, iters,
                                          reg, frac, w0, tol, return_chain_counts=True)
    wr, hr, cr = oracle.run(mat, offs, "logistic", upd, step, iters, reg, w0, tol=tol, fraction=frac,
                            num_classes=K, n_threads=8)
    tag = f"K={K} {upd} tol={tol} f={frac}"
    assert [list(map(int, c)) for c in counts] == [list(map(int, c)) for c in cr], tag
    assert_close(w, wr, what=tag + " weights")
    assert_close(h, hr, what=tag + " loss")
    return w


@pytest.mark.parametrize("upd", ["simple", "squared_l2", "l1", "adagrad", "adam"])
def test_multinomial_dense(pkg, oracle, upd):
    rng = np.random.default_rng(40 + len(upd))
    n, d, K = 2400, 200, 10
    X, y = dense_case(rng, n, d, K)
    offs = [0, 700, 701, 1600, 2400]
    parts = [pkg.DensePartition(y[a:b], X[a:b]) for a, b in zip(offs[:-1], offs[1:])]
    mat = oracle.Matrix(y, X)
    run_both(pkg, oracle, parts, mat, offs, K, upd, d)
    assert pkg.optimization.get_context(0).last_kernel() == 500
    run_both(pkg, oracle, parts, mat, offs, K, upd, d, tol=0.002,
             w0=0.05 * rng.standard_normal((K - 1) * d))


@pytest.mark.parametrize("upd", ["simple", "squared_l2", "l1", "adagrad", "adam"])
def test_multinomial_csr(pkg, oracle, upd):
    rng = np.random.default_rng(50 + len(upd))
    n, d, K = 1500, 3000, 6
    rp, col, val, y = csr_case(rng, n, d, K, 60)
    offs = [0, 400, 400, 1500]
    parts = [pkg.CsrPartition(y[a:b], rp[a:b + 1] - rp[a], col[rp[a]:rp[b]], val[rp[a]:rp[b]], d)
             for a, b in zip(offs[:-1], offs[1:])]
    mat = oracle.Matrix(y, row_ptr=rp, col=col, val=val, d=d)
    run_both(pkg, oracle, parts, mat, offs, K, upd, d, step=0.5)
    assert pkg.optimization.get_context(0).last_kernel() == 501
    run_both(pkg, oracle, parts, mat, offs, K, upd, d, step=0.5, tol=0.01)


def test_multinomial_f32_storage_and_sampling(pkg, oracle):
    rng = np.random.default_rng(61)
    n, d, K = 3000, 64, 4
    X, y = dense_case(rng, n, d, K)
    X32 = X.astype(np.float32)
    offs = [0, 1000, 3000]
    parts = [pkg.DensePartition(y[a:b], X32[a:b]) for a, b in zip(offs[:-1], offs[1:])]
    mat = oracle.Matrix(y, X32.astype(np.float64))
    for frac in (1.0, 0.3, 0.7):
        run_both(pkg, oracle, parts, mat, offs, K, "squared_l2", d, frac=frac, iters=4)


def test_multinomial_rejects_fp32_compute(pkg):
    X = np.ones((4, 3))
    data = pkg.PartitionedData([pkg.DensePartition(np.zeros(4), X)])
    with pytest.raises(pkg.UnsupportedOperationException):
        pkg.runParallelizedSGD(data, pkg.LogisticGradient(3), pkg.SimpleSGDUpdater(), 1.0, 1, 0.0, 1.0,
                               np.zeros(6), 0.0, compute_dtype="f32")
