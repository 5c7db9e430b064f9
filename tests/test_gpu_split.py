"""chain_split (psgd_split.hip): the dense per-sample chain with its features split over H compute
waves, the throughput kernel of AdaGrad / Adam / L1 (SGDUpdater.scala:120-148, :193-286) at tol = 0.

Every gradient x the three updaters (L1 with regParam > 0), f32 and f64 rows, full and ragged row vectors, H = 2 and 4, fp64
compute at 1e-9 with exact counts against the oracle (ParallelizedSGD.scala:243-276), fp32
compute at the fp32 tolerance; sampled batches (the loader's row-index path), 1-row and empty
partitions."""
import numpy as np
import pytest

from conftest import has_gpu
from test_gpu_parity import FP32_LOSS_REL, FP32_REL, G, U, assert_close, block64_variant, stateful_variant

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not has_gpu():
        pytest.skip("no GPU")


def synth(rng, n, d, grad):
    X = (rng.standard_normal((n, d)) / np.sqrt(d)).astype(np.float32)
    w = rng.standard_normal(d)
    z = X.astype(np.float64) @ w
    if grad == "least_squares":
        y = z + 0.1 * rng.standard_normal(n)
    else:
        y = (z + rng.logistic(size=n) > 0).astype(np.float64)
    return X, y


def nv_of(d, storage):
    vec = 4 if storage == np.float32 else 2
    nv = 1
    while nv * 64 * vec < d:
        nv *= 2
    return nv


def run_both(pkg, oracle, X, y, storage, P, grad, upd, step, compute="f64", frac=1.0, iters=3):
    n, d = X.shape
    reg = 0.002 if upd == "l1" else 0.0   # L1: the soft threshold and regVal = reg ||w||_1
    data = pkg.PartitionedData.parallelize(y, X.astype(storage), P, dtype=storage)
    offs = [i * n // P for i in range(P)] + [n]
    w, h, counts = pkg.runParallelizedSGD(data, getattr(pkg, G[grad])(), getattr(pkg, U[upd])(), step, iters,
                                          reg, frac, np.zeros(d), 0.0, compute_dtype=compute,
                                          return_chain_counts=True)
    variant = pkg.optimization.get_context(0).last_kernel()
    wr, hr, cr = oracle.run(oracle.Matrix(y, X.astype(np.float64)), offs, grad, upd, step, iters, reg,
                            np.zeros(d), tol=0.0, fraction=frac, n_threads=8)
    return w, h, counts, wr, hr, cr, variant


@pytest.mark.parametrize("upd", ["adagrad", "adam", "l1"])
@pytest.mark.parametrize("grad", ["logistic", "least_squares", "hinge"])
@pytest.mark.parametrize("d,storage", [(300, np.float32), (700, np.float32), (1024, np.float32),
                                       (2048, np.float32), (256, np.float64), (1000, np.float64)])
def test_split_fp64_parity(pkg, oracle, grad, upd, d, storage):
    rng = np.random.default_rng(d + 7 * len(grad) + len(upd))
    X, y = synth(rng, 1600, d, grad)
    w, h, counts, wr, hr, cr, variant = run_both(pkg, oracle, X, y, storage, 4, grad, upd, 0.1)
    assert variant == stateful_variant(upd, 0.0, nv_of(d, storage)) and variant >= 800
    tag = f"{grad} {upd} d={d} {np.dtype(storage).name}"
    assert [list(c) for c in counts] == [list(c) for c in cr], tag
    assert_close(w, wr, what=tag + " weights")
    assert_close(h, hr, what=tag + " loss")


@pytest.mark.parametrize("upd", ["adagrad", "adam", "l1"])
@pytest.mark.parametrize("grad", ["logistic", "least_squares", "hinge"])
@pytest.mark.parametrize("d", [700, 1024])
def test_split_fp32(pkg, oracle, grad, upd, d):
    rng = np.random.default_rng(d + 3 * len(grad) + len(upd))
    X, y = synth(rng, 4000, d, grad)
    w, h, counts, wr, hr, cr, variant = run_both(pkg, oracle, X, y, np.float32, 4, grad, upd, 0.05, compute="f32")
    assert variant == 844
    assert [list(c) for c in counts] == [list(c) for c in cr]
    scale = np.max(np.abs(wr))
    err = np.max(np.abs(w - wr)) / scale
    assert err <= FP32_REL, f"{grad} {upd} d={d}: weights {err:.3g} x max|w|"
    assert_close(h, hr, rel=FP32_LOSS_REL, what=f"{grad} {upd} d={d} fp32 loss")


@pytest.mark.parametrize("upd", ["adagrad", "adam"])
def test_split_sampled_batches(pkg, oracle, upd):
    # miniBatchFraction < 1: the loader streams the sampled rows by index (PSGD.scala:242)
    rng = np.random.default_rng(21)
    X, y = synth(rng, 3000, 512, "logistic")
    w, h, counts, wr, hr, cr, variant = run_both(pkg, oracle, X, y, np.float32, 3, "logistic", upd, 0.1, frac=0.4)
    assert variant == 822
    assert [list(c) for c in counts] == [list(c) for c in cr]
    assert_close(w, wr, what="sampled weights")
    assert_close(h, hr, what="sampled loss")


@pytest.mark.parametrize("n,P", [(7, 5), (3, 5)])
def test_split_tiny_and_empty_partitions(pkg, oracle, n, P):
    # 1-row chains (no prefetch), and partitions with no rows (count 0, w_in)
    rng = np.random.default_rng(n * P)
    X, y = synth(rng, n, 600, "logistic")
    for upd in ("adagrad", "adam"):
        w, h, counts, wr, hr, cr, variant = run_both(pkg, oracle, X, y, np.float32, P, "logistic", upd, 0.5)
        assert variant == 844
        assert [list(c) for c in counts] == [list(c) for c in cr]
        assert_close(w, wr, what=f"{upd} n={n} P={P} weights")
        assert_close(h, hr, what=f"{upd} n={n} P={P} loss")


@pytest.mark.parametrize("upd", ["simple", "squared_l2", "l1", "adagrad", "adam"])
@pytest.mark.parametrize("grad", ["logistic", "least_squares", "hinge"])
@pytest.mark.parametrize("d,storage,tol", [(700, np.float32, 0.002), (1024, np.float32, 0.02),
                                           (256, np.float64, 0.005)])
def test_split_per_sample_convergence(pkg, oracle, monkeypatch, grad, upd, d, storage, tol):
    """tol > 0: the per-sample isConverged break (PSGD.scala:262, :324-336) on chain_split, its
    test of sample t - 1 carried by the exchange of sample t; every updater (Simple / SquaredL2
    take this kernel only with the test, and in fp64 only with PSGD_B64_CONV=0: chain_block64
    runs their break by default, test_gpu_parity.py::test_block64_per_sample_break). fp64 at 1e-9
    with exact per-chain counts."""
    monkeypatch.setenv("PSGD_B64_CONV", "0")
    rng = np.random.default_rng(d + 11 * len(grad) + 5 * len(upd))
    X, y = synth(rng, 2400, d, grad)
    n = X.shape[0]
    P = 4
    reg = {"l1": 0.002, "squared_l2": 0.05}.get(upd, 0.0)
    data = pkg.PartitionedData.parallelize(y, X.astype(storage), P, dtype=storage)
    offs = [i * n // P for i in range(P)] + [n]
    w, h, counts = pkg.runParallelizedSGD(data, getattr(pkg, G[grad])(), getattr(pkg, U[upd])(), 0.2, 3,
                                          reg, 1.0, np.zeros(d), tol, return_chain_counts=True)
    assert pkg.optimization.get_context(0).last_kernel() == stateful_variant(upd, tol, nv_of(d, storage))
    wr, hr, cr = oracle.run(oracle.Matrix(y, X.astype(np.float64)), offs, grad, upd, 0.2, 3, reg,
                            np.zeros(d), tol=tol, n_threads=8)
    tag = f"{grad} {upd} d={d} tol={tol}"
    assert [list(c) for c in counts] == [list(c) for c in cr[: len(counts)]], tag
    assert_close(w, wr, what=tag + " weights")
    assert_close(h, hr, what=tag + " loss")


@pytest.mark.parametrize("upd", ["l1", "squared_l2"])
@pytest.mark.parametrize("d,storage", [(1024, np.float32), (256, np.float64)])
def test_split_break_same_parity_final_exchange(pkg, oracle, monkeypatch, upd, d, storage):
    """The regVal exchange after a per-sample break: a chain that breaks at sample t
    with t = n (mod 2) must not publish its final norms into slot t & 1, which a slower wave may
    still be polling for sample t. Many short chains of ragged lengths (37 / 38 rows) at a tol that
    breaks most of them early: both parities of the break against n occur, every chain's count is
    exact and the run finishes (no watchdog). (fp64 SquaredL2 takes chain_split here only with
    PSGD_B64_CONV=0.)"""
    monkeypatch.setenv("PSGD_B64_CONV", "0")
    rng = np.random.default_rng(4242 + d)
    P = 128
    n = P * 37 + 61
    X, y = synth(rng, n, d, "logistic")
    reg = {"l1": 0.002, "squared_l2": 0.05}[upd]
    tol = 0.05
    data = pkg.PartitionedData.parallelize(y, X.astype(storage), P, dtype=storage)
    offs = [i * n // P for i in range(P)] + [n]
    sizes = np.diff(offs)
    w, h, counts = pkg.runParallelizedSGD(data, pkg.LogisticGradient(), getattr(pkg, U[upd])(), 0.5, 3,
                                          reg, 1.0, np.zeros(d), tol, return_chain_counts=True)
    wr, hr, cr = oracle.run(oracle.Matrix(y, X.astype(np.float64)), offs, "logistic", upd, 0.5, 3, reg,
                            np.zeros(d), tol=tol, n_threads=8)
    assert [list(c) for c in counts] == [list(c) for c in cr[: len(counts)]]
    same = sum(int(c < s and c % 2 == s % 2) for it in cr for c, s in zip(it, sizes))
    other = sum(int(c < s and c % 2 != s % 2) for it in cr for c, s in zip(it, sizes))
    assert same > 0 and other > 0, (same, other)
    assert_close(w, wr, what=f"{upd} break-parity weights")
    assert_close(h, hr, what=f"{upd} break-parity loss")
