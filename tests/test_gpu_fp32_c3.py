"""fp32 throughput mode at BASELINE config 3's own hyper-parameters (Logistic, dense d = 1,024,
step 1.0, 3 iterations, 256 chains per GPU) against the fp64 oracle on the same (fp32-stored)
rows: SURVEY §8c asks for a stated fp32 tolerance; ParallelizedSGD.scala:283 is the loss history
it is stated on.

At this step size fp32 compute is a throughput mode WITHOUT a uniform weight tolerance
(DESIGN.md §4): with ||x||^2 ~ 1,024 every early sample moves w by O(1), so the fp32/fp64
weight difference depends on the trajectory (measured 4.8e-6 .. 3.7e-3 x max|w| over these chain
lengths; the standard 2e-4 holds at 40, 200 and 48,828 rows per chain, not at 2,000). What is
asserted uniformly, for every chain length: the fp64 parity mode (chain_block64) at 1e-9 of the
oracle, and the fp32 loss history within FP32_C3_LOSS_REL of the oracle's. The fp32 weight
difference is printed, not asserted.
"""
import numpy as np
import pytest

from conftest import has_gpu

pytestmark = pytest.mark.gpu

# the fp32 loss history at C3's hyper-parameters, relative to the fp64 oracle: one bound for
# every chain length (no weight bound: see the module docstring)
FP32_C3_LOSS_REL = 1e-3


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not has_gpu():
        pytest.skip("no GPU")


def c3_prefix(P=256, per=200, d=1024, seed=44):
    """X ~ N(0,1) stored fp32, w* ~ N(0, 1/d), y = 1{w*.x + Logistic(0,1) > 0}."""
    rng = np.random.default_rng(seed)
    n = P * per
    X = rng.standard_normal((n, d), dtype=np.float32)
    w = rng.standard_normal(d) / np.sqrt(d)
    y = ((X.astype(np.float64) @ w + rng.logistic(size=n)) > 0).astype(np.float64)
    offs = [i * n // P for i in range(P)] + [n]
    return X, y, offs


@pytest.mark.parametrize("P,per", [(256, 40), (256, 200), (64, 2000), (8, 48828)])
def test_fp32_at_c3_hyper_parameters(pkg, oracle, P, per):
    X, y, offs = c3_prefix(P=P, per=per)
    d = X.shape[1]
    parts = [pkg.DensePartition(y[a:b], X[a:b]) for a, b in zip(offs[:-1], offs[1:])]
    data = pkg.PartitionedData(parts)
    args = (pkg.LogisticGradient(), pkg.SimpleSGDUpdater(), 1.0, 3, 0.0, 1.0, np.zeros(d), 0.0)
    w32, h32 = pkg.runParallelizedSGD(data, *args, compute_dtype="f32")
    assert pkg.optimization.get_context(0).last_kernel() == 304   # chain_block, NV = 4
    w64, h64 = pkg.runParallelizedSGD(data, *args)                 # fp64 parity mode (chain_block64)
    wr, hr, _ = oracle.run(oracle.Matrix(y, X.astype(np.float64)), offs, "logistic", "simple", 1.0, 3, 0.0,
                           np.zeros(d), tol=0.0, n_threads=8)
    scale = np.max(np.abs(wr))
    rel64 = np.max(np.abs(w64 - wr)) / scale
    err_w = np.max(np.abs(w32 - wr)) / scale
    big = np.abs(wr) > 0.1 * scale
    err_w_elem = np.max(np.abs(w32 - wr)[big] / np.abs(wr[big]))
    err_h = np.max(np.abs(h32 - hr) / np.abs(hr))
    print(f"\nC3 prefix {len(offs) - 1} chains x {per} rows, step 1.0, 3 iterations: fp32 weights "
          f"{err_w:.3g} x max|w| (element-wise {err_w_elem:.3g} where |w| > 0.1 max), loss {err_h:.3g} "
          f"relative; fp64 mode {rel64:.3g}")
    assert rel64 < 1e-9
    assert np.isfinite(w32).all()
    assert err_h <= FP32_C3_LOSS_REL, err_h
