"""fp32 throughput mode at BASELINE config 3's own hyper-parameters (Logistic, dense d = 1,024,
step 1.0, 3 iterations, 256 chains per GPU) against the fp64 oracle on the same (fp32-stored)
rows: SURVEY §8c asks for a stated fp32 tolerance; ParallelizedSGD.scala:253-268 is the chain and
:283 the loss history it is stated on.

The stated fp32 tolerance at C3: weights within FP32_C3_W_REL x max|w| of the fp64
oracle AND within FP32_C3_VS_SEQ x the largest error of the three fp32 restatements of the
reference on the same data (oracle.run_f32: the same chain with float operands -- left-fold dots,
tree dots, and float weights with double dots; floor 2e-4) -- the fp32 kernel is no further from the
fp64 reference than plain fp32 evaluations of the reference's own loop are. The loss history within
FP32_C3_LOSS_REL. Why the weight bound is looser than the 2e-4 x max|w| that holds on the other
configs: with ||x||^2 ~ 1,024 and step 1.0 every early sample moves w by O(1), and over thousands of
rows per chain the trajectory amplifies the rounding of fp32 WEIGHTS ~1e5-fold -- at 64 x 2,000 the
left-fold restatement is 8.1e-3 x max|w| from the fp64 oracle, the tree one 2.9e-3, and even exact
dots over float weights 7.3e-4 (tests/test_oracle_f32.py pins these on the CPU; the sweep over
chain lengths, up to 2.9e-2, is in DESIGN.md §4).
"""
import numpy as np
import pytest

from conftest import has_gpu

pytestmark = pytest.mark.gpu

# the fp32 mode's stated tolerance at C3's hyper-parameters, against the fp64 oracle
FP32_C3_W_REL = 5e-2       # weights, x max|w|, every chain length
FP32_C3_VS_SEQ = 2.0       # weights, x the largest fp32 restatement error on the same data (floor 2e-4)
FP32_C3_LOSS_REL = 1e-3    # loss history, relative


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


@pytest.mark.parametrize("P,per", [(256, 40), (256, 200), (64, 2000), (8, 4000), (64, 4000), (8, 48828)])
def test_fp32_at_c3_hyper_parameters(pkg, oracle, P, per):
    X, y, offs = c3_prefix(P=P, per=per)
    d = X.shape[1]
    parts = [pkg.DensePartition(y[a:b], X[a:b]) for a, b in zip(offs[:-1], offs[1:])]
    data = pkg.PartitionedData(parts)
    args = (pkg.LogisticGradient(), pkg.SimpleSGDUpdater(), 1.0, 3, 0.0, 1.0, np.zeros(d), 0.0)
    w32, h32 = pkg.runParallelizedSGD(data, *args, compute_dtype="f32")
    assert pkg.optimization.get_context(0).last_kernel() == 304   # chain_block, NV = 4
    w64, h64 = pkg.runParallelizedSGD(data, *args)                 # fp64 parity mode (chain_block64)
    mat = oracle.Matrix(y, X.astype(np.float64))
    oargs = (mat, offs, "logistic", "simple", 1.0, 3, 0.0, np.zeros(d))
    wr, hr, _ = oracle.run(*oargs, tol=0.0, n_threads=8)
    scale = np.max(np.abs(wr))
    # the fp32 restatements: left-fold dots, tree dots, float weights with double dots
    err_r = [np.max(np.abs(oracle.run_f32(*oargs, order=o, tol=0.0, n_threads=8)[0] - wr)) / scale
             for o in (0, 1, 2)]
    err_seq = max(err_r)
    rel64 = np.max(np.abs(w64 - wr)) / scale
    err_w = np.max(np.abs(w32 - wr)) / scale
    err_h = np.max(np.abs(h32 - hr) / np.abs(hr))
    print(f"\nC3 prefix {len(offs) - 1} chains x {per} rows, step 1.0, 3 iterations (x max|w|): "
          f"fp32 kernel {err_w:.3g}, fp32 restatements {err_r[0]:.3g} / {err_r[1]:.3g} / {err_r[2]:.3g} "
          f"(left fold / tree / float weights only); loss {err_h:.3g} relative; fp64 mode {rel64:.3g}")
    assert rel64 < 1e-9
    assert np.isfinite(w32).all()
    assert err_w <= FP32_C3_W_REL, err_w
    assert err_w <= FP32_C3_VS_SEQ * max(err_seq, 2e-4), (err_w, err_seq)
    assert err_h <= FP32_C3_LOSS_REL, err_h
