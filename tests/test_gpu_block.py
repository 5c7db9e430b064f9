"""The blocked fp32 chain kernel (psgd_block.hip) against the fp64 CPU oracle.

fp32 compute is the throughput mode; its stated tolerance is weights within
FP32_REL * max|w| and the loss history within FP32_LOSS_REL relative of the fp64 oracle on the
same inputs, for well-conditioned steps. Chain counts are exact at tol = 0; with the per-sample
convergence test (tol > 0, decided inside the block from the recurrence's norms) a break may fall
one side of the fp32/fp64 rounding or the other, so counts are compared chain by chain with a
small allowance (test_block_per_sample_break).

Cases: every gradient x {Simple, SquaredL2}, f32 and f64 storage, feature counts that do and do
not fill the lanes' 16-byte vectors (FULL / partial rows), partitions whose length is not a
multiple of the 8-row block, partitions shorter than a block, empty partitions, and 256 chains
(one per CU, the bench geometry).
"""
import numpy as np
import pytest

from conftest import has_gpu
from test_gpu_parity import fp32_break_counts_agree

pytestmark = pytest.mark.gpu

FP32_REL = 2e-4
FP32_LOSS_REL = 1e-4

G = {"logistic": "LogisticGradient", "least_squares": "LeastSquaresGradient", "hinge": "HingeGradient"}
U = {"simple": "SimpleSGDUpdater", "squared_l2": "SquaredL2SGDUpdater"}


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not has_gpu():
        pytest.skip("no GPU")


def synth(rng, n, d, grad, dtype):
    X = rng.standard_normal((n, d)).astype(dtype)
    wt = rng.standard_normal(d) / np.sqrt(d)
    z = X.astype(np.float64) @ wt
    if grad == "least_squares":
        y = z + 0.1 * rng.standard_normal(n)
    else:
        y = ((z + rng.logistic(size=n)) > 0).astype(np.float64)
    return X, y


def step_for(grad, d):
    # well-conditioned: s * ||x||^2 < 1 for least squares; logistic/hinge steps that keep the
    # fp32 and fp64 trajectories from separating for reasons unrelated to the kernel
    return {"least_squares": 0.5 / d, "logistic": 2.0 / d, "hinge": 1.0 / d}[grad]


def check(pkg, oracle, X, y, offs, grad, upd, step, reg, iters, dtype, expect_variant=None, w0=None):
    d = X.shape[1]
    parts = [pkg.DensePartition(y[a:b], X[a:b]) for a, b in zip(offs[:-1], offs[1:])]
    data = pkg.PartitionedData(parts)
    w0 = np.zeros(d) if w0 is None else w0
    w, h, counts = pkg.runParallelizedSGD(data, getattr(pkg, G[grad])(), getattr(pkg, U[upd])(), step,
                                          iters, reg, 1.0, w0, 0.0, compute_dtype="f32",
                                          return_chain_counts=True)
    if expect_variant is not None:
        assert pkg.optimization.get_context(0).last_kernel() == expect_variant
    wr, hr, cr = oracle.run(oracle.Matrix(y, X.astype(np.float64)), offs, grad, upd, step, iters, reg,
                            w0, tol=0.0, n_threads=8)
    tag = f"d={d} {grad} {upd} {np.dtype(dtype).name}"
    assert [list(c) for c in counts] == [list(c) for c in cr[: len(counts)]], tag
    scale = max(np.max(np.abs(wr)), 1e-30)
    err = np.max(np.abs(w - wr)) / scale
    assert err <= FP32_REL, f"{tag}: weights max err {err:.3g} x max|w|"
    herr = np.max(np.abs(h - hr) / np.maximum(np.abs(hr), 1e-30))
    assert herr <= FP32_LOSS_REL, f"{tag}: loss rel err {herr:.3g}"
    return w, h


@pytest.mark.parametrize("d", [3, 100, 512, 700, 1024, 2048])
@pytest.mark.parametrize("grad", ["least_squares", "logistic", "hinge"])
@pytest.mark.parametrize("upd", ["simple", "squared_l2"])
def test_block_fp32_storage(pkg, oracle, d, grad, upd):
    rng = np.random.default_rng(d * 31 + len(grad) + len(upd))
    n, P = 2403, 5                      # 480/481-row partitions: ragged last block
    X, y = synth(rng, n, d, grad, np.float32)
    offs = [i * n // P for i in range(P)] + [n]
    nv = 1
    while nv * 256 < d:
        nv *= 2
    check(pkg, oracle, X, y, offs, grad, upd, step_for(grad, d), 0.05, 3, np.float32,
          expect_variant=300 + nv)


@pytest.mark.parametrize("d", [5, 128, 512, 1000])
def test_block_fp64_storage(pkg, oracle, d):
    rng = np.random.default_rng(d + 1)
    n, P = 1605, 4
    for grad in ("least_squares", "logistic"):
        X, y = synth(rng, n, d, grad, np.float64)
        offs = [i * n // P for i in range(P)] + [n]
        nv = 1
        while nv * 128 < d:
            nv *= 2
        check(pkg, oracle, X, y, offs, grad, "simple", step_for(grad, d), 0.0, 2, np.float64,
              expect_variant=300 + nv)


def test_block_short_and_empty_partitions(pkg, oracle):
    """Partitions of 0, 1, 3, 7, 8, 9 and 17 rows: the tail block and a block-less chain."""
    rng = np.random.default_rng(12)
    sizes = [1, 3, 7, 8, 0, 9, 17, 2]
    n, d = sum(sizes), 64
    offs = list(np.cumsum([0] + sizes))
    for grad in ("least_squares", "logistic", "hinge"):
        for upd in ("simple", "squared_l2"):
            X, y = synth(rng, n, d, grad, np.float32)
            check(pkg, oracle, X, y, offs, grad, upd, step_for(grad, d), 0.1, 3, np.float32,
                  w0=0.05 * np.ones(d))


def test_block_many_chains_bench_geometry(pkg, oracle):
    """256 chains (one per CU, the largest LDS ring), d = 512 f32, least squares: the bench's
    kernel instance on a 1000-row-per-chain sample, plus run-to-run determinism."""
    rng = np.random.default_rng(21)
    P, m, d = 256, 1001, 512
    n = P * m
    X, y = synth(rng, n, d, "least_squares", np.float32)
    offs = [i * n // P for i in range(P)] + [n]
    w1, h1 = check(pkg, oracle, X, y, offs, "least_squares", "simple", 1e-3, 0.0, 2, np.float32,
                   expect_variant=302)
    data = pkg.PartitionedData([pkg.DensePartition(y[a:b], X[a:b]) for a, b in zip(offs[:-1], offs[1:])])
    w2, h2 = pkg.runParallelizedSGD(data, pkg.LeastSquaresGradient(), pkg.SimpleSGDUpdater(), 1e-3, 2,
                                    0.0, 1.0, np.zeros(d), 0.0, compute_dtype="f32")
    assert np.array_equal(w1, w2) and np.array_equal(h1, h2)


def test_block_device_registration(pkg, oracle):
    """Rows registered zero-copy from HBM (the bench path) give the same bits as host rows."""
    import torch
    rng = np.random.default_rng(13)
    n, d, P = 4001, 512, 6
    X, y = synth(rng, n, d, "logistic", np.float32)
    offs = [i * n // P for i in range(P)] + [n]
    host = pkg.PartitionedData([pkg.DensePartition(y[a:b], X[a:b]) for a, b in zip(offs[:-1], offs[1:])])
    Xd, yd = torch.from_numpy(X).cuda(), torch.from_numpy(y).cuda()
    dev = pkg.PartitionedData([pkg.DevicePartition(yd[a:b], Xd[a:b], d) for a, b in zip(offs[:-1], offs[1:])])
    args = (pkg.LogisticGradient(), pkg.SquaredL2SGDUpdater(), 0.004, 2, 0.01, 1.0, np.zeros(d), 0.0)
    w1, h1 = pkg.runParallelizedSGD(host, *args, compute_dtype="f32")
    w2, h2 = pkg.runParallelizedSGD(dev, *args, compute_dtype="f32")
    assert np.array_equal(w1, w2) and np.array_equal(h1, h2)


def test_block_per_sample_kernel_on_request(pkg, oracle, monkeypatch):
    """PSGD_B64_CONV=0 keeps tol > 0 on the per-sample kernels (A/B measurements)."""
    monkeypatch.setenv("PSGD_B64_CONV", "0")
    rng = np.random.default_rng(14)
    X, y = synth(rng, 400, 64, "logistic", np.float32)
    data = pkg.PartitionedData.parallelize(y, X, 2, dtype=np.float32)
    pkg.runParallelizedSGD(data, pkg.LogisticGradient(), pkg.SimpleSGDUpdater(), 0.03, 1, 0.0, 1.0,
                           np.zeros(64), 0.01, compute_dtype="f32")
    assert pkg.optimization.get_context(0).last_kernel() == 101


@pytest.mark.parametrize("grad", ["logistic", "least_squares", "hinge"])
@pytest.mark.parametrize("upd", ["simple", "squared_l2"])
@pytest.mark.parametrize("d,dtype", [(60, np.float32), (512, np.float32), (1024, np.float32), (300, np.float64)])
def test_block_per_sample_break(pkg, oracle, grad, upd, d, dtype):
    """tol > 0 on chain_block (variant 340 + NV): the per-sample isConverged break (PSGD.scala:262,
    :324-336) from the block recurrence's norms, against the fp64 oracle. 64 ragged chains at tols
    that break most of them at assorted rows of their blocks: at least 90 % of the per-chain counts
    equal the oracle's (a break may land a row off across the fp32/fp64 rounding), and where every
    count agrees the weights and losses are within the fp32 tolerance."""
    rng = np.random.default_rng(d + 17 * len(grad) + len(upd))
    P = 64
    n = P * 45 + 29
    X, y = synth(rng, n, d, grad, dtype)
    data = pkg.PartitionedData.parallelize(y, X, P, dtype=dtype)
    offs = [i * n // P for i in range(P)] + [n]
    sizes = np.diff(offs)
    vec = 4 if dtype == np.float32 else 2
    nv = 1
    while nv * 64 * vec < d:
        nv *= 2
    step = {"least_squares": 0.5 / d, "logistic": 4.0 / d, "hinge": 2.0 / d}[grad]
    breaks = 0
    for tol in (0.01, 0.03):
        w, h, counts = pkg.runParallelizedSGD(data, getattr(pkg, G[grad])(), getattr(pkg, U[upd])(), step, 3,
                                              0.05, 1.0, np.zeros(d), tol, compute_dtype="f32",
                                              return_chain_counts=True)
        assert pkg.optimization.get_context(0).last_kernel() == 340 + nv
        wr, hr, cr, mg = oracle.run_with_margins(oracle.Matrix(y, X.astype(np.float64)), offs, grad, upd, step,
                                                 3, 0.05, np.zeros(d), tol=tol, n_threads=8)
        tag = f"{grad} {upd} d={d} tol={tol}"
        breaks += sum(int(c < s) for it in cr for c, s in zip(it, sizes))
        if fp32_break_counts_agree(counts, cr, mg, tag) and len(h) == len(hr):
            scale = max(np.max(np.abs(wr)), 1e-30)
            err = np.max(np.abs(w - wr)) / scale
            assert err <= FP32_REL, f"{tag}: weights max err {err:.3g} x max|w|"
            herr = np.max(np.abs(h - hr) / np.maximum(np.abs(hr), 1e-30))
            assert herr <= FP32_LOSS_REL, f"{tag}: loss rel err {herr:.3g}"
    assert breaks > 0
