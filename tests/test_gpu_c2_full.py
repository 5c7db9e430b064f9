"""BASELINE config 2 at its full geometry against the oracle: LeastSquares, dense 10M x 512 f32
rows, 256 chains of 39,062 / 39,063 rows, step 1e-3, one iteration.

The 20 GB row buffer puts chain offsets past 2^32 bytes, and every chain runs its real length,
so the offset arithmetic of the registration, the ring loader and the folds meets the oracle at
the size the bench runs (the other C2 tests use 1,001-row chains). fp64 compute (chain_block64,
the parity mode) at 1e-9 with exact counts; fp32 compute (chain_block, the headline kernel) at
the fp32 tolerance. Rows: a 65,537-row N(0,1) block tiled over the 10M rows (a prime period, so
no two chains see the same sequence) -- the host needs the f64 copy for the oracle (41 GB).
Reference: ParallelizedSGD.scala:243-276."""
import numpy as np
import pytest

from conftest import has_gpu
from test_gpu_parity import assert_close

pytestmark = pytest.mark.gpu

N, D, P = 10_000_000, 512, 256


@pytest.fixture(scope="module")
def c2_full():
    if not has_gpu():
        pytest.skip("no GPU")
    rng = np.random.default_rng(43)
    base = rng.standard_normal((65_537, D), dtype=np.float32)
    w_star = rng.standard_normal(D) / np.sqrt(D)
    yb = base.astype(np.float64) @ w_star
    idx = np.arange(N, dtype=np.int64) % base.shape[0]
    X = base[idx]
    y = yb[idx] + 0.01 * rng.standard_normal(N)
    return X, y


def test_c2_full_geometry(pkg, oracle, c2_full):
    X, y = c2_full
    data = pkg.PartitionedData.parallelize(y, X, P, dtype=np.float32)
    offs = [i * N // P for i in range(P)] + [N]
    assert max(b - a for a, b in zip(offs[:-1], offs[1:])) == 39_063
    args = (pkg.LeastSquaresGradient(), pkg.SimpleSGDUpdater(), 1e-3, 1, 0.0, 1.0, np.zeros(D), 0.0)
    w64, h64, c64 = pkg.runParallelizedSGD(data, *args, return_chain_counts=True)
    assert pkg.optimization.get_context(0).last_kernel() == 712   # chain_block64 NV 2, 2 chain waves
    w32, h32 = pkg.runParallelizedSGD(data, *args, compute_dtype="f32")
    assert pkg.optimization.get_context(0).last_kernel() == 302   # chain_block NV 2
    del data
    wr, hr, cr = oracle.run(oracle.Matrix(y, X), offs, "least_squares", "simple", 1e-3, 1, 0.0,
                            np.zeros(D), tol=0.0, n_threads=16)
    assert [list(c) for c in c64] == [list(c) for c in cr]
    assert_close(w64, wr, what="C2 full fp64 weights")
    assert_close(h64, hr, what="C2 full fp64 loss")
    scale = np.max(np.abs(wr))
    assert np.max(np.abs(w32 - wr)) <= 2e-4 * scale
    assert np.max(np.abs(h32 - hr) / np.abs(hr)) <= 1e-4
