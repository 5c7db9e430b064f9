"""chain_block64 with LeastSquares + Simple (the fp64 parity mode of BASELINE config 2) on ragged
partitions -- every chain ends in a partial block -- at steps from small to the edge of stability,
with and without the per-sample break, f32 and f64 rows, one and two chain waves and the Gram split
by features (NV = 8), against the oracle (ParallelizedSGD.scala:243-270, SGDUpdater.scala:86-98) at
the fp64 bar: 1e-9 relative and exact per-chain counts."""
import numpy as np
import pytest

from conftest import has_gpu
from test_gpu_parity import assert_close, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not has_gpu():
        pytest.skip("no GPU")


# (d, row dtype, stepSize): d = 60 f64 rows is one chain wave (NV = 1); 512 / 700 f32 rows two
# (NV = 2 / 4); 1,000 f64 rows NV = 8 (the Gram split by features). The Gram terms s G[k][i] of a
# block reach ~1 at d = 60, step 0.02 (the recurrence far from the identity) and stay ~0.05 at the
# small steps.
CASES = [(60, np.float64, 0.02), (60, np.float64, 0.002), (512, np.float32, 0.003),
         (700, np.float32, 0.002), (1000, np.float64, 0.0015)]


@pytest.mark.parametrize("d,dtype,step", CASES)
@pytest.mark.parametrize("tol", [0.0, 2e-4])
def test_block64_least_squares_ragged(pkg, oracle, d, dtype, step, tol):
    rng = np.random.default_rng(int(d * 1000 * step) + 7)
    # ragged partitions: every chain ends in a partial block
    sizes = [203, 157, 98, 61, 250, 13]
    n = sum(sizes)
    offs = np.concatenate([[0], np.cumsum(sizes)]).tolist()
    X, y = synth(rng, n, d, "least_squares", dtype)
    data = pkg.PartitionedData([pkg.DensePartition(y[a:b], X[a:b]) for a, b in zip(offs[:-1], offs[1:])])
    w0 = 0.01 * np.ones(d)
    w, h, c = pkg.runParallelizedSGD(data, pkg.LeastSquaresGradient(), pkg.SimpleSGDUpdater(), step, 3,
                                     0.0, 1.0, w0, tol, return_chain_counts=True)
    v = pkg.optimization.get_context(0).last_kernel()
    assert 700 <= v < 800, v
    wr, hr, cr = oracle.run(oracle.Matrix(y, X.astype(np.float64)), offs, "least_squares", "simple", step, 3,
                            0.0, w0, tol=tol)
    assert np.array_equal(np.asarray(c), np.asarray(cr)), (c, cr)
    assert_close(w, wr, what="weights")
    assert_close(h, hr, what="loss history")
