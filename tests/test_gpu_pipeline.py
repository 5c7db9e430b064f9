"""The driver's pipelined loop on the GPU (ParallelizedSGD._run_pipelined: tol == 0, full
batches; each epoch enqueued with the previous epoch's folded weights before that epoch's
scalars are read back) against the loop's synchronous form (ParallelizedSGD.scala:237-297, one
scalar read per epoch) and the oracle; the context's per-launch chain timings."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _data(pkg, seed, n, d, P, f32=False):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, d))
    if f32:
        X = X.astype(np.float32)
    y = (rng.random(n) < 0.5).astype(np.float64)
    return (pkg.PartitionedData.parallelize(y, X, P, dtype=np.float32 if f32 else np.float64),
            X.astype(np.float64), y)


def _sync_loop(pkg, data, g, u, step, iters, reg, w0, compute):
    """The synchronous loop, step by step (the shape runParallelizedSGD has when its branches are
    not known ahead: scalars read after every epoch)."""
    eng = pkg.HipEngine(data, 0, 1, weight_dim=len(w0))
    params = pkg.make_params(g, u, step, reg, 1.0, 0.0, compute)
    w = eng.weights(np.asarray(w0, dtype=np.float64))
    regval = eng.initial_regval(params, np.asarray(w0, dtype=np.float64))
    hist = []
    for i in range(1, iters + 1):
        params.iteration = i
        folded, _ = eng.epoch(params, w)
        rv, loss, cnt = eng.scalars(folded)
        assert cnt > 0
        hist.append(loss / cnt + regval)
        w = eng.adopt(folded)
        regval = rv
    return eng.to_host(w), np.array(hist)


@pytest.mark.parametrize("compute", ["f64", "f32"])
@pytest.mark.parametrize("grad,upd,reg", [("LogisticGradient", "SimpleSGDUpdater", 0.0),
                                          ("LeastSquaresGradient", "SquaredL2SGDUpdater", 0.05)])
def test_pipelined_driver_matches_synchronous_loop(pkg, grad, upd, reg, compute):
    """Bit for bit: the same epochs in the same order on the same weights."""
    data, _, _ = _data(pkg, 11, 3000, 256, 8, f32=compute == "f32")
    w0 = np.full(256, 0.01)
    g, u = getattr(pkg, grad)(), getattr(pkg, upd)()
    w_p, h_p = pkg.runParallelizedSGD(data, g, u, 0.05, 7, reg, 1.0, w0, 0.0, compute_dtype=compute)
    w_s, h_s = _sync_loop(pkg, data, g, u, 0.05, 7, reg, w0, compute)
    assert len(h_p) == 7
    np.testing.assert_array_equal(w_p, w_s)
    np.testing.assert_array_equal(h_p, h_s)


@pytest.mark.parametrize("compute", ["f64", "f32"])
def test_pipelined_driver_matches_synchronous_loop_csr(pkg, compute):
    """CSR rows (chain_sparse_lds with an HBM tail; the fold over the chains' vectors writes the
    mirror), Hinge + Simple and Logistic + SquaredL2: bit for bit against the synchronous loop."""
    rng = np.random.default_rng(19)
    n, d, P, k = 6000, 30000, 8, 24
    rp = np.arange(n + 1, dtype=np.int64) * k
    col = (np.sort(rng.choice(d - k, size=(n, k)), axis=1) + np.arange(k)[None, :]).astype(np.int32).reshape(-1)
    val = rng.standard_normal(n * k)
    if compute == "f32":
        val = val.astype(np.float32)
    y = (rng.uniform(size=n) > 0.5).astype(np.float64)
    data = pkg.PartitionedData.parallelize_csr(y, rp, col, val, d, P,
                                               dtype=np.float32 if compute == "f32" else np.float64)
    w0 = np.zeros(d)
    for g, u, reg in ((pkg.HingeGradient(), pkg.SimpleSGDUpdater(), 0.0),
                      (pkg.LogisticGradient(), pkg.SquaredL2SGDUpdater(), 0.01)):
        w_p, h_p = pkg.runParallelizedSGD(data, g, u, 0.5, 5, reg, 1.0, w0, 0.0, compute_dtype=compute)
        w_s, h_s = _sync_loop(pkg, data, g, u, 0.5, 5, reg, w0, compute)
        np.testing.assert_array_equal(w_p, w_s)
        np.testing.assert_array_equal(h_p, h_s)


def test_pipelined_driver_against_oracle(pkg, oracle):
    """fp64 at 1e-9 against the CPU restatement over enough iterations that the pipeline runs
    PIPELINE_LAG epochs ahead for most of them."""
    n, d, P, iters = 4000, 100, 4, 9
    data, X, y = _data(pkg, 5, n, d, P)
    w0 = np.zeros(d)
    w, h = pkg.runParallelizedSGD(data, pkg.LogisticGradient(), pkg.SimpleSGDUpdater(), 1.0, iters, 0.0,
                                  1.0, w0, 0.0)
    offs = [p * n // P for p in range(P)] + [n]
    ew, eh, _ = oracle.run(oracle.Matrix(y, X), offs, "logistic", "simple", 1.0, iters, 0.0, w0, tol=0.0)
    np.testing.assert_allclose(w, ew, rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(h, eh, rtol=1e-9)


def test_chain_launch_timings(pkg):
    """psgd_ctx_chain_launches counts every chain launch; psgd_ctx_chain_ms reads any of the
    last 64 after later ones were enqueued, and refuses older or future launches."""
    data, _, _ = _data(pkg, 3, 2000, 128, 4)
    eng = pkg.HipEngine(data, 0, 1)
    params = pkg.make_params(pkg.LogisticGradient(), pkg.SimpleSGDUpdater(), 0.1, 0.0, 1.0, 0.0)
    w = eng.weights(np.zeros(128))
    first = eng.ctx.chain_launches()
    for i in range(70):
        params.iteration = i + 1
        folded, _ = eng.epoch(params, w)
        w = eng.adopt(folded)
    end = eng.ctx.chain_launches()
    assert end - first == 70
    ms = [eng.ctx.chain_ms(k) for k in range(end - 64, end)]
    assert all(t > 0 for t in ms)
    assert eng.ctx.last_chain_ms() == ms[-1]
    for bad in (end - 65, end, -1):
        with pytest.raises(Exception, match="not among the last 64"):
            eng.ctx.chain_ms(bad)
