"""The placement re-roll of the CSR chains' weight-vector sets (psgd_capi.cpp reroll_vectors,
psgd_probe.hip): a freshly allocated set below the VMM threshold is chosen
from PSGD_REROLL candidates by a probe of the chains' scattered access pattern. The epoch's results
do not depend on which candidate is kept (the vectors are re-initialised every epoch), so the CSR
chain on a re-rolled set matches the oracle (ParallelizedSGD.scala:243-270) at the fp32 tolerance,
and PSGD_REROLL=1 turns the re-roll off."""
import numpy as np
import pytest

from conftest import has_gpu

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not has_gpu():
        pytest.skip("no GPU")


def csr(rng, n, d, nnz=24):
    width = d // nnz
    col = (np.arange(nnz) * width)[None, :] + rng.integers(0, width, (n, nnz))
    val = rng.uniform(size=(n, nnz))
    val = (val / np.linalg.norm(val, axis=1, keepdims=True)).astype(np.float32)
    y = (rng.uniform(size=n) > 0.5).astype(np.float64)
    rp = np.arange(n + 1, dtype=np.int64) * nnz
    return y, rp, col.reshape(-1).astype(np.int32), val.reshape(-1)


@pytest.mark.parametrize("reroll", ["8", "1"])
def test_reroll_keeps_results(pkg, oracle, monkeypatch, reroll):
    N = pkg._native
    monkeypatch.setenv("PSGD_REROLL", reroll)
    rng = np.random.default_rng(31)
    d, P, per = 30_000, 16, 300
    y, rp, col, val = csr(rng, P * per, d)
    offs = [p * per for p in range(P + 1)]
    s0 = N.reroll_stats()
    ctx = N.Context(0)
    for p in range(P):
        a, b = offs[p], offs[p + 1]
        ctx.register_csr(p, y[a:b], rp[a:b + 1] - rp[a], col[rp[a]:rp[b]], val[rp[a]:rp[b]], d)
    prm = pkg.optimization.make_params(pkg.HingeGradient(), pkg.SimpleSGDUpdater(), 0.5, 0.0, 1.0, 0.0, "f32")
    w, _, loss, cnt, counts = ctx.run_epoch(prm, np.zeros(d))
    s1 = N.reroll_stats()
    ctx.close()
    assert s1["sets"] - s0["sets"] == (1 if reroll == "8" else 0), (s0, s1)
    wr, _, lr, cr = oracle.run_chains(oracle.Matrix(y, row_ptr=rp, col=col, val=val.astype(np.float64), d=d),
                                      offs, "hinge", "simple", 0.5, 0.0, np.zeros(d))
    assert list(counts) == list(cr) and cnt == P * per
    # the fold of the chains (PSGD.scala:271-276: equal counts -> the mean), fp32 tolerance
    wmean = wr.mean(axis=0)
    assert np.max(np.abs(w - wmean)) <= 2e-4 * np.max(np.abs(wmean)), np.max(np.abs(w - wmean))
    assert abs(loss - lr.sum()) <= 1e-4 * abs(lr.sum())
