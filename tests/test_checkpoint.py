"""Checkpoint / resume of the driver loop (optional row; the reference returns the
weights only, ParallelizedSGD.scala:304). A run stopped after k iterations and resumed from its
checkpoint must equal the uninterrupted run bit for bit: weights, loss history, regVal lag
(:283) and the driver-side convergence test (:289-294) included.

CPU tests drive the product's loop with the oracle computing the chains (the OracleEngine of
test_distributed_gloo.py, world 1); the GPU test uses the real HipEngine."""
import numpy as np
import pytest

from conftest import has_gpu
from test_distributed_gloo import make_oracle_engine


def _data(pkg, n=300, d=5, P=3, seed=7):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, d))
    y = (rng.uniform(size=n) > 0.5).astype(float)
    return pkg.PartitionedData.parallelize(y, X, P), d


def _run(pkg, O, data, d, iters, tol=0.0, **kw):
    eng = make_oracle_engine(pkg, O)(data, 0, 1)
    return pkg.runParallelizedSGD(data, pkg.LogisticGradient(), pkg.SquaredL2SGDUpdater(), 0.5, iters,
                                  0.01, 1.0, np.zeros(d), tol, engine=eng, **kw)


@pytest.mark.parametrize("stop", [1, 2, 4])
def test_resume_equals_uninterrupted(tmp_path, pkg, oracle, stop):
    data, d = _data(pkg)
    w_full, h_full = _run(pkg, oracle, data, d, 5)
    ck = str(tmp_path / "loop.npz")
    w_a, h_a = _run(pkg, oracle, data, d, stop, checkpoint=ck)
    assert len(h_a) == stop
    w_b, h_b = _run(pkg, oracle, data, d, 5, checkpoint=ck)
    assert np.array_equal(w_b, w_full) and np.array_equal(h_b, h_full)


def test_resume_keeps_convergence_state(tmp_path, pkg, oracle):
    # tol large enough to stop at the driver's second comparison: the resumed run must stop
    # where the uninterrupted one did (have_current survives the checkpoint)
    data, d = _data(pkg)
    w_full, h_full = _run(pkg, oracle, data, d, 50, tol=0.2)
    assert len(h_full) < 50
    ck = str(tmp_path / "loop.npz")
    _run(pkg, oracle, data, d, 1, tol=0.2, checkpoint=ck)
    w_b, h_b = _run(pkg, oracle, data, d, 50, tol=0.2, checkpoint=ck)
    assert np.array_equal(w_b, w_full) and np.array_equal(h_b, h_full)
    # a converged checkpoint: nothing more runs
    w_c, h_c = _run(pkg, oracle, data, d, 50, tol=0.2, checkpoint=ck)
    assert np.array_equal(w_c, w_full) and np.array_equal(h_c, h_full)


def test_checkpoint_interval(tmp_path, pkg, oracle):
    data, d = _data(pkg)
    ck = str(tmp_path / "loop.npz")
    _run(pkg, oracle, data, d, 5, checkpoint=ck, checkpoint_every=2)
    z = np.load(ck, allow_pickle=False)
    assert int(z["i"]) == 6 and len(z["history"]) == 5   # the last iteration is always saved
    with pytest.raises(pkg.IllegalArgumentException):
        _run(pkg, oracle, data, d, 5, checkpoint=str(tmp_path / "x.npz"), checkpoint_every=0)


def test_checkpoint_of_other_parameters_is_refused(tmp_path, pkg, oracle):
    data, d = _data(pkg)
    ck = str(tmp_path / "loop.npz")
    _run(pkg, oracle, data, d, 2, checkpoint=ck)
    eng = make_oracle_engine(pkg, oracle)(data, 0, 1)
    with pytest.raises(pkg.IllegalArgumentException, match="other parameters"):
        pkg.runParallelizedSGD(data, pkg.LogisticGradient(), pkg.SquaredL2SGDUpdater(), 0.25, 5,
                               0.01, 1.0, np.zeros(d), 0.0, engine=eng, checkpoint=ck)
    data2, _ = _data(pkg, n=301)
    eng = make_oracle_engine(pkg, oracle)(data2, 0, 1)
    with pytest.raises(pkg.IllegalArgumentException, match="other parameters"):
        pkg.runParallelizedSGD(data2, pkg.LogisticGradient(), pkg.SquaredL2SGDUpdater(), 0.5, 5,
                               0.01, 1.0, np.zeros(d), 0.0, engine=eng, checkpoint=ck)


@pytest.mark.gpu
def test_resume_on_device(tmp_path, pkg):
    if not has_gpu():
        pytest.skip("no GPU")
    rng = np.random.default_rng(3)
    n, d, P = 4096, 64, 8
    X = rng.standard_normal((n, d))
    y = (rng.uniform(size=n) > 0.5).astype(float)
    data = pkg.PartitionedData.parallelize(y, X, P)
    args = (pkg.LogisticGradient(), pkg.SquaredL2SGDUpdater(), 0.5, 4, 0.01, 0.5, np.zeros(d), 0.0)
    w_full, h_full = pkg.runParallelizedSGD(data, *args)
    ck = str(tmp_path / "dev.npz")
    pkg.runParallelizedSGD(data, *args[:3], 2, *args[4:], checkpoint=ck)
    w_b, h_b = pkg.runParallelizedSGD(data, *args, checkpoint=ck)
    assert np.array_equal(w_b, w_full) and np.array_equal(h_b, h_full)
