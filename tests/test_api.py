"""Host-side API mirror of ParallelizedSGD.scala: setters, validation messages, partitioning,
driver rules (with a scripted engine -- no device needed)."""
import numpy as np
import pytest


def test_defaults_and_setters(pkg):
    o = pkg.ParallelizedSGD(pkg.LogisticGradient(), pkg.SimpleSGDUpdater())
    assert (o.stepSize, o.numIterations, o.regParam, o.miniBatchFraction, o.convergenceTol) == \
        (1.0, 100, 0.0, 1.0, 0.001)
    assert o.setStepSize(0.5).setNumIterations(3).setRegParam(0.1).setConvergenceTol(0.0) is o
    assert (o.stepSize, o.numIterations, o.regParam, o.convergenceTol) == (0.5, 3, 0.1, 0.0)


@pytest.mark.parametrize("call,msg", [
    (lambda o: o.setStepSize(0.0), "requirement failed: Initial step size must be positive but got 0.0"),
    (lambda o: o.setStepSize(-1), "requirement failed: Initial step size must be positive but got -1.0"),
    (lambda o: o.setMiniBatchFraction(0.0),
     "requirement failed: Fraction for mini-batch SGD must be in range (0, 1] but got 0.0"),
    (lambda o: o.setMiniBatchFraction(1.5),
     "requirement failed: Fraction for mini-batch SGD must be in range (0, 1] but got 1.5"),
    (lambda o: o.setNumIterations(-1), "requirement failed: Number of iterations must be nonnegative but got -1"),
    (lambda o: o.setRegParam(-0.5), "requirement failed: Regularization parameter must be nonnegative but got -0.5"),
    (lambda o: o.setConvergenceTol(1.5),
     "requirement failed: Convergence tolerance must be in range [0, 1] but got 1.5"),
])
def test_setter_validation_messages(pkg, call, msg):
    o = pkg.ParallelizedSGD(pkg.LogisticGradient(), pkg.SimpleSGDUpdater())
    with pytest.raises(pkg.IllegalArgumentException) as ei:
        call(o)
    assert str(ei.value) == msg


def test_parallelize_slices_like_spark(pkg):
    y = np.arange(10.0)
    d = pkg.PartitionedData.parallelize(y, np.ones((10, 2)), 3)
    assert [list(p.labels) for p in d.partitions] == [[0, 1, 2], [3, 4, 5], [6, 7, 8, 9]]
    d = pkg.PartitionedData.parallelize(y[:2], np.ones((2, 2)), 4)
    assert [p.n_rows for p in d.partitions] == [0, 1, 0, 1]
    assert d.count() == 2


def test_shard_ranges_cover_partitions(pkg):
    for P in (1, 2, 5, 256, 2048):
        for G in (1, 2, 3, 8):
            spans = [pkg.shard_range(P, r, G) for r in range(G)]
            assert spans[0][0] == 0 and spans[-1][1] == P
            assert all(spans[i][1] == spans[i + 1][0] for i in range(G - 1))
            for r, (lo, hi) in enumerate(spans):
                assert all(p * G // P == r for p in range(lo, hi))


def test_csr_from_points(pkg):
    pts = [(1.0, ([0, 3], [0.5, 1.0], 4)), (0.0, ([1], [2.0], 4)), (1.0, ([], [], 4))]
    d = pkg.PartitionedData.from_points(pts, 2)
    assert d.num_features == 4 and d.count() == 3
    p0, p1 = d.partitions
    assert list(p0.row_ptr) == [0, 2] and list(p1.row_ptr) == [0, 1, 1]


def test_unsupported_plugins_raise(pkg):
    class MyGradient(pkg.Gradient):
        pass

    with pytest.raises(pkg.IllegalArgumentException):
        pkg.make_params(MyGradient(), pkg.SimpleSGDUpdater(), 1.0, 0.0, 1.0, 0.0)
    with pytest.raises(pkg.IllegalArgumentException):
        pkg.LogisticGradient(numClasses=1)


def test_multinomial_params_and_weight_size(pkg):
    """LogisticGradient(numClasses = K): params carry K, and the weight vector must be (K-1)*d
    (MLlib's require(weights.size % dataSize == 0 && numClasses == weights.size / dataSize + 1))."""
    g = pkg.LogisticGradient(numClasses=4)
    p = pkg.make_params(g, pkg.SimpleSGDUpdater(), 1.0, 0.0, 1.0, 0.0)
    assert p.num_classes == 4 and p.gradient == 0
    assert pkg.make_params(pkg.HingeGradient(), pkg.SimpleSGDUpdater(), 1.0, 0.0, 1.0, 0.0).num_classes == 2
    X = np.ones((4, 3))
    data = pkg.PartitionedData([pkg.DensePartition(np.zeros(4), X)])
    for bad in (3, 7, 12):   # (K-1)*d = 9
        with pytest.raises(pkg.IllegalArgumentException, match="requirement failed"):
            pkg.runParallelizedSGD(data, g, pkg.SimpleSGDUpdater(), 1.0, 1, 0.0, 1.0, np.zeros(bad), 0.0)
    with pytest.raises(pkg.IllegalArgumentException, match="requirement failed"):
        pkg.runParallelizedSGD(data, pkg.LogisticGradient(), pkg.SimpleSGDUpdater(), 1.0, 1, 0.0, 1.0,
                               np.zeros(9), 0.0)


class ScriptedEngine:
    """Returns canned fold results to exercise the driver's bookkeeping (PSGD.scala:237-299)."""

    def __init__(self, results, d, terms=(1.0, 1.0), rv0=0.25):
        self.results, self.d, self.terms, self.rv0, self.calls = list(results), d, terms, rv0, 0

    def weights(self, w):
        return np.array(w, dtype=float)

    def initial_regval(self, params, w):
        return self.rv0

    def epoch(self, params, w, with_counts=False):
        self.calls += 1
        return self.results.pop(0), None

    def scalars(self, f):
        return f[self.d], f[self.d + 1], int(f[self.d + 2])

    def adopt(self, f):
        return np.array(f[: self.d])

    def convergence_terms(self, prev, cur):
        return self.terms

    def to_host(self, w):
        return np.array(w)


def test_driver_regval_lag_and_empty_batch(pkg):
    data = pkg.PartitionedData.parallelize(np.ones(4), np.ones((4, 2)), 2)
    res = [np.array([1.0, 2.0, 0.5, 8.0, 4.0]),   # rv 0.5, lossSum 8, count 4
           np.array([9.0, 9.0, 0.0, 0.0, 0.0]),   # empty batch: skipped
           np.array([3.0, 4.0, 0.7, 2.0, 4.0])]
    eng = ScriptedEngine(res, 2, terms=(100.0, 1.0))
    w, h = pkg.runParallelizedSGD(data, pkg.LogisticGradient(), pkg.SquaredL2SGDUpdater(), 1.0, 3,
                                  0.1, 1.0, [0.0, 0.0], 0.001, engine=eng)
    # loss_i = lossSum/batch + regVal of the previous iteration (:283)
    assert list(h) == [8.0 / 4 + 0.25, 2.0 / 4 + 0.5]
    assert list(w) == [3.0, 4.0]


def test_driver_convergence_from_second_success(pkg):
    data = pkg.PartitionedData.parallelize(np.ones(4), np.ones((4, 2)), 2)
    res = [np.array([1.0, 2.0, 0.0, 8.0, 4.0]) for _ in range(5)]
    eng = ScriptedEngine(res, 2, terms=(0.0, 1.0))  # ||diff|| = 0 < tol -> converged
    w, h = pkg.runParallelizedSGD(data, pkg.LogisticGradient(), pkg.SimpleSGDUpdater(), 1.0, 5,
                                  0.0, 1.0, [0.0, 0.0], 0.001, engine=eng)
    assert eng.calls == 2 and len(h) == 2


def test_driver_empty_data_returns_initial_weights(pkg):
    data = pkg.PartitionedData.parallelize(np.zeros(0), np.zeros((0, 3)), 2)
    w, h = pkg.runParallelizedSGD(data, pkg.LogisticGradient(), pkg.SimpleSGDUpdater(), 1.0, 5,
                                  0.0, 1.0, [1.0, 2.0, 3.0])
    assert list(w) == [1.0, 2.0, 3.0] and len(h) == 0


def test_driver_zero_iterations(pkg):
    data = pkg.PartitionedData.parallelize(np.ones(4), np.ones((4, 2)), 2)
    eng = ScriptedEngine([], 2)
    w, h = pkg.runParallelizedSGD(data, pkg.LogisticGradient(), pkg.SimpleSGDUpdater(), 1.0, 0,
                                  0.0, 1.0, [0.5, 0.5], engine=eng)
    assert list(w) == [0.5, 0.5] and len(h) == 0 and eng.calls == 0


class PipelinedScriptedEngine(ScriptedEngine):
    """ScriptedEngine with HipEngine's asynchronous epochs (epoch_async / scalars_wait /
    adopt_view); logs the order of enqueues and reads."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.log = []

    def epoch(self, params, w, with_counts=False):
        self.log.append(("epoch", params.iteration, tuple(np.asarray(w, dtype=float))))
        return super().epoch(params, w, with_counts)

    def epoch_async(self, params, w):
        f, _ = self.epoch(params, w)
        return f, np.array(f)

    def scalars_wait(self, token):
        self.log.append(("wait",))
        return self.scalars(token)

    def adopt_view(self, f):
        return f[: self.d]


def _scripted_results(k):
    return [np.array([1.0 + i, 2.0 - i, 0.1 * (i + 1), 3.0 + i, 4.0]) for i in range(k)]


def test_driver_pipelined_matches_synchronous_loop(pkg):
    """tol == 0 and miniBatchFraction == 1: the pipelined loop (ParallelizedSGD._run_pipelined)
    gives the synchronous loop's weights and loss history (regVal lag :283, adoption :286), each
    epoch runs on the previous epoch's folded weights, and epochs are enqueued PIPELINE_LAG ahead
    of the scalar reads."""
    data = pkg.PartitionedData.parallelize(np.ones(4), np.ones((4, 2)), 2)
    args = (data, pkg.LogisticGradient(), pkg.SquaredL2SGDUpdater(), 1.0, 6, 0.1, 1.0, [0.5, -0.5], 0.0)
    w_s, h_s = pkg.runParallelizedSGD(*args, engine=ScriptedEngine(_scripted_results(6), 2))
    eng = PipelinedScriptedEngine(_scripted_results(6), 2)
    w_p, h_p = pkg.runParallelizedSGD(*args, engine=eng)
    assert list(w_p) == list(w_s) and list(h_p) == list(h_s) and len(h_p) == 6
    epochs = [e for e in eng.log if e[0] == "epoch"]
    assert [e[1] for e in epochs] == [1, 2, 3, 4, 5, 6]
    assert epochs[0][2] == (0.5, -0.5)
    for i in range(1, 6):   # epoch i+1 runs on epoch i's folded weights
        assert epochs[i][2] == (1.0 + (i - 1), 2.0 - (i - 1))
    lag = pkg.ParallelizedSGD.PIPELINE_LAG
    kinds = [e[0] for e in eng.log]
    assert kinds[: lag + 2] == ["epoch"] * (lag + 1) + ["wait"]
    assert kinds.count("wait") == 6


def test_driver_pipelined_only_when_branches_are_known(pkg):
    """tol > 0 (isConverged may stop the loop), miniBatchFraction < 1 (a batch may be empty) or
    per-iteration chain counts keep the synchronous loop: no asynchronous reads."""
    data = pkg.PartitionedData.parallelize(np.ones(4), np.ones((4, 2)), 2)
    for tol, frac, counts in ((0.001, 1.0, False), (0.0, 0.5, False), (0.0, 1.0, True)):
        eng = PipelinedScriptedEngine(_scripted_results(3), 2, terms=(100.0, 1.0))
        pkg.runParallelizedSGD(data, pkg.LogisticGradient(), pkg.SimpleSGDUpdater(), 1.0, 3, 0.0, frac,
                               [0.0, 0.0], tol, engine=eng, return_chain_counts=counts)
        assert ("wait",) not in eng.log and eng.calls == 3


def test_driver_pipelined_error_drains_inflight_epochs(pkg):
    """An error while epochs are in flight (e.g. a watchdog NaN count read back) waits for the
    engine's stream before it propagates: the in-flight folds write into the engine's page-locked
    slots."""
    data = pkg.PartitionedData.parallelize(np.ones(4), np.ones((4, 2)), 2)

    class Failing(PipelinedScriptedEngine):
        drained = False

        def scalars_wait(self, token):
            raise RuntimeError("watchdog")

        def drain(self):
            self.drained = True

    eng = Failing(_scripted_results(5), 2)
    with pytest.raises(RuntimeError, match="watchdog"):
        pkg.runParallelizedSGD(data, pkg.LogisticGradient(), pkg.SimpleSGDUpdater(), 1.0, 5, 0.0, 1.0,
                               [0.0, 0.0], 0.0, engine=eng)
    assert eng.drained
