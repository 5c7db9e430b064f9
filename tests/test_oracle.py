"""The CPU oracle: pinned against the reference suite's known-answer properties
(ParallelizedSGDSuite.scala), cross-checked against the independent pure-Python restatement,
and against the committed golden fixtures."""
import math
import random

import numpy as np
import pytest

import psgd_ref as R


def suite_data(O, n, bias_first=False):
    x, y = O.generate_gd_input(2.0, -1.5, n, 42)
    X = np.stack([np.ones(n), x], 1) if bias_first else np.stack([x, np.ones(n)], 1)
    return X, y


def test_generator_matches_python_restatement(oracle):
    x, y = oracle.generate_gd_input(2.0, -1.5, 3000, 42)
    xp, yp = R.generate_gd_input(2.0, -1.5, 3000, 42)
    assert list(x) == xp and list(y) == yp


def test_fdlibm_log_within_one_ulp_of_libm(oracle):
    rs = random.Random(5)
    for _ in range(20000):
        v = rs.random() * 10 ** rs.uniform(-300, 300)
        a, b = oracle.fdlibm_log(v), math.log(v)
        assert a == R.fdlibm_log(v)
        assert abs(a - b) <= math.ulp(b)
    assert oracle.fdlibm_log(1.0) == 0.0 and oracle.fdlibm_log(0.0) == -math.inf


def test_java_random_known_sequence(oracle):
    # java.util.Random(42): nextDouble() published first value 0.7275636800328681
    assert oracle.jrandom_doubles(42, 1)[0] == 0.7275636800328681
    g = oracle.jrandom_gaussians(42, 2)
    assert list(g) == [R.JavaRandom(42).next_gaussian(), g[1]]


def test_suite_loss_decreasing(oracle):
    """ParallelizedSGDSuite.scala:67-105 -- loss.last - loss.head < 0."""
    X, y = suite_data(oracle, 10000)
    w, h, c = oracle.run(oracle.Matrix(y, X), [0, 5000, 10000], "logistic", "simple", 1.0, 10,
                         0.0, [-1.0, 1.0], tol=0.001)
    assert len(h) == 10 and h[-1] - h[0] < 0
    assert list(c[0]) == [153, 35]  # per-sample convergence breaks fire early


def test_suite_first_iteration_with_regularization(oracle):
    """ParallelizedSGDSuite.scala:107-142 -- L2: loss1 = loss0 + |w0|^2/2, w1 = w0' - w0."""
    X, y = suite_data(oracle, 2, bias_first=True)
    m = oracle.Matrix(y, X)
    w0 = np.array([1.0, 0.5])
    nw0, l0, _ = oracle.run(m, [0, 1, 2], "logistic", "squared_l2", 1.0, 1, 0.0, w0)
    nw1, l1, _ = oracle.run(m, [0, 1, 2], "logistic", "squared_l2", 1.0, 1, 1.0, w0)
    assert abs(l1[0] - (l0[0] + (w0[0] ** 2 + w0[1] ** 2) / 2)) < 1e-5
    assert abs(nw1[0] - (nw0[0] - w0[0])) < 1e-5 and abs(nw1[1] - (nw0[1] - w0[1])) < 1e-5


def test_suite_convergence_tolerance(oracle):
    """ParallelizedSGDSuite.scala:144-181 -- tol 0.5 stops before numIterations."""
    X, y = suite_data(oracle, 10000)
    _, h, _ = oracle.run(oracle.Matrix(y, X), [0, 5000, 10000], "logistic", "simple", 1.0, 10,
                         0.0, [-1.0, 1.0], tol=0.5)
    assert len(h) < 10


def test_survey_scratch_anchors_with_glibc_log(oracle, monkeypatch):
    """SURVEY §8c anchors came from a scratch port that used libm log instead of StrictMath.log;
    substituting it reproduces them bit for bit (so the chain/combine/driver logic agrees with
    that independent port; the 1-ulp differences are the generator's log only)."""
    monkeypatch.setattr(R, "fdlibm_log", math.log)
    x, y = R.generate_gd_input(2.0, -1.5, 10000, 42)
    assert x[:3] == [1.141905315473055, 0.919407948982788, -0.9498666368908959]
    assert sum(y) / len(y) == 0.8133
    parts = [([[1.0, x[0]]], [y[0]]), ([[1.0, x[1]]], [y[1]])]
    w, h, _ = R.run(parts, 0, 1, 1.0, 1, 0.0, [1.0, 0.5])
    assert w == [1.180296615483073, 0.6849098844205752] and h == [0.19886296441133905]
    w, h, _ = R.run(parts, 0, 1, 1.0, 1, 1.0, [1.0, 0.5])
    assert w == [0.18029661548307302, 0.18490988442057515] and h == [0.8238629644113391]


@pytest.mark.parametrize("gi", range(3))
@pytest.mark.parametrize("ui", range(5))
def test_c_matches_python_bitwise_small(oracle, gi, ui):
    rng = np.random.default_rng(100 + 10 * gi + ui)
    n, d = 60, 5
    X = rng.standard_normal((n, d))
    y = (rng.uniform(size=n) > 0.5).astype(float) if gi != 1 else 0.3 * rng.standard_normal(n)
    offs = [0, 20, 20, 60]
    for tol in (0.0, 0.05):
        w, h, c = oracle.run(oracle.Matrix(y, X), offs, gi, ui, 0.3, 3, 0.05, np.zeros(d), tol=tol)
        parts = [([list(X[r]) for r in range(a, b)], list(y[a:b])) for a, b in zip(offs[:-1], offs[1:])]
        wp, hp, cp = R.run(parts, gi, ui, 0.3, 3, 0.05, [0.0] * d, tol=tol)
        assert list(w) == wp and list(h) == hp
        assert [list(r) for r in c[:len(cp)]] == cp


def test_two_level_combine_order(oracle):
    rng = np.random.default_rng(3)
    X = rng.standard_normal((90, 4))
    y = (rng.uniform(size=90) > 0.5).astype(float)
    offs = [0, 20, 45, 70, 90]
    w, h, _ = oracle.run(oracle.Matrix(y, X), offs, "logistic", "simple", 0.5, 2, 0.0, np.zeros(4),
                         tol=0.0, groups=[0, 2, 4])
    parts = [([list(X[r]) for r in range(a, b)], list(y[a:b])) for a, b in zip(offs[:-1], offs[1:])]
    wp, hp, _ = R.run(parts, 0, 0, 0.5, 2, 0.0, [0.0] * 4, tol=0.0, groups=[0, 2, 4])
    assert list(w) == wp and list(h) == hp


def test_empty_partitions_combine(oracle):
    """Two empty partitions merged first give 0/0 = NaN weights (the reference's combiner,
    ParallelizedSGD.scala:272-274); one empty partition merges harmlessly."""
    X = np.array([[1.0, 2.0], [0.5, -1.0]])
    y = np.array([1.0, 0.0])
    m = oracle.Matrix(y, X)
    w, h, _ = oracle.run(m, [0, 0, 2], "logistic", "simple", 1.0, 1, 0.0, [0.1, 0.2], tol=0.0)
    assert np.all(np.isfinite(w)) and len(h) == 1
    w, h, _ = oracle.run(m, [0, 0, 0, 2], "logistic", "simple", 1.0, 1, 0.0, [0.1, 0.2], tol=0.0)
    assert np.all(np.isnan(w))


def test_golden_fixtures_reproduce(oracle, golden):
    for case in golden:
        if case["source"] == "suite":
            X, y = suite_data(oracle, case["n"], case["bias_first"])
            m = oracle.Matrix(y, X)
        elif "X" in case:
            m = oracle.Matrix(np.array(case["y"]), np.array(case["X"]))
        else:
            m = oracle.Matrix(np.array(case["y"]), row_ptr=np.array(case["row_ptr"]),
                              col=np.array(case["col"]), val=np.array(case["val"]), d=case["d"])
        w, h, c = oracle.run(m, case["offsets"], case["gradient"], case["updater"], case["step"],
                             case["iters"], case["reg"], np.array(case["w0"]), tol=case["tol"],
                             fraction=case.get("fraction", 1.0), num_classes=case.get("num_classes", 2),
                             margin_check=False)
        e = case["expected"]
        assert list(map(float, w)) == e["weights"], case["name"]
        assert list(map(float, h)) == e["loss_history"], case["name"]


def test_murmur3_published_vectors():
    """XORShiftRandom.hashSeed's MurmurHash3 (scala.util.hashing.MurmurHash3.bytesHash, the
    x86_32 algorithm) against the algorithm's published test vectors."""
    import psgd_ref as R
    vec = [(b"", 0, 0), (b"", 1, 0x514E28B7), (b"", 0xFFFFFFFF, 0x81F16F39), (b"\0\0\0\0", 0, 0x2362F9DE),
           (b"\x21\x43\x65\x87", 0, 0xF55B516B), (b"\x21\x43\x65\x87", 0x5082EDEE, 0x2362F9DE),
           (b"\x21\x43\x65", 0, 0x7E4A8634), (b"\x21\x43", 0, 0xA0F7B07A), (b"\x21", 0, 0x72661CF4),
           (b"\xff\xff\xff\xff", 0, 0x76293B50), (b"\0\0\0", 0, 0x85F0B427), (b"\0\0", 0, 0x30F4C306)]
    for data, seed, want in vec:
        assert R.murmur3_bytes_hash(data, seed) & 0xFFFFFFFF == want, (data, seed)


def test_sampler_c_and_python_agree(oracle):
    """RDD.sample(false, f, seed) restated twice: the C oracle and the pure-Python one select the
    same rows (java.util.Random(42).nextLong() = -5025562857975149833, the JDK's known value)."""
    import psgd_ref as R
    assert int(oracle.partition_seeds(42, 1)[0]) == -5025562857975149833
    rng = np.random.default_rng(5)
    for s in rng.integers(-2**63, 2**63 - 1, 40):
        assert R.xorshift_hash_seed(int(s)) == oracle.xorshift_hash_seed(int(s))
    assert R.partition_seeds(43, 7) == [int(v) for v in oracle.partition_seeds(43, 7)]
    for f in (1e-6, 0.01, 0.2, 0.4, 0.400001, 0.6, 0.999, 1.0, 0.0):
        for sd in oracle.partition_seeds(44, 3):
            a = R.bernoulli_sample(int(sd), 3000, f)
            b = oracle.sample_partition(int(sd), 3000, f)
            assert a == b.tolist(), (f, len(a), len(b))
    # the filter keeps about f of the rows, gap sampling too
    for f in (0.1, 0.7):
        m = sum(len(oracle.sample_partition(int(sd), 20000, f)) for sd in oracle.partition_seeds(46, 5))
        assert abs(m / 100000 - f) < 0.01


def test_multinomial_gradient_is_softmax_cross_entropy():
    """The multinomial LogisticGradient restatement (C and Python) against the textbook form:
    loss = logsumexp([0, m_1..m_{K-1}]) - m_y, gradient block i = (p_{i+1} - [y == i+1]) x,
    in both regimes of the reference's max-margin shift (M > 0 and M <= 0) -- a property check
    independent of the reference's evaluation order."""
    import psgd_ref as R
    rng = np.random.default_rng(5)
    for K, scale in ((3, 0.1), (5, 3.0), (7, 0.5)):
        d = 6
        for _ in range(20):
            x = rng.standard_normal(d)
            x[rng.uniform(size=d) < 0.2] = 0.0
            w = scale * rng.standard_normal((K - 1) * d)
            y = float(rng.integers(0, K))
            (_, g), loss = R.multinomial(list(x), y, list(w), K)
            m = np.concatenate([[0.0], w.reshape(K - 1, d) @ x])
            lse = np.log(np.sum(np.exp(m - m.max()))) + m.max()
            assert abs(loss - (lse - m[int(y)])) <= 1e-12 * max(1.0, abs(loss))
            p = np.exp(m - lse)
            want = np.concatenate([(p[i + 1] - (1.0 if y == i + 1 else 0.0)) * x for i in range(K - 1)])
            assert np.allclose(g, want, rtol=1e-12, atol=1e-15)
    # the C restatement agrees with the Python one bit for bit on a one-sample chain
    X = rng.standard_normal((1, 4))
    w0 = rng.standard_normal(12)
    for lab in (0.0, 2.0, 3.0, 4.0, 1.5):
        import oracle as O
        mat = O.Matrix(np.array([lab]), X)
        w, h, _ = O.run(mat, [0, 1], "logistic", "simple", 1.0, 1, 0.0, w0, tol=0.0, num_classes=4)
        wp, hp, _ = R.run([([list(X[0])], [lab])], R.GRAD_LOGISTIC, R.UPD_SIMPLE, 1.0, 1, 0.0, list(w0),
                          tol=0.0, num_classes=4)
        assert list(map(float, w)) == wp and list(map(float, h)) == hp


def test_break_margin_probe(oracle):
    """The break-margin probe leaves every decision unchanged and reports, per
    iteration and chain, the closest |diff / (tol max(norm, 1)) - 1|; the tol-free ratio trace puts
    a break exactly where tol = r_k (1 +- 1e-13) says: at sample k just above r_k, past it just
    below (the adversarial cases of tests/test_gpu_break_margin.py)."""
    rng = np.random.default_rng(5)
    n, d, P = 400, 12, 4
    X = rng.standard_normal((n, d)) / np.sqrt(d)
    y = (X @ rng.standard_normal(d) + rng.logistic(size=n) > 0).astype(float)
    m = oracle.Matrix(y, X)
    offs = [i * n // P for i in range(P)] + [n]
    w, h, c = oracle.run(m, offs, "logistic", "simple", 0.5, 3, 0.0, np.zeros(d), tol=0.02, margin_check=False)
    w2, h2, c2, mg = oracle.run_with_margins(m, offs, "logistic", "simple", 0.5, 3, 0.0, np.zeros(d), tol=0.02)
    assert np.array_equal(w, w2) and np.array_equal(h, h2) and np.array_equal(c, c2)
    assert mg.shape == c.shape and np.all(mg > 0) and np.all(np.isfinite(mg))
    r = oracle.ratio_trace(m, offs, 1, "logistic", "simple", 0.5, 0.0, np.zeros(d))
    assert len(r) == offs[2] - offs[1]
    # a record low of the trace (every earlier sample's r larger by far more than 1e-13)
    k = next(k for k in range(5, len(r)) if r[k] < r[:k].min() * (1 - 1e-9))
    for e, want_at_k in ((1e-13, True), (-1e-13, False)):
        tol = r[k] * (1 + e)
        _, _, cc = oracle.run(m, offs, "logistic", "simple", 0.5, 1, 0.0, np.zeros(d), tol=tol, margin_check=False)
        assert (cc[0][1] == k + 1) == want_at_k, (e, cc[0][1], k)
        _, _, _, mm = oracle.run_with_margins(m, offs, "logistic", "simple", 0.5, 1, 0.0, np.zeros(d), tol=tol)
        assert mm[0][1] < 2e-13
