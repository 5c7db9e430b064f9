"""Parity of the HIP path (libpsgd.so through the C ABI) with the CPU oracle.

fp64 mode: weights and loss history within 1e-9 relative (TestingUtils relTol semantics,
TestingUtils.scala:34-46, with an absolute floor of 1e-12 near zero) and per-iteration chain
counts EXACTLY equal (including the per-sample convergence breaks).
fp32 storage + fp64 compute: the oracle runs on the same (fp32-representable) inputs: 1e-9.
fp32 compute (throughput mode): stated tolerance FP32_REL below, versus the fp64 oracle.
"""
import numpy as np
import pytest

from conftest import has_gpu

pytestmark = pytest.mark.gpu

REL = 1e-9
ABS_FLOOR = 1e-12
FP32_REL = 2e-4       # weights, fp32 compute vs fp64 oracle
FP32_LOSS_REL = 1e-4  # loss history


# fp32 compute decides isConverged on fp32 weights and norms: a chain whose reference decisions
# all sit further than this (relative) from flipping must break where the reference does
FP32_BREAK_MARGIN = 1e-3


def fp32_break_counts_agree(counts, cr, margins, tag):
    """fp32-compute per-sample breaks against the fp64 oracle: per outer iteration,
    every chain whose oracle margin (conftest.CheckedOracle) exceeds FP32_BREAK_MARGIN has the
    oracle's exact count; only chains with a decision within that margin of flipping may differ.
    Checked up to the first iteration where any count differs -- after it the folded weights, and
    so every later trajectory, differ. Returns True when every count of every iteration agreed
    (the caller then checks weights and losses at the fp32 tolerance)."""
    assert len(counts) >= 1
    for it in range(min(len(counts), len(cr))):
        got, ref, mg = list(counts[it]), list(cr[it]), margins[it]
        assert len(got) == len(ref), tag
        far = [p for p in range(len(ref)) if got[p] != ref[p] and mg[p] > FP32_BREAK_MARGIN]
        assert not far, (f"{tag} iteration {it + 1}: chains {far} break elsewhere than the reference "
                         f"(margins {[float(mg[p]) for p in far]}, counts {[(got[p], ref[p]) for p in far]})")
        if got != ref:
            return False
    return len(counts) == len(cr)


def assert_close(a, b, rel=REL, floor=ABS_FLOOR, what=""):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    both_nan = np.isnan(a) & np.isnan(b)
    diff = np.abs(a - b)
    ok = both_nan | (diff <= rel * np.maximum(np.abs(a), np.abs(b))) | (diff <= floor)
    if not ok.all():
        i = int(np.argmax(~ok))
        raise AssertionError(f"{what}: {int((~ok).sum())} mismatches; first at {i}: {a.flat[i]!r} vs "
                             f"{b.flat[i]!r} (max rel {np.nanmax(diff / np.maximum(np.abs(b), 1e-300)):.3g})")


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not has_gpu():
        pytest.skip("no GPU")


G = {"logistic": "LogisticGradient", "least_squares": "LeastSquaresGradient", "hinge": "HingeGradient"}
U = {"simple": "SimpleSGDUpdater", "squared_l2": "SquaredL2SGDUpdater", "l1": "L1SGDUpdater",
     "adagrad": "AdaGradSGDUpdater", "adam": "AdamSGDUpdater"}


def stateful_variant(upd, tol, nv):
    """Kernel of a dense per-sample epoch (AdaGrad / Adam / L1 at any tol, every updater at
    tol > 0 in fp32 compute or with PSGD_B64_CONV=0): the feature-split chain_split (800 + 10 H +
    NV, H = min(NV, 4) compute waves) from two row vectors on, else the one-wave chain_dense
    (100 + NV)."""
    if (upd in ("adagrad", "adam", "l1") or tol > 0.0) and nv >= 2:
        return 800 + 10 * min(nv, 4) + nv
    return 100 + nv


def block64_variant(tol, nv):
    """fp64 Simple / SquaredL2 epochs on dense rows of <= 8 vectors: chain_block64, 700 + 40 (the
    per-sample break, tol > 0) + 10 (H - 1) + NV, H = 2 chain waves from two row vectors on."""
    return 700 + (40 if tol > 0.0 else 0) + (10 if nv >= 2 else 0) + nv


def data_for(pkg, oracle, case):
    offs = case["offsets"]
    P = len(offs) - 1
    if case["source"] == "suite":
        x, y = oracle.generate_gd_input(2.0, -1.5, case["n"], 42)
        X = np.stack([np.ones(len(x)), x], 1) if case["bias_first"] else np.stack([x, np.ones(len(x))], 1)
        assert [float(v) for v in X[: len(case["x_head"]), 1 if case["bias_first"] else 0]] == case["x_head"]
        parts = [pkg.DensePartition(y[a:b], X[a:b]) for a, b in zip(offs[:-1], offs[1:])]
    elif "X" in case:
        X, y = np.array(case["X"]), np.array(case["y"])
        parts = [pkg.DensePartition(y[a:b], X[a:b]) for a, b in zip(offs[:-1], offs[1:])]
    else:
        rp, col, val, y = (np.array(case["row_ptr"]), np.array(case["col"], np.int32),
                           np.array(case["val"]), np.array(case["y"]))
        parts = [pkg.CsrPartition(y[a:b], rp[a:b + 1] - rp[a], col[rp[a]:rp[b]], val[rp[a]:rp[b]], case["d"])
                 for a, b in zip(offs[:-1], offs[1:])]
    assert len(parts) == P
    return pkg.PartitionedData(parts)


def run_case(pkg, data, case, **kw):
    g = getattr(pkg, G[case["gradient"]])(*([case["num_classes"]] if "num_classes" in case else []))
    u = getattr(pkg, U[case["updater"]])()
    return pkg.runParallelizedSGD(data, g, u, case["step"], case["iters"], case["reg"],
                                  case.get("fraction", 1.0), np.array(case["w0"]), case["tol"],
                                  return_chain_counts=True, **kw)


def test_golden_cases_fp64(pkg, oracle, golden):
    for case in golden:
        data = data_for(pkg, oracle, case)
        w, h, counts = run_case(pkg, data, case)
        e = case["expected"]
        assert [list(map(int, c)) for c in counts] == e["chain_counts"], case["name"]
        assert_close(w, e["weights"], what=case["name"] + " weights")
        assert_close(h, e["loss_history"], what=case["name"] + " loss")


def test_suite_known_answers_on_gpu(pkg, oracle, golden):
    """The reference suite's three assertions, re-run on the HIP path."""
    by = {c["name"]: c for c in golden}
    c = by["suite_loss_decreasing"]
    _, h, _ = run_case(pkg, data_for(pkg, oracle, c), c)
    assert h[-1] - h[0] < 0                                   # ParallelizedSGDSuite.scala:101
    c0, c1 = by["suite_first_iteration_l2_reg0"], by["suite_first_iteration_l2_reg1"]
    w0, l0, _ = run_case(pkg, data_for(pkg, oracle, c0), c0)
    w1, l1, _ = run_case(pkg, data_for(pkg, oracle, c1), c1)
    assert abs(l1[0] - (l0[0] + (1.0 + 0.25) / 2)) < 1e-5      # :132-135
    assert abs(w1[0] - (w0[0] - 1.0)) < 1e-5 and abs(w1[1] - (w0[1] - 0.5)) < 1e-5  # :137-141
    c = by["suite_convergence_tol"]
    _, h, _ = run_case(pkg, data_for(pkg, oracle, c), c)
    assert len(h) < 10                                        # :180


def synth(rng, n, d, grad, dtype=np.float64):
    X = rng.standard_normal((n, d)).astype(dtype)
    wt = rng.standard_normal(d) / np.sqrt(d)
    z = X.astype(np.float64) @ wt
    if grad == "least_squares":
        y = z + 0.1 * rng.standard_normal(n)
    else:
        y = ((z + rng.logistic(size=n)) > 0).astype(np.float64)
    return X, y


@pytest.mark.parametrize("d", [3, 100, 256, 300, 512, 700, 1024, 2048, 3000])
@pytest.mark.parametrize("grad", ["logistic", "least_squares", "hinge"])
def test_dense_fp64_sizes(pkg, oracle, d, grad):
    rng = np.random.default_rng(d * 7 + len(grad))
    n, P = 1200, 5
    X, y = synth(rng, n, d, grad)
    data = pkg.PartitionedData.parallelize(y, X, P)
    offs = [i * n // P for i in range(P)] + [n]
    step = 0.002 if grad == "least_squares" else 0.5
    for upd in ("simple", "squared_l2", "l1"):
        for tol in (0.0, 0.002):
            w0 = 0.01 * np.ones(d)
            w, h, c = pkg.runParallelizedSGD(data, getattr(pkg, G[grad])(), getattr(pkg, U[upd])(),
                                             step, 3, 0.01, 1.0, w0, tol, return_chain_counts=True)
            wr, hr, cr = oracle.run(oracle.Matrix(y, X), offs, grad, upd, step, 3, 0.01, w0, tol=tol,
                                    n_threads=8)
            tag = f"d={d} {grad} {upd} tol={tol}"
            assert [list(x) for x in c] == [list(x) for x in cr[: len(c)]], tag
            assert_close(w, wr, what=tag + " weights")
            assert_close(h, hr, what=tag + " loss")


@pytest.mark.parametrize("upd", ["adagrad", "adam"])
def test_dense_stateful_updaters(pkg, oracle, upd):
    rng = np.random.default_rng(11)
    n, d, P = 600, 40, 3
    X, y = synth(rng, n, d, "logistic")
    data = pkg.PartitionedData.parallelize(y, X, P)
    offs = [i * n // P for i in range(P)] + [n]
    for tol in (0.0, 0.01):
        w, h = pkg.runParallelizedSGD(data, pkg.LogisticGradient(), getattr(pkg, U[upd])(), 0.3, 3,
                                      0.0, 1.0, np.zeros(d), tol)
        wr, hr, _ = oracle.run(oracle.Matrix(y, X), offs, "logistic", upd, 0.3, 3, 0.0, np.zeros(d), tol=tol)
        assert_close(w, wr, what=f"{upd} tol={tol}")
        assert_close(h, hr, what=f"{upd} tol={tol} loss")


@pytest.mark.parametrize("upd", ["adagrad", "adam", "l1"])
@pytest.mark.parametrize("d,dtype", [(40, np.float64), (512, np.float32), (1024, np.float64), (2048, np.float32)])
def test_dense_fp32_throughput_updaters(pkg, oracle, upd, d, dtype):
    """AdaGrad / Adam / L1 in the fp32 throughput mode: chain_dense / chain_split with the updater
    status in registers (stateful_variant), against the fp64 oracle at the fp32 tolerance, tol 0
    and tol > 0 (per-sample breaks: counts may differ only when tol > 0)."""
    rng = np.random.default_rng(d + len(upd))
    n, P = 8000, 4
    X, y = synth(rng, n, d, "logistic", dtype)
    data = pkg.PartitionedData.parallelize(y, X, P, dtype=dtype)
    offs = [i * n // P for i in range(P)] + [n]
    step = 0.01
    reg = 0.001 if upd == "l1" else 0.0
    for tol in (0.0, 0.001):
        w, h = pkg.runParallelizedSGD(data, pkg.LogisticGradient(), getattr(pkg, U[upd])(), step, 3, reg, 1.0,
                                      np.zeros(d), tol, compute_dtype="f32")
        es = np.dtype(dtype).itemsize
        nv = 1
        while nv * 64 * 16 // es < d:
            nv *= 2
        assert pkg.optimization.get_context(0).last_kernel() == stateful_variant(upd, tol, nv)
        wr, hr, _ = oracle.run(oracle.Matrix(y, X.astype(np.float64)), offs, "logistic", upd, step, 3, reg,
                               np.zeros(d), tol=tol, n_threads=8, margin_check=False)   # fp32 decisions
        if tol > 0 and len(h) != len(hr):
            continue   # a break on the other side of the fp32/fp64 rounding (allowed when tol > 0)
        scale = np.max(np.abs(wr))
        err = np.max(np.abs(w - wr)) / scale
        assert err <= FP32_REL, f"{upd} d={d} tol={tol}: weights {err:.3g} x max|w|"
        assert_close(h, hr, rel=FP32_LOSS_REL, what=f"{upd} d={d} tol={tol} fp32 loss")


def test_kernel_selection(pkg, oracle):
    """fp64 compute: tol = 0 with Simple/SquaredL2 runs the blocked fp64 kernel (70x one chain
    wave, 71x two), tol > 0 the per-sample kernels (chain_dense 10x for one row vector,
    chain_split 8xx from two), d past the register-resident range chain_general (200)."""
    rng = np.random.default_rng(1)
    for d, dtype, tol, expect in ((100, np.float64, 0.0, 701), (512, np.float32, 0.0, 712),
                                  (1024, np.float32, 0.0, 714), (2048, np.float32, 0.0, 718),
                                  (1024, np.float64, 0.0, 718),
                                  (100, np.float64, 0.001, 741), (512, np.float32, 0.001, 752),
                                  (3000, np.float64, 0.0, 200)):
        X, y = synth(rng, 64, d, "logistic", dtype)
        data = pkg.PartitionedData.parallelize(y, X, 2, dtype=dtype)
        pkg.runParallelizedSGD(data, pkg.LogisticGradient(), pkg.SimpleSGDUpdater(), 1.0, 1, 0.0, 1.0,
                               np.zeros(d), tol)
        ctx = pkg.optimization.get_context(0)
        assert ctx.last_kernel() == expect, (d, dtype, tol, ctx.last_kernel())


def test_fp32_storage_fp64_compute(pkg, oracle):
    rng = np.random.default_rng(5)
    n, d, P = 4000, 512, 8
    X, y = synth(rng, n, d, "least_squares", np.float32)
    data = pkg.PartitionedData.parallelize(y, X, P, dtype=np.float32)
    offs = [i * n // P for i in range(P)] + [n]
    w, h = pkg.runParallelizedSGD(data, pkg.LeastSquaresGradient(), pkg.SimpleSGDUpdater(), 1e-3, 3,
                                  0.0, 1.0, np.zeros(d), 0.0)
    wr, hr, _ = oracle.run(oracle.Matrix(y, X.astype(np.float64)), offs, "least_squares", "simple",
                           1e-3, 3, 0.0, np.zeros(d), tol=0.0, n_threads=8)
    assert_close(w, wr, what="f32 storage weights")
    assert_close(h, hr, what="f32 storage loss")


@pytest.mark.parametrize("grad,d", [("least_squares", 512), ("logistic", 1024), ("hinge", 100)])
def test_fp32_compute_mode_tolerance(pkg, oracle, grad, d):
    rng = np.random.default_rng(9)
    n, P = 20000, 4
    X, y = synth(rng, n, d, grad, np.float32)
    data = pkg.PartitionedData.parallelize(y, X, P, dtype=np.float32)
    offs = [i * n // P for i in range(P)] + [n]
    # a well-conditioned step (||x||^2 ~ d): at step 1.0 a d=1024 logistic chain is chaotic and
    # fp32 vs fp64 trajectories separate for reasons unrelated to the kernel
    step = 1e-3 if grad == "least_squares" else 0.01
    w, h = pkg.runParallelizedSGD(data, getattr(pkg, G[grad])(), pkg.SimpleSGDUpdater(), step, 3, 0.0,
                                  1.0, np.zeros(d), 0.0, compute_dtype="f32")
    wr, hr, _ = oracle.run(oracle.Matrix(y, X.astype(np.float64)), offs, grad, "simple", step, 3, 0.0,
                           np.zeros(d), tol=0.0, n_threads=8)
    scale = np.max(np.abs(wr))
    assert np.max(np.abs(w - wr)) <= FP32_REL * scale, np.max(np.abs(w - wr)) / scale
    assert_close(h, hr, rel=FP32_LOSS_REL, what="fp32 loss")


def test_csr_stateful_updater(pkg, oracle):
    # CSR rows with AdaGrad/Adam (UPD.scala:199-285 on a gradient that is zero outside the row's
    # indices); the golden cases csr_*_adagrad/adam cover every gradient, this one a wide sparse d
    rng = np.random.default_rng(11)
    n, d = 90, 700
    rp, col, val = [0], [], []
    for _ in range(n):
        idx = np.sort(rng.choice(d, size=int(rng.integers(1, 12)), replace=False))
        col += idx.tolist()
        val += rng.uniform(0, 1, size=len(idx)).tolist()
        rp.append(len(col))
    rp, col, val = np.array(rp), np.array(col, np.int32), np.array(val)
    y = (rng.uniform(size=n) > 0.5).astype(float)
    offs = [0, 30, 90]
    parts = [pkg.CsrPartition(y[a:b], rp[a:b + 1] - rp[a], col[rp[a]:rp[b]], val[rp[a]:rp[b]], d)
             for a, b in zip(offs[:-1], offs[1:])]
    data = pkg.PartitionedData(parts)
    # tol > 0: the per-sample break (AdaGrad carries ||w||^2 over the row's coordinates, O(nnz))
    for upd, tol in (("adagrad", 0.0), ("adam", 0.0), ("adagrad", 0.05), ("adam", 0.05)):
        w, h, counts = pkg.runParallelizedSGD(data, pkg.HingeGradient(), getattr(pkg, U[upd])(), 0.5, 3,
                                              0.0, 1.0, np.zeros(d), tol, return_chain_counts=True)
        wr, hr, cr = oracle.run(oracle.Matrix(y, row_ptr=rp, col=col, val=val, d=d), offs, "hinge", upd,
                                0.5, 3, 0.0, np.zeros(d), tol=tol)
        assert [list(map(int, c)) for c in counts] == [list(map(int, c)) for c in cr], (upd, tol)
        assert_close(w, wr, what=f"{upd} tol={tol} weights")
        assert_close(h, hr, what=f"{upd} tol={tol} loss")
        if tol > 0:
            assert any(c < s for it in cr for c, s in zip(it, np.diff(offs))), "no chain broke"


def alpha_in_range(step, reg, n):
    """The host's test for the fp64 CSR kernel's alpha-scaled form (psgd_capi.cpp alpha_in_range)."""
    a = 1.0
    for j in range(1, n + 1):
        a *= 1.0 - (step / np.sqrt(float(j))) * reg
        if not (2.0 ** -400 <= abs(a) <= 2.0 ** 400):
            return False
    return True


@pytest.mark.parametrize("reg,step", [(0.01, 0.5), (0.999, 1.0), (1.0, 1.0), (3.0, 1.0), (1e-6, 0.5)])
def test_csr_squared_l2_alpha_scaled(pkg, oracle, reg, step):
    """fp64 CSR SquaredL2 without a convergence test keeps w = alpha * v (O(nnz) per sample):
    against the oracle's O(d) scale per sample at the 1e-9 bar, including alpha leaving
    [2^-400, 2^400] (folded back into v), 1 - s*lambda == 0 exactly (reg 1, step 1 at j = 1)
    and negative factors (reg 3)."""
    rng = np.random.default_rng(int(reg * 1000) + 7)
    n, d = 1200, 5000
    rp, col, val = [0], [], []
    for _ in range(n):
        k = int(rng.integers(0, 40))
        col += sorted(rng.choice(d, size=k, replace=False).tolist())
        val += rng.uniform(0, 1, size=k).tolist()
        rp.append(len(col))
    rp, col, val = np.array(rp), np.array(col, np.int32), np.array(val)
    y = (rng.uniform(size=n) > 0.5).astype(float)
    offs = [0, 500, 500, 1200]
    parts = [pkg.CsrPartition(y[a:b], rp[a:b + 1] - rp[a], col[rp[a]:rp[b]], val[rp[a]:rp[b]], d)
             for a, b in zip(offs[:-1], offs[1:])]
    w0 = 0.1 * rng.standard_normal(d)
    for grad in ("logistic", "hinge"):
        w, h, counts = pkg.runParallelizedSGD(pkg.PartitionedData(parts), getattr(pkg, G[grad])(),
                                              pkg.SquaredL2SGDUpdater(), step, 3, reg, 1.0, w0, 0.0,
                                              return_chain_counts=True)
        # chain_sparse_lds in fp64 (62x) while every prefix product of (1 - s_j lambda) stays in
        # [2^-400, 2^400]; else chain_general (201), which renormalises
        assert pkg.optimization.get_context(0).last_kernel() == (620 if alpha_in_range(step, reg, 700) else 201)
        wr, hr, cr = oracle.run(oracle.Matrix(y, row_ptr=rp, col=col, val=val, d=d), offs, grad, "squared_l2",
                                step, 3, reg, w0, tol=0.0)
        assert [list(map(int, c)) for c in counts] == [list(map(int, c)) for c in cr]
        assert_close(w, wr, what=f"{grad} reg={reg} weights")
        assert_close(h, hr, what=f"{grad} reg={reg} loss")


def test_mini_batch_fraction(pkg, oracle):
    """miniBatchFraction < 1: batch i = data.sample(false, f, 42 + i) (PSGD.scala:242) through
    the fp32 block kernel and the per-sample kernels (the fp64 path is in the golden cases);
    both branches of the sampler (gap sampling f <= 0.4, the filter above)."""
    rng = np.random.default_rng(2)
    X, y = synth(rng, 3000, 64, "logistic")
    offs = [0, 1000, 1001, 2000, 3000]
    parts = [pkg.DensePartition(y[a:b], X[a:b]) for a, b in zip(offs[:-1], offs[1:])]
    data = pkg.PartitionedData(parts)
    for frac in (0.1, 0.75):
        # fp64 per-sample kernel (dense d = 64 fits the LDS-ring kernel)
        w, h, counts = pkg.runParallelizedSGD(data, pkg.LogisticGradient(), pkg.SimpleSGDUpdater(), 0.5, 4,
                                              0.0, frac, np.zeros(64), 0.0, return_chain_counts=True)
        wr, hr, cr = oracle.run(oracle.Matrix(y, X), offs, "logistic", "simple", 0.5, 4, 0.0, np.zeros(64),
                                tol=0.0, fraction=frac)
        assert [list(map(int, c)) for c in counts] == [list(map(int, c)) for c in cr]
        assert 0 < cr[0][0] < 1000
        assert_close(w, wr, what=f"f={frac} weights")
        assert_close(h, hr, what=f"f={frac} loss")
        # fp32 block kernel: same batches, the fp32 tolerance
        w, h = pkg.runParallelizedSGD(data, pkg.LogisticGradient(), pkg.SimpleSGDUpdater(), 0.01, 4, 0.0,
                                      frac, np.zeros(64), 0.0, compute_dtype="f32")
        wr, hr, _ = oracle.run(oracle.Matrix(y, X.astype(np.float64)), offs, "logistic", "simple", 0.01, 4,
                               0.0, np.zeros(64), tol=0.0, fraction=frac)
        assert np.max(np.abs(w - wr)) <= FP32_REL * np.max(np.abs(wr))
        assert_close(h, hr, rel=FP32_LOSS_REL, what="fp32 loss")


@pytest.mark.parametrize("fraction", [1e-9, 0.001, 0.1, 0.4, 0.4000001, 0.75, 0.999999])
def test_device_sampler_matches_oracle(pkg, oracle, fraction):
    """The device sampler (jump-ahead over the XORShift sequence, 16384 draws a round) selects
    exactly the rows the sequential restatement of BernoulliSampler does: partitions smaller
    than one round, exactly one round, and many rounds; both samplers (gap <= 0.4 < filter)."""
    native = pkg._native
    seeds = oracle.partition_seeds(42 + 3, 4)
    for n, seed in zip((1, 16384, 16385, 1_000_003), seeds):
        got = native.sample_partition(int(seed), n, fraction)
        want = oracle.sample_partition(int(seed), n, fraction)
        assert got.shape == want.shape, (n, fraction, got.shape, want.shape)
        assert np.array_equal(got, want), (n, fraction)
    assert native.sample_partition(7, 0, fraction).size == 0


def test_sampled_epoch_large_partitions(pkg, oracle):
    """Sampled epochs over partitions of several sampler rounds through the fp64 chain: chain
    counts exact, weights at the fp64 tolerance."""
    rng = np.random.default_rng(21)
    X, y = synth(rng, 90_000, 8, "least_squares")
    offs = [0, 40_000, 40_001, 90_000]
    parts = [pkg.DensePartition(y[a:b], X[a:b]) for a, b in zip(offs[:-1], offs[1:])]
    data = pkg.PartitionedData(parts)
    for frac in (0.05, 0.6):
        w, h, counts = pkg.runParallelizedSGD(data, pkg.LeastSquaresGradient(), pkg.SimpleSGDUpdater(), 0.01,
                                              2, 0.0, frac, np.zeros(8), 0.0, return_chain_counts=True)
        wr, hr, cr = oracle.run(oracle.Matrix(y, X), offs, "least_squares", "simple", 0.01, 2, 0.0,
                                np.zeros(8), tol=0.0, fraction=frac)
        assert [list(map(int, c)) for c in counts] == [list(map(int, c)) for c in cr]
        assert_close(w, wr, what=f"f={frac} weights")
        assert_close(h, hr, what=f"f={frac} loss")


def test_empty_partitions_nan_poisoning(pkg, oracle):
    """Two leading empty partitions: (w*0 + w*0)/0 = NaN, as the reference's combiner gives when
    Spark merges them first (ParallelizedSGD.scala:272-274)."""
    X = np.array([[1.0, 2.0], [0.5, -1.0]])
    y = np.array([1.0, 0.0])
    parts = [pkg.DensePartition(y[:0], X[:0]), pkg.DensePartition(y[:0], X[:0]), pkg.DensePartition(y, X)]
    w, h = pkg.runParallelizedSGD(pkg.PartitionedData(parts), pkg.LogisticGradient(), pkg.SimpleSGDUpdater(),
                                  1.0, 1, 0.0, 1.0, np.array([0.1, 0.2]), 0.0)
    wr, hr, _ = oracle.run(oracle.Matrix(y, X), [0, 0, 0, 2], "logistic", "simple", 1.0, 1, 0.0,
                           np.array([0.1, 0.2]), tol=0.0)
    assert np.all(np.isnan(w)) and np.all(np.isnan(wr))
    assert_close(h, hr, what="loss")


def test_device_registration_matches_host(pkg, oracle):
    import torch
    rng = np.random.default_rng(3)
    n, d, P = 3000, 512, 6
    X, y = synth(rng, n, d, "logistic", np.float32)
    host = pkg.PartitionedData.parallelize(y, X, P, dtype=np.float32)
    Xd = torch.from_numpy(X).cuda()
    yd = torch.from_numpy(y).cuda()
    offs = [i * n // P for i in range(P)] + [n]
    dev = pkg.PartitionedData([pkg.DevicePartition(yd[a:b], Xd[a:b], d) for a, b in zip(offs[:-1], offs[1:])])
    args = (pkg.LogisticGradient(), pkg.SimpleSGDUpdater(), 1.0, 2, 0.0, 1.0, np.zeros(d), 0.0)
    w1, h1 = pkg.runParallelizedSGD(host, *args)
    w2, h2 = pkg.runParallelizedSGD(dev, *args)
    assert np.array_equal(w1, w2) and np.array_equal(h1, h2)


def test_host_pointer_epoch_abi(pkg, oracle):
    """psgd_run_epoch (the JNI-shaped call with host buffers) = one oracle iteration."""
    rng = np.random.default_rng(4)
    n, d, P = 900, 64, 3
    X, y = synth(rng, n, d, "hinge")
    ctx = pkg._native.Context(0)
    offs = [i * n // P for i in range(P)] + [n]
    for p in range(P):
        ctx.register_dense(p, y[offs[p]:offs[p + 1]], X[offs[p]:offs[p + 1]])
    prm = pkg.make_params(pkg.HingeGradient(), pkg.SimpleSGDUpdater(), 0.7, 0.0, 1.0, 0.0)
    w, rv, loss, cnt, counts = ctx.run_epoch(prm, np.zeros(d))
    wr, rvr, lr, cr = oracle.run_chains(oracle.Matrix(y, X), offs, "hinge", "simple", 0.7, 0.0, np.zeros(d))
    assert list(counts) == list(cr) and cnt == n
    acc_w, acc_c = wr[0].copy(), cr[0]
    for p in range(1, P):
        acc_w = (acc_w * acc_c + wr[p] * cr[p]) / (acc_c + cr[p])
        acc_c += cr[p]
    assert_close(w, acc_w, what="weights")
    assert_close(loss, lr.sum(), what="loss")
    ctx.close()


def test_determinism_many_chains(pkg):
    rng = np.random.default_rng(6)
    n, d, P = 256 * 300, 512, 256
    X, y = synth(rng, n, d, "least_squares", np.float32)
    data = pkg.PartitionedData.parallelize(y, X, P, dtype=np.float32)
    args = (pkg.LeastSquaresGradient(), pkg.SimpleSGDUpdater(), 1e-3, 2, 0.0, 1.0, np.zeros(d), 0.0)
    w1, h1 = pkg.runParallelizedSGD(data, *args)
    w2, h2 = pkg.runParallelizedSGD(data, *args)
    assert np.array_equal(w1, w2) and np.array_equal(h1, h2)


def test_libsvm_file_to_chains(pkg, oracle, tmp_path):
    """MLUtils.loadLibSVMFile -> runParallelizedSGD: the natively parsed CSR partitions through
    the fp64 chain, against the oracle on the same rows and partition boundaries."""
    rng = np.random.default_rng(21)
    lines = []
    for _ in range(600):
        idx = np.sort(rng.choice(40, size=int(rng.integers(1, 8)), replace=False)) + 1
        lines.append(f"{int(rng.integers(0, 2))} " + " ".join(f"{i}:{rng.uniform(0, 1):.5f}" for i in idx))
    f = tmp_path / "train.libsvm"
    f.write_text("\n".join(lines) + "\n")
    data = pkg.loadLibSVMFile(str(f), -1, 3)
    assert len(data.partitions) >= 3
    w, h = pkg.runParallelizedSGD(data, pkg.HingeGradient(), pkg.SquaredL2SGDUpdater(), 0.5, 3, 0.01, 1.0,
                                  np.zeros(data.partitions[0].d), 0.0)
    y = np.concatenate([p.labels for p in data.partitions])
    rp, col, val, offs = [0], [], [], [0]
    for p in data.partitions:
        col.append(p.col)
        val.append(p.val)
        rp += list(p.row_ptr[1:] + rp[-1])
        offs.append(offs[-1] + p.n_rows)
    mat = oracle.Matrix(y, row_ptr=np.array(rp), col=np.concatenate(col), val=np.concatenate(val),
                        d=data.partitions[0].d)
    wr, hr, _ = oracle.run(mat, offs, "hinge", "squared_l2", 0.5, 3, 0.01, np.zeros(data.partitions[0].d), tol=0.0)
    assert_close(w, wr, what="weights")
    assert_close(h, hr, what="loss")


@pytest.mark.parametrize("d", [100, 300, 700, 1024])
@pytest.mark.parametrize("grad", ["least_squares", "logistic", "hinge"])
@pytest.mark.parametrize("upd", ["simple", "squared_l2"])
@pytest.mark.parametrize("storage", [np.float32, np.float64])
def test_fp64_block_rows_in_registers(pkg, oracle, d, grad, upd, storage):
    """chain_block64 (NV = 1, 2, 4 f32 / 1, 2, 4, 8 f64; the c2 / c3 fp64 instances, f32 and the
    reference's Double rows): one chain wave at NV = 1, else two chain waves that split the
    features and exchange their partial dots per block, every row of a block held in registers.
    d = 100 / 300 / 700 exercise the zero-masked row end, 903-row partitions a ragged last block;
    1e-9 and exact counts against the oracle."""
    rng = np.random.default_rng(d + len(grad) * 3 + len(upd))
    n, P = 2709, 3
    X, y = synth(rng, n, d, grad, np.float32)
    data = pkg.PartitionedData.parallelize(y, X.astype(storage), P, dtype=storage)
    offs = [i * n // P for i in range(P)] + [n]
    step = 2.0 / d if grad == "logistic" else 0.5 / d   # non-chaotic trajectories (1e-9 bar)
    G = {"logistic": pkg.LogisticGradient, "least_squares": pkg.LeastSquaresGradient, "hinge": pkg.HingeGradient}
    U = {"simple": pkg.SimpleSGDUpdater, "squared_l2": pkg.SquaredL2SGDUpdater}
    w, h, counts = pkg.runParallelizedSGD(data, G[grad](), U[upd](), step, 3, 0.05, 1.0, np.zeros(d), 0.0,
                                          return_chain_counts=True)
    vec = 4 if storage == np.float32 else 2
    nv = 1
    while nv * 64 * vec < d:
        nv *= 2
    waves = 2 if nv >= 2 else 1
    assert pkg.optimization.get_context(0).last_kernel() == 700 + 10 * (waves - 1) + nv
    wr, hr, cr = oracle.run(oracle.Matrix(y, X.astype(np.float64)), offs, grad, upd, step, 3, 0.05,
                            np.zeros(d), tol=0.0, n_threads=8)
    assert [list(c) for c in counts] == [list(c) for c in cr[: len(counts)]]
    assert_close(w, wr, what=f"d={d} {grad} {upd} weights")
    assert_close(h, hr, what=f"d={d} {grad} {upd} loss")


@pytest.mark.parametrize("upd", ["adagrad", "adam"])
@pytest.mark.parametrize("d,storage", [(40, np.float64), (300, np.float32), (1024, np.float32),
                                       (1024, np.float64)])
def test_dense_fp64_stateful_updaters_in_registers(pkg, oracle, upd, d, storage):
    """AdaGrad / Adam (SGDUpdater.scala:193-286) in the fp64 parity mode on chain_dense /
    chain_split: the weights and the updater status in registers (stateful_variant), f32 and f64 rows,
    tol 0 and tol > 0 (per-sample breaks). 1e-9 and exact counts against the oracle."""
    rng = np.random.default_rng(d * 3 + len(upd))
    n, P = 2400, 4
    X, y = synth(rng, n, d, "logistic", np.float32)
    data = pkg.PartitionedData.parallelize(y, X.astype(storage), P, dtype=storage)
    offs = [i * n // P for i in range(P)] + [n]
    step = 0.05
    vec = 4 if storage == np.float32 else 2
    nv = 1
    while nv * 64 * vec < d:
        nv *= 2
    for tol in (0.0, 0.001):
        w, h, counts = pkg.runParallelizedSGD(data, pkg.LogisticGradient(), getattr(pkg, U[upd])(), step, 3,
                                              0.0, 1.0, np.zeros(d), tol, return_chain_counts=True)
        assert pkg.optimization.get_context(0).last_kernel() == stateful_variant(upd, tol, nv)
        wr, hr, cr = oracle.run(oracle.Matrix(y, X.astype(np.float64)), offs, "logistic", upd, step, 3, 0.0,
                                np.zeros(d), tol=tol, n_threads=8)
        tag = f"{upd} d={d} {np.dtype(storage).name} tol={tol}"
        assert [list(c) for c in counts] == [list(c) for c in cr[: len(counts)]], tag
        assert_close(w, wr, what=tag + " weights")
        assert_close(h, hr, what=tag + " loss")


@pytest.mark.parametrize("grad", ["logistic", "least_squares", "hinge"])
@pytest.mark.parametrize("upd", ["simple", "squared_l2"])
@pytest.mark.parametrize("d,storage", [(60, np.float64), (200, np.float32), (256, np.float64),
                                       (700, np.float32), (1024, np.float64), (2048, np.float32)])
def test_block64_per_sample_break(pkg, oracle, grad, upd, d, storage):
    """tol > 0 on chain_block64 (fp64 Simple / SquaredL2): the per-sample isConverged break
    (PSGD.scala:262, :324-336) decided from the block recurrence's norms (psgd_block64.hip header:
    ||w'||^2 and ||w - w'||^2 from z, c and the Gram diagonal). 64 ragged chains (45-46 rows:
    full blocks and a tail block) at tols whose breaks fall on every row of a block, and one that
    breaks few chains: exact per-chain counts and 1e-9 against the oracle."""
    rng = np.random.default_rng(d + len(grad) * 13 + len(upd))
    P = 64
    n = P * 45 + 29
    X, y = synth(rng, n, d, grad)
    X = X.astype(storage)
    data = pkg.PartitionedData.parallelize(y, X, P, dtype=storage)
    offs = [i * n // P for i in range(P)] + [n]
    sizes = np.diff(offs)
    vec = 4 if storage == np.float32 else 2
    nv = 1
    while nv * 64 * vec < d:
        nv *= 2
    step = {"least_squares": 0.5 / d, "logistic": 4.0 / d, "hinge": 2.0 / d}[grad]
    rows_hit = set()
    for tol in (0.01, 0.03, 0.1):
        w, h, counts = pkg.runParallelizedSGD(data, getattr(pkg, G[grad])(), getattr(pkg, U[upd])(), step, 3,
                                              0.05, 1.0, np.zeros(d), tol, return_chain_counts=True)
        assert pkg.optimization.get_context(0).last_kernel() == block64_variant(tol, nv)
        wr, hr, cr = oracle.run(oracle.Matrix(y, X.astype(np.float64)), offs, grad, upd, step, 3, 0.05,
                                np.zeros(d), tol=tol, n_threads=8)
        tag = f"{grad} {upd} d={d} {np.dtype(storage).name} tol={tol}"
        assert [list(c) for c in counts] == [list(c) for c in cr[: len(counts)]], tag
        assert_close(w, wr, what=tag + " weights")
        assert_close(h, hr, what=tag + " loss")
        rows_hit |= {(c - 1) % 8 for it in cr for c, s in zip(it, sizes) if 0 < c < s}
    assert len(rows_hit) >= 2, rows_hit   # breaks at more than one row position of a block


def test_block64_break_every_block_row(pkg, oracle):
    """Breaks on each of the 8 rows of a block, in full and tail blocks, with f32 and f64 rows
    (the H = 1 and H = 2 chain-wave forms), against the oracle's exact counts."""
    for d, storage, nvh in ((60, np.float64, 1), (700, np.float32, 2)):
        rng = np.random.default_rng(99 + d)
        P = 96
        n = P * 45 + 29
        X, y = synth(rng, n, d, "logistic")
        X = X.astype(storage)
        data = pkg.PartitionedData.parallelize(y, X, P, dtype=storage)
        offs = [i * n // P for i in range(P)] + [n]
        sizes = np.diff(offs)
        hit = set()
        for tol in (0.01, 0.015, 0.02, 0.03):
            w, h, counts = pkg.runParallelizedSGD(data, pkg.LogisticGradient(), pkg.SimpleSGDUpdater(),
                                                  4.0 / d, 2, 0.0, 1.0, np.zeros(d), tol,
                                                  return_chain_counts=True)
            wr, hr, cr = oracle.run(oracle.Matrix(y, X.astype(np.float64)), offs, "logistic", "simple",
                                    4.0 / d, 2, 0.0, np.zeros(d), tol=tol, n_threads=8)
            assert [list(c) for c in counts] == [list(c) for c in cr[: len(counts)]], (d, tol)
            assert_close(w, wr, what=f"d={d} tol={tol} weights")
            hit |= {((c - 1) % 8, c > s // 8 * 8) for it in cr for c, s in zip(it, sizes) if 0 < c < s}
        assert {r for r, _ in hit} == set(range(8)), (d, sorted(hit))
