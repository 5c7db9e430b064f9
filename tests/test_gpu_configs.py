"""BASELINE.json's configs at their own workload shapes, and the multi-rank device path.

* C1 (Logistic dense 100k x 100 fp64, 4 partitions, 10 iterations) at full size, tol 0 and
  tol 0.001 (the per-sample break): exact chain counts, 1e-9 weights/loss.
* C4 (Hinge CSR, rcv1-like: d = 47,236, 60-128 nnz/row, rows L2-normalised) on 256 chains:
  fp32 through chain_sparse_lds (variant 601: an LDS head of ~22k features, the tail in HBM) and
  chain_sparse_spec (variant 411, its 94 KB LDS tag table at this d), and fp64
  through chain_sparse_lds in fp64 (variant 620: an LDS head of ~5k doubles, the tail in HBM).
* C5 (L2 Logistic CSR, d = 2^22, 100 nnz/row, lambda 1e-6, step 0.5): fp32 chain_sparse
  (variant 401, HBM-resident weights) and fp64 chain_sparse64 (variant 420: double vectors in HBM,
  alpha-scaled SquaredL2).
* psgd_fold_partials_device (the cross-GPU level of the treeReduce, PSGD.scala:271-276) bit for
  bit against the combiner restated in numpy, incl. a zero-count and a NaN-count rank.
* The engine's two-level fold over partition subsets (what two ranks do) against the oracle's
  two-level fold, and HipEngine at world size 2 (two processes over gloo sharing cuda:0).

Tolerances: fp64 1e-9 relative (TestingUtils relTol, abs floor 1e-12), counts exact; fp32
compute FP32_REL * max|w| on weights and FP32_LOSS_REL relative on the loss.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT, has_gpu
from test_gpu_parity import ABS_FLOOR, REL, assert_close

pytestmark = pytest.mark.gpu

FP32_REL = 2e-4
FP32_LOSS_REL = 1e-4


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not has_gpu():
        pytest.skip("no GPU")


def c1_data(n=100_000, d=100, seed=42):
    """X ~ N(0,1), w* ~ N(0, 1/d), y = 1{w*.x + Logistic(0,1) > 0}."""
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, d))
    w = rng.standard_normal(d) / np.sqrt(d)
    y = ((X @ w + rng.logistic(size=n)) > 0).astype(np.float64)
    return X, y


def csr_rows(rng, n, d, nnz_lo, nnz_hi, normal_vals=False):
    """Distinct sorted column indices per row; values U(0,1) L2-normalised per row (rcv1 style)
    or N(0,1)/10 (C5)."""
    rp = np.zeros(n + 1, np.int64)
    cols, vals = [], []
    for i in range(n):
        k = int(rng.integers(nnz_lo, nnz_hi + 1))
        c = np.sort(rng.choice(d, size=k, replace=False)).astype(np.int32)
        if normal_vals:
            v = rng.standard_normal(k) / 10.0
        else:
            v = rng.uniform(size=k)
            v /= np.linalg.norm(v)
        cols.append(c)
        vals.append(v)
        rp[i + 1] = rp[i] + k
    return rp, np.concatenate(cols), np.concatenate(vals)


def planted_labels(rng, rp, col, val, d):
    wt = rng.standard_normal(d)
    z = np.add.reduceat(val * wt[col], rp[:-1]) if len(val) else np.zeros(len(rp) - 1)
    return ((z + rng.logistic(size=len(rp) - 1)) > 0).astype(np.float64)


def csr_parts(pkg, y, rp, col, val, d, offs):
    return pkg.PartitionedData([
        pkg.CsrPartition(y[a:b], rp[a:b + 1] - rp[a], col[rp[a]:rp[b]], val[rp[a]:rp[b]], d)
        for a, b in zip(offs[:-1], offs[1:])])


def check_fp32(w, h, wr, hr, tag):
    scale = max(np.max(np.abs(wr)), 1e-30)
    err = np.max(np.abs(w - wr)) / scale
    assert err <= FP32_REL, f"{tag}: weights max err {err:.3g} x max|w|"
    herr = np.max(np.abs(h - hr) / np.maximum(np.abs(hr), 1e-30))
    assert herr <= FP32_LOSS_REL, f"{tag}: loss rel err {herr:.3g}"


# ------------------------------------------------------------------------------------------
# C1 at full size
# ------------------------------------------------------------------------------------------
@pytest.mark.parametrize("tol", [0.0, 0.001])
def test_c1_full_size(pkg, oracle, tol):
    X, y = c1_data()
    n, d, P = X.shape[0], X.shape[1], 4
    data = pkg.PartitionedData.parallelize(y, X, P)
    offs = [i * n // P for i in range(P)] + [n]
    w0 = np.zeros(d)
    w, h, counts = pkg.runParallelizedSGD(data, pkg.LogisticGradient(), pkg.SimpleSGDUpdater(), 1.0, 10,
                                          0.0, 1.0, w0, tol, return_chain_counts=True)
    wr, hr, cr = oracle.run(oracle.Matrix(y, X), offs, "logistic", "simple", 1.0, 10, 0.0, w0, tol=tol,
                            n_threads=4)
    assert [list(map(int, c)) for c in counts] == [list(map(int, c)) for c in cr[: len(counts)]]
    if tol == 0.0:
        assert len(h) == 10 and all(int(c.sum()) == n for c in counts)
    else:
        assert all(int(c.sum()) < n for c in counts)   # the per-sample break fires
    assert_close(w, wr, what=f"c1 tol={tol} weights")
    assert_close(h, hr, what=f"c1 tol={tol} loss")


# ------------------------------------------------------------------------------------------
# C4: rcv1-like Hinge CSR at d = 47,236
# ------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def c4():
    rng = np.random.default_rng(404)
    d, P, per = 47_236, 256, 100
    n = P * per
    rp, col, val = csr_rows(rng, n, d, 60, 128)
    y = planted_labels(rng, rp, col, val, d)
    offs = [i * n // P for i in range(P)] + [n]
    return d, rp, col, val, y, offs


@pytest.mark.parametrize("kernel,variant", [("lds", 601), ("spec", 411)])
def test_c4_rcv1_shape_fp32(pkg, oracle, c4, kernel, variant, monkeypatch):
    # chain_sparse_lds (LDS head of ~22k features, tail in HBM) and chain_sparse_spec (94 KB tag table)
    monkeypatch.setenv("PSGD_SPARSE_KERNEL", kernel)
    d, rp, col, val, y, offs = c4
    v32 = val.astype(np.float32)
    data = csr_parts(pkg, y, rp, col, v32, d, offs)
    w, h, counts = pkg.runParallelizedSGD(data, pkg.HingeGradient(), pkg.SimpleSGDUpdater(), 1.0, 3, 0.0, 1.0,
                                          np.zeros(d), 0.0, compute_dtype="f32", return_chain_counts=True)
    assert pkg.optimization.get_context(0).last_kernel() == variant
    mat = oracle.Matrix(y, row_ptr=rp, col=col, val=v32.astype(np.float64), d=d)
    wr, hr, cr = oracle.run(mat, offs, "hinge", "simple", 1.0, 3, 0.0, np.zeros(d), tol=0.0, n_threads=8)
    assert [list(map(int, c)) for c in counts] == [list(map(int, c)) for c in cr]
    check_fp32(w, h, wr, hr, "c4 fp32")


def test_c4_rcv1_shape_fp64(pkg, oracle, c4):
    d, rp, col, val, y, offs = c4
    data = csr_parts(pkg, y, rp, col, val, d, offs)
    w, h, counts = pkg.runParallelizedSGD(data, pkg.HingeGradient(), pkg.SimpleSGDUpdater(), 1.0, 2, 0.0, 1.0,
                                          np.zeros(d), 0.0, return_chain_counts=True)
    assert pkg.optimization.get_context(0).last_kernel() == 620   # chain_sparse_lds<double, double>
    mat = oracle.Matrix(y, row_ptr=rp, col=col, val=val, d=d)
    wr, hr, cr = oracle.run(mat, offs, "hinge", "simple", 1.0, 2, 0.0, np.zeros(d), tol=0.0, n_threads=8)
    assert [list(map(int, c)) for c in counts] == [list(map(int, c)) for c in cr]
    assert_close(w, wr, what="c4 fp64 weights")
    assert_close(h, hr, what="c4 fp64 loss")


# ------------------------------------------------------------------------------------------
# C5: L2 Logistic CSR at d = 2^22 (weights HBM-resident)
# ------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def c5():
    rng = np.random.default_rng(505)
    d, P, per = 1 << 22, 32, 64
    n = P * per
    rp, col, val = csr_rows(rng, n, d, 100, 100, normal_vals=True)
    y = planted_labels(rng, rp, col, val, d)
    offs = [i * n // P for i in range(P)] + [n]
    w0 = np.zeros(d)
    return d, rp, col, val, y, offs, w0


@pytest.mark.parametrize("compute,want", [("f32", 401), ("f64", 420)])
def test_c5_wide_sparse_l2(pkg, oracle, c5, compute, want):
    # f32: chain_sparse (HBM-resident weights); f64: chain_sparse64 (double vectors in HBM, alpha-scaled SquaredL2)
    d, rp, col, val, y, offs, w0 = c5
    vs = val.astype(np.float32) if compute == "f32" else val
    data = csr_parts(pkg, y, rp, col, vs, d, offs)
    iters = 2
    w, h, counts = pkg.runParallelizedSGD(data, pkg.LogisticGradient(), pkg.SquaredL2SGDUpdater(), 0.5, iters,
                                          1e-6, 1.0, w0, 0.0, compute_dtype=compute, return_chain_counts=True)
    assert pkg.optimization.get_context(0).last_kernel() == want
    mat = oracle.Matrix(y, row_ptr=rp, col=col, val=vs.astype(np.float64), d=d)
    wr, hr, cr = oracle.run(mat, offs, "logistic", "squared_l2", 0.5, iters, 1e-6, w0, tol=0.0, n_threads=8)
    assert [list(map(int, c)) for c in counts] == [list(map(int, c)) for c in cr]
    if compute == "f32":
        check_fp32(w, h, wr, hr, "c5 fp32")
    else:
        assert_close(w, wr, what="c5 fp64 weights")
        assert_close(h, hr, what="c5 fp64 loss")


# ------------------------------------------------------------------------------------------
# The cross-GPU fold and the multi-rank engine
# ------------------------------------------------------------------------------------------
def np_fold(parts, d):
    """The reference combiner (PSGD.scala:271-276) over (d+3)-vectors, left fold in order."""
    acc = parts[0].copy()
    for q in parts[1:]:
        c1, c2 = acc[d + 2], q[d + 2]
        acc[:d] = (acc[:d] * c1 + q[:d] * c2) / (c1 + c2)
        acc[d] = (acc[d] * c1 + q[d] * c2) / (c1 + c2)
        acc[d + 1] = acc[d + 1] + q[d + 1]
        acc[d + 2] = c1 + c2
    return acc


def test_fold_partials_device_bitwise(pkg):
    import warnings
    warnings.simplefilter("ignore", RuntimeWarning)   # 0/0 in the restated combiner (intended)
    import torch
    rng = np.random.default_rng(31)
    ctx = pkg.optimization.get_context(0)
    for d in (1, 7, 300, 5000):
        for counts in ([3.0, 5.0, 11.0], [7.0, 0.0, 4.0, 9.0], [0.0, 6.0], [5.0], [2.0, float("nan"), 3.0],
                       [0.0, 0.0, 8.0]):
            world = len(counts)
            g = np.zeros((world, d + 3))
            g[:, :d] = rng.standard_normal((world, d))
            g[:, d] = rng.uniform(size=world)
            g[:, d + 1] = rng.uniform(1, 100, size=world)
            g[:, d + 2] = counts
            # a real stream handle (NULL would select the library's own stream)
            st = torch.cuda.Stream()
            with torch.cuda.stream(st):
                dev = torch.from_numpy(g.reshape(-1)).cuda()
                out = torch.empty(d + 3, dtype=torch.float64, device="cuda")
                ctx.fold_partials_device(world, d, dev.data_ptr(), out.data_ptr(), st.cuda_stream)
                got = out.cpu().numpy()
            want = np_fold(list(g), d)
            same = (got == want) | (np.isnan(got) & np.isnan(want))
            assert same.all(), (d, counts)


def _adversarial_values(rng, shape):
    """f64 values over the whole range: binary exponents -1074 .. 1023 (denormals, the tiny and
    huge ends where v_div_scale rescales), signed zeros, infinities and NaN among normal ones."""
    e = rng.integers(-1074, 1024, size=shape)
    v = np.ldexp(rng.uniform(0.5, 1.0, size=shape), e) * rng.choice([-1.0, 1.0], size=shape)
    u = rng.uniform(size=shape)
    v = np.where(u < 0.5, rng.standard_normal(shape) * 10.0 ** rng.integers(-3, 4, size=shape), v)
    v = np.where(u > 0.97, 0.0, v)
    v = np.where(u > 0.98, -0.0, v)
    v = np.where(u > 0.99, np.inf, v)
    v = np.where(u > 0.995, np.nan, v)
    return v


def test_fold_step_bitwise_over_the_f64_range(pkg):
    """The fold kernel's division (fold_step: the compiler's f64 division sequence with the
    reciprocal of the count sum computed beside the running value, a stage folded again with `/`
    when a step leaves its ranges) against numpy's IEEE division in the combiner's order, bit for
    bit -- signed zeros and NaN included -- over weights and regVals spread across every binary
    exponent, counts from 0 to 2^40, 2 to 700 items (two LDS stages) per fold."""
    import warnings
    warnings.simplefilter("ignore", RuntimeWarning)
    import torch
    rng = np.random.default_rng(77)
    ctx = pkg.optimization.get_context(0)
    st = torch.cuda.Stream()
    for trial in range(24):
        world = int(rng.choice([2, 3, 17, 255, 700]))
        d = int(rng.choice([1, 63, 640]))
        g = np.zeros((world, d + 3))
        g[:, :d] = _adversarial_values(rng, (world, d))
        g[:, d] = _adversarial_values(rng, world)
        g[:, d + 1] = rng.standard_normal(world)
        cnt = rng.integers(0, 40000, size=world).astype(np.float64)
        if trial % 4 == 1:
            cnt = np.floor(2.0 ** rng.uniform(0, 40, size=world))
        if trial % 4 == 2:
            cnt[: world // 3] = 0.0
        g[:, d + 2] = cnt
        with torch.cuda.stream(st):
            dev = torch.from_numpy(g.reshape(-1)).cuda()
            out = torch.empty(d + 3, dtype=torch.float64, device="cuda")
            ctx.fold_partials_device(world, d, dev.data_ptr(), out.data_ptr(), st.cuda_stream)
            got = out.cpu().numpy()
        want = np_fold(list(g), d)
        same = ((got == want) & (np.signbit(got) == np.signbit(want))) | (np.isnan(got) & np.isnan(want))
        assert same.all(), (trial, world, d, np.nonzero(~same)[0][:5], got[~same][:5], want[~same][:5])


def test_two_level_fold_of_partition_subsets(pkg, oracle):
    """What two ranks do, in one process: the engine's epoch over each rank's partition block
    (its on-device fold), then psgd_fold_partials_device over the two partials -- bit for bit
    against the combiner restated on those partials, and within 1e-9 of the oracle's two-level
    fold (oracle.run(groups=...))."""
    import torch
    rng = np.random.default_rng(32)
    n, d, P = 2400, 48, 5
    X = rng.standard_normal((n, d))
    y = (rng.uniform(size=n) > 0.5).astype(float)
    data = pkg.PartitionedData.parallelize(y, X, P)
    offs = [i * n // P for i in range(P)] + [n]
    bounds = [pkg.shard_range(P, r, 2) for r in range(2)]
    prm = pkg.make_params(pkg.LogisticGradient(), pkg.SquaredL2SGDUpdater(), 0.5, 0.01, 1.0, 0.0)
    w_in = torch.from_numpy(0.01 * rng.standard_normal(d)).cuda()
    partials = []
    for r in range(2):
        eng = pkg.HipEngine(data, r, 2, device=0)   # registers partitions [lo, hi) only
        eng.stream.wait_stream(torch.cuda.current_stream())
        part, _ = eng.local_partial(prm, w_in, False)
        eng.stream.synchronize()
        partials.append(part.clone())
    ctx = pkg.optimization.get_context(0)
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        g = torch.cat(partials)
        out = torch.empty(d + 3, dtype=torch.float64, device="cuda")
        ctx.fold_partials_device(2, d, g.data_ptr(), out.data_ptr(), st.cuda_stream)
        got = out.cpu().numpy()
    assert np.array_equal(got, np_fold([p.cpu().numpy() for p in partials], d))
    groups = [0, bounds[0][1], bounds[1][1]]
    wr, hr, cr = oracle.run(oracle.Matrix(y, X), offs, "logistic", "squared_l2", 0.5, 1, 0.01,
                            w_in.cpu().numpy(), tol=0.0, groups=groups)
    assert int(got[d + 2]) == n
    assert_close(got[:d], wr, what="two-level fold weights")
    # loss history entry 1 = lossSum / count + regVal_0 (PSGD.scala:283)
    rv0 = ctx.initial_regval(prm, w_in.cpu().numpy())
    assert_close([got[d + 1] / got[d + 2] + rv0], hr, what="two-level fold loss")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("P", [5, 1])
def test_hip_engine_two_ranks(tmp_path, pkg, oracle, P):
    """HipEngine at world size 2: two fresh processes (started as children, gloo over
    127.0.0.1, both on cuda:0) run runParallelizedSGD through the real engine -- partition
    blocks per rank, on-device fold, all-gather of the partials, psgd_fold_partials_device in
    rank order, the empty-rank identity when P = 1. Against the oracle's two-level fold."""
    out = str(tmp_path / "res.npz")
    script = os.path.join(ROOT, "tests", "two_rank_hip.py")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), PSGD_TEST_P=str(P))
    r = subprocess.run([sys.executable, script, out], env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = np.load(out)
    X, y, n, d = (res["X"], res["y"], int(res["n"]), int(res["d"]))
    offs = [i * n // P for i in range(P)] + [n]
    bounds = [pkg.shard_range(P, rk, 2) for rk in range(2)]
    groups = [0, bounds[0][1], bounds[1][1]] if P > 1 else None
    wr, hr, cr = oracle.run(oracle.Matrix(y, X), offs, "logistic", "squared_l2", 0.5, 4, 0.01, np.zeros(d),
                            tol=0.001, groups=groups)
    assert_close(res["w"], wr, what=f"P={P} weights")
    assert_close(res["h"], hr, what=f"P={P} loss")
    # each rank's chain counts, per iteration, are the oracle's for its partitions
    c0, c1 = res["c0"], res["c1"]
    lo1 = bounds[1][0]
    assert [list(c) for c in c0] == [list(c[:lo1]) for c in cr[: len(c0)]]
    if P > 1:
        assert [list(c) for c in c1] == [list(c[lo1:]) for c in cr[: len(c1)]]
    # the pipelined loop (tol = 0): 5 iterations, all rows every time
    wr0, hr0, _ = oracle.run(oracle.Matrix(y, X), offs, "logistic", "squared_l2", 0.5, 5, 0.01, np.zeros(d),
                             tol=0.0, groups=groups)
    assert len(res["hp"]) == 5
    assert_close(res["wp"], wr0, what=f"P={P} pipelined weights")
    assert_close(res["hp"], hr0, what=f"P={P} pipelined loss")


def test_rccl_exchange_single_rank(tmp_path):
    """The engine's RCCL leg (ShardedEngine.exchange: dist.all_gather_into_tensor into the gather
    buffer, then psgd_fold_partials_device) in a one-rank nccl process group: bit for bit the
    single-process epoch's partial, for dense fp64 and CSR fp32 partitions."""
    out = str(tmp_path / "rccl.npz")
    script = os.path.join(ROOT, "tests", "one_rank_nccl.py")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    r = subprocess.run([sys.executable, script, out], env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = np.load(out)
    for name in ("dense", "csr"):
        single, rccl = res[name + "_single"], res[name + "_rccl"]
        assert np.isfinite(single).all() and single[-1] > 0, name
        assert np.array_equal(single, rccl), name
        assert np.array_equal(single, res[name + "_default"]), name + " read on the default stream"


def test_epoch_result_on_default_stream(pkg):
    """HipEngine.epoch returns tensors written on the engine's stream; a caller that reads them on
    its own (default) stream, with no stream block, must see the finished epoch (a
    CSR fp32 partial once came back all zeros with count 0, which the driver would take for an
    empty batch and skip the update, ParallelizedSGD.scala:295-297). The partial buffer is
    poisoned first and the chains run long enough (256 chains x 4,000 rows) that an unordered
    read would see the poison."""
    import torch
    rng = np.random.default_rng(9)
    n, d, P, k = 1_024_000, 40_000, 256, 32
    rp = np.arange(n + 1, dtype=np.int64) * k
    col = np.sort(rng.choice(d - k, size=(n, k)), axis=1) + np.arange(k)[None, :]
    col = col.astype(np.int32).reshape(-1)
    val = rng.standard_normal(n * k).astype(np.float32)
    y = (rng.uniform(size=n) > 0.5).astype(np.float64)
    offs = [i * n // P for i in range(P + 1)]
    data = pkg.PartitionedData([pkg.CsrPartition(y[a:b], rp[a:b + 1] - rp[a], col[rp[a]:rp[b]], val[rp[a]:rp[b]], d)
                                for a, b in zip(offs[:-1], offs[1:])])
    eng = pkg.HipEngine(data, 0, 1, device=0)
    prm = pkg.make_params(pkg.HingeGradient(), pkg.SimpleSGDUpdater(), 0.5, 0.0, 1.0, 0.0, "f32")
    w = eng.weights(np.zeros(d))
    ref = None
    for _ in range(3):
        for b in eng._partials:   # (the result buffers alternate by epoch)
            b.fill_(-7.0)
        torch.cuda.synchronize()
        partial, _ = eng.epoch(prm, w)
        got = partial.cpu().numpy()          # the default stream, no stream block
        assert got[-1] == n, got[-3:]
        torch.cuda.synchronize()
        ref = got if ref is None else ref
        assert np.array_equal(got, ref)


@pytest.fixture(scope="module")
def c5_full_chains(oracle):
    """C5's per-GPU geometry: 1,024 chains over d = 2^22 (1,024 f32 weight vectors = 17 GB of
    wf32 in the fp32 mode), 2-4 rows each (ragged), 100 nnz per row; f32-representable values,
    so that one oracle run (2 iterations, ~1 min on 16 threads) serves both compute modes."""
    rng = np.random.default_rng(5050)
    d, P = 1 << 22, 1024
    per = rng.integers(2, 5, size=P)
    offs = [0] + [int(o) for o in np.cumsum(per)]
    n = offs[-1]
    rp, col, val = csr_rows(rng, n, d, 100, 100, normal_vals=True)
    val = val.astype(np.float32).astype(np.float64)
    y = planted_labels(rng, rp, col, val, d)
    mat = oracle.Matrix(y, row_ptr=rp, col=col, val=val, d=d)
    ref = oracle.run(mat, offs, "logistic", "squared_l2", 0.5, 2, 1e-6, np.zeros(d), tol=0.0, n_threads=16)
    return d, rp, col, val, y, offs, ref


@pytest.mark.parametrize("compute,want", [("f32", 401), ("f64", 420)])
def test_c5_1024_chains(pkg, c5_full_chains, compute, want):
    """C5 at its real chain count: wf32_init_kernel over 1,024 chains x 2^22 features, the
    chains, fold_f32_kernel over 1,024 fp32 vectors (f32); w64_init_kernel, chain_sparse64's
    alpha-scaled SquaredL2 and the fold over 1,024 f64 vectors (f64). Against the oracle: counts exact,
    fp64 at 1e-9, fp32 at its stated tolerance."""
    d, rp, col, val, y, offs, (wr, hr, cr) = c5_full_chains
    vs = val.astype(np.float32) if compute == "f32" else val
    data = csr_parts(pkg, y, rp, col, vs, d, offs)
    w, h, counts = pkg.runParallelizedSGD(data, pkg.LogisticGradient(), pkg.SquaredL2SGDUpdater(), 0.5, 2,
                                          1e-6, 1.0, np.zeros(d), 0.0, compute_dtype=compute,
                                          return_chain_counts=True)
    assert pkg.optimization.get_context(0).last_kernel() == want
    assert [list(map(int, c)) for c in counts] == [list(map(int, c)) for c in cr]
    if compute == "f32":
        check_fp32(w, h, wr, hr, "c5 1024 chains fp32")
    else:
        assert_close(w, wr, what="c5 1024 chains fp64 weights")
        assert_close(h, hr, what="c5 1024 chains fp64 loss")


def test_bench_two_ranks_gloo():
    """bench.py's multi-rank path -- the placeholder partitions of the other rank, the n * world
    count check, the prewarm MAX agreement, the world > 1 timing and the cross-rank all-gather +
    fold -- run with two ranks sharing cuda:0 over gloo (RCCL refuses two ranks on one device;
    the driver's 8-GPU node runs the nccl form). The line reports both ranks' samples."""
    import json
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
           "--rows", "200000", "--secondary", "c3:f32,c5:f32", "--secondary-rows", "100000",
           "--steps", "3", "--warmup", "1", "--prewarm-s", "0.2"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 3 and out["warmup"] == 1
    assert out["config"]["parallelism"].startswith("dp2"), out["config"]
    assert out["value"] > 0 and out["prewarm"]["epochs"] >= 2
    # both ranks' rows were counted: value = 2 * 200,000 samples per step / the step time
    assert abs(out["value"] * out["ms_per_step"] / 1e3 - 400_000) < 1.0, out
    # every rank's chain-kernel and all-gather + fold times, and the step-level roofline
    assert len(out["ranks"]["kernel_ms"]) == 2 and len(out["ranks"]["xchg_ms"]) == 2, out["ranks"]
    assert all(t > 0 for t in out["ranks"]["kernel_ms"] + out["ranks"]["xchg_ms"])
    assert 0 < out["roofline"]["frac_step"] <= out["roofline"]["frac"] * 1.05
    # the N > 1 secondary: BASELINE configs[2]'s per-GPU shard (c3), here at 100,000 rows per rank
    sec = out["secondary_summary"]
    assert [e["spec"] for e in sec] == ["c3:f32", "c5:f32"] and all("error" not in e for e in sec), sec
    assert len(sec[0]["ranks"]["kernel_ms"]) == 2 and sec[0]["frac_step"] > 0
    # c5 (configs[4]'s shard, here 100,000 rows per rank) with its store-mode probe on each rank
    assert len(sec[1]["ranks"]["xchg_ms"]) == 2 and "c5_store_probe" in sec[1], sec[1]
