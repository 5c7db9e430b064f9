"""The fp32 CSR chain kernels (psgd_sparse_lds.hip, psgd_sparse.hip) against the fp64 CPU oracle.

Every case runs on each kernel variant (PSGD_SPARSE_KERNEL forces one): chain_sparse_lds with
all weights in LDS, with an LDS head of d/3 features and the rest in HBM (PSGD_SPARSE_LDS_HEAD:
exercises the tail gathers and their corrections at small d) at speculation depths 4 and 8,
chain_sparse_spec, and chain_sparse.

fp32 compute is the throughput mode; its stated tolerance is weights within
FP32_REL * max|w| and the loss history within FP32_LOSS_REL relative of the fp64 oracle on the
same inputs. Chain counts are exact.

Cases: every gradient x {Simple, SquaredL2 (alpha-scaled lazy form)}; a narrow d where
consecutive rows share features all the time (the kernel's gather after its own scatter);
rows wider than 128 non-zeros (the per-lane loop past two entries); empty rows, empty and
one-row partitions; sampled batches (miniBatchFraction < 1); device-resident CSR registration.
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


KERNELS = {  # name: (environment, variant base without the storage digit)
    "lds": ({"PSGD_SPARSE_KERNEL": "lds"}, 600),
    "lds_tail": ({"PSGD_SPARSE_KERNEL": "lds", "PSGD_SPARSE_LDS_HEAD": "third"}, 600),
    "lds_tail_sk8": ({"PSGD_SPARSE_KERNEL": "lds", "PSGD_SPARSE_LDS_HEAD": "third", "PSGD_SPARSE_SK": "8"}, 610),
    "spec": ({"PSGD_SPARSE_KERNEL": "spec"}, 410),
    "plain": ({"PSGD_SPARSE_KERNEL": "plain"}, 400),
}


@pytest.fixture(params=sorted(KERNELS))
def kernel(request, monkeypatch):
    env, base = KERNELS[request.param]
    for k in ("PSGD_SPARSE_KERNEL", "PSGD_SPARSE_LDS_HEAD", "PSGD_SPARSE_SK"):
        monkeypatch.delenv(k, raising=False)

    def apply(d):
        for k, v in env.items():
            monkeypatch.setenv(k, str(max(d // 3, 0)) if v == "third" else v)
        return base
    return apply


def synth_csr(rng, n, d, kmin, kmax, grad):
    rp, col, val = [0], [], []
    for _ in range(n):
        k = int(rng.integers(kmin, kmax + 1))
        idx = np.sort(rng.choice(d, size=min(k, d), replace=False))
        col += idx.tolist()
        v = rng.uniform(0.1, 1.0, size=len(idx))
        v /= max(np.linalg.norm(v), 1e-12)
        val += v.astype(np.float32).tolist()
        rp.append(len(col))
    rp, col, val = np.array(rp, np.int64), np.array(col, np.int32), np.array(val, np.float64)
    wt = rng.standard_normal(d)
    z = np.array([val[rp[i]:rp[i + 1]] @ wt[col[rp[i]:rp[i + 1]]] for i in range(n)])
    if grad == "least_squares":
        y = z + 0.1 * rng.standard_normal(n)
    else:
        y = ((z + rng.logistic(size=n)) > 0).astype(np.float64)
    return rp, col, val, y


def check(pkg, oracle, rp, col, val, y, d, offs, grad, upd, step, reg, iters, frac=1.0, dtype=np.float32,
          kernel=None):
    base = kernel(d) if kernel else None
    vstore = val.astype(dtype)
    parts = [pkg.CsrPartition(y[a:b], rp[a:b + 1] - rp[a], col[rp[a]:rp[b]], vstore[rp[a]:rp[b]], d)
             for a, b in zip(offs[:-1], offs[1:])]
    data = pkg.PartitionedData(parts)
    w, h, counts = pkg.runParallelizedSGD(data, getattr(pkg, G[grad])(), getattr(pkg, U[upd])(), step,
                                          iters, reg, frac, np.zeros(d), 0.0, compute_dtype="f32",
                                          return_chain_counts=True)
    # 63x: Gram recurrence; 60x/61x: weights in LDS; 41x: gathers SK samples ahead (tag table in LDS); 40x: one per
    # sample. Rows of more than 128 non-zeros always take 40x.
    wide = int(np.max(np.diff(rp))) > 128
    if base is None:
        base = 600
    want = (400 if wide else base) + (1 if dtype == np.float32 else 0)
    assert pkg.optimization.get_context(0).last_kernel() == want
    mat = oracle.Matrix(y, row_ptr=rp, col=col, val=vstore.astype(np.float64), d=d)
    wr, hr, cr = oracle.run(mat, offs, grad, upd, step, iters, reg, np.zeros(d), tol=0.0, fraction=frac,
                            n_threads=8)
    tag = f"d={d} {grad} {upd} f={frac}"
    assert [list(c) for c in counts] == [list(c) for c in cr[: len(counts)]], tag
    scale = max(np.max(np.abs(wr)), 1e-30)
    err = np.max(np.abs(w - wr)) / scale
    assert err <= FP32_REL, f"{tag}: weights max err {err:.3g} x max|w|"
    herr = np.max(np.abs(h - hr) / np.maximum(np.abs(hr), 1e-30))
    assert herr <= FP32_LOSS_REL, f"{tag}: loss rel err {herr:.3g}"


@pytest.mark.parametrize("grad", ["least_squares", "logistic", "hinge"])
@pytest.mark.parametrize("upd", ["simple", "squared_l2"])
def test_sparse_wide(pkg, oracle, grad, upd, kernel):
    rng = np.random.default_rng(len(grad) * 7 + len(upd))
    n, d = 1500, 3000
    rp, col, val, y = synth_csr(rng, n, d, 0, 40, grad)
    offs = [0, 500, 500, 501, 1500]
    check(pkg, oracle, rp, col, val, y, d, offs, grad, upd, 0.3, 0.05, 3, kernel=kernel)


@pytest.mark.parametrize("grad", ["least_squares", "logistic", "hinge"])
def test_sparse_narrow_overlapping_rows(pkg, oracle, grad, kernel):
    # d = 12 with up to 9 non-zeros per row: nearly every feature is shared by consecutive rows
    rng = np.random.default_rng(3 + len(grad))
    n, d = 900, 12
    rp, col, val, y = synth_csr(rng, n, d, 1, 9, grad)
    offs = [0, 300, 600, 900]
    check(pkg, oracle, rp, col, val, y, d, offs, grad, "simple", 0.2, 0.0, 3, kernel=kernel)
    check(pkg, oracle, rp, col, val, y, d, offs, grad, "squared_l2", 0.2, 0.1, 2, kernel=kernel)


def test_sparse_rows_wider_than_128(pkg, oracle):
    rng = np.random.default_rng(9)
    n, d = 400, 1000
    rp, col, val, y = synth_csr(rng, n, d, 100, 300, "logistic")
    check(pkg, oracle, rp, col, val, y, d, [0, 200, 400], "logistic", "simple", 0.5, 0.0, 2)
    check(pkg, oracle, rp, col, val, y, d, [0, 200, 400], "hinge", "squared_l2", 0.5, 0.02, 2)


def test_sparse_sampled_batches(pkg, oracle, kernel):
    rng = np.random.default_rng(12)
    n, d = 2000, 500
    rp, col, val, y = synth_csr(rng, n, d, 0, 30, "hinge")
    for frac in (0.15, 0.6):
        check(pkg, oracle, rp, col, val, y, d, [0, 1000, 2000], "hinge", "simple", 0.5, 0.0, 3, frac=frac,
              kernel=kernel)


def test_sparse_f64_storage(pkg, oracle, kernel):
    rng = np.random.default_rng(13)
    n, d = 800, 200
    rp, col, val, y = synth_csr(rng, n, d, 0, 20, "logistic")
    check(pkg, oracle, rp, col, val, y, d, [0, 400, 800], "logistic", "simple", 0.5, 0.0, 2,
          dtype=np.float64, kernel=kernel)


def test_sparse_device_registration(pkg, oracle):
    import torch
    rng = np.random.default_rng(14)
    n, d = 1000, 700
    rp, col, val, y = synth_csr(rng, n, d, 1, 50, "least_squares")
    dev = torch.device("cuda", 0)
    t_rp = torch.from_numpy(rp).to(dev)
    t_col = torch.from_numpy(col).to(dev)
    t_val = torch.from_numpy(val.astype(np.float32)).to(dev)
    t_y = torch.from_numpy(y).to(dev)
    offs = [0, 250, 1000]
    parts = [pkg.DeviceCsrPartition(t_y[a:b], t_rp[a:b + 1], t_col, t_val, d) for a, b in zip(offs[:-1], offs[1:])]
    w, h = pkg.runParallelizedSGD(pkg.PartitionedData(parts), pkg.LeastSquaresGradient(), pkg.SimpleSGDUpdater(),
                                  0.3, 3, 0.0, 1.0, np.zeros(d), 0.0, compute_dtype="f32")
    mat = oracle.Matrix(y, row_ptr=rp, col=col, val=val.astype(np.float32).astype(np.float64), d=d)
    wr, hr, _ = oracle.run(mat, offs, "least_squares", "simple", 0.3, 3, 0.0, np.zeros(d), tol=0.0)
    assert np.max(np.abs(w - wr)) <= FP32_REL * np.max(np.abs(wr))
    assert np.max(np.abs(h - hr) / np.abs(hr)) <= FP32_LOSS_REL


# ------------------------------------------------------------------------------------------
# fp64 compute (the parity mode) on chain_sparse_lds<., double> and chain_sparse64 (rows wider than
# 128 entries, d past the LDS kernel's reach, or forced): 1e-9 and exact counts.
# ------------------------------------------------------------------------------------------
KERNELS64 = {  # name: (environment, variant base without the storage digit)
    "lds64": ({}, 620),
    "lds64_tail": ({"PSGD_SPARSE_LDS_HEAD": "third"}, 620),
    "lds64_tail_sk8": ({"PSGD_SPARSE_LDS_HEAD": "third", "PSGD_SPARSE_SK": "8"}, 630),
    "hbm64": ({"PSGD_SPARSE_KERNEL": "hbm64"}, 420),   # chain_sparse64: weights as doubles in HBM
}


@pytest.fixture(params=sorted(KERNELS64))
def kernel64(request, monkeypatch):
    env, base = KERNELS64[request.param]
    for k in ("PSGD_SPARSE_KERNEL", "PSGD_SPARSE_LDS_HEAD", "PSGD_SPARSE_SK"):
        monkeypatch.delenv(k, raising=False)

    def apply(d):
        for k, v in env.items():
            monkeypatch.setenv(k, str(max(d // 3, 0)) if v == "third" else v)
        return base
    return apply


def check64(pkg, oracle, rp, col, val, y, d, offs, grad, upd, step, reg, iters, frac=1.0, dtype=np.float64,
            kernel=None, want=None):
    from test_gpu_parity import assert_close
    base = kernel(d) if kernel else 620
    vstore = val.astype(dtype)
    parts = [pkg.CsrPartition(y[a:b], rp[a:b + 1] - rp[a], col[rp[a]:rp[b]], vstore[rp[a]:rp[b]], d)
             for a, b in zip(offs[:-1], offs[1:])]
    w, h, counts = pkg.runParallelizedSGD(pkg.PartitionedData(parts), getattr(pkg, G[grad])(),
                                          getattr(pkg, U[upd])(), step, iters, reg, frac, np.zeros(d), 0.0,
                                          return_chain_counts=True)
    if want is None:
        wide = int(np.max(np.diff(rp))) > 128
        want = (420 if wide else base) + (1 if dtype == np.float32 else 0)
    assert pkg.optimization.get_context(0).last_kernel() == want
    mat = oracle.Matrix(y, row_ptr=rp, col=col, val=vstore.astype(np.float64), d=d)
    wr, hr, cr = oracle.run(mat, offs, grad, upd, step, iters, reg, np.zeros(d), tol=0.0, fraction=frac,
                            n_threads=8)
    tag = f"fp64 d={d} {grad} {upd} f={frac}"
    assert [list(c) for c in counts] == [list(c) for c in cr[: len(counts)]], tag
    assert_close(w, wr, what=tag + " weights")
    assert_close(h, hr, what=tag + " loss")


@pytest.mark.parametrize("grad", ["least_squares", "logistic", "hinge"])
@pytest.mark.parametrize("upd", ["simple", "squared_l2"])
def test_sparse_fp64_wide(pkg, oracle, grad, upd, kernel64):
    rng = np.random.default_rng(len(grad) * 11 + len(upd))
    n, d = 1500, 3000
    rp, col, val, y = synth_csr(rng, n, d, 0, 40, grad)
    offs = [0, 500, 500, 501, 1500]
    check64(pkg, oracle, rp, col, val, y, d, offs, grad, upd, 0.3, 0.05, 3, kernel=kernel64)


@pytest.mark.parametrize("grad", ["least_squares", "logistic", "hinge"])
def test_sparse_fp64_narrow_overlapping_rows(pkg, oracle, grad, kernel64):
    rng = np.random.default_rng(23 + len(grad))
    n, d = 900, 12
    rp, col, val, y = synth_csr(rng, n, d, 1, 9, grad)
    offs = [0, 300, 600, 900]
    check64(pkg, oracle, rp, col, val, y, d, offs, grad, "simple", 0.2, 0.0, 3, kernel=kernel64)
    check64(pkg, oracle, rp, col, val, y, d, offs, grad, "squared_l2", 0.2, 0.1, 2, kernel=kernel64)


def test_sparse_fp64_f32_rows_and_sampled_batches(pkg, oracle, kernel64):
    rng = np.random.default_rng(24)
    n, d = 2000, 500
    rp, col, val, y = synth_csr(rng, n, d, 0, 30, "hinge")
    check64(pkg, oracle, rp, col, val, y, d, [0, 1000, 2000], "hinge", "squared_l2", 0.5, 0.01, 2,
            dtype=np.float32, kernel=kernel64)
    for frac in (0.15, 0.6):
        check64(pkg, oracle, rp, col, val, y, d, [0, 1000, 2000], "hinge", "simple", 0.5, 0.0, 3, frac=frac,
                kernel=kernel64)


def test_sparse_fp64_alpha_out_of_range_takes_chain_general(pkg, oracle):
    """SquaredL2 with 1 - s*lambda = 0 at the first sample (alpha = 0): the alpha-scaled form
    without renormalisation does not apply, chain_general (which renormalises) runs."""
    rng = np.random.default_rng(25)
    n, d = 600, 300
    rp, col, val, y = synth_csr(rng, n, d, 1, 20, "logistic")
    check64(pkg, oracle, rp, col, val, y, d, [0, 300, 600], "logistic", "squared_l2", 1.0, 1.0, 2, want=201)


@pytest.mark.parametrize("upd", ["simple", "squared_l2"])
def test_sparse_fp64_rows_wider_than_128(pkg, oracle, upd):
    """Rows of 100-300 entries: chain_sparse64's per-lane loop past two entries (gathers, dot and
    stores), both storage dtypes."""
    rng = np.random.default_rng(27)
    n, d = 400, 1000
    rp, col, val, y = synth_csr(rng, n, d, 100, 300, "logistic")
    for dtype in (np.float64, np.float32):
        check64(pkg, oracle, rp, col, val, y, d, [0, 200, 400], "logistic", upd, 0.5, 0.02, 2, dtype=dtype)


@pytest.mark.parametrize("grad", ["least_squares", "logistic", "hinge"])
def test_sparse_fp64_beyond_lds(pkg, oracle, grad):
    """d = 200,000: past the fp64 LDS kernel's ~61k features, so chain_sparse64 (weights as
    doubles in HBM) runs by default; SquaredL2 (alpha-scaled) and Simple, ragged and empty
    partitions, f32 and f64 rows."""
    rng = np.random.default_rng(31 + len(grad))
    n, d = 3000, 200_000
    rp, col, val, y = synth_csr(rng, n, d, 0, 120, grad)
    offs = [0, 1000, 1000, 1001, 2200, 3000]
    check64(pkg, oracle, rp, col, val, y, d, offs, grad, "squared_l2", 0.4, 0.01, 3, want=420)
    check64(pkg, oracle, rp, col, val, y, d, offs, grad, "simple", 0.4, 0.0, 2, dtype=np.float32, want=421)


# ------------------------------------------------------------------------------------------
# The per-sample break (tol > 0, PSGD.scala:262, :324-336) on chain_sparse_lds (variant 640 +
# ...): the chain wave tests isConverged from z, x.x, c and the ||w||^2 recurrence. fp64: exact
# per-chain counts and 1e-9; fp32: chain by chain against the fp64 oracle (a break may land a
# row off across the rounding). Step 1.0 with tols 0.01 / 0.03 / 0.1 gives chains that never
# break, break early and break late for every gradient (checked on the oracle).
# ------------------------------------------------------------------------------------------
def break_case(rng, grad, P=64):
    n = P * 45 + 29
    d = 3000
    rp, col, val, y = synth_csr(rng, n, d, 5, 40, grad)
    offs = [i * n // P for i in range(P)] + [n]
    return rp, col, val, y, d, offs


@pytest.mark.parametrize("grad", ["least_squares", "logistic", "hinge"])
@pytest.mark.parametrize("upd", ["simple", "squared_l2"])
@pytest.mark.parametrize("head", ["all", "third"])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_sparse_lds64_per_sample_break(pkg, oracle, monkeypatch, grad, upd, head, dtype):
    from test_gpu_parity import assert_close
    monkeypatch.delenv("PSGD_SPARSE_KERNEL", raising=False)
    monkeypatch.delenv("PSGD_SPARSE_SK", raising=False)
    rng = np.random.default_rng(len(grad) * 5 + len(upd))
    rp, col, val, y, d, offs = break_case(rng, grad)
    if head == "third":
        monkeypatch.setenv("PSGD_SPARSE_LDS_HEAD", str(d // 3))
    else:
        monkeypatch.delenv("PSGD_SPARSE_LDS_HEAD", raising=False)
    vstore = val.astype(dtype)
    parts = [pkg.CsrPartition(y[a:b], rp[a:b + 1] - rp[a], col[rp[a]:rp[b]], vstore[rp[a]:rp[b]], d)
             for a, b in zip(offs[:-1], offs[1:])]
    data = pkg.PartitionedData(parts)
    mat = oracle.Matrix(y, row_ptr=rp, col=col, val=vstore.astype(np.float64), d=d)
    breaks = 0
    for tol in (0.01, 0.03, 0.1):
        w, h, counts = pkg.runParallelizedSGD(data, getattr(pkg, G[grad])(), getattr(pkg, U[upd])(), 1.0, 3,
                                              0.05, 1.0, np.zeros(d), tol, return_chain_counts=True)
        assert pkg.optimization.get_context(0).last_kernel() == 660 + (1 if dtype == np.float32 else 0)
        wr, hr, cr = oracle.run(mat, offs, grad, upd, 1.0, 3, 0.05, np.zeros(d), tol=tol, n_threads=8)
        tag = f"fp64 {grad} {upd} head={head} tol={tol}"
        assert [list(c) for c in counts] == [list(c) for c in cr[: len(counts)]], tag
        assert_close(w, wr, what=tag + " weights")
        assert_close(h, hr, what=tag + " loss")
        breaks += sum(int(c < s) for it in cr for c, s in zip(it, np.diff(offs)))
    assert breaks > 0


@pytest.mark.parametrize("grad", ["least_squares", "logistic", "hinge"])
@pytest.mark.parametrize("upd", ["simple", "squared_l2"])
@pytest.mark.parametrize("head", ["all", "third"])
def test_sparse_lds_per_sample_break_fp32(pkg, oracle, monkeypatch, grad, upd, head):
    for k in ("PSGD_SPARSE_KERNEL", "PSGD_SPARSE_SK", "PSGD_SPARSE_LDS_HEAD"):
        monkeypatch.delenv(k, raising=False)
    rng = np.random.default_rng(len(grad) * 5 + len(upd))
    rp, col, val, y, d, offs = break_case(rng, grad)
    if head == "third":
        monkeypatch.setenv("PSGD_SPARSE_LDS_HEAD", str(d // 3))
    vstore = val.astype(np.float32)
    parts = [pkg.CsrPartition(y[a:b], rp[a:b + 1] - rp[a], col[rp[a]:rp[b]], vstore[rp[a]:rp[b]], d)
             for a, b in zip(offs[:-1], offs[1:])]
    data = pkg.PartitionedData(parts)
    mat = oracle.Matrix(y, row_ptr=rp, col=col, val=vstore.astype(np.float64), d=d)
    for tol in (0.01, 0.03, 0.1):
        w, h, counts = pkg.runParallelizedSGD(data, getattr(pkg, G[grad])(), getattr(pkg, U[upd])(), 1.0, 3,
                                              0.05, 1.0, np.zeros(d), tol, compute_dtype="f32",
                                              return_chain_counts=True)
        assert pkg.optimization.get_context(0).last_kernel() == 641
        wr, hr, cr, mg = oracle.run_with_margins(mat, offs, grad, upd, 1.0, 3, 0.05, np.zeros(d), tol=tol,
                                                 n_threads=8)
        tag = f"fp32 {grad} {upd} head={head} tol={tol}"
        if fp32_break_counts_agree(counts, cr, mg, tag) and len(h) == len(hr):
            scale = max(np.max(np.abs(wr)), 1e-30)
            assert np.max(np.abs(w - wr)) / scale <= FP32_REL, tag
            assert np.max(np.abs(h - hr) / np.maximum(np.abs(hr), 1e-30)) <= FP32_LOSS_REL, tag


@pytest.mark.parametrize("compute", ["f32", "f64"])
@pytest.mark.parametrize("upd", ["simple", "squared_l2"])
def test_sparse_break_beyond_lds(pkg, oracle, monkeypatch, compute, upd):
    """tol > 0 with d past the LDS kernel's range: the HBM-weight kernels chain_sparse (fp32,
    variant 440 + storage) and chain_sparse64 (fp64, 460 + storage) run the break from the same
    norm recurrence; exact in fp64. The per-sample fallback (PSGD_PER_SAMPLE=1: chain_general)
    carries ||w||^2 from sample to sample (O(nnz)) and gives the same counts."""
    from test_gpu_parity import assert_close
    for k in ("PSGD_SPARSE_KERNEL", "PSGD_SPARSE_SK", "PSGD_SPARSE_LDS_HEAD"):
        monkeypatch.delenv(k, raising=False)
    rng = np.random.default_rng(77)
    n, d = 300, 200_000
    rp, col, val, y = synth_csr(rng, n, d, 5, 40, "logistic")
    offs = [0, 150, 300]
    parts = [pkg.CsrPartition(y[a:b], rp[a:b + 1] - rp[a], col[rp[a]:rp[b]], val[rp[a]:rp[b]], d)
             for a, b in zip(offs[:-1], offs[1:])]
    reg = 0.05 if upd == "squared_l2" else 0.0
    w, h, counts = pkg.runParallelizedSGD(pkg.PartitionedData(parts), pkg.LogisticGradient(),
                                          getattr(pkg, U[upd])(), 1.0, 2, reg, 1.0, np.zeros(d), 0.1,
                                          compute_dtype=compute, return_chain_counts=True)
    assert pkg.optimization.get_context(0).last_kernel() == (440 if compute == "f32" else 460)
    wr, hr, cr = oracle.run(oracle.Matrix(y, row_ptr=rp, col=col, val=val, d=d), offs, "logistic", upd,
                            1.0, 2, reg, np.zeros(d), tol=0.1, n_threads=8)
    assert sum(int(c < s) for it in cr for c, s in zip(it, np.diff(offs))) > 0   # breaks happen
    if compute == "f64":
        assert [list(c) for c in counts] == [list(c) for c in cr[: len(counts)]]
        assert_close(w, wr, what="beyond-LDS break weights")
        assert_close(h, hr, what="beyond-LDS break loss")
        # the per-sample fallback (chain_general, O(nnz) norms) gives the same counts
        monkeypatch.setenv("PSGD_PER_SAMPLE", "1")
        w2, h2, c2 = pkg.runParallelizedSGD(pkg.PartitionedData(parts), pkg.LogisticGradient(),
                                            getattr(pkg, U[upd])(), 1.0, 2, reg, 1.0, np.zeros(d), 0.1,
                                            compute_dtype=compute, return_chain_counts=True)
        assert [list(c) for c in c2] == [list(c) for c in cr[: len(c2)]]
        assert_close(w2, wr, what="chain_general break weights")
