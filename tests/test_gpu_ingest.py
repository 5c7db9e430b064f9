"""Host -> HBM ingest (the .cache() analogue, ParallelizedSGDSuite.scala:88):
psgd_register_dense / psgd_register_csr through the pinned staging ring (pageable sources,
several 8 MiB chunks, padded rows), direct DMA from psgd_host_alloc'd memory, concurrent
registration from several threads (Spark local[N] task threads), CSR validation failing in a late
chunk, and the epoch's device-side wait for copies still in flight. Each registration is checked
bit for bit against the zero-copy device registration of the same rows (same kernel, same
inputs), and one against the oracle."""
import threading
import time

import numpy as np
import pytest

from conftest import has_gpu
from test_gpu_parity import assert_close

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not has_gpu():
        pytest.skip("no GPU")


def epoch(pkg, ctx, grad, d, step=0.5, compute=None):
    prm = pkg.make_params(grad, pkg.SimpleSGDUpdater(), step, 0.0, 1.0, 0.0)
    if compute is not None:
        prm.compute_dtype = compute
    return ctx.run_epoch(prm, np.zeros(d))


def same(a, b):
    for x, y in zip(a, b):
        assert np.array_equal(np.asarray(x), np.asarray(y)), (x, y)


@pytest.mark.parametrize("dtype,d", [(np.float32, 101), (np.float64, 100), (np.float32, 512)])
def test_dense_staged_pinned_device_agree(pkg, oracle, dtype, d):
    import torch
    rng = np.random.default_rng(11)
    P, n = 4, 60_000          # >= 3 staging chunks per partition at d = 101 f32 (416-byte rows)
    X = rng.standard_normal((n, d)).astype(dtype)
    y = (rng.standard_normal(n) > 0).astype(np.float64)
    offs = [i * n // P for i in range(P)] + [n]
    grad = pkg.LogisticGradient()
    res = {}
    # pageable (staged)
    ctx = pkg._native.Context(0)
    for p in range(P):
        ctx.register_dense(p, y[offs[p]:offs[p + 1]], X[offs[p]:offs[p + 1]])
    res["staged"] = epoch(pkg, ctx, grad, d)
    # pinned (direct DMA)
    ctx2 = pkg._native.Context(0)
    Xp = ctx2.host_array(X.shape, dtype)
    yp = ctx2.host_array(y.shape, np.float64)
    Xp[:] = X
    yp[:] = y
    for p in range(P):
        ctx2.register_dense(p, yp[offs[p]:offs[p + 1]], Xp[offs[p]:offs[p + 1]])
    res["pinned"] = epoch(pkg, ctx2, grad, d)
    # zero-copy device registration of the same rows (padded to 16-byte rows)
    es = np.dtype(dtype).itemsize
    ld = (d * es + 15) // 16 * 16 // es
    Xd = torch.zeros((n, ld), dtype=torch.float32 if dtype == np.float32 else torch.float64, device="cuda")
    Xd[:, :d] = torch.from_numpy(X).cuda()
    yd = torch.from_numpy(y).cuda()
    ctx3 = pkg._native.Context(0)
    dt = pkg._native.F32 if dtype == np.float32 else pkg._native.F64
    for p in range(P):
        a = offs[p]
        ctx3.register_dense_device(p, offs[p + 1] - a, d, ld, yd[a:].data_ptr(), Xd[a:].data_ptr(), dt)
    res["device"] = epoch(pkg, ctx3, grad, d)
    same(res["staged"], res["device"])
    same(res["pinned"], res["device"])
    if d == 100:
        wr, rvr, lr, cr = oracle.run_chains(oracle.Matrix(y, X.astype(np.float64)), offs, "logistic", "simple",
                                            0.5, 0.0, np.zeros(d))
        w, _, loss, cnt, counts = res["staged"]
        assert list(counts) == list(cr) and cnt == n
        acc_w, acc_c = wr[0].copy(), cr[0]
        for p in range(1, P):
            acc_w = (acc_w * acc_c + wr[p] * cr[p]) / (acc_c + cr[p])
            acc_c += cr[p]
        assert_close(w, acc_w, what="weights")
        assert_close(loss, lr.sum(), what="loss")
    del Xp, yp
    for c in (ctx, ctx2, ctx3):
        c.close()


def csr_random(rng, n, d, lo, hi):
    k = rng.integers(lo, hi + 1, size=n)
    rp = np.zeros(n + 1, np.int64)
    rp[1:] = np.cumsum(k)
    col = np.empty(rp[-1], np.int32)
    for i in range(n):
        col[rp[i]:rp[i + 1]] = np.sort(rng.choice(d, size=int(k[i]), replace=False))
    val = rng.uniform(0, 1, size=rp[-1]).astype(np.float32)
    y = (rng.standard_normal(n) > 0).astype(np.float64)
    return y, rp, col, val


def test_csr_staged_pinned_device_agree(pkg):
    import torch
    rng = np.random.default_rng(12)
    P, n, d = 4, 80_000, 5000     # ~2.4M entries per partition pair: several col/val chunks
    y, rp, col, val = csr_random(rng, n, d, 30, 90)
    offs = [i * n // P for i in range(P)] + [n]
    grad = pkg.HingeGradient()
    res = {}
    ctx = pkg._native.Context(0)
    for p in range(P):
        a, b = offs[p], offs[p + 1]
        # row_ptr keeps its absolute offsets (row_ptr[0] != 0): the library rebases
        ctx.register_csr(p, y[a:b], rp[a:b + 1], col, val, d)
    res["staged"] = epoch(pkg, ctx, grad, d, compute=pkg._native.F64)
    ctx2 = pkg._native.Context(0)
    colp = ctx2.host_array(col.shape, np.int32)
    valp = ctx2.host_array(val.shape, np.float32)
    colp[:] = col
    valp[:] = val
    for p in range(P):
        a, b = offs[p], offs[p + 1]
        ctx2.register_csr(p, y[a:b], rp[a:b + 1], colp, valp, d)
    res["pinned"] = epoch(pkg, ctx2, grad, d, compute=pkg._native.F64)
    ctx3 = pkg._native.Context(0)
    rpd, cold, vald, yd = (torch.from_numpy(rp).cuda(), torch.from_numpy(col).cuda(),
                           torch.from_numpy(val).cuda(), torch.from_numpy(y).cuda())
    for p in range(P):
        a, b = offs[p], offs[p + 1]
        ctx3.register_csr_device(p, b - a, d, yd[a:].data_ptr(), rpd[a:].data_ptr(), cold.data_ptr(),
                                 vald.data_ptr(), pkg._native.F32)
    res["device"] = epoch(pkg, ctx3, grad, d, compute=pkg._native.F64)
    same(res["staged"], res["device"])
    same(res["pinned"], res["device"])
    del colp, valp
    for c in (ctx, ctx2, ctx3):
        c.close()


def test_csr_validation_in_a_late_chunk(pkg):
    rng = np.random.default_rng(13)
    n, d = 60_000, 4000
    y, rp, col, val = csr_random(rng, n, d, 40, 80)
    ctx = pkg._native.Context(0)
    bad = col.copy()
    bad[-5] = d                        # out of range, several chunks in
    with pytest.raises(pkg.IllegalArgumentException, match="out of range"):
        ctx.register_csr(0, y, rp, bad, val, d)
    bad = col.copy()
    r = n - 3
    bad[rp[r] + 1] = bad[rp[r]]        # not strictly increasing inside row r
    with pytest.raises(pkg.IllegalArgumentException, match="strictly increasing"):
        ctx.register_csr(0, y, rp, bad, val, d)
    assert ctx.num_partitions() == (0, 0)
    # the context is still usable
    ctx.register_csr(0, y, rp, col, val, d)
    w, _, _, cnt, _ = epoch(pkg, ctx, pkg.HingeGradient(), d, compute=pkg._native.F64)
    assert cnt == n and np.all(np.isfinite(w))
    ctx.close()


def test_concurrent_registration(pkg):
    """Spark local[N]: N task threads register their partitions at once (the copies run without
    the context lock); the epoch equals the one over sequentially registered partitions."""
    rng = np.random.default_rng(14)
    P, n, d = 16, 64_000, 256
    X = rng.standard_normal((n, d)).astype(np.float32)
    y = (rng.standard_normal(n) > 0).astype(np.float64)
    offs = [i * n // P for i in range(P)] + [n]
    grad = pkg.LogisticGradient()
    seq = pkg._native.Context(0)
    for p in range(P):
        seq.register_dense(p, y[offs[p]:offs[p + 1]], X[offs[p]:offs[p + 1]])
    ref = epoch(pkg, seq, grad, d)
    seq.close()
    ctx = pkg._native.Context(0)
    errs = []

    def task(parts):
        try:
            for p in parts:
                ctx.register_dense(p, y[offs[p]:offs[p + 1]], X[offs[p]:offs[p + 1]])
        except Exception as e:   # noqa: BLE001
            errs.append(e)

    ts = [threading.Thread(target=task, args=(list(range(k, P, 4)),)) for k in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs
    assert ctx.num_partitions() == (P, n)
    same(epoch(pkg, ctx, grad, d), ref)
    ctx.close()


def test_ingest_rate(pkg):
    """Registration throughput of a 1 GiB dense partition set, pageable (staged) and pinned
    (direct): printed for DESIGN.md, asserted only to be sane and to agree."""
    rng = np.random.default_rng(15)
    P, d = 8, 512
    n = (1 << 30) // (d * 4)
    X = rng.standard_normal((n, d), dtype=np.float32)
    y = np.zeros(n)
    offs = [i * n // P for i in range(P)] + [n]
    ctx = pkg._native.Context(0)
    # first registration warms the staging ring and the allocator
    ctx.register_dense(0, y[:offs[1]], X[:offs[1]])
    ctx.register_wait()
    t0 = time.perf_counter()
    for p in range(P):
        ctx.register_dense(p, y[offs[p]:offs[p + 1]], X[offs[p]:offs[p + 1]])
    ctx.register_wait()
    t_staged = time.perf_counter() - t0
    Xp = ctx.host_array(X.shape, np.float32)
    Xp[:] = X
    yp = ctx.host_array(y.shape, np.float64)
    yp[:] = y
    t0 = time.perf_counter()
    for p in range(P):
        ctx.register_dense(p, yp[offs[p]:offs[p + 1]], Xp[offs[p]:offs[p + 1]])
    ctx.register_wait()
    t_pinned = time.perf_counter() - t0
    gb = (X.nbytes + y.nbytes) / 1e9
    print(f"\ningest: {gb:.2f} GB dense f32 rows: pageable (staged) {gb / t_staged:.1f} GB/s, "
          f"pinned (direct) {gb / t_pinned:.1f} GB/s")
    assert gb / t_staged > 0.5 and gb / t_pinned > 0.5
    w, _, _, cnt, _ = epoch(pkg, ctx, pkg.LeastSquaresGradient(), d, step=1e-4)
    assert cnt == n and np.all(np.isfinite(w))
    del Xp, yp
    ctx.close()
