"""The CSR chains' weight vectors mapped through the virtual-memory API (DevBuf::vmm_map,
psgd_capi.cpp): every chunk is unmapped and released when the buffer regrows and when the context
is destroyed, and the device memory comes back (the release used to unmap the whole
range in one call and ignore every return code). PSGD_VMM_MIN_MB / PSGD_VMM_CHUNK_MB are read at
every allocation, so small vectors take the several-chunk path here."""
import os

import numpy as np
import pytest

from conftest import has_gpu

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not has_gpu():
        pytest.skip("no GPU")


def csr_rows(rng, n, d, nnz=16):
    # strictly increasing per row: one draw per bucket of d / nnz columns
    width = d // nnz
    col = (np.arange(nnz) * width)[None, :] + rng.integers(0, width, (n, nnz))
    val = rng.uniform(size=(n, nnz))
    y = (rng.uniform(size=n) > 0.5).astype(np.float64)
    rp = np.arange(n + 1, dtype=np.int64) * nnz
    return y, rp, col.reshape(-1).astype(np.int32), val.reshape(-1)


def register(ctx, rng, parts, d, per=64):
    for p in parts:
        y, rp, col, val = csr_rows(rng, per, d)
        ctx.register_csr(p, y, rp, col, val, d)


def cycle(pkg, d=200_000, seed=5, probe=None):
    """8 chains (fp32) -> 16 chains (fp32, regrow) -> 16 chains (fp64 vectors, regrow) -> destroy;
    probe(stage) is called after each stage."""
    N = pkg._native
    rng = np.random.default_rng(seed)
    ctx = N.Context(0)
    register(ctx, rng, range(8), d)
    grad, upd = pkg.HingeGradient(), pkg.SimpleSGDUpdater()
    w = np.zeros(d)
    f32 = pkg.optimization.make_params(grad, upd, 0.5, 0.0, 1.0, 0.0, "f32")
    f64 = pkg.optimization.make_params(grad, upd, 0.5, 0.0, 1.0, 0.0, "f64")
    ctx.run_epoch(f32, w)
    probe and probe(1)
    register(ctx, rng, range(8, 16), d)
    ctx.run_epoch(f32, w)
    probe and probe(2)
    ctx.run_epoch(f64, w)
    probe and probe(3)
    ctx.close()
    probe and probe(4)


def test_vmm_chunks_released_on_regrow_and_destroy(pkg, monkeypatch):
    import torch
    N = pkg._native
    # the same sequence once through hipMalloc first: the kernels' code objects and scratch are
    # loaded, so the free-memory comparison below sees only the mapped chunks
    monkeypatch.setenv("PSGD_VMM", "0")
    cycle(pkg)
    monkeypatch.setenv("PSGD_VMM", "1")
    monkeypatch.setenv("PSGD_VMM_MIN_MB", "1")
    monkeypatch.setenv("PSGD_VMM_CHUNK_MB", "2")
    torch.cuda.synchronize()
    free0, _ = torch.cuda.mem_get_info()
    s = {0: N.vmm_stats()}
    free = {}

    def probe(stage):
        torch.cuda.synchronize()
        s[stage] = N.vmm_stats()
        free[stage] = torch.cuda.mem_get_info()[0]
    cycle(pkg, probe=probe)
    s0, s1, s2, s3, s4 = (s[i] for i in range(5))
    if s1["mapped"] == s0["mapped"]:
        pytest.skip("the device's VMM granularity does not divide 2 MiB chunks: hipMalloc path taken")
    d = 200_000
    assert s1["live_bytes"] - s0["live_bytes"] >= 8 * d * 4          # 8 chains' fp32 vectors
    # the regrow released the first set chunk by chunk and mapped a larger one
    assert s2["unmapped"] - s1["unmapped"] == s1["mapped"] - s0["mapped"]
    assert s2["mapped"] - s1["mapped"] > s1["mapped"] - s0["mapped"]
    mine = s3["live_bytes"] - s0["live_bytes"]   # (the counters are process-wide: other contexts' too)
    assert s3["mapped"] > s2["mapped"] and mine >= 16 * d * 8
    # while mapped, the chunks are visible in the device's free memory ...
    assert free[3] <= free0 - mine + (8 << 20), (free0, free[3], s0, s3)
    # ... and after psgd_ctx_destroy every chunk is unmapped and released, none failed
    assert s4["failures"] == s0["failures"], s4
    assert s4["mapped"] - s0["mapped"] == s4["unmapped"] - s0["unmapped"], s4
    assert s4["live_bytes"] == s0["live_bytes"], s4
    assert free[4] >= free0 - (8 << 20), (free0, free[4])
    print(f"\nVMM: {s4['mapped'] - s0['mapped']} chunks mapped and unmapped over 3 sizes; free memory "
          f"{free0 >> 20} -> {free[3] >> 20} (mapped) -> {free[4] >> 20} MiB")
