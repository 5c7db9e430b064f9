"""The N > 1 path on CPU: world_size 2 over gloo.

The product's multi-process logic (partition sharding, the all-gather of per-rank partials,
the rank-order fold, the empty-rank identity, the driver loop) is exercised with the chains
computed by the CPU oracle instead of the GPU (OracleEngine below implements ShardedEngine's
local hooks; everything else is the product's code). The result must equal, bit for bit, the
oracle's single-process run with the same two-level combine tree."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def make_oracle_engine(pkg, O):
    class OracleEngine(pkg.ShardedEngine):
        def __init__(self, data, rank, world):
            super().__init__(data, rank, world)
            self.data = data

        def weights(self, w):
            return torch.tensor(np.asarray(w, dtype=np.float64))

        def initial_regval(self, params, w):
            prm = O.params(params.gradient, params.updater, params.step_size, params.reg_param,
                           params.convergence_tol)
            import ctypes as C
            w = np.ascontiguousarray(w, dtype=np.float64)
            return O.lib().or_initial_regval(len(w), w.ctypes.data_as(C.POINTER(C.c_double)), C.byref(prm))

        def _mat(self):
            parts = self.data.partitions[self.lo:self.hi]
            X = np.concatenate([p.x for p in parts])
            y = np.concatenate([p.labels for p in parts])
            offs = np.cumsum([0] + [p.n_rows for p in parts])
            return O.Matrix(y, X), offs

        def local_partial(self, params, w, with_counts):
            mat, offs = self._mat()
            cw, rv, loss, cnt = O.run_chains(mat, offs, params.gradient, params.updater,
                                             params.step_size, params.reg_param, w.numpy(),
                                             tol=params.convergence_tol)
            acc_w, acc_rv, acc_l, acc_c = cw[0].copy(), rv[0], loss[0], int(cnt[0])
            for p in range(1, len(cnt)):  # the reference combiner, partition order
                c1, c2 = float(acc_c), float(cnt[p])
                acc_w = (acc_w * c1 + cw[p] * c2) / float(acc_c + cnt[p])
                acc_rv = (acc_rv * c1 + rv[p] * c2) / float(acc_c + cnt[p])
                acc_l = acc_l + loss[p]
                acc_c += int(cnt[p])
            return torch.tensor(np.concatenate([acc_w, [acc_rv, acc_l, float(acc_c)]])), cnt

        def empty_partial(self, w):
            return torch.cat([w, torch.zeros(3, dtype=torch.float64)])

        def gather_buffer(self):
            return torch.empty(self.world * (self.d + 3), dtype=torch.float64)

        def fold_partials(self, g):
            g = g.view(self.world, self.d + 3).numpy()
            acc = g[0].copy()
            for r in range(1, self.world):
                c1, c2 = acc[self.d + 2], g[r][self.d + 2]
                acc[: self.d] = (acc[: self.d] * c1 + g[r][: self.d] * c2) / (c1 + c2)
                acc[self.d] = (acc[self.d] * c1 + g[r][self.d] * c2) / (c1 + c2)
                acc[self.d + 1] = acc[self.d + 1] + g[r][self.d + 1]
                acc[self.d + 2] = c1 + c2
            return torch.tensor(acc)

        def scalars(self, f):
            return float(f[self.d]), float(f[self.d + 1]), int(f[self.d + 2])

        def adopt(self, f):
            return f[: self.d].clone()

        def convergence_terms(self, prev, cur):
            p, c = prev.numpy(), cur.numpy()
            dsq = 0.0
            nsq = 0.0
            for a, b in zip(p, c):
                dsq += (a - b) * (a - b)
                nsq += b * b
            return dsq, nsq

        def to_host(self, w):
            return w.numpy().copy()

    return OracleEngine


def _worker(rank, world, port, P, result_path):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import __graft_entry__ as g
    import oracle as O
    pkg = g.load_package()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(12)
        n, d = 500, 6
        X = rng.standard_normal((n, d))
        y = (rng.uniform(size=n) > 0.4).astype(float)
        data = pkg.PartitionedData.parallelize(y, X, P)
        eng = make_oracle_engine(pkg, O)(data, rank, world)
        w, h = pkg.runParallelizedSGD(data, pkg.LogisticGradient(), pkg.SquaredL2SGDUpdater(), 0.5, 4,
                                      0.01, 1.0, np.zeros(d), 0.001, engine=eng)
        if rank == 0:
            np.savez(result_path, w=w, h=h)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("P", [5, 1])
def test_two_ranks_match_single_process_oracle(tmp_path, oracle, pkg, P):
    world = 2
    out = str(tmp_path / "res.npz")
    mp.start_processes(_worker, args=(world, _free_port(), P, out), nprocs=world, start_method="spawn")
    res = np.load(out)
    rng = np.random.default_rng(12)
    n, d = 500, 6
    X = rng.standard_normal((n, d))
    y = (rng.uniform(size=n) > 0.4).astype(float)
    offs = [i * n // P for i in range(P)] + [n]
    bounds = [pkg.shard_range(P, r, world) for r in range(world)]
    groups = [bounds[0][0]] + [b[1] for b in bounds]
    groups = [g for i, g in enumerate(groups) if i == 0 or g != groups[i - 1]] if P > 1 else [0, 1]
    w, h, _ = oracle.run(oracle.Matrix(y, X), offs, "logistic", "squared_l2", 0.5, 4, 0.01, np.zeros(d),
                         tol=0.001, groups=groups)
    if P == 1:
        # rank 1 owns no partition: its identity partial (w_in, 0, 0, 0) folds away exactly
        # except for the rounding of (w*c + w_in*0) / c
        np.testing.assert_allclose(res["w"], w, rtol=1e-14)
        np.testing.assert_allclose(res["h"], h, rtol=1e-14)
    else:
        assert np.array_equal(res["w"], w) and np.array_equal(res["h"], h)


def _ckpt_worker(rank, world, port, ck, stop, result_path, w0_shift=0.0):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import __graft_entry__ as g
    import oracle as O
    pkg = g.load_package()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(21)
        n, d = 400, 5
        X = rng.standard_normal((n, d))
        y = (rng.uniform(size=n) > 0.5).astype(float)
        data = pkg.PartitionedData.parallelize(y, X, 4)
        eng = make_oracle_engine(pkg, O)(data, rank, world)
        if isinstance(ck, (list, tuple)):   # per-rank paths (a node-local checkpoint directory)
            ck = ck[rank]
        w0 = np.zeros(d) + (w0_shift if rank == 1 else 0.0)
        try:
            w, h = pkg.runParallelizedSGD(data, pkg.LogisticGradient(), pkg.SquaredL2SGDUpdater(), 0.5, stop,
                                          0.01, 1.0, w0, 0.0, engine=eng, checkpoint=ck)
        except pkg.IllegalArgumentException as e:
            if result_path:
                np.savez(f"{result_path}.rank{rank}.err", msg=str(e))
            return
        dist.barrier()   # rank 0's checkpoint is on disk before any rank resumes from it
        if rank == 0 and result_path:
            np.savez(result_path, w=w, h=h)
    finally:
        dist.destroy_process_group()


def test_two_ranks_checkpoint_resume(tmp_path):
    """Checkpoint / resume with world size 2: rank 0 writes, every rank resumes from the file; the
    resumed run equals the uninterrupted one bit for bit."""
    world = 2
    full, res = str(tmp_path / "full.npz"), str(tmp_path / "res.npz")
    mp.start_processes(_ckpt_worker, args=(world, _free_port(), str(tmp_path / "a.npz"), 5, full),
                       nprocs=world, start_method="spawn")
    ck = str(tmp_path / "b.npz")
    mp.start_processes(_ckpt_worker, args=(world, _free_port(), ck, 2, ""), nprocs=world, start_method="spawn")
    mp.start_processes(_ckpt_worker, args=(world, _free_port(), ck, 5, res), nprocs=world, start_method="spawn")
    a, b = np.load(full), np.load(res)
    assert len(a["h"]) == 5 and np.array_equal(a["w"], b["w"]) and np.array_equal(a["h"], b["h"])


def test_two_ranks_checkpoint_rank0_broadcast(tmp_path):
    """Resume reads the checkpoint on rank 0 only and broadcasts it: rank 1's path
    holds no file (a node-local directory) and the resumed run still equals the uninterrupted
    one; a rank whose parameters differ from rank 0's makes both ranks raise."""
    world = 2
    full, res = str(tmp_path / "full.npz"), str(tmp_path / "res.npz")
    mp.start_processes(_ckpt_worker, args=(world, _free_port(), str(tmp_path / "a.npz"), 5, full),
                       nprocs=world, start_method="spawn")
    paths = [str(tmp_path / "r0.npz"), str(tmp_path / "elsewhere" / "r1.npz")]
    mp.start_processes(_ckpt_worker, args=(world, _free_port(), paths, 2, ""), nprocs=world, start_method="spawn")
    assert not os.path.exists(paths[1])
    mp.start_processes(_ckpt_worker, args=(world, _free_port(), paths, 5, res), nprocs=world, start_method="spawn")
    a, b = np.load(full), np.load(res)
    assert np.array_equal(a["w"], b["w"]) and np.array_equal(a["h"], b["h"])
    bad = str(tmp_path / "bad.npz")
    mp.start_processes(_ckpt_worker, args=(world, _free_port(), paths, 5, bad, 0.25), nprocs=world,
                       start_method="spawn")
    for r in range(world):
        msg = str(np.load(f"{bad}.rank{r}.err.npz")["msg"])
        assert "other parameters or data than rank 0" in msg, msg


@pytest.mark.timeout(180)
@pytest.mark.parametrize("kind", ["truncated", "old_format"])
def test_two_ranks_unreadable_checkpoint_raises_on_every_rank(tmp_path, kind):
    """an unreadable checkpoint on rank 0 (a truncated zip, an .npz without the
    version key) is forwarded through the broadcast, so both ranks raise the same error instead
    of rank 1 waiting in the broadcast for the process-group timeout."""
    world = 2
    ck = tmp_path / "ck.npz"
    if kind == "truncated":
        np.savez(ck, weights=np.zeros(5), i=np.int64(2))
        ck.write_bytes(ck.read_bytes()[:40])
    else:
        np.savez(ck, weights=np.zeros(5), i=np.int64(2))   # no version / fingerprint keys
    res = str(tmp_path / "res.npz")
    mp.start_processes(_ckpt_worker, args=(world, _free_port(), str(ck), 3, res), nprocs=world,
                       start_method="spawn")
    for r in range(world):
        msg = str(np.load(f"{res}.rank{r}.err.npz")["msg"])
        assert "unreadable" in msg and "ck.npz" in msg, msg
