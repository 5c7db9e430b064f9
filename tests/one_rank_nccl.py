"""The engine's RCCL leg in a single-rank nccl process group (run by
tests/test_gpu_configs.py::test_rccl_exchange_single_rank as a child process).

usage: python tests/one_rank_nccl.py OUT.npz   (env: MASTER_ADDR, MASTER_PORT)

Initialises torch.distributed with the nccl backend (RCCL on ROCm) at world size 1 on cuda:0,
runs one epoch of HipEngine over a dense fp64 and a CSR fp32 dataset (the chain kernel and the
on-device fold: the single-process partial), then sends that partial through
ShardedEngine.exchange -- dist.all_gather_into_tensor into the engine's gather buffer and
psgd_fold_partials_device over the gathered ranks -- the call that replaces the cross-GPU
treeReduce (ParallelizedSGD.scala:271-276) when the bench runs N > 1 ranks. Writes both
results for a bit-for-bit comparison."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def main():
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    import __graft_entry__ as g
    pkg = g.load_package()
    out = sys.argv[1]
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl", dist.get_backend()
        rng = np.random.default_rng(88)
        res = {}
        # dense fp64 rows (chain_block64), CSR fp32 rows (chain_sparse_lds)
        n, d, P = 4000, 300, 6
        X = rng.standard_normal((n, d))
        y = (rng.uniform(size=n) > 0.5).astype(np.float64)
        dense = pkg.PartitionedData.parallelize(y, X, P)
        rp = np.arange(n + 1, dtype=np.int64) * 20
        col = np.sort(rng.choice(5000, size=(n, 20)), axis=1)
        col = (col + np.arange(20)[None, :]).astype(np.int32).reshape(-1)   # strictly increasing
        val = rng.standard_normal(n * 20).astype(np.float32)
        csr = pkg.PartitionedData([pkg.CsrPartition(y[a:b], rp[a:b + 1] - rp[a], col[rp[a]:rp[b]],
                                                    val[rp[a]:rp[b]], 5020)
                                   for a, b in zip([i * n // P for i in range(P)],
                                                   [(i + 1) * n // P for i in range(P)])])
        for name, data, dd, compute in (("dense", dense, d, "f64"), ("csr", csr, 5020, "f32")):
            eng = pkg.HipEngine(data, 0, 1, device=0)
            prm = pkg.make_params(pkg.LogisticGradient(), pkg.SquaredL2SGDUpdater(), 0.5, 0.01, 1.0, 0.0,
                                  compute)
            w = eng.weights(0.01 * rng.standard_normal(dd))
            # everything on the engine's stream (its kernels and copies run there)
            with torch.cuda.stream(eng.stream):
                partial, _ = eng.epoch(prm, w)            # world 1: the single-process result
                single = partial.clone()
                folded = eng.exchange(single.clone())    # RCCL all-gather + the rank-order fold
                got = folded.cpu().numpy()
                res[name + "_single"] = single.cpu().numpy()
            res[name + "_rccl"] = got
            # the same epoch read on the default stream, with no stream block (HipEngine.epoch
            # makes the caller's stream wait for the engine's): the partial as it ends the epoch
            for b in eng._partials:   # (the result buffers alternate by epoch)
                b.fill_(-7.0)
            torch.cuda.synchronize()
            partial, _ = eng.epoch(prm, w)
            res[name + "_default"] = partial.cpu().numpy()
        np.savez(out, **res)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
