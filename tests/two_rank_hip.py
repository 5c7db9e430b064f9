"""Two ranks of the real HipEngine over gloo on one GPU (run by
tests/test_gpu_configs.py::test_hip_engine_two_ranks as a child process).

usage: python tests/two_rank_hip.py OUT.npz   (env: MASTER_ADDR, MASTER_PORT, PSGD_TEST_P)

Starts two fresh worker processes (torch.multiprocessing spawn); each initialises gloo, builds
the same PartitionedData, and calls runParallelizedSGD with no engine argument, so the product
picks HipEngine(rank, world=2) on cuda:0 -- its partition block, the on-device fold, the
all-gather of the (d+3)-double partials and psgd_fold_partials_device in rank order. Rank 0
writes the result and both ranks' chain counts."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def make_data(n=3000, d=64):
    rng = np.random.default_rng(77)
    X = rng.standard_normal((n, d))
    w = rng.standard_normal(d) / np.sqrt(d)
    y = ((X @ w + rng.logistic(size=n)) > 0).astype(np.float64)
    return X, y


def worker(rank, world, P, out):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    import __graft_entry__ as g
    pkg = g.load_package()
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        X, y = make_data()
        data = pkg.PartitionedData.parallelize(y, X, P)
        w, h, counts = pkg.runParallelizedSGD(data, pkg.LogisticGradient(), pkg.SquaredL2SGDUpdater(), 0.5, 4,
                                              0.01, 1.0, np.zeros(X.shape[1]), 0.001, return_chain_counts=True)
        eng_counts = np.array([c if c is not None else [] for c in counts], dtype=np.int64)
        # tol = 0, full batches: the driver's pipelined loop (the cross-rank fold writes the host
        # mirror of the scalars)
        wp, hp = pkg.runParallelizedSGD(data, pkg.LogisticGradient(), pkg.SquaredL2SGDUpdater(), 0.5, 5,
                                        0.01, 1.0, np.zeros(X.shape[1]), 0.0)
        if rank == 1:
            np.save(out + ".c1.npy", eng_counts)
        dist.barrier()
        if rank == 0:
            c1 = np.load(out + ".c1.npy")
            np.savez(out, w=w, h=h, c0=eng_counts, c1=c1, X=X, y=y, n=X.shape[0], d=X.shape[1], wp=wp, hp=hp)
    finally:
        dist.destroy_process_group()


def main():
    import torch.multiprocessing as mp
    out = sys.argv[1]
    P = int(os.environ.get("PSGD_TEST_P", "5"))
    mp.start_processes(worker, args=(2, P, out), nprocs=2, start_method="spawn")


if __name__ == "__main__":
    main()
