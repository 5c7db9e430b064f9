"""c4's per-process mode: is it the rows' placement or the chains' weight
vectors'? One process, the c4 shard generated twice (two row allocations) and run through four
device contexts (four allocations of the chains' fp32 vectors, psgd_capi.cpp wf32), every
(rows, context) pair timed over a few epochs with the chain kernel's HIP events.

usage: python tools/c4_placement.py [--rows 20000000] [--epochs 6] [--contexts 4] [--compute f32|f64]
       [--shards 2]   (PSGD_REROLL=1: no placement re-roll; PSGD_REROLL_LOG=1 prints the probes)
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=20_000_000)
    ap.add_argument("--epochs", type=int, default=6)
    ap.add_argument("--contexts", type=int, default=4)
    ap.add_argument("--compute", default="f32", choices=["f32", "f64"])
    ap.add_argument("--shards", type=int, default=2)
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    import __graft_entry__ as ge
    pkg = ge.load_package()
    N = pkg._native
    dev = torch.device("cuda", 0)
    grad, _, d, P, step, sdt = bench.WORKLOADS["c4"][:6]
    nnz = bench.CSR_NNZ["c4"]
    shards = [bench.make_csr_shard(torch, dev, a.rows, d, P, grad, sdt, 1000 + s, nnz) for s in range(a.shards)]
    torch.cuda.synchronize()
    params = pkg.make_params(pkg.HingeGradient(), pkg.SimpleSGDUpdater(), step, 0.0, 1.0, 0.0, a.compute)
    w = torch.zeros(d, dtype=torch.float64, device=dev)
    partial = torch.empty(d + 3, dtype=torch.float64, device=dev)
    ctxs = [N.Context(0) for _ in range(a.contexts)]
    out = {}
    for rnd in range(2):
        for si, (rp, col, val, y, offs) in enumerate(shards):
            for ci, ctx in enumerate(ctxs):
                ctx.clear()
                for p in range(P):
                    lo, hi = offs[p], offs[p + 1]
                    ctx.register_csr_device(p, hi - lo, d, y[lo:].data_ptr(), rp[lo:].data_ptr(), col.data_ptr(),
                                            val.data_ptr(), N.F32)
                ms = []
                for e in range(a.epochs):
                    params.iteration = e + 1
                    ctx.run_epoch_device(params, w.data_ptr(), partial.data_ptr())
                    ms.append(ctx.last_chain_ms())
                key = f"round{rnd} rows{si} ctx{ci}"
                out[key] = {"variant": ctx.last_kernel(), "ms": [round(x, 3) for x in ms],
                            "best": round(min(ms[1:]), 3)}
                print(key, out[key], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
