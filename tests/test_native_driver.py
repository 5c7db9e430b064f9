"""The native host driver (spark-parallelized-sgd_amd/psgd_run, C++ over the C ABI, no Python in
the loop): MLUtils.loadLibSVMFile partitions -> runParallelizedSGD (ParallelizedSGD.scala:188-306)
against the oracle on the same rows and partition boundaries. fp64: weights and loss history
within 1e-9 relative, per-iteration chain counts exactly equal (per-sample breaks included)."""
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, has_gpu
from test_gpu_parity import assert_close

BIN = os.path.join(ROOT, "spark-parallelized-sgd_amd", "psgd_run")


def need_bin():
    if not os.path.exists(BIN):
        pytest.skip("psgd_run not built (__graft_entry__.build())")


def test_usage_and_argument_errors():
    need_bin()
    assert subprocess.run([BIN], capture_output=True).returncode == 2
    r = subprocess.run([BIN, "x.libsvm", "--gradient", "softmax"], capture_output=True, text=True)
    assert r.returncode == 2 and "unknown gradient" in r.stderr


def write_libsvm(path, n, d, seed, max_nnz=8):
    rng = np.random.default_rng(seed)
    lines = []
    for _ in range(n):
        idx = np.sort(rng.choice(d, size=int(rng.integers(1, max_nnz)), replace=False)) + 1
        lines.append(f"{int(rng.integers(0, 2))} " + " ".join(f"{i}:{rng.uniform(-1, 1):.6f}" for i in idx))
    path.write_text("\n".join(lines) + "\n")


CASES = [
    # gradient, updater, step, iterations, reg, tol
    ("logistic", "simple", 1.0, 5, 0.0, 0.001),
    ("hinge", "squared_l2", 0.5, 3, 0.01, 0.0),
    ("least_squares", "l1", 0.1, 4, 0.05, 0.0),
    ("logistic", "adagrad", 0.5, 3, 0.0, 0.0),
]


@pytest.mark.gpu
@pytest.mark.parametrize("grad,upd,step,iters,reg,tol", CASES)
def test_native_driver_matches_oracle(pkg, oracle, tmp_path, grad, upd, step, iters, reg, tol):
    if not has_gpu():
        pytest.skip("no GPU")
    need_bin()
    f = tmp_path / "train.libsvm"
    write_libsvm(f, 900, 50, seed=len(grad) * 7 + iters)
    r = subprocess.run([BIN, str(f), "--partitions", "3", "--gradient", grad, "--updater", upd,
                        "--step", str(step), "--iterations", str(iters), "--reg", str(reg),
                        "--tol", str(tol)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    # the same partitions through the host package's loader (same native parser)
    data = pkg.loadLibSVMFile(str(f), -1, 3)
    P = len(data.partitions)
    assert out["partitions"] == P and out["d"] == data.partitions[0].d
    y = np.concatenate([p.labels for p in data.partitions])
    rp, col, val, offs = [0], [], [], [0]
    for p in data.partitions:
        col.append(p.col)
        val.append(p.val)
        rp += list(p.row_ptr[1:] + rp[-1])
        offs.append(offs[-1] + p.n_rows)
    d = data.partitions[0].d
    mat = oracle.Matrix(y, row_ptr=np.array(rp), col=np.concatenate(col), val=np.concatenate(val), d=d)
    wr, hr, cr = oracle.run(mat, offs, grad, upd, step, iters, reg, np.zeros(d), tol=tol)
    assert_close(out["weights"], wr, what="weights")
    assert_close(out["loss"], hr, what="loss")
    counts = np.array(out["chain_counts"], dtype=np.int64).reshape(-1, P)
    np.testing.assert_array_equal(counts, np.asarray(cr, dtype=np.int64).reshape(-1, P))


@pytest.mark.gpu
def test_native_driver_checkpoint_resume(tmp_path):
    """--checkpoint FILE: a run stopped after 2 iterations and resumed to 6 prints the weights and
    loss history of the uninterrupted 6-iteration run, bit for bit; a checkpoint of other
    parameters is refused (exit 2)."""
    if not has_gpu():
        pytest.skip("no GPU")
    need_bin()
    f = tmp_path / "train.libsvm"
    write_libsvm(f, 900, 50, seed=5)
    base = [BIN, str(f), "--partitions", "3", "--gradient", "logistic", "--updater", "squared_l2",
            "--step", "0.5", "--reg", "0.01", "--tol", "0"]
    run = lambda *extra: subprocess.run(base + list(extra), capture_output=True, text=True, timeout=120)
    full = run("--iterations", "6")
    assert full.returncode == 0, full.stderr
    ck = str(tmp_path / "loop.ck")
    first = run("--iterations", "2", "--checkpoint", ck)
    assert first.returncode == 0, first.stderr
    res = run("--iterations", "6", "--checkpoint", ck)
    assert res.returncode == 0 and "resuming at iteration 3" in res.stderr, res.stderr
    a = json.loads(full.stdout.strip().splitlines()[-1])
    b = json.loads(res.stdout.strip().splitlines()[-1])
    assert a["weights"] == b["weights"] and a["loss"] == b["loss"] and len(b["loss"]) == 6
    other = subprocess.run(base[:-1] + ["0.001", "--iterations", "6", "--checkpoint", ck],
                           capture_output=True, text=True, timeout=120)
    assert other.returncode == 2 and "other parameters" in other.stderr
