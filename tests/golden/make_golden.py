"""Generate the golden fixtures in tests/golden/ from the CPU restatement (oracle/).

Every case is computed twice -- by the C oracle and by the independent pure-Python restatement
(oracle/psgd_ref.py) -- and only written if both agree bit for bit. Inputs are stored with the
expected outputs (or regenerated deterministically from the suite's generator, whose first
values are stored as a check).

Run: python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402
import psgd_ref as R  # noqa: E402

GRAD = {"logistic": 0, "least_squares": 1, "hinge": 2}
UPD = {"simple": 0, "squared_l2": 1, "l1": 2, "adagrad": 3, "adam": 4}


def suite_data(n, bias_first=False):
    x, y = O.generate_gd_input(2.0, -1.5, n, 42)
    X = np.stack([np.ones(n), x], 1) if bias_first else np.stack([x, np.ones(n)], 1)
    return X, y


def py_partitions_dense(X, y, offs):
    return [([list(map(float, X[r])) for r in range(a, b)], [float(v) for v in y[a:b]])
            for a, b in zip(offs[:-1], offs[1:])]


def py_partitions_csr(rp, col, val, y, offs):
    parts = []
    for a, b in zip(offs[:-1], offs[1:]):
        rows = [([int(c) for c in col[rp[r]:rp[r + 1]]], [float(v) for v in val[rp[r]:rp[r + 1]]])
                for r in range(a, b)]
        parts.append((rows, [float(v) for v in y[a:b]]))
    return parts


def run_both(case, mat, py_parts, offs):
    frac = case.get("fraction", 1.0)
    nc = case.get("num_classes", 2)
    kw = dict(tol=case["tol"], fraction=frac, num_classes=nc)
    w, h, c = O.run(mat, offs, case["gradient"], case["updater"], case["step"], case["iters"],
                    case["reg"], np.array(case["w0"]), **kw)
    wp, hp, cp = R.run(py_parts, GRAD[case["gradient"]], UPD[case["updater"]], case["step"],
                       case["iters"], case["reg"], list(case["w0"]), tol=case["tol"], fraction=frac,
                       num_classes=nc)
    same = lambda a, b: len(a) == len(b) and all(x == y or (x != x and y != y) for x, y in zip(a, b))
    assert same(list(map(float, w)), wp), (case["name"], "weights differ between C and Python")
    assert same(list(map(float, h)), hp), (case["name"], "loss history differs")
    assert [list(map(int, r)) for r in c[:len(cp)]] == cp, (case["name"], "counts differ")
    case["expected"] = {"weights": [float(v) for v in w], "loss_history": [float(v) for v in h],
                        "chain_counts": [list(map(int, r)) for r in c[:len(h) if len(h) else 0]]}
    case["expected"]["chain_counts"] = cp
    return case


def main():
    cases = []
    # --- the reference suite's three tests (ParallelizedSGDSuite.scala) ---
    X, y = suite_data(10000)
    x0 = [float(v) for v in X[:3, 0]]
    offs = [0, 5000, 10000]
    for name, tol in (("suite_loss_decreasing", 0.001), ("suite_loss_decreasing_tol0", 0.0),
                      ("suite_convergence_tol", 0.5)):
        c = dict(name=name, source="suite", n=10000, bias_first=False, offsets=offs,
                 gradient="logistic", updater="simple", step=1.0, iters=10, reg=0.0, tol=tol,
                 w0=[-1.0, 1.0], x_head=x0)
        cases.append(run_both(c, O.Matrix(y, X), py_partitions_dense(X, y, offs), offs))
    X2, y2 = suite_data(2, bias_first=True)
    for lam in (0.0, 1.0):
        c = dict(name=f"suite_first_iteration_l2_reg{int(lam)}", source="suite", n=2, bias_first=True,
                 offsets=[0, 1, 2], gradient="logistic", updater="squared_l2", step=1.0, iters=1,
                 reg=lam, tol=0.001, w0=[1.0, 0.5], x_head=[float(v) for v in X2[:2, 1]])
        cases.append(run_both(c, O.Matrix(y2, X2), py_partitions_dense(X2, y2, [0, 1, 2]), [0, 1, 2]))

    # --- random dense cases: every gradient x updater, tol 0 and > 0 ---
    rng = np.random.default_rng(2024)
    n, d = 240, 10
    for gi, g in enumerate(GRAD):
        for u in UPD:
            for tol in (0.0, 0.01):
                Xr = rng.standard_normal((n, d)).round(6)
                wt = rng.standard_normal(d)
                if g == "least_squares":
                    yr = (Xr @ wt + 0.1 * rng.standard_normal(n)).round(6)
                else:
                    yr = ((Xr @ wt + rng.logistic(size=n)) > 0).astype(float)
                offs = [0, 70, 160, 240]
                step = 0.05 if g == "least_squares" else 0.5
                if g == "least_squares" and u == "adam":
                    # keep r = (1-gamma) g^2 < 1: the reference's Adam takes sqrt(1 - r^iter),
                    # NaN otherwise (covered separately in tests/test_oracle.py)
                    Xr = (0.2 * Xr).round(6)
                    yr = (Xr @ wt + 0.1 * rng.standard_normal(n)).round(6)
                c = dict(name=f"dense_{g}_{u}_tol{tol}", source="random", n=n, d=d, offsets=offs,
                         gradient=g, updater=u, step=step, iters=4, reg=0.01, tol=tol,
                         w0=list(map(float, (0.1 * rng.standard_normal(d)).round(6))),
                         X=Xr.tolist(), y=yr.tolist())
                cases.append(run_both(c, O.Matrix(yr, Xr), py_partitions_dense(Xr, yr, offs), offs))

    # --- random CSR cases (hinge / logistic / least squares, simple / l2 / l1) ---
    for g in GRAD:
        for u in ("simple", "squared_l2", "l1"):
            for tol in (0.0, 0.01):
                n, d = 150, 64
                rp = [0]
                col, val = [], []
                for r in range(n):
                    k = int(rng.integers(0, 9))
                    idx = sorted(rng.choice(d, size=k, replace=False).tolist())
                    col += idx
                    val += list(map(float, rng.uniform(0, 1, size=k).round(6)))
                    rp.append(len(col))
                rp, col, val = np.array(rp), np.array(col, np.int32), np.array(val)
                yr = (rng.uniform(size=n) > 0.5).astype(float)
                offs = [0, 50, 50, 150]  # includes an empty partition
                c = dict(name=f"csr_{g}_{u}_tol{tol}", source="random", n=n, d=d, offsets=offs,
                         gradient=g, updater=u, step=0.5, iters=3, reg=0.01, tol=tol,
                         w0=[0.0] * d, row_ptr=rp.tolist(), col=col.tolist(), val=val.tolist(),
                         y=yr.tolist())
                mat = O.Matrix(yr, row_ptr=rp, col=col, val=val, d=d)
                cases.append(run_both(c, mat, py_partitions_csr(rp, col, val, yr, offs), offs))

    # --- random CSR cases with the stateful updaters (appended: the cases above keep their data) ---
    for g in GRAD:
        for u in ("adagrad", "adam"):
            for tol in (0.0, 0.01):
                n, d = 120, 48
                rp = [0]
                col, val = [], []
                for r in range(n):
                    k = int(rng.integers(0, 7))
                    idx = sorted(rng.choice(d, size=k, replace=False).tolist())
                    col += idx
                    val += list(map(float, rng.uniform(0, 1, size=k).round(6)))
                    rp.append(len(col))
                rp, col, val = np.array(rp), np.array(col, np.int32), np.array(val)
                if g == "least_squares":
                    # |g| < 1 keeps Adam's sqrt(1 - r^iter) real (see the dense Adam cases)
                    yr = (rng.uniform(size=n) * 0.5).round(6)
                    val = (0.3 * val).round(6)
                else:
                    yr = (rng.uniform(size=n) > 0.5).astype(float)
                offs = [0, 40, 40, 120]  # includes an empty partition
                c = dict(name=f"csr_{g}_{u}_tol{tol}", source="random", n=n, d=d, offsets=offs,
                         gradient=g, updater=u, step=0.5, iters=3, reg=0.01, tol=tol,
                         w0=[0.0] * d, row_ptr=rp.tolist(), col=col.tolist(), val=val.tolist(),
                         y=yr.tolist())
                mat = O.Matrix(yr, row_ptr=rp, col=col, val=val, d=d)
                cases.append(run_both(c, mat, py_partitions_csr(rp, col, val, yr, offs), offs))

    # --- miniBatchFraction < 1: RDD.sample(false, f, 42 + i) per iteration (PSGD.scala:242) ---
    for g, u, frac, tol in (("logistic", "simple", 0.3, 0.0), ("logistic", "squared_l2", 0.7, 0.0),
                            ("least_squares", "simple", 0.05, 0.0), ("hinge", "l1", 0.5, 0.01),
                            ("logistic", "adagrad", 0.2, 0.0), ("least_squares", "squared_l2", 0.9, 0.001),
                            ("hinge", "simple", 0.02, 0.0)):
        n, d = 400, 6
        Xr = rng.standard_normal((n, d)).round(6)
        wt = rng.standard_normal(d)
        if g == "least_squares":
            yr = (Xr @ wt + 0.1 * rng.standard_normal(n)).round(6)
        else:
            yr = ((Xr @ wt + rng.logistic(size=n)) > 0).astype(float)
        offs = [0, 250, 251, 251, 400]   # a one-row and an empty partition
        c = dict(name=f"sampled_{g}_{u}_f{frac}_tol{tol}", source="random", n=n, d=d, offsets=offs,
                 gradient=g, updater=u, step=0.05 if g == "least_squares" else 0.5, iters=6,
                 reg=0.01, tol=tol, fraction=frac,
                 w0=list(map(float, (0.1 * rng.standard_normal(d)).round(6))),
                 X=Xr.tolist(), y=yr.tolist())
        cases.append(run_both(c, O.Matrix(yr, Xr), py_partitions_dense(Xr, yr, offs), offs))
    for g, u, frac in (("hinge", "simple", 0.25), ("logistic", "adam", 0.6)):
        n, d = 200, 40
        rp, col, val = [0], [], []
        for r in range(n):
            k = int(rng.integers(0, 8))
            col += sorted(rng.choice(d, size=k, replace=False).tolist())
            val += list(map(float, rng.uniform(0, 1, size=k).round(6)))
            rp.append(len(col))
        rp, col, val = np.array(rp), np.array(col, np.int32), np.array(val)
        yr = (rng.uniform(size=n) > 0.5).astype(float)
        offs = [0, 90, 200]
        c = dict(name=f"sampled_csr_{g}_{u}_f{frac}", source="random", n=n, d=d, offsets=offs,
                 gradient=g, updater=u, step=0.5, iters=4, reg=0.01, tol=0.0, fraction=frac,
                 w0=[0.0] * d, row_ptr=rp.tolist(), col=col.tolist(), val=val.tolist(), y=yr.tolist())
        mat = O.Matrix(yr, row_ptr=rp, col=col, val=val, d=d)
        cases.append(run_both(c, mat, py_partitions_csr(rp, col, val, yr, offs), offs))

    # --- multinomial LogisticGradient(numClasses > 2) [ext MLlib 1.6.1]: weights (K-1)*d ---
    for K, u, tol, layout in ((3, "simple", 0.0, "dense"), (3, "squared_l2", 0.01, "dense"),
                              (5, "l1", 0.0, "dense"), (4, "adagrad", 0.0, "dense"),
                              (3, "adam", 0.01, "dense"), (6, "simple", 0.0, "csr"),
                              (3, "squared_l2", 0.0, "csr"), (4, "adagrad", 0.01, "csr"),
                              (5, "adam", 0.0, "csr"), (3, "l1", 0.01, "csr")):
        n, d = 180, 7 if layout == "dense" else 30
        W = rng.standard_normal((K, d))
        # labels 0..K-1, a few out of range (K) and a non-integer one: the reference accepts them
        if layout == "dense":
            Xr = rng.standard_normal((n, d)).round(6)
            Xr[rng.uniform(size=(n, d)) < 0.15] = 0.0   # zero values are skipped by foreachActive
            logits = Xr @ W.T
        else:
            rp, col, val = [0], [], []
            for r in range(n):
                k = int(rng.integers(0, 9))
                col += sorted(rng.choice(d, size=k, replace=False).tolist())
                val += list(map(float, rng.uniform(-1, 1, size=k).round(6)))
                rp.append(len(col))
            rp, col, val = np.array(rp), np.array(col, np.int32), np.array(val)
            dense = np.zeros((n, d))
            for r in range(n):
                dense[r, col[rp[r]:rp[r + 1]]] = val[rp[r]:rp[r + 1]]
            logits = dense @ W.T
        yr = np.argmax(logits + rng.gumbel(size=logits.shape), 1).astype(float)
        yr[:3] = [float(K), 1.5, -1.0]
        offs = [0, 60, 61, 180]
        w0 = list(map(float, (0.5 * rng.standard_normal((K - 1) * d)).round(6)))
        step = 0.3
        c = dict(name=f"multinomial_k{K}_{layout}_{u}_tol{tol}", source="random", n=n, d=d, offsets=offs,
                 gradient="logistic", num_classes=K, updater=u, step=step, iters=3, reg=0.01, tol=tol,
                 w0=w0, y=yr.tolist())
        if layout == "dense":
            c["X"] = Xr.tolist()
            cases.append(run_both(c, O.Matrix(yr, Xr), py_partitions_dense(Xr, yr, offs), offs))
        else:
            c.update(row_ptr=rp.tolist(), col=col.tolist(), val=val.tolist())
            mat = O.Matrix(yr, row_ptr=rp, col=col, val=val, d=d)
            cases.append(run_both(c, mat, py_partitions_csr(rp, col, val, yr, offs), offs))

    out = os.path.join(HERE, "golden_cases.json")
    with open(out, "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "oracle": "oracle/psgd_oracle.c",
                   "cases": cases}, f)
    print(f"wrote {len(cases)} cases to {out}")


if __name__ == "__main__":
    main()
