"""CPU model of chain_sparse_gram's algorithm (tools/experimental/psgd_sparse_gram.hip at commit 3c55d48, since removed from the tree: a measured
negative result kept out of libpsgd.so), checked against the
sequential chain of ParallelizedSGD.scala:243-270 in f64.

The kernel splits a CSR chain into batches of 8 rows and takes each row's dot against a weight
snapshot that lags by up to 15 rows (the updates of the two latest batches are missing), then
adds the missing part from the sparse Gram terms of the row with those rows:

    z_t = x_t . w_snap + sum_{r in window(t)} c_r (x_t . x_r)     (Simple; v-space for SquaredL2)

The Gram terms are found through a bucket table with exchange-linked chains (each entry keeps
the tag its insertion displaced). This model follows the kernel's indexing (bucket hash, 24-bit
row tags, walk bounds) so that the walk's termination and match rules are tested here, on CPU,
with duplicate features, empty rows and narrow feature spaces. Pure numpy/Python; small sizes.
"""
import numpy as np
import pytest

B = 8          # rows per batch
H_BITS = 12    # bucket table: 4096 entries
ROW_MASK = 0xFFFFFF


def bucket(j, h_bits=H_BITS):
    return ((j * 2654435761) & 0xFFFFFFFF) >> (32 - h_bits)


def tag_of(u, e):
    return 0x80000000 | ((u & ROW_MASK) << 7) | e


def sequential(rows, y, steps, reg, w0, coef):
    """The reference chain (PSGD:253-268), α-scaled for SquaredL2 exactly as the fp32 kernels."""
    v = w0.astype(np.float64).copy()
    alpha = 1.0
    cs = []
    for t, (cols, vals) in enumerate(rows):
        z = alpha * float(np.dot(vals, v[cols])) if len(cols) else 0.0
        alpha_n = alpha * (1.0 - steps[t] * reg)
        c = coef(z, y[t], steps[t])
        cv = c / alpha_n
        np.add.at(v, cols, cv * vals)
        alpha = alpha_n
        cs.append(cv)
    return v, alpha, np.array(cs)


def gram_model(rows, y, steps, reg, w0, coef, h_bits=H_BITS):
    """The kernel's schedule: P of batch b from the weights after batch b-2, G from the chains."""
    n = len(rows)
    nb = (n + B - 1) // B
    rows = rows + [(np.zeros(0, np.int64), np.zeros(0))] * (nb * B - n)
    steps = np.concatenate([steps, np.zeros(nb * B - n)])
    y = np.concatenate([y, np.zeros(nb * B - n)])
    v = w0.astype(np.float64).copy()
    buckets = np.zeros(1 << h_bits, np.uint64)
    prev = {}                      # (row, entry) -> displaced tag
    P = {}

    def dots(b):
        return [float(np.dot(rows[u][1], v[rows[u][0]])) if len(rows[u][0]) else 0.0
                for u in range(B * b, B * b + B)]

    P[0] = dots(0)
    if nb > 1:
        P[1] = dots(1)
    cprev = np.zeros(B)
    alpha = 1.0
    cs = []
    max_hops = 0
    for b in range(nb):
        # --- Gram wave: insert the batch's entries in row order, then walk each entry's chain
        for i in range(B):
            u = B * b + i
            for e, j in enumerate(rows[u][0]):
                h = bucket(int(j), h_bits)
                prev[(u, e)] = int(buckets[h])
                buckets[h] = tag_of(u, e)
        G = np.zeros((B, 2 * B))
        for i in range(B):
            u = B * b + i
            wlim = i + (B if b > 0 else 0)
            for e, j in enumerate(rows[u][0]):
                cur, last, hops = prev[(u, e)], 0, 0
                while cur != 0 and hops < 2048:
                    dist = (u - ((cur >> 7) & ROW_MASK)) & ROW_MASK
                    if dist > wlim or dist < last:
                        break
                    r, er = u - dist, cur & 127
                    if dist > 0 and rows[r][0][er] == j:
                        G[i, i + B - dist] += rows[u][1][e] * rows[r][1][er]
                    cur, last, hops = prev[(r, er)], dist, hops + 1
                max_hops = max(max_hops, hops)
        # --- chain wave: cross terms with batch b-1, then the in-batch recurrence
        yv = np.array(P[b]) + G[:, :B] @ cprev
        cv = np.zeros(B)
        for k in range(B):
            u = B * b + k
            alpha_n = alpha * (1.0 - steps[u] * reg)
            c = coef(alpha * yv[k], y[u], steps[u])
            cv[k] = c / alpha_n
            alpha = alpha_n
            yv += cv[k] * G[:, B + k]
        cs += list(cv)
        cprev = cv
        # --- apply wave: the batch's updates, then P of batch b+2
        for k in range(B):
            cols, vals = rows[B * b + k]
            np.add.at(v, cols, cv[k] * vals)
        if b + 2 < nb:
            P[b + 2] = dots(b + 2)
    return v, alpha, np.array(cs[:n]), max_hops


COEF = {
    "least_squares": lambda z, yl, s: -s * (z - yl),
    "logistic": lambda z, yl, s: -s * (1.0 / (1.0 + np.exp(-z)) - yl),
    "hinge": lambda z, yl, s: (s * (2 * yl - 1)) if 1.0 > (2 * yl - 1) * z else 0.0,
}


def synth(rng, n, d, kmin, kmax, dup=False):
    rows = []
    for _ in range(n):
        k = int(rng.integers(kmin, kmax + 1))
        if dup:
            idx = np.sort(rng.integers(0, d, size=k))
        else:
            idx = np.sort(rng.choice(d, size=min(k, d), replace=False))
        vals = rng.uniform(0.1, 1.0, size=len(idx))
        vals /= max(np.linalg.norm(vals), 1e-12)
        rows.append((idx.astype(np.int64), vals))
    return rows


@pytest.mark.parametrize("grad", sorted(COEF))
@pytest.mark.parametrize("reg", [0.0, 0.05])
@pytest.mark.parametrize("shape", [(203, 3000, 0, 40, False), (77, 12, 1, 9, False), (150, 40, 0, 30, True),
                                   (5, 100, 0, 3, False), (1, 10, 2, 2, False)])
def test_gram_schedule_matches_sequential_chain(grad, reg, shape):
    n, d, kmin, kmax, dup = shape
    rng = np.random.default_rng(n + d)
    rows = synth(rng, n, d, kmin, kmax, dup)
    y = (rng.random(n) > 0.5).astype(np.float64) if grad != "least_squares" else rng.standard_normal(n)
    steps = 0.3 / np.sqrt(1.0 + np.arange(n) % 7)
    w0 = rng.standard_normal(d) * 0.1
    vs, as_, cs_ = sequential(rows, y, steps, reg, w0, COEF[grad])
    vg, ag, cg, _ = gram_model(rows, y, steps, reg, w0, COEF[grad])
    assert ag == as_
    # only sums are reassociated: f64 agreement far inside the fp32 tolerance
    np.testing.assert_allclose(cg, cs_, rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(vg, vs, rtol=1e-9, atol=1e-12)


def test_gram_walk_with_tiny_bucket_table():
    # 16 buckets: every chain is long and full of collisions; the walk must still find every
    # shared feature exactly once (and stop at the window's end)
    rng = np.random.default_rng(5)
    rows = synth(rng, 120, 500, 0, 20)
    y = rng.standard_normal(120)
    steps = np.full(120, 0.2)
    w0 = np.zeros(500)
    vs, _, cs_ = sequential(rows, y, steps, 0.0, w0, COEF["least_squares"])[:3]
    vg, _, cg, hops = gram_model(rows, y, steps, 0.0, w0, COEF["least_squares"], h_bits=4)
    assert hops > 16
    np.testing.assert_allclose(cg, cs_, rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(vg, vs, rtol=1e-9, atol=1e-12)
