"""CPU model of chain_block64's per-block break test (psgd_block64.hip, conv_test; psgd_device.h,
kpair / ballot_rows), checked against the sequential isConverged of ParallelizedSGD.scala:262,
:324-336 in f64.

After a block's recurrence every lane l carries the terms of row k(l) = l5 | l4<<1 | l3<<2 (the
transposed reduction's layout). Row k's norm step is an affine map of ||w_k||^2:

    N_{k+1} = A_k N_k + B_k,   A_k = a^2,   B_k = c (2 a z + c q)
    D_k     = b^2 N_k + E_k,   E_k = c (c q - 2 b z),   b = s lambda   (Simple: a = 1, b = 0)

and the kernel composes the maps in k order with a butterfly over lane bits 5, 4, 3 (partners
l ^ 32 by permlane32_swap, l ^ 16 by permlane16_swap, l ^ 8 by DPP row_ror 8; each returns the
pair's values with the member whose bit is clear first). This model runs that exact schedule on
64 lanes and compares every lane's N_k, N_{k+1}, D_k and the first passing row with the
sequential definitions. Pure numpy; the GPU tests hold the kernel itself to the oracle.
"""
import numpy as np
import pytest

KB = 8


def krow(lane):
    return ((lane >> 5) & 1) | (((lane >> 4) & 1) << 1) | (((lane >> 3) & 1) << 2)


def kbit(j):
    return (32, 16, 8)[j]


def kpair(v, j):
    """Every lane's (lo, hi): the values of the pair {l, l ^ kbit(j)} in k order."""
    lanes = np.arange(64)
    partner = v[lanes ^ kbit(j)]
    up = (lanes & kbit(j)) != 0
    lo = np.where(up, partner, v)
    hi = np.where(up, v, partner)
    return lo, hi


def butterfly_l2(A, B, n0):
    """conv_test's SquaredL2 form: exclusive prefix maps (eA, eB), then N_k, N_{k+1}."""
    lanes = np.arange(64)
    eA, eB = np.ones(64), np.zeros(64)
    tA, tB = A.copy(), B.copy()
    for j in range(3):
        pAlo, pAhi = kpair(tA, j)
        pBlo, pBhi = kpair(tB, j)
        up = (lanes & kbit(j)) != 0
        nA = eA * pAlo
        nB = eA * pBlo + eB
        eA = np.where(up, nA, eA)
        eB = np.where(up, nB, eB)
        if j < 2:
            tA, tB = pAhi * pAlo, pAhi * pBlo + pBhi
    Nk = eA * n0 + eB
    return Nk, A * Nk + B


def butterfly_simple(B, n0):
    """conv_test's Simple form: the inclusive sum of B in k order."""
    lanes = np.arange(64)
    incl, tot = B.copy(), B.copy()
    for j in range(3):
        lo, hi = kpair(tot, j)
        incl = np.where((lanes & kbit(j)) != 0, lo + incl, incl)
        if j < 2:
            tot = lo + hi
    return n0 + incl


def ballot_rows(mask):
    """psgd_device.h ballot_rows: rows (bit k) of a ballot over lanes 8g."""
    rows = 0
    for g in range(8):
        if (mask >> (8 * g)) & 1:
            rows |= 1 << (((g >> 2) & 1) | (((g >> 1) & 1) << 1) | ((g & 1) << 2))
    return rows


def block_terms(rng, l2):
    c = rng.normal(size=KB) * 0.1
    z = rng.normal(size=KB)
    q = rng.uniform(0.5, 2.0, size=KB)
    s = rng.uniform(0.01, 0.1, size=KB)
    lam = 0.3 if l2 else 0.0
    a = 1.0 - s * lam
    b = s * lam
    return c, z, q, a, b


def sequential(c, z, q, a, b, n0, tol):
    """isConverged after each row (PSGD.scala:333-335) from the norm recurrence."""
    N = n0
    Nk, Nn, D, first = [], [], [], -1
    for k in range(KB):
        Nk.append(N)
        D.append(b[k] ** 2 * N + c[k] * (c[k] * q[k] - 2 * b[k] * z[k]))
        N = a[k] ** 2 * N + c[k] * (2 * a[k] * z[k] + c[k] * q[k])
        Nn.append(N)
        if first < 0 and D[k] < tol * tol * max(N, 1.0):
            first = k
    return np.array(Nk), np.array(Nn), np.array(D), first


@pytest.mark.parametrize("l2", [False, True])
@pytest.mark.parametrize("seed", range(6))
def test_butterfly_matches_sequential_norms(l2, seed):
    rng = np.random.default_rng(seed)
    c, z, q, a, b = block_terms(rng, l2)
    n0 = float(rng.uniform(0.5, 5.0))
    Nk, Nn, D, _ = sequential(c, z, q, a, b, n0, 0.0)
    lanes = np.arange(64)
    k = np.array([krow(l) for l in lanes])
    if l2:
        A = a[k] ** 2
        B = c[k] * (2 * a[k] * z[k] + c[k] * q[k])
        E = c[k] * (c[k] * q[k] - 2 * b[k] * z[k])
        gNk, gNn = butterfly_l2(A, B, n0)
        gD = b[k] ** 2 * gNk + E
        np.testing.assert_allclose(gNk, Nk[k], rtol=1e-13)
    else:
        gNn = butterfly_simple(c[k] * (2 * z[k] + c[k] * q[k]), n0)
        gD = c[k] * (c[k] * q[k])
    np.testing.assert_allclose(gNn, Nn[k], rtol=1e-13)
    np.testing.assert_allclose(gD, D[k], rtol=1e-12, atol=1e-300)


@pytest.mark.parametrize("l2", [False, True])
def test_first_passing_row_every_position(l2):
    """A tol between consecutive rows' ratios makes each row in turn the first to pass; the
    ballot over lanes 8g decoded by ballot_rows names it."""
    rng = np.random.default_rng(7 + l2)
    hits = set()
    for trial in range(200):
        c, z, q, a, b = block_terms(rng, l2)
        n0 = float(rng.uniform(0.5, 5.0))
        _, Nn, D, _ = sequential(c, z, q, a, b, n0, 0.0)
        ratio = np.sqrt(np.maximum(D, 0.0) / np.maximum(Nn, 1.0))
        tol = float(np.sort(ratio)[trial % KB]) * (1 + 1e-9)
        _, _, _, first = sequential(c, z, q, a, b, n0, tol)
        lanes = np.arange(64)
        k = np.array([krow(l) for l in lanes])
        live = np.ones(64, bool)
        if l2:
            A = a[k] ** 2
            B = c[k] * (2 * a[k] * z[k] + c[k] * q[k])
            E = c[k] * (c[k] * q[k] - 2 * b[k] * z[k])
            gNk, gNn = butterfly_l2(A, B, n0)
            gD = b[k] ** 2 * gNk + E
        else:
            gNn = butterfly_simple(c[k] * (2 * z[k] + c[k] * q[k]), n0)
            gD = c[k] * c[k] * q[k]
        passing = ((lanes & 7) == 0) & live & (gD < tol * tol * np.maximum(gNn, 1.0))
        mask = sum(1 << int(l) for l in lanes[passing])
        rows = ballot_rows(mask)
        got = (rows & -rows).bit_length() - 1 if rows else -1
        assert got == first, (trial, got, first)
        hits.add(first)
    assert hits == set(range(KB)), hits


def test_row_lanes_and_pairs():
    """Lane 8g carries row rev3(g); kpair's levels pair rows k and k ^ (1 << j)."""
    for g in range(8):
        assert krow(8 * g) == (((g >> 2) & 1) | (((g >> 1) & 1) << 1) | ((g & 1) << 2))
    v = np.array([krow(l) for l in range(64)], dtype=float)
    for j in range(3):
        lo, hi = kpair(v, j)
        assert np.all(hi - lo == (1 << j))
