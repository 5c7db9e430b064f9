"""Pure-Python restatement of the reference's parallelized-SGD hot path (fp64, small cases).

TEST INFRASTRUCTURE ONLY: imported by tests/ (and the golden-fixture script) as an independent
second restatement; it must agree bit-for-bit with the C oracle (oracle/psgd_oracle.c) before
the C oracle's outputs are committed as golden vectors.

Parity status: PARTIALLY PINNED (see oracle/psgd_oracle.h).

Every function cites the reference it restates (paths under /root/reference):
  PSGD = src/main/scala/org/apache/spark/mllib/optimization/ParallelizedSGD.scala
  UPD  = src/main/scala/org/apache/spark/mllib/optimization/SGDUpdater.scala
  SUITE= src/test/scala/org/apache/spark/mllib/optimization/ParallelizedSGDSuite.scala
Third-party semantics ([ext], Spark MLlib 1.6.1 / Breeze 0.11 / netlib F2J / JDK) are restated
from their published algorithms; they are not vendored in the reference.

Python floats are IEEE binary64 and every operator rounds once, exactly as the JVM does.
"""
from __future__ import annotations

import math
import struct

GRAD_LOGISTIC, GRAD_LEAST_SQUARES, GRAD_HINGE = 0, 1, 2
UPD_SIMPLE, UPD_SQUARED_L2, UPD_L1, UPD_ADAGRAD, UPD_ADAM = 0, 1, 2, 3, 4


# ----------------------------------------------------------------------------- JDK restatements
class JavaRandom:
    """java.util.Random (48-bit LCG), as scala.util.Random(seed) wraps it [ext JDK]."""

    MULT = 0x5DEECE66D
    MASK = (1 << 48) - 1

    def __init__(self, seed: int):
        self.seed = (seed ^ self.MULT) & self.MASK
        self._have_next = False
        self._next_gaussian = 0.0

    def _next(self, bits: int) -> int:
        self.seed = (self.seed * self.MULT + 0xB) & self.MASK
        v = self.seed >> (48 - bits)
        if v >= 1 << 31:  # (int) cast
            v -= 1 << 32
        return v

    def next_double(self) -> float:
        return ((self._next(26) << 27) + self._next(27)) * (1.0 / (1 << 53))

    def next_gaussian(self) -> float:
        if self._have_next:
            self._have_next = False
            return self._next_gaussian
        while True:
            v1 = 2 * self.next_double() - 1
            v2 = 2 * self.next_double() - 1
            s = v1 * v1 + v2 * v2
            if not (s >= 1 or s == 0):
                break
        multiplier = math.sqrt(-2 * fdlibm_log(s) / s)
        self._next_gaussian = v2 * multiplier
        self._have_next = True
        return v1 * multiplier


def _hi_lo(x: float):
    u = struct.unpack("<Q", struct.pack("<d", x))[0]
    hi = u >> 32
    if hi >= 1 << 31:
        hi -= 1 << 32
    return hi, u & 0xFFFFFFFF


def _from_hi_lo(hi: int, lo: int) -> float:
    return struct.unpack("<d", struct.pack("<Q", ((hi & 0xFFFFFFFF) << 32) | lo))[0]


def fdlibm_log(x: float) -> float:
    """StrictMath.log == fdlibm 5.3 __ieee754_log (public algorithm) [ext JDK]."""
    ln2_hi = 6.93147180369123816490e-01
    ln2_lo = 1.90821492927058770002e-10
    two54 = 1.80143985094819840000e16
    Lg1, Lg2, Lg3 = 6.666666666666735130e-01, 3.999999999940941908e-01, 2.857142874366239149e-01
    Lg4, Lg5, Lg6 = 2.222219843214978396e-01, 1.818357216161805012e-01, 1.531383769920937332e-01
    Lg7 = 1.479819860511658591e-01
    hx, lx = _hi_lo(x)
    k = 0
    if hx < 0x00100000:
        if ((hx & 0x7FFFFFFF) | lx) == 0:
            return -math.inf
        if hx < 0:
            return math.nan
        k -= 54
        x *= two54
        hx, lx = _hi_lo(x)
    if hx >= 0x7FF00000:
        return x + x
    k += (hx >> 20) - 1023
    hx &= 0x000FFFFF
    i = (hx + 0x95F64) & 0x100000
    x = _from_hi_lo(hx | (i ^ 0x3FF00000), lx)
    k += i >> 20
    f = x - 1.0
    if (0x000FFFFF & (2 + hx)) < 3:
        if f == 0.0:
            if k == 0:
                return 0.0
            dk = float(k)
            return dk * ln2_hi + dk * ln2_lo
        R = f * f * (0.5 - 0.33333333333333333 * f)
        if k == 0:
            return f - R
        dk = float(k)
        return dk * ln2_hi - ((R - dk * ln2_lo) - f)
    s = f / (2.0 + f)
    dk = float(k)
    z = s * s
    i = hx - 0x6147A
    w = z * z
    j = 0x6B851 - hx
    t1 = w * (Lg2 + w * (Lg4 + w * Lg6))
    t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)))
    i |= j
    R = t2 + t1
    if i > 0:
        hfsq = 0.5 * f * f
        if k == 0:
            return f - (hfsq - s * (hfsq + R))
        return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f)
    if k == 0:
        return f - s * (f - R)
    return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f)


def generate_gd_input(offset: float, scale: float, n: int, seed: int):
    """ParallelizedSGDSuite.generateGDInput (SUITE:42-62): returns (x list, y list)."""
    rnd = JavaRandom(seed)
    x1 = [rnd.next_gaussian() for _ in range(n)]
    unif = JavaRandom(45)
    r_logis = []
    for _ in range(n):
        u = unif.next_double()
        r_logis.append(fdlibm_log(u) - fdlibm_log(1.0 - u))
    y = [1.0 if (offset + scale * x1[i] + r_logis[i]) > 0 else 0.0 for i in range(n)]
    return x1, y


# ----------------------------------------------------------------------------- MLlib / Breeze
def _jmax(a: float, b: float) -> float:
    if a != a:
        return a
    if b != b:
        return b
    return a if a >= b else b


def _signum(x: float) -> float:
    if x != x or x == 0.0:
        return x
    return 1.0 if x > 0.0 else -1.0


def _jsqrt(x: float) -> float:
    """Math.pow(x, 0.5) / Math.sqrt: NaN (not an exception) for negative x."""
    return math.sqrt(x) if x >= 0 else math.nan


def log1p_exp(x: float) -> float:
    """[ext] MLlib 1.6.1 MLUtils.log1pExp."""
    if x > 0:
        return x + math.log1p(math.exp(-x))
    return math.log1p(math.exp(x))


def _dot(row, w) -> float:
    """[ext] MLlib BLAS.dot (F2J ddot left fold / sparse loop)."""
    s = 0.0
    if isinstance(row, tuple):  # sparse (indices, values)
        idx, val = row
        for k in range(len(idx)):
            s = s + val[k] * w[idx[k]]
    else:
        for i in range(len(row)):
            s = s + row[i] * w[i]
    return s


def _norm2(w) -> float:
    s = 0.0
    for v in w:
        s = s + v * v
    return math.sqrt(s)


def is_converged(prev, cur, tol: float) -> bool:
    """PSGD:324-336."""
    s = 0.0
    for a, b in zip(prev, cur):
        t = a - b
        s = s + t * t
    return math.sqrt(s) < tol * _jmax(_norm2(cur), 1.0)


def _d2i(x: float) -> int:
    """Double.toInt: NaN -> 0, saturating, truncation toward zero."""
    if x != x:
        return 0
    if x >= 2147483647.0:
        return 2147483647
    if x <= -2147483648.0:
        return -2147483648
    return int(x)


def _active(row):
    """data.foreachActive order: (index, value) pairs."""
    if isinstance(row, tuple):
        return list(zip(row[0], row[1]))
    return list(enumerate(row))


def multinomial(row, label: float, w, num_classes: int):
    """[ext] MLlib 1.6.1 LogisticGradient(numClasses > 2).compute(data, label, weights):
    pivot class 0, weights in numClasses - 1 blocks of dataSize, zero values skipped, margins
    shifted by maxMargin when it is positive -> (('dense', grad), loss)."""
    nc1 = num_classes - 1
    d = len(w) // nc1
    act = _active(row)
    ly = _d2i(label) - 1
    margin_y, max_margin, max_idx = 0.0, -math.inf, 0
    margins = []
    for i in range(nc1):
        m = 0.0
        for j, v in act:
            if v != 0.0:
                m += v * w[i * d + j]
        if i == ly:
            margin_y = m
        if m > max_margin:
            max_margin, max_idx = m, i
        margins.append(m)
    s = 0.0
    if max_margin > 0:
        for i in range(nc1):
            margins[i] -= max_margin
            s += math.exp(-max_margin) if i == max_idx else math.exp(margins[i])
    else:
        for i in range(nc1):
            s += math.exp(margins[i])
    g = [0.0] * len(w)
    for i in range(nc1):
        mult = math.exp(margins[i]) / (s + 1.0) - (1.0 if (label != 0.0 and label == float(i + 1)) else 0.0)
        for j, v in act:
            if v != 0.0:
                g[i * d + j] += mult * v
    loss = math.log1p(s) - margin_y if label > 0.0 else math.log1p(s)
    return ("dense", g), (loss + max_margin if max_margin > 0 else loss)


def gradient(kind: int, row, label: float, w, num_classes: int = 2):
    """[ext] MLlib 1.6.1 {Logistic,LeastSquares,Hinge}Gradient.compute -> (grad, loss).

    grad is ('dense', list) or ('sparse', idx, vals)."""
    if kind == GRAD_LOGISTIC and num_classes > 2:
        return multinomial(row, label, w, num_classes)
    d = len(w)
    dotv = _dot(row, w)
    sparse = isinstance(row, tuple)
    if kind == GRAD_LOGISTIC:
        margin = -1.0 * dotv
        mult = (1.0 / (1.0 + math.exp(margin))) - label
        g = [0.0] * d
        if sparse:
            for i, v in zip(*row):
                g[i] = g[i] + mult * v
        elif mult != 0.0:
            g = [g[i] + mult * row[i] for i in range(d)]
        loss = log1p_exp(margin) if label > 0 else log1p_exp(margin) - margin
        return ("dense", g), loss
    if kind == GRAD_LEAST_SQUARES:
        diff = dotv - label
        loss = diff * diff / 2.0
        if sparse:
            return ("sparse", list(row[0]), [diff * v for v in row[1]]), loss
        return ("dense", [diff * v for v in row]), loss
    ls = 2 * label - 1.0
    if 1.0 > ls * dotv:
        a = -ls
        if sparse:
            return ("sparse", list(row[0]), [a * v for v in row[1]]), 1.0 - ls * dotv
        return ("dense", [a * v for v in row]), 1.0 - ls * dotv
    return ("sparse", [], []), 0.0


def _axpy(a: float, g, w):
    if g[0] == "dense":
        for i, gi in enumerate(g[1]):
            w[i] = w[i] + a * gi
    else:
        for i, gi in zip(g[1], g[2]):
            w[i] = w[i] + a * gi


def _dense(g, d):
    if g[0] == "dense":
        return g[1]
    out = [0.0] * d
    for i, v in zip(g[1], g[2]):
        out[i] = v
    return out


class UpdaterState:
    def __init__(self):
        self.a = None  # AdaGrad accum / Adam v
        self.b = None  # Adam r


def updater(kind: int, w, g, step: float, it: int, reg: float, st: UpdaterState,
            beta=0.9, gamma=0.999, eps=1e-8) -> float:
    """UPD: SimpleSGDUpdater :86-98, SquaredL2 :163-181, L1 :126-148, AdaGrad :199-227,
    Adam :252-285.  Updates w in place (the reference's toDenseVector copy); returns regVal."""
    s = step / math.sqrt(it)
    d = len(w)
    if kind == UPD_SIMPLE:
        _axpy(-s, g, w)
        return 0.0
    if kind == UPD_SQUARED_L2:
        c = 1.0 - s * reg
        for i in range(d):
            w[i] = w[i] * c
        _axpy(-s, g, w)
        n = _norm2(w)
        return 0.5 * reg * n * n
    if kind == UPD_L1:
        _axpy(-s, g, w)
        shrink = reg * s
        for i in range(d):
            wi = w[i]
            w[i] = _signum(wi) * _jmax(0.0, abs(wi) - shrink)
        t = 0.0
        for v in w:
            t = t + abs(v)
        return t * reg
    gd = _dense(g, d)
    if kind == UPD_ADAGRAD:
        sq = [v * v for v in gd]
        st.a = sq if st.a is None else [st.a[i] + sq[i] for i in range(d)]
        for i in range(d):
            w[i] = w[i] + (-s) * (gd[i] / _jsqrt(st.a[i] + 1.0))
        return 0.0
    if kind == UPD_ADAM:
        sq = [v * v for v in gd]
        if st.a is None:
            st.a = [v * (1 - beta) for v in gd]
            st.b = [v * (1 - gamma) for v in sq]
        else:
            st.a = [st.a[i] * beta + gd[i] * (1 - beta) for i in range(d)]
            st.b = [st.b[i] * gamma + sq[i] * (1 - gamma) for i in range(d)]
        lr = s / (1.0 - math.pow(beta, float(it)))
        for i in range(d):
            fix1 = _jsqrt(1.0 - math.pow(st.b[i], float(it))) + eps
            w[i] = w[i] + (-lr) * (st.a[i] / fix1)
        return 0.0
    raise ValueError(kind)


def chain(rows, labels, grad_kind, upd_kind, step, reg, tol, w_in, num_classes=2, **kw):
    """PSGD:243-270 -> (w, regVal, lossSum, count)."""
    st = UpdaterState()
    w = list(w_in)
    old = list(w_in)
    rv, loss_sum, count, j = 0.0, 0.0, 0, 1
    for row, y in zip(rows, labels):
        g, loss = gradient(grad_kind, row, y, w, num_classes)
        rv = updater(upd_kind, w, g, step, j, reg, st, **kw)
        loss_sum += loss
        count += 1
        j += 1
        if is_converged(old, w, tol):
            break
        old = list(w)
    return w, rv, loss_sum, count


def combine(a, b):
    """PSGD:271-276."""
    w1, rv1, l1, c1 = a
    w2, rv2, l2, c2 = b
    s = float(c1 + c2)
    w = [_jdiv(w1[i] * float(c1) + w2[i] * float(c2), s) for i in range(len(w1))]
    return w, _jdiv(rv1 * float(c1) + rv2 * float(c2), s), l1 + l2, c1 + c2


def _jdiv(a: float, b: float) -> float:
    """Java double division (IEEE 754: x/0 is +-Infinity or NaN, never an exception)."""
    if b != 0.0:
        return a / b
    if a != a or a == 0.0:
        return math.nan
    return math.copysign(math.inf, a) * math.copysign(1.0, b)


# ----------------------------------------------------------------------------- RDD.sample
# [ext] Spark 1.6.1 RDD.sample(false, fraction, seed) -> PartitionwiseSampledRDD(BernoulliSampler),
# restated from the published sources (not runnable here: no JVM): per-partition seeds from
# java.util.Random(seed).nextLong() in partition order; BernoulliSampler.setSeed(s) seeds an
# XORShiftRandom with hashSeed(s) = scala.util.hashing.MurmurHash3.bytesHash of the 64-byte
# ByteBuffer.allocate(java.lang.Long.SIZE).putLong(s) (Int, sign-extended).

M32 = 0xFFFFFFFF
M64 = 0xFFFFFFFFFFFFFFFF


def _rotl32(x, r):
    return ((x << r) | (x >> (32 - r))) & M32


def murmur3_bytes_hash(data: bytes, seed: int = 0x3C074A61) -> int:
    """scala.util.hashing.MurmurHash3.bytesHash (MurmurHash3 x86_32), as a signed Int."""
    def mix_last(h, k):
        k = (k * 0xCC9E2D51) & M32
        k = _rotl32(k, 15)
        k = (k * 0x1B873593) & M32
        return h ^ k
    h = seed & M32
    n4 = len(data) // 4
    for i in range(n4):
        k = data[4 * i] | (data[4 * i + 1] << 8) | (data[4 * i + 2] << 16) | (data[4 * i + 3] << 24)
        h = mix_last(h, k)
        h = _rotl32(h, 13)
        h = (h * 5 + 0xE6546B64) & M32
    tail = len(data) & 3
    k = 0
    i = 4 * n4
    if tail == 3:
        k ^= data[i + 2] << 16
    if tail >= 2:
        k ^= data[i + 1] << 8
    if tail >= 1:
        k ^= data[i]
        h = mix_last(h, k)
    h ^= len(data)
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & M32
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & M32
    h ^= h >> 16
    return h - (1 << 32) if h >= 1 << 31 else h


def xorshift_hash_seed(s: int) -> int:
    data = (s & M64).to_bytes(8, "big") + bytes(56)
    return murmur3_bytes_hash(data)


class XORShiftRandom:
    """[ext] org.apache.spark.util.random.XORShiftRandom (1.6.1)."""

    def __init__(self, seed: int):
        self.seed = xorshift_hash_seed(seed) & M64

    def next(self, bits: int) -> int:
        x = self.seed
        x ^= (x << 21) & M64
        x ^= x >> 35
        x ^= (x << 4) & M64
        self.seed = x
        return x & ((1 << bits) - 1)

    def next_double(self) -> float:
        return ((self.next(26) << 27) + self.next(27)) * (1.0 / (1 << 53))


def partition_seeds(seed: int, P: int):
    r = JavaRandom(seed)
    out = []
    for _ in range(P):
        hi = r._next(32)
        lo = r._next(32)
        v = ((hi << 32) + lo) & M64
        out.append(v - (1 << 64) if v >= 1 << 63 else v)
    return out


def bernoulli_sample(seed: int, n: int, fraction: float):
    """BernoulliSampler(fraction).sample over n rows after setSeed(seed): the kept offsets."""
    if fraction <= 0.0:
        return []
    if fraction >= 1.0:
        return list(range(n))
    rng = XORShiftRandom(seed)
    out = []
    if fraction <= 0.4:  # GapSamplingIterator, epsilon 5e-11
        lnq = math.log1p(-fraction)
        pos = 0
        while True:
            u = max(rng.next_double(), 5e-11)
            q = math.log(u) / lnq
            pos += 2147483647 if q >= 2147483647.0 else int(q)
            if pos >= n:
                break
            out.append(pos)
            pos += 1
    else:
        for t in range(n):
            if rng.next_double() <= fraction:
                out.append(t)
    return out


def run(partitions, grad_kind, upd_kind, step, iters, reg, w0, tol=0.001, groups=None,
        fraction=1.0, num_classes=2, **kw):
    """PSGD:188-306, batch i = data.sample(false, fraction, 42 + i) (:242).
    partitions: list of (rows, labels).
    groups: optional list of partition-index boundaries for the two-level combine tree.
    Returns (weights, loss_history, per-iteration chain counts)."""
    n = sum(len(p[1]) for p in partitions)
    if n == 0:
        return list(w0), [], []
    weights = list(w0)
    d = len(weights)
    reg_val = updater(upd_kind, list(weights), ("dense", [0.0] * d), 0, 1, reg, UpdaterState(), **kw)
    hist, counts = [], []
    prev = cur = None
    converged = False
    i = 1
    P = len(partitions)
    bounds = groups if groups else [0, P]
    while not converged and i <= iters:
        batch_parts = partitions
        if fraction < 1.0:
            seeds = partition_seeds(42 + i, P)
            batch_parts = []
            for (rows, labels), sd in zip(partitions, seeds):
                keep = bernoulli_sample(sd, len(labels), fraction)
                batch_parts.append(([rows[k] for k in keep], [labels[k] for k in keep]))
        res = [chain(rows, labels, grad_kind, upd_kind, step, reg, tol, weights, num_classes, **kw)
               for rows, labels in batch_parts]
        counts.append([r[3] for r in res])
        acc = None
        for gi in range(len(bounds) - 1):
            grp = res[bounds[gi]:bounds[gi + 1]]
            if not grp:
                continue
            ga = (list(grp[0][0]), grp[0][1], grp[0][2], grp[0][3])
            for r in grp[1:]:
                ga = combine(ga, r)
            acc = ga if acc is None else combine(acc, ga)
        w_avg, rv_avg, loss_sum, batch = acc
        if batch > 0:
            hist.append(loss_sum / float(batch) + reg_val)
            weights = w_avg
            reg_val = rv_avg
            prev, cur = cur, weights
            if prev is not None:
                converged = is_converged(prev, cur, tol)
        i += 1
    return weights, hist, counts


def parallelize_slices(n: int, num_slices: int):
    """[ext] Spark ParallelCollectionRDD.slice positions: partition i = [i*n/P, (i+1)*n/P)."""
    return [((i * n) // num_slices, ((i + 1) * n) // num_slices) for i in range(num_slices)]
