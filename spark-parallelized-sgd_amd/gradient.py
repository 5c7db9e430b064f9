"""Gradient plugins -- the MLlib `Gradient` surface the reference's chain calls at
ParallelizedSGD.scala:254 ([ext] Spark MLlib 1.6.1 mllib/optimization/Gradient.scala).

These are descriptors: the per-sample arithmetic they name runs inside the HIP chain kernel
(spark-parallelized-sgd_amd/csrc/psgd_kernels.hip, `gradient_scalar`). An unsupported gradient
class raises IllegalArgumentException when the optimizer maps it to a kernel; there is no
second (CPU) code path.
"""
from __future__ import annotations

from ._native import IllegalArgumentException, UnsupportedOperationException


class Gradient:
    """Abstract MLlib Gradient: compute(data, label, weights) -> (gradient, loss)."""

    kind: int = -1

    def __repr__(self) -> str:
        return f"{type(self).__name__}()"


class LogisticGradient(Gradient):
    """Binary logistic loss: margin = -dot(x, w); mult = 1/(1+exp(margin)) - y;
    grad = mult * x; loss = y > 0 ? log1pExp(margin) : log1pExp(margin) - margin."""

    kind = 0

    def __init__(self, numClasses: int = 2):
        if numClasses < 2:
            raise IllegalArgumentException(
                f"requirement failed: numClasses must be >= 2 but got {numClasses}")
        if numClasses != 2:
            raise UnsupportedOperationException(
                "multinomial LogisticGradient(numClasses > 2) is not built (SURVEY §8f rank 4)")
        self.numClasses = numClasses

    def __repr__(self) -> str:
        return f"LogisticGradient(numClasses={self.numClasses})"


class LeastSquaresGradient(Gradient):
    """diff = dot(x, w) - y; grad = diff * x; loss = diff * diff / 2.0."""

    kind = 1


class HingeGradient(Gradient):
    """ls = 2y - 1; if 1 > ls * dot(x, w): grad = -ls * x, loss = 1 - ls * dot; else 0, 0."""

    kind = 2


def gradient_kind(g) -> int:
    if isinstance(g, Gradient) and g.kind >= 0:
        return g.kind
    raise IllegalArgumentException(
        f"unsupported Gradient {type(g).__name__}: expected LogisticGradient, "
        "LeastSquaresGradient or HingeGradient")
