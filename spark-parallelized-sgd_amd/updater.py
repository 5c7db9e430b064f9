"""SGDUpdater plugins -- SGDUpdater.scala:40-286 (reference). Called at
ParallelizedSGD.scala:255 as updater.compute(weights, grad, stepSize, j, regParam, status).

Descriptors for the HIP chain kernel: the per-sample update runs on the device
(csrc/psgd_kernels.hip). `thisIterStepSize = stepSize / sqrt(iter)` with iter restarting at 1
in every partition on every outer iteration (ParallelizedSGD.scala:250).
"""
from __future__ import annotations

from ._native import IllegalArgumentException


class SGDUpdater:
    """Abstract SGDUpdater (SGDUpdater.scala:40-73)."""

    kind: int = -1

    def __repr__(self) -> str:
        return f"{type(self).__name__}()"


class SimpleSGDUpdater(SGDUpdater):
    """w' = w - (stepSize/sqrt(iter)) * g; regVal 0 (SGDUpdater.scala:80-99)."""

    kind = 0


class SquaredL2SGDUpdater(SGDUpdater):
    """w' = w * (1 - s*regParam) - s*g; regVal = 0.5*regParam*||w'||^2 (SGDUpdater.scala:157-182)."""

    kind = 1


class L1SGDUpdater(SGDUpdater):
    """w' = softThreshold(w - s*g, regParam*s); regVal = regParam*||w'||_1
    (SGDUpdater.scala:120-149)."""

    kind = 2


class AdaGradSGDUpdater(SGDUpdater):
    """accum += g*g; w' = w - s * g / sqrt(accum + 1.0) (SGDUpdater.scala:193-228).
    Per-chain status (accum): in the chain's registers on dense rows (chain_split / chain_dense),
    in HBM on CSR rows and past the register-resident width (chain_general); dense and CSR rows."""

    kind = 3


class AdamSGDUpdater(SGDUpdater):
    """The reference's Adam variant, reproduced literally (SGDUpdater.scala:240-286):
    v = beta*v + (1-beta)*g; r = gamma*r + (1-gamma)*g*g;
    w' = w - s/(1-beta^iter) * v / (sqrt(1 - r^iter) + eps).  Dense and CSR rows."""

    kind = 4

    def __init__(self, beta: float = 0.9, gamma: float = 0.999, eps: float = 1e-8):
        self.beta, self.gamma, self.eps = float(beta), float(gamma), float(eps)

    def __repr__(self) -> str:
        return f"AdamSGDUpdater({self.beta}, {self.gamma}, {self.eps})"


def updater_kind(u) -> int:
    if isinstance(u, SGDUpdater) and u.kind >= 0:
        return u.kind
    raise IllegalArgumentException(
        f"unsupported SGDUpdater {type(u).__name__}: expected one of SimpleSGDUpdater, "
        "SquaredL2SGDUpdater, L1SGDUpdater, AdaGradSGDUpdater, AdamSGDUpdater")
