"""MI355X-native parallelized SGD: a drop-in for the hot path of
Patrickgsheng/spark-parallelized-sgd (ParallelizedSGD.runParallelizedSGD / optimize).

The per-partition SGD chains, the Gradient/SGDUpdater per-sample math and the model averaging
run as HIP kernels for gfx950 (csrc/, built into libpsgd.so, C ABI in include/psgd.h). This
package is the host side: the reference's Optimizer API and driver loop.

The directory name contains dashes; import it through __graft_entry__.load_package() (which
registers it as `spark_parallelized_sgd_amd`).
"""
from ._native import (DeviceError, IllegalArgumentException, UnsupportedOperationException,
                      build)
from .data import (CsrPartition, DensePartition, DeviceCsrPartition, DevicePartition, PartitionedData,
                   shard_range)
from .gradient import Gradient, HingeGradient, LeastSquaresGradient, LogisticGradient
from .optimization import (DriverCheckpoint, HipEngine, ParallelizedSGD, ShardedEngine, make_params,
                           runParallelizedSGD)
from .updater import (AdaGradSGDUpdater, AdamSGDUpdater, L1SGDUpdater, SGDUpdater,
                      SimpleSGDUpdater, SquaredL2SGDUpdater)
from .util import loadLibSVMFile

__all__ = [
    "ParallelizedSGD", "runParallelizedSGD", "HipEngine", "ShardedEngine", "make_params",
    "Gradient", "LogisticGradient", "LeastSquaresGradient", "HingeGradient",
    "SGDUpdater", "SimpleSGDUpdater", "SquaredL2SGDUpdater", "L1SGDUpdater",
    "AdaGradSGDUpdater", "AdamSGDUpdater",
    "PartitionedData", "DensePartition", "CsrPartition", "DevicePartition", "DeviceCsrPartition",
    "shard_range", "loadLibSVMFile",
    "IllegalArgumentException", "UnsupportedOperationException", "DeviceError", "build",
]
