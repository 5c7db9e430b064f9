"""MLUtils.loadLibSVMFile [ext Spark MLlib 1.6.1]: the data-loading caller side of the path.

The reference's users build the RDD[(Double, Vector)] that ParallelizedSGD.runParallelizedSGD
(ParallelizedSGD.scala:188) takes with MLUtils.loadLibSVMFile(sc, path, numFeatures,
minPartitions). Here the parsing runs natively (libpsgd.so, psgd_libsvm_read: one host thread
per text split) and yields a PartitionedData of CSR partitions with the partitioning
sc.textFile(path, minPartitions) gives a local file.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _native as N
from .data import CsrPartition, PartitionedData


def loadLibSVMFile(path: str, numFeatures: int = -1, minPartitions: int = 2) -> PartitionedData:
    """Rows "label idx:val ..." (1-based, strictly increasing indices; '#' lines and blank lines
    skipped); numFeatures <= 0 infers max index + 1. minPartitions defaults to Spark's
    sc.defaultMinPartitions (2)."""
    L = N.lib()
    out = C.POINTER(N.psgd_libsvm)()
    N.check(L.psgd_libsvm_read(str(path).encode(), int(numFeatures), int(minPartitions), C.byref(out)))
    try:
        r = out.contents
        n, P = int(r.n_rows), int(r.n_parts)
        offs = np.ctypeslib.as_array(r.part_offsets, shape=(P + 1,)).copy()
        labels = np.ctypeslib.as_array(r.labels, shape=(max(n, 1),))[:n].copy()
        row_ptr = np.ctypeslib.as_array(r.row_ptr, shape=(n + 1,)).copy()
        nnz = int(row_ptr[-1])
        col = np.ctypeslib.as_array(r.col, shape=(max(nnz, 1),))[:nnz].copy()
        val = np.ctypeslib.as_array(r.val, shape=(max(nnz, 1),))[:nnz].copy()
        d = int(r.d)
    finally:
        L.psgd_libsvm_free(out)
    parts = []
    for a, b in zip(offs[:-1], offs[1:]):
        ka, kb = row_ptr[a], row_ptr[b]
        parts.append(CsrPartition(labels[a:b], row_ptr[a:b + 1] - ka, col[ka:kb], val[ka:kb], d))
    return PartitionedData(parts)
