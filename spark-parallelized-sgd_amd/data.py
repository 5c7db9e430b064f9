"""The RDD[(Double, Vector)] side of the boundary: partitions packed once into contiguous dense
or CSR buffers, in iterator order.

`PartitionedData.parallelize` reproduces Spark's `sc.parallelize(seq, numSlices)` slicing
([ext] Spark 1.6.1 ParallelCollectionRDD.slice: partition i holds rows
[floor(i*N/P), floor((i+1)*N/P))), which is the partition -> chain assignment the reference's
suite relies on (ParallelizedSGDSuite.scala:88, :119, :166).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np


@dataclass
class DensePartition:
    labels: np.ndarray  # float64 [n]
    x: np.ndarray       # [n, d] float32 or float64, row-major

    @property
    def n_rows(self) -> int:
        return int(self.labels.shape[0])

    @property
    def num_features(self) -> int:
        return int(self.x.shape[1])


@dataclass
class CsrPartition:
    labels: np.ndarray   # float64 [n]
    row_ptr: np.ndarray  # int64 [n+1]
    col: np.ndarray      # int32 [nnz], strictly increasing within a row
    val: np.ndarray      # float32/float64 [nnz]
    d: int

    @property
    def n_rows(self) -> int:
        return int(self.labels.shape[0])

    @property
    def num_features(self) -> int:
        return int(self.d)


@dataclass
class DevicePartition:
    """A dense partition already resident in HBM (torch tensors on the context's device),
    registered zero-copy (psgd_register_dense_device)."""

    labels: object  # torch.float64 [n] on cuda
    x: object       # torch [n, ld] float32/float64 on cuda; columns [d, ld) zero
    d: int

    @property
    def n_rows(self) -> int:
        return int(self.labels.shape[0])

    @property
    def num_features(self) -> int:
        return int(self.d)


@dataclass
class DeviceCsrPartition:
    """A CSR partition already resident in HBM (torch tensors on the context's device),
    registered zero-copy (psgd_register_csr_device): row_ptr int64 [n+1] absolute offsets into
    col (int32, strictly increasing per row) and val (float32/float64)."""

    labels: object
    row_ptr: object
    col: object
    val: object
    d: int

    @property
    def n_rows(self) -> int:
        return int(self.labels.shape[0])

    @property
    def num_features(self) -> int:
        return int(self.d)


def slice_positions(n: int, num_slices: int):
    """[ext] Spark ParallelCollectionRDD.slice.positions."""
    if num_slices < 1:
        from ._native import IllegalArgumentException
        raise IllegalArgumentException("requirement failed: Positive number of slices required")
    return [((i * n) // num_slices, ((i + 1) * n) // num_slices) for i in range(num_slices)]


class PartitionedData:
    """An ordered list of partitions: partition index = chain id."""

    def __init__(self, partitions: Sequence):
        self.partitions: List = list(partitions)
        feats = {p.num_features for p in self.partitions}
        if len(feats) > 1:
            from ._native import IllegalArgumentException
            raise IllegalArgumentException(
                f"requirement failed: all rows must have the same size, got {sorted(feats)}")
        self._num_features = feats.pop() if feats else 0

    # RDD-like API ----------------------------------------------------------------------------
    def count(self) -> int:
        return sum(p.n_rows for p in self.partitions)

    @property
    def num_partitions(self) -> int:
        return len(self.partitions)

    @property
    def num_features(self) -> int:
        return self._num_features

    def cache(self) -> "PartitionedData":
        """Registration copies to HBM once per optimizer context (the .cache() analogue)."""
        return self

    # constructors ----------------------------------------------------------------------------
    @staticmethod
    def parallelize(labels, x, num_slices: int, dtype=np.float64) -> "PartitionedData":
        labels = np.ascontiguousarray(labels, dtype=np.float64)
        x = np.ascontiguousarray(x, dtype=dtype)
        if x.ndim != 2 or x.shape[0] != labels.shape[0]:
            raise ValueError("x must be [n, d] with one label per row")
        parts = [DensePartition(labels[a:b], x[a:b]) for a, b in
                 slice_positions(labels.shape[0], num_slices)]
        return PartitionedData(parts)

    @staticmethod
    def parallelize_csr(labels, row_ptr, col, val, d: int, num_slices: int,
                        dtype=np.float64) -> "PartitionedData":
        labels = np.ascontiguousarray(labels, dtype=np.float64)
        row_ptr = np.ascontiguousarray(row_ptr, dtype=np.int64)
        col = np.ascontiguousarray(col, dtype=np.int32)
        val = np.ascontiguousarray(val, dtype=dtype)
        parts = []
        for a, b in slice_positions(labels.shape[0], num_slices):
            s, e = row_ptr[a], row_ptr[b]
            parts.append(CsrPartition(labels[a:b], row_ptr[a:b + 1] - s, col[s:e], val[s:e], d))
        return PartitionedData(parts)

    @staticmethod
    def from_points(points, num_slices: int, dtype=np.float64) -> "PartitionedData":
        """points: sequence of (label, features) with features a dense sequence, or a
        (indices, values, size) triple for a sparse vector (MLlib SparseVector)."""
        points = list(points)
        if points and isinstance(points[0][1], tuple):
            d = int(points[0][1][2])
            labels = np.array([p[0] for p in points], dtype=np.float64)
            row_ptr = np.zeros(len(points) + 1, dtype=np.int64)
            cols, vals = [], []
            for i, (_, (idx, v, _size)) in enumerate(points):
                cols.extend(idx)
                vals.extend(v)
                row_ptr[i + 1] = row_ptr[i] + len(idx)
            return PartitionedData.parallelize_csr(labels, row_ptr, np.array(cols, np.int32),
                                                   np.array(vals, dtype=dtype), d, num_slices, dtype)
        labels = np.array([p[0] for p in points], dtype=np.float64)
        x = np.array([np.asarray(p[1], dtype=np.float64) for p in points], dtype=dtype)
        if x.ndim == 1:
            x = x.reshape(len(points), -1)
        return PartitionedData.parallelize(labels, x, num_slices, dtype)


def shard_range(num_partitions: int, rank: int, world: int):
    """Contiguous partition block of `rank` (partition p -> GPU floor(p*G/P))."""
    # partition p belongs to rank floor(p * world / P); the block of rank r is
    # [ceil(r * P / world), ceil((r + 1) * P / world))
    lo = -(-(rank * num_partitions) // world)
    hi = -(-((rank + 1) * num_partitions) // world)
    return lo, hi


def default_dtype_of(data: PartitionedData) -> Optional[np.dtype]:
    for p in data.partitions:
        if isinstance(p, DensePartition):
            return p.x.dtype
        if isinstance(p, CsrPartition):
            return p.val.dtype
    return None
