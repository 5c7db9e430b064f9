"""ParallelizedSGD -- the reference's Optimizer API and driver loop, with the per-partition
chains, the per-sample Gradient/SGDUpdater math and the model averaging on MI355X.

Reference: src/main/scala/org/apache/spark/mllib/optimization/ParallelizedSGD.scala
  class ParallelizedSGD(gradient, updater)  :41-159   -> class ParallelizedSGD below
  object ParallelizedSGD.runParallelizedSGD :188-306  -> ParallelizedSGD.runParallelizedSGD
  8-argument alias (tol 0.001)              :311-321  -> the default of convergenceTol
  isConverged                               :324-336  -> device terms + the comparison here

What runs where: the driver loop below is the reference's, statement for statement (loss
history, regVal lag, driver-side convergence test, empty-data and empty-batch rules). The block
the reference ships to executors (:238-276: broadcast, sample, mapPartitions chain, treeReduce)
is one psgd_run_epoch_device call per process (HIP chain kernel + on-device fold in partition
order), then -- with several processes -- an all-gather of the per-process partial results over
RCCL and the same fold in rank order (the cross-GPU level of the treeReduce).
"""
from __future__ import annotations

import collections
import logging
import math
import threading
import time
import uuid
from typing import List, Optional, Tuple

import numpy as np

from . import _native as N
from .data import (CsrPartition, DensePartition, DeviceCsrPartition, DevicePartition, PartitionedData,
                   shard_range)
from .gradient import Gradient, LogisticGradient, gradient_kind, num_classes, weight_dim
from .updater import AdamSGDUpdater, SGDUpdater, updater_kind

log = logging.getLogger("org.apache.spark.mllib.optimization.ParallelizedSGD")

IllegalArgumentException = N.IllegalArgumentException


def _require(cond: bool, msg: str) -> None:
    if not cond:
        raise IllegalArgumentException("requirement failed: " + msg)


def _jstr(x) -> str:
    """Scala string interpolation of a Double/Int."""
    if isinstance(x, float):
        return repr(x) if math.isfinite(x) else ("NaN" if x != x else ("Infinity" if x > 0 else "-Infinity"))
    return str(x)


def make_params(gradient, updater, stepSize, regParam, miniBatchFraction, convergenceTol,
                compute_dtype="f64", iteration=1) -> N.psgd_params:
    p = N.psgd_params()
    p.gradient = gradient_kind(gradient)
    p.num_classes = num_classes(gradient)
    p.updater = updater_kind(updater)
    p.compute_dtype = {"f64": N.F64, "f32": N.F32}[compute_dtype]
    p.iteration = iteration
    p.step_size = float(stepSize)
    p.reg_param = float(regParam)
    p.mini_batch_fraction = float(miniBatchFraction)
    p.convergence_tol = float(convergenceTol)
    if isinstance(updater, AdamSGDUpdater):
        p.adam_beta, p.adam_gamma, p.adam_eps = updater.beta, updater.gamma, updater.eps
    else:
        p.adam_beta, p.adam_gamma, p.adam_eps = 0.9, 0.999, 1e-8
    return p


def _dist():
    """(rank, world, process_group_available) from torch.distributed, if initialised."""
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist.get_rank(), dist.get_world_size(), True
    except ImportError:
        pass
    return 0, 1, False


# ---------------------------------------------------------------------------------------------
# Engines: who runs the chains of this process's partitions.
# ---------------------------------------------------------------------------------------------
_contexts = {}


def get_context(device: int) -> N.Context:
    ctx = _contexts.get(device)
    if ctx is None:
        ctx = N.Context(device)
        ctx.registered_token = None
        # serialises (re-)registration + epoch of the engines that share this device's context
        ctx.engine_lock = threading.RLock()
        _contexts[device] = ctx
    return ctx


class ShardedEngine:
    """The multi-process part of an epoch, shared by every engine.

    Partition p belongs to rank floor(p * world / P) (contiguous blocks). Each rank
    folds its own chains (partition order) into a (d+3)-vector [w, regVal, lossSum, count];
    the ranks all-gather those partials and fold them in rank order with the reference's
    combiner -- a two-level treeReduce (ParallelizedSGD.scala:271-276). A rank without
    partitions contributes the fold's identity element (w_in, 0, 0, 0): an empty partition's
    result (ParallelizedSGD.scala:270 with count 0)."""

    def __init__(self, data: PartitionedData, rank: int, world: int, weight_dim: Optional[int] = None):
        # length of the weight vector: num_features, (K-1)*num_features for multinomial Logistic
        self.d = int(weight_dim) if weight_dim else data.num_features
        self.rank, self.world = rank, world
        self.lo, self.hi = shard_range(data.num_partitions, rank, world)
        self.n_local = self.hi - self.lo

    # subclass hooks: local_partial(params, w, with_counts) -> (partial[d+3], counts | None);
    # empty_partial(w) -> partial; fold_partials(gathered[world*(d+3)]) -> partial;
    # gather_buffer() -> tensor[world*(d+3)]
    def epoch(self, params, w, with_counts: bool = False):
        """ParallelizedSGD.scala:238-276 over all ranks: the folded [w_avg, regVal, lossSum,
        count] and (optionally) this rank's chain counts."""
        if self.n_local > 0:
            partial, counts = self.local_partial(params, w, with_counts)
        else:
            partial, counts = self.empty_partial(w), None
        if self.world == 1:
            return partial, counts
        return self.exchange(partial), counts

    def exchange(self, partial):
        """The cross-process level of the treeReduce: all-gather every rank's (d+3) partial
        (RCCL over xGMI with the nccl backend; gloo's list form on CPU) and fold them in rank
        order with the reference's combiner (ParallelizedSGD.scala:271-276)."""
        import torch.distributed as dist
        out = self.gather_buffer()
        if dist.get_backend() == "gloo":
            dist.all_gather(list(out.view(self.world, self.d + 3).unbind(0)), partial)
        else:
            dist.all_gather_into_tensor(out, partial)
        return self.fold_partials(out)


class HipEngine(ShardedEngine):
    """Runs this process's chains on one MI355X through the psgd C ABI.

    Weights and the (d+3)-double partial results stay in HBM (torch tensors serve as device
    allocations and as the RCCL all-gather buffers); every kernel and copy runs on
    `self.stream`."""

    def __init__(self, data: PartitionedData, rank: int = 0, world: int = 1,
                 device: Optional[int] = None, weight_dim: Optional[int] = None):
        import torch
        if not torch.cuda.is_available():
            raise N.DeviceError("HipEngine needs a visible MI355X (torch.cuda.is_available() is False)")
        super().__init__(data, rank, world, weight_dim)
        if device is None:
            device = torch.cuda.current_device()
        self.torch = torch
        self.device = device
        self.dev = torch.device("cuda", device)
        self.ctx = get_context(device)
        # a real stream handle: NULL would select the library's own stream
        self.stream = torch.cuda.Stream(device=self.dev)
        # two of each result buffer, alternating by epoch: an epoch's folded weights stay intact
        # while the next epoch, which reads them, runs (adopt_view)
        self._partials = [torch.empty(self.d + 3, dtype=torch.float64, device=self.dev) for _ in range(2)]
        self._folds = [torch.empty(self.d + 3, dtype=torch.float64, device=self.dev) for _ in range(2)]
        self._slot = 0
        self._partial, self._folded = self._partials[0], self._folds[0]
        self._gather = torch.empty(self.world * (self.d + 3), dtype=torch.float64, device=self.dev)
        self._counts = torch.empty(max(self.n_local, 1), dtype=torch.int64, device=self.dev)
        self._data = data
        with self.ctx.engine_lock:
            self._register(data)

    def _register(self, data: PartitionedData):
        """Register partitions [lo, hi) with the device context unless they are what it holds
        (ctx.engine_lock held). Engines on one device share its context; the key records whose
        partitions it holds."""
        token = getattr(data, "_psgd_token", None)
        if token is None:
            token = uuid.uuid4().hex
            data._psgd_token = token
        key = (token, self.lo, self.hi)
        self._key = key
        if self.ctx.registered_token == key:
            return
        self.ctx.clear()
        self.ctx.registered_token = None
        for p in range(self.lo, self.hi):
            part = data.partitions[p]
            if isinstance(part, DensePartition):
                self.ctx.register_dense(p, part.labels, part.x)
            elif isinstance(part, CsrPartition):
                self.ctx.register_csr(p, part.labels, part.row_ptr, part.col, part.val, part.d)
            elif isinstance(part, DevicePartition):
                dt = N.F32 if part.x.dtype == self.torch.float32 else N.F64
                self.ctx.register_dense_device(p, part.n_rows, part.d, int(part.x.stride(0)),
                                               part.labels.data_ptr(), part.x.data_ptr(), dt)
            elif isinstance(part, DeviceCsrPartition):
                dt = N.F32 if part.val.dtype == self.torch.float32 else N.F64
                self.ctx.register_csr_device(p, part.n_rows, part.d, part.labels.data_ptr(),
                                             part.row_ptr.data_ptr(), part.col.data_ptr(),
                                             part.val.data_ptr(), dt)
            else:
                raise IllegalArgumentException(f"unsupported partition type {type(part).__name__}")
        self.ctx.registered_token = key

    # driver hooks ---------------------------------------------------------------------------
    def weights(self, w_host: np.ndarray):
        with self.torch.cuda.stream(self.stream):
            return self.torch.from_numpy(np.ascontiguousarray(w_host, dtype=np.float64)).to(self.dev)

    def initial_regval(self, params, w_host: np.ndarray) -> float:
        return self.ctx.initial_regval(params, w_host)

    def epoch(self, params, w_dev, with_counts: bool = False):
        """The folded partial is written on `self.stream`. Its readers may be on any stream: the
        caller's current stream is made to wait for the epoch before this returns, so a read
        there (e.g. `.cpu()` on the default stream) sees the finished result -- never the
        buffer's previous contents, which the driver would take for an empty batch (count 0,
        ParallelizedSGD.scala:295-297)."""
        caller = self.torch.cuda.current_stream(self.dev)
        # order after whatever produced the inputs on the caller's stream
        self.stream.wait_stream(caller)
        out = self._enqueue(params, w_dev, with_counts)
        caller.wait_stream(self.stream)
        return out

    def _enqueue(self, params, w_dev, with_counts=False):
        """The epoch on self.stream (into the next pair of result buffers), no cross-stream order."""
        self._slot ^= 1
        self._partial, self._folded = self._partials[self._slot], self._folds[self._slot]
        with self.torch.cuda.stream(self.stream):
            return super().epoch(params, w_dev, with_counts)

    def local_partial(self, params, w_dev, with_counts):
        # The lock serialises re-registration and the enqueue; the device order of epochs that
        # share the context's scratch buffers from different streams is the library's
        # (psgd_run_epoch_device waits for the previous epoch's end event on another stream).
        with self.ctx.engine_lock:
            # another engine on this device may have registered its own partitions since
            if self.ctx.registered_token != self._key:
                self._register(self._data)
            counts_ptr = self._counts.data_ptr() if with_counts else None
            if self._mirror_next is not None and self.world == 1:
                self.ctx.run_epoch_device_mirror(params, w_dev.data_ptr(), self._partial.data_ptr(), counts_ptr,
                                                 self.stream.cuda_stream, self._mirror_next)
                self._mirror_used = True
            else:
                self.ctx.run_epoch_device(params, w_dev.data_ptr(), self._partial.data_ptr(), counts_ptr,
                                          self.stream.cuda_stream)
        counts = self._counts[: self.n_local].cpu().numpy() if with_counts else None
        return self._partial, counts

    def empty_partial(self, w_dev):
        self._partial[: self.d].copy_(w_dev)
        self._partial[self.d:].zero_()
        return self._partial

    def gather_buffer(self):
        return self._gather

    # (diagnostics) when a list, every cross-process exchange appends a pair of HIP events recorded
    # around it on self.stream: the all-gather plus the rank-order fold (bench.py times them)
    exchange_events = None

    def exchange(self, partial):
        if self.exchange_events is None:
            return super().exchange(partial)
        a = self.torch.cuda.Event(enable_timing=True)
        b = self.torch.cuda.Event(enable_timing=True)
        a.record(self.stream)
        out = super().exchange(partial)
        b.record(self.stream)
        self.exchange_events.append((a, b))
        return out

    def fold_partials(self, gathered):
        if self._mirror_next is not None:
            self.ctx.fold_partials_device_mirror(self.world, self.d, gathered.data_ptr(), self._folded.data_ptr(),
                                                 self.stream.cuda_stream, self._mirror_next)
            self._mirror_used = True
        else:
            self.ctx.fold_partials_device(self.world, self.d, gathered.data_ptr(),
                                          self._folded.data_ptr(), self.stream.cuda_stream)
        return self._folded

    def scalars(self, folded) -> Tuple[float, float, int]:
        with self.torch.cuda.stream(self.stream):
            h = folded[self.d:].cpu().numpy()
        if not math.isfinite(h[2]):
            raise N.DeviceError("chain kernel watchdog fired (loader/compute waves stalled)")
        return float(h[0]), float(h[1]), int(h[2])

    def adopt(self, folded):
        with self.torch.cuda.stream(self.stream):
            return folded[: self.d].clone()

    # the driver's pipelined loop (ParallelizedSGD._run_pipelined) ------------------------------
    # An epoch's three scalars reach the host without a copy: the epoch's last fold kernel writes
    # them to a page-locked slot as well (psgd_run_epoch_device_mirror /
    # psgd_fold_partials_device_mirror), the count last; the host polls the count.
    _PIN_SLOTS = 16
    _mirror = None
    _mirror_next = None
    _mirror_used = False

    def epoch_async(self, params, w_dev):
        """epoch() that returns (folded, token) at once; scalars_wait(token) gives its scalars.
        Tokens are read in the order they were made, fewer than _PIN_SLOTS behind the newest.
        Unlike epoch() it orders nothing against the caller's stream (each cross-stream wait
        costs the device ~20 us between epochs): w_dev must have been produced on self.stream
        (weights(), adopt(), adopt_view() all are), and `folded` is read on self.stream or after
        scalars_wait(token)."""
        if self._mirror is None:
            self._mirror = self.ctx.host_array((self._PIN_SLOTS, 3), np.float64)
            self._pin_owner = [-1] * self._PIN_SLOTS
            self._pin_seq = 0
        seq = self._pin_seq
        k = seq % self._PIN_SLOTS
        if self._pin_owner[k] >= 0:
            self._poll(k)   # (a slot is reused only after its last epoch's fold has written it)
        self._mirror[k, 2] = self._UNSET   # the fold's count replaces it (psgd.h)
        self._mirror_next, self._mirror_used = self._mirror[k].ctypes.data, False
        try:
            folded, _ = self._enqueue(params, w_dev)
        finally:
            used, self._mirror_next = self._mirror_used, None
        if not used:   # (no fold of this epoch ran on this rank's context: copy the scalars)
            with self.torch.cuda.stream(self.stream):
                self.torch.from_numpy(self._mirror[k]).copy_(folded[self.d:])
        self._pin_owner[k] = seq
        self._pin_seq = seq + 1
        return folded, (seq, k)

    _UNSET = -1.0            # no count is negative
    _WAIT_LIMIT_S = 600.0    # a chain kernel's own watchdog ends a stalled epoch in seconds

    def scalars_wait(self, token) -> Tuple[float, float, int]:
        """scalars() of the epoch behind `token`: polls its slot until the fold kernel's count
        lands (no event: each event recorded between epochs costs the device a few us)."""
        seq, k = token
        if self._pin_owner[k] != seq:
            raise RuntimeError(f"the scalars of epoch token {seq} were overwritten before they were read")
        self._poll(k)
        h = self._mirror[k].copy()
        if not math.isfinite(h[2]):
            raise N.DeviceError("chain kernel watchdog fired (loader/compute waves stalled)")
        return float(h[0]), float(h[1]), int(h[2])

    def _poll(self, k):
        slot = self._mirror[k]
        if slot[2] != self._UNSET:
            return
        t0 = time.perf_counter()
        spins = 0
        while slot[2] == self._UNSET:
            spins += 1
            if spins > 2000:   # past the first ~ms: yield between polls
                time.sleep(20e-6)
                if time.perf_counter() - t0 > self._WAIT_LIMIT_S:
                    raise N.DeviceError("an epoch's fold did not complete")

    def drain(self):
        """Wait for everything enqueued on the engine's stream."""
        self.stream.synchronize()

    def adopt_view(self, folded):
        """adopt() without the copy: the folded weights in place, intact until the second epoch
        after the one that produced them is enqueued (the result buffers alternate)."""
        return folded[: self.d]

    def convergence_terms(self, prev, cur) -> Tuple[float, float]:
        return self.ctx.convergence_terms_device(self.d, prev.data_ptr(), cur.data_ptr(),
                                                 self.stream.cuda_stream)

    def to_host(self, w_dev) -> np.ndarray:
        with self.torch.cuda.stream(self.stream):
            return w_dev.detach().cpu().numpy().astype(np.float64)


# ---------------------------------------------------------------------------------------------
# The optimizer.
# ---------------------------------------------------------------------------------------------
class ParallelizedSGD:
    """:: Experimental :: Parallelized Stochastic Gradient Descent (Zinkevich et al.).

    Mirrors ParallelizedSGD.scala:41-159: same defaults (:46-50), same validated setters
    (:56-134, same messages), optimize(data, initialWeights) -> weights (:144-157)."""

    def __init__(self, gradient: Gradient, updater: SGDUpdater):
        self.gradient = gradient
        self.updater = updater
        self.stepSize = 1.0
        self.numIterations = 100
        self.regParam = 0.0
        self.miniBatchFraction = 1.0
        self.convergenceTol = 0.001
        self.compute_dtype = "f64"

    def setStepSize(self, step: float) -> "ParallelizedSGD":
        _require(step > 0, f"Initial step size must be positive but got {_jstr(float(step))}")
        self.stepSize = float(step)
        return self

    def setMiniBatchFraction(self, fraction: float) -> "ParallelizedSGD":
        _require(fraction > 0 and fraction <= 1.0,
                 f"Fraction for mini-batch SGD must be in range (0, 1] but got {_jstr(float(fraction))}")
        self.miniBatchFraction = float(fraction)
        return self

    def setNumIterations(self, iters: int) -> "ParallelizedSGD":
        _require(iters >= 0, f"Number of iterations must be nonnegative but got {iters}")
        self.numIterations = int(iters)
        return self

    def setRegParam(self, regParam: float) -> "ParallelizedSGD":
        _require(regParam >= 0,
                 f"Regularization parameter must be nonnegative but got {_jstr(float(regParam))}")
        self.regParam = float(regParam)
        return self

    def setConvergenceTol(self, tolerance: float) -> "ParallelizedSGD":
        _require(tolerance >= 0.0 and tolerance <= 1.0,
                 f"Convergence tolerance must be in range [0, 1] but got {_jstr(float(tolerance))}")
        self.convergenceTol = float(tolerance)
        return self

    def setGradient(self, gradient: Gradient) -> "ParallelizedSGD":
        self.gradient = gradient
        return self

    def setUpdater(self, updater: SGDUpdater) -> "ParallelizedSGD":
        self.updater = updater
        return self

    def setComputeDtype(self, dtype: str) -> "ParallelizedSGD":
        """Build extension: "f64" (reference arithmetic, default) or "f32" (throughput mode)."""
        _require(dtype in ("f64", "f32"), f"compute dtype must be f64 or f32 but got {dtype}")
        self.compute_dtype = dtype
        return self

    def optimize(self, data: PartitionedData, initialWeights) -> np.ndarray:
        weights, _ = ParallelizedSGD.runParallelizedSGD(
            data, self.gradient, self.updater, self.stepSize, self.numIterations, self.regParam,
            self.miniBatchFraction, initialWeights, self.convergenceTol,
            compute_dtype=self.compute_dtype)
        return weights

    # object ParallelizedSGD ---------------------------------------------------------------------
    @staticmethod
    def runParallelizedSGD(data: PartitionedData, gradient: Gradient, updater: SGDUpdater,
                           stepSize: float, numIterations: int, regParam: float,
                           miniBatchFraction: float, initialWeights, convergenceTol: float = 0.001,
                           *, compute_dtype: str = "f64", engine=None,
                           return_chain_counts: bool = False,
                           checkpoint: Optional[str] = None, checkpoint_every: int = 1):
        """ParallelizedSGD.scala:188-306 (and the 8-argument alias :311-321 via the default).
        Returns (weights, stochasticLossHistory) [, per-iteration chain counts].

        checkpoint: a file path (extension): the loop state is saved there every
        `checkpoint_every` iterations and after the last one, and a run that finds a checkpoint of
        the same parameters and data resumes from it (DriverCheckpoint). The chain counts of
        iterations before the resume are not in it."""
        if miniBatchFraction < 1.0 and convergenceTol > 0.0:  # :200-203
            log.warning("Testing against a convergenceTol when using miniBatchFraction "
                        "< 1.0 can be unstable because of the stochasticity in sampling.")
        history: List[float] = []
        chain_counts: List[np.ndarray] = []
        w0 = np.ascontiguousarray(np.asarray(initialWeights, dtype=np.float64))

        numExamples = data.count()  # :211
        if numExamples == 0:  # :214-217
            log.warning("GradientDescent.runMiniBatchSGD returning initial weights, no data found")
            out = (w0, np.array(history))
            return out + (chain_counts,) if return_chain_counts else out
        if numExamples * miniBatchFraction < 1:  # :219-221
            log.warning("The miniBatchFraction is too small")
        nf = data.num_features
        if isinstance(gradient, LogisticGradient):
            # LogisticGradient.compute: require(weights.size % dataSize == 0 &&
            # numClasses == weights.size / dataSize + 1) [ext MLlib 1.6.1]
            if nf == 0 or w0.shape[0] % nf != 0 or num_classes(gradient) != w0.shape[0] // nf + 1:
                raise IllegalArgumentException("requirement failed")
        elif w0.shape[0] != nf:
            raise IllegalArgumentException(
                f"requirement failed: BLAS.dot(x: Vector, y: Vector) was given Vectors with "
                f"non-matching sizes: x.size = {nf}, y.size = {w0.shape[0]}")

        if engine is None:
            rank, world, _ = _dist()
            engine = HipEngine(data, rank, world, weight_dim=weight_dim(gradient, nf))

        params = make_params(gradient, updater, stepSize, regParam, miniBatchFraction,
                             convergenceTol, compute_dtype)
        ckpt = DriverCheckpoint(checkpoint, checkpoint_every) if checkpoint else None
        fp = _ckpt_fingerprint(params, data, w0) if ckpt else None
        state = ckpt.load(fp) if ckpt else None
        if state is None:
            weights = engine.weights(w0)                  # :224
            regVal = engine.initial_regval(params, w0)    # :231-233
            have_current = False
            converged = False
            i = 1
        else:
            weights = engine.weights(state["weights"])
            regVal, history = state["regVal"], state["history"]
            have_current, converged, i = state["have_current"], state["converged"], state["i"]
            log.warning("resuming at iteration %d from checkpoint %s", i, checkpoint)
        last_saved = i
        if (convergenceTol == 0.0 and miniBatchFraction >= 1.0 and ckpt is None and not return_chain_counts
                and hasattr(engine, "epoch_async")):
            weights, regVal = ParallelizedSGD._run_pipelined(engine, params, weights, regVal, i,
                                                             numIterations, history)
            i = numIterations + 1
        while not converged and i <= numIterations:       # :237
            params.iteration = i
            folded, counts = engine.epoch(params, weights, with_counts=return_chain_counts)
            avgRegVal, lossSum, batchSize = engine.scalars(folded)
            if return_chain_counts:
                chain_counts.append(counts)
            if batchSize > 0:                              # :278
                stochasticLoss = lossSum / batchSize + regVal   # :283
                history.append(stochasticLoss)
                log.warning("stochastic loss at step%d: %s", i, stochasticLoss)
                new_weights = engine.adopt(folded)         # :286-287
                regVal = avgRegVal
                if have_current:                           # :289-294
                    dsq, nsq = engine.convergence_terms(weights, new_weights)
                    converged = math.sqrt(dsq) < convergenceTol * max_j(math.sqrt(nsq), 1.0)
                weights = new_weights
                have_current = True
            else:                                          # :295-297
                log.warning("Iteration (%d/%d). The size of sampled batch is zero", i, numIterations)
            i += 1
            if ckpt and (i - last_saved >= ckpt.every or converged or i > numIterations):
                ckpt.save(fp, engine.to_host(weights), i, regVal, history, have_current, converged)
                last_saved = i
        log.info("GradientDescent.runMiniBatchSGD finished. Last 10 stochastic losses %s",
                 ", ".join(str(v) for v in history[-10:]))
        out = (engine.to_host(weights), np.array(history))
        return out + (chain_counts,) if return_chain_counts else out

    # (the number of epochs enqueued ahead of the one whose scalars are read)
    PIPELINE_LAG = 2

    @staticmethod
    def _run_pipelined(engine, params, weights, regVal: float, i: int, numIterations: int,
                       history: List[float]):
        """The loop :237-297 when its branches are known before an epoch's scalars are: with
        convergenceTol == 0 `isConverged` (:324-336) is `norm < 0.0 * max(.)`, never true, and
        with miniBatchFraction == 1 every row of the (non-empty, :214-217) data is in every batch
        (:242), so batchSize > 0 (:278) and the folded weights are always adopted (:286). Each
        epoch is enqueued with the previous epoch's folded weights before that epoch's three
        scalars are read back, up to PIPELINE_LAG epochs ahead, so the device runs epoch after
        epoch without waiting for the host; the loss history, regVal lag (:283, :287) and log
        lines follow in iteration order as each epoch's scalars arrive. Returns (weights, regVal)."""
        pending = collections.deque()

        def settle(regVal):
            it, token = pending.popleft()
            avgRegVal, lossSum, batchSize = engine.scalars_wait(token)
            if batchSize <= 0:   # a full batch of non-empty data: cannot happen
                raise RuntimeError(f"iteration {it}: an empty batch in a full-batch epoch")
            stochasticLoss = lossSum / batchSize + regVal          # :283
            history.append(stochasticLoss)
            log.warning("stochastic loss at step%d: %s", it, stochasticLoss)
            return avgRegVal                                       # :287

        try:
            while i <= numIterations:
                params.iteration = i
                folded, token = engine.epoch_async(params, weights)
                pending.append((i, token))
                # (valid while the next epoch reads it; every later use is after its own epoch)
                weights = engine.adopt_view(folded)                # :286
                if len(pending) > ParallelizedSGD.PIPELINE_LAG:
                    regVal = settle(regVal)
                i += 1
            while pending:
                regVal = settle(regVal)
        except BaseException:
            # epochs still in flight write their scalars to the engine's page-locked slots:
            # let them finish before the error unwinds (and may free the engine)
            if hasattr(engine, "drain"):
                engine.drain()
            raise
        # the last epoch's weights, copied out of the alternating result buffers
        return engine.adopt(weights), regVal


_CKPT_VERSION = 1


def _ckpt_fingerprint(params, data: PartitionedData, w0: np.ndarray) -> np.ndarray:
    """What an iteration's result depends on besides (w, i): the plugins and hyper-parameters
    (the psgd_params fields), the data's shape, the initial weights (the first regVal and the
    driver's first convergence reference). numIterations is left out, so a finished run can be
    resumed with a larger iteration budget and continue exactly where it stopped."""
    import hashlib
    h = hashlib.sha256()
    for f, _ in N.psgd_params._fields_:
        if f != "iteration":
            h.update(f"{f}={getattr(params, f)!r};".encode())
    h.update(f"n={data.count()};P={data.num_partitions};d={data.num_features};".encode())
    h.update(np.ascontiguousarray(w0, dtype=np.float64).tobytes())
    return np.frombuffer(h.digest(), dtype=np.uint8)


class DriverCheckpoint:
    """Checkpoint / resume of the driver loop (the reference has none and returns the
    weights only, ParallelizedSGD.scala:304). The loop's whole state between iterations is
    (weights, i, regVal, stochasticLossHistory, whether `currentWeights` is defined, converged):
    an epoch is a pure function of (weights, i, data) -- the sample seed is 42 + i (:240), every
    chain starts its updater status afresh (:246) -- so a resumed run continues bit for bit.

    Written by rank 0 only (every rank holds the same folded state), atomically (temp file +
    os.replace), as an .npz read back with allow_pickle=False."""

    def __init__(self, path: str, every: int = 1):
        _require(every >= 1, f"checkpoint interval must be positive but got {every}")
        self.path, self.every = str(path), int(every)

    def load(self, fingerprint: np.ndarray):
        """The saved loop state, or None. With world > 1 only rank 0 reads the file (it is the
        rank that writes it; other ranks may see a node-local path or none) and broadcasts the
        state, so every rank resumes at the same iteration; a rank whose own parameter/data
        fingerprint differs from rank 0's makes every rank raise, rather than issue mismatched
        collectives. The fingerprint covers the parameters, the data's shape and the initial
        weights, not the data's values."""
        rank, world, _ = _dist()
        state, err = None, None
        if rank == 0:
            try:
                state = self._read(fingerprint)
            except IllegalArgumentException as e:
                err = str(e)
            except Exception as e:   # unreadable file (truncated zip, old format, I/O error):
                # forwarded, so every rank raises after the broadcast instead of ranks >= 1
                # waiting in it for the process-group timeout
                err = f"checkpoint {self.path}: unreadable ({e!r})"
        if world > 1:
            import torch.distributed as dist
            box = [(state, err, np.asarray(fingerprint).tobytes())]
            dist.broadcast_object_list(box, src=0)
            state, err, fp0 = box[0]
            agree = [None] * world
            dist.all_gather_object(agree, fp0 == np.asarray(fingerprint).tobytes())
            if err is None and not all(agree):
                err = (f"checkpoint {self.path}: ranks {[r for r, a in enumerate(agree) if not a]} "
                       f"run with other parameters or data than rank 0")
        if err is not None:
            raise IllegalArgumentException(err)
        return state

    def _read(self, fingerprint: np.ndarray):
        import os
        if not os.path.exists(self.path):
            return None
        with np.load(self.path, allow_pickle=False) as z:
            if int(z["version"]) != _CKPT_VERSION or not np.array_equal(z["fingerprint"], fingerprint):
                raise IllegalArgumentException(
                    f"checkpoint {self.path} was written by a run with other parameters or data")
            return dict(weights=z["weights"].copy(), i=int(z["i"]), regVal=float(z["regVal"]),
                        history=[float(v) for v in z["history"]],
                        have_current=bool(z["have_current"]), converged=bool(z["converged"]))

    def save(self, fingerprint, weights_host, i, regVal, history, have_current, converged):
        import os
        rank, _, _ = _dist()
        if rank != 0:
            return
        tmp = f"{self.path}.tmp{os.getpid()}"
        with open(tmp, "wb") as f:
            np.savez(f, version=np.int64(_CKPT_VERSION), fingerprint=fingerprint,
                     weights=np.asarray(weights_host, dtype=np.float64), i=np.int64(i),
                     regVal=np.float64(regVal), history=np.asarray(history, dtype=np.float64),
                     have_current=np.bool_(have_current), converged=np.bool_(converged))
        os.replace(tmp, self.path)


def max_j(a: float, b: float) -> float:
    """java.lang.Math.max (NaN-propagating)."""
    if a != a:
        return a
    if b != b:
        return b
    return a if a >= b else b


runParallelizedSGD = ParallelizedSGD.runParallelizedSGD
