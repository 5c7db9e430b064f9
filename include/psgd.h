/*
 * psgd.h -- C ABI of the MI355X-native parallelized-SGD hot path.
 *
 * This is the drop-in boundary for the reference's per-partition SGD loop. The host (a Scala
 * shim over JNI/Panama, or the Python package in this repo over ctypes) keeps the driver loop of
 * ParallelizedSGD.runParallelizedSGD (ParallelizedSGD.scala:188-306) and replaces the
 * broadcast + mapPartitions + treeReduce block (ParallelizedSGD.scala:238-276) with one
 * psgd_run_epoch call per process and iteration.
 *
 * All file:line citations are into the reference (Patrickgsheng/spark-parallelized-sgd):
 *   PSGD = src/main/scala/org/apache/spark/mllib/optimization/ParallelizedSGD.scala
 *   UPD  = src/main/scala/org/apache/spark/mllib/optimization/SGDUpdater.scala
 *
 * Conventions: plain C types only; 0 = success, negative = error (psgd_last_error() holds the
 * thread-local message). PSGD_EINVAL maps to IllegalArgumentException on the JVM side (the
 * reference's `require` failures), everything else to RuntimeException.
 * Pointers named d_* are device pointers on the context's device; all others are host memory
 * owned by the caller. `stream` arguments are hipStream_t passed as void* (NULL = the context's
 * own stream).
 */
#ifndef PSGD_H
#define PSGD_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PSGD_ABI_VERSION 1

typedef struct psgd_ctx psgd_ctx;

/* Gradient plugins -- [ext] Spark MLlib 1.6.1 Gradient.scala; called at PSGD.scala:254. */
enum psgd_gradient {
    PSGD_GRADIENT_LOGISTIC = 0,      /* LogisticGradient(numClasses = 2) */
    PSGD_GRADIENT_LEAST_SQUARES = 1, /* LeastSquaresGradient */
    PSGD_GRADIENT_HINGE = 2          /* HingeGradient */
};

/* Updater plugins -- UPD.scala:40-286; called at PSGD.scala:255. */
enum psgd_updater {
    PSGD_UPDATER_SIMPLE = 0,     /* SimpleSGDUpdater      UPD.scala:80-99   */
    PSGD_UPDATER_SQUARED_L2 = 1, /* SquaredL2SGDUpdater   UPD.scala:157-182 */
    PSGD_UPDATER_L1 = 2,         /* L1SGDUpdater          UPD.scala:120-149 */
    PSGD_UPDATER_ADAGRAD = 3,    /* AdaGradSGDUpdater     UPD.scala:193-228 */
    PSGD_UPDATER_ADAM = 4        /* AdamSGDUpdater        UPD.scala:240-286 */
};

/* Element types. Storage dtype is chosen per registered partition; compute dtype per epoch:
 * PSGD_F64 reproduces the reference's double arithmetic (parity mode); PSGD_F32 computes the
 * chain in float (throughput mode, looser stated tolerance). */
enum psgd_dtype { PSGD_F64 = 0, PSGD_F32 = 1 };

enum psgd_status {
    PSGD_OK = 0,
    PSGD_EINVAL = -1,       /* bad argument (IllegalArgumentException) */
    PSGD_EUNSUPPORTED = -2, /* valid in the reference, not built here yet */
    PSGD_EDEVICE = -3,      /* HIP runtime failure */
    PSGD_ENOMEM = -4,
    PSGD_ESTATE = -5        /* call sequence error (e.g. no partitions registered) */
};

/* Hyper-parameters of one outer iteration (ParallelizedSGD.scala:46-50 defaults; validation
 * mirrors the setters' `require`s at :57-113). */
typedef struct {
    int32_t gradient;           /* enum psgd_gradient */
    int32_t updater;            /* enum psgd_updater */
    int32_t compute_dtype;      /* enum psgd_dtype */
    int32_t iteration;          /* outer iteration i (1-based), sampling seed 42+i (PSGD:242) */
    double step_size;           /* stepSize > 0 */
    double reg_param;           /* regParam >= 0 */
    double mini_batch_fraction; /* [0, 1]: batch = RDD.sample(false, f, 42 + iteration) per
                                   partition (BernoulliSampler [ext Spark 1.6.1]); 1 = every row */
    double convergence_tol;     /* [0, 1]; 0 disables the per-sample break (PSGD.scala:262) */
    double adam_beta, adam_gamma, adam_eps; /* AdamSGDUpdater(beta, gamma, eps), UPD:241-244 */
    int32_t num_classes;        /* LogisticGradient(numClasses) [ext MLlib 1.6.1]: <= 2 binary;
                                   K > 2 multinomial, weights of (K - 1) * d (class blocks of d),
                                   every weight-sized buffer of the epoch calls is (K - 1) * d;
                                   fp64 compute only */
} psgd_params;

int32_t psgd_abi_version(void);
const char* psgd_last_error(void);

/* Context: one device, its stream, the partition registry and all device buffers. */
int32_t psgd_ctx_create(int32_t device, psgd_ctx** out);
int32_t psgd_ctx_destroy(psgd_ctx* ctx);

/* Register partition `part` (its index in the RDD = its chain id) from host memory; the data
 * is copied to HBM once (the analogue of RDD.cache(), ParallelizedSGDSuite.scala:88) and no host
 * pointer is kept. Rows are in the partition's iterator order. labels[n_rows] are doubles;
 * x is row-major n_rows x d of `dtype`. Thread-safe (Spark local[N] registers from N task
 * threads; their copies run concurrently). Empty partitions (n_rows == 0) must be registered
 * too: they take part in the combine with count 0 (PSGD.scala:270-276). Replaces the
 * mapPartitions closure input at PSGD.scala:243-253.
 * Ingest: pinned sources (psgd_host_alloc) are DMA'd directly; pageable ones are packed through
 * a pinned staging ring, the DMA of one chunk overlapping the packing of the next, on a copy
 * stream of their own. The call returns once every copy it enqueued has landed in HBM (the
 * staging ring is drained before it goes back to the pool), so concurrent registrations from
 * several threads overlap each other, not the caller's next statement; an epoch that starts
 * while another thread's registration is in flight waits for it on the device. */
int32_t psgd_register_dense(psgd_ctx* ctx, int64_t part, int64_t n_rows, int32_t d,
                            const double* labels, const void* x, int32_t dtype);

/* Same for CSR rows: row_ptr[n_rows+1] (row_ptr[0] may be non-zero), col[] strictly
 * increasing within a row and < d, val[] of `dtype` (MLlib SparseVector rows). */
int32_t psgd_register_csr(psgd_ctx* ctx, int64_t part, int64_t n_rows, int32_t d,
                          const double* labels, const int64_t* row_ptr, const int32_t* col,
                          const void* val, int32_t dtype);

/* Zero-copy registration of a dense partition already resident on the context's device:
 * d_x row-major with leading dimension ld >= d elements (16-byte aligned rows; columns
 * [d, ld) must hold zeros), d_labels[n_rows]. The caller keeps both alive. */
int32_t psgd_register_dense_device(psgd_ctx* ctx, int64_t part, int64_t n_rows, int32_t d,
                                   int64_t ld, const double* d_labels, const void* d_x,
                                   int32_t dtype);

/* Zero-copy registration of a CSR partition already resident on the context's device:
 * d_row_ptr[n_rows+1] int64 absolute offsets into d_col/d_val (non-decreasing), d_col[] int32
 * strictly increasing within a row and < d, d_val[] of `dtype`, d_labels[n_rows]. The contents
 * are not validated (they are on the device); the caller keeps the buffers alive. */
int32_t psgd_register_csr_device(psgd_ctx* ctx, int64_t part, int64_t n_rows, int32_t d,
                                 const double* d_labels, const int64_t* d_row_ptr,
                                 const int32_t* d_col, const void* d_val, int32_t dtype);

/* Page-locked host buffers for packing partitions in place (the JVM shim wraps them as direct
 * ByteBuffers, NewDirectByteBuffer): registration from them skips the staging copy. */
int32_t psgd_host_alloc(psgd_ctx* ctx, int64_t bytes, void** out);
int32_t psgd_host_free(psgd_ctx* ctx, void* p);

/* Block until every registration copy enqueued so far has landed in HBM. */
int32_t psgd_register_wait(psgd_ctx* ctx);

int32_t psgd_clear_partitions(psgd_ctx* ctx);
int32_t psgd_num_partitions(psgd_ctx* ctx, int64_t* n_parts, int64_t* n_rows_total);

/* One outer iteration over this process's partitions (PSGD.scala:238-276):
 * every chain starts from w_in (the broadcast, :238/:245), runs its partition in iterator
 * order with j restarting at 1 (:243-269), and the chains' (w, regVal, lossSum, count) are
 * folded with the reference's combiner (:271-276) in partition-index order.
 * Host pointers: w_in[d] -> w_out[d] (the fold's averaged weights), *regval_out, *loss_sum_out,
 * *count_out; chain_counts[n_parts] (nullable) receives each chain's processed count.
 * A count of 0 means an empty batch (:295-297): the caller keeps its weights. */
int32_t psgd_run_epoch(psgd_ctx* ctx, const psgd_params* params, const double* w_in,
                       double* w_out, double* regval_out, double* loss_sum_out,
                       int64_t* count_out, int64_t* chain_counts);

/* Device-resident form of psgd_run_epoch for hosts that keep the weights in HBM across
 * iterations (the broadcast at PSGD.scala:238 disappears): d_w_in[d] on the device;
 * d_partial[d+3] receives {w_avg[0..d), regVal, lossSum, (double)count}; d_chain_counts
 * (nullable) [n_parts] int64. Enqueued on `stream`; no host synchronisation. */
int32_t psgd_run_epoch_device(psgd_ctx* ctx, const psgd_params* params, const double* d_w_in,
                              double* d_partial, int64_t* d_chain_counts, void* stream);

/* psgd_run_epoch_device whose fold kernel also writes {regVal, lossSum, (double)count} to
 * h_scalars[3], page-locked host memory (psgd_host_alloc; nullable): no copy is enqueued. The
 * count is stored last, with release order: a host that set h_scalars[2] to a value no count
 * takes (e.g. -1) before the call may poll it and then read the other two; or it waits for an
 * event recorded after the call. For a host loop that keeps several epochs in flight. */
int32_t psgd_run_epoch_device_mirror(psgd_ctx* ctx, const psgd_params* params, const double* d_w_in,
                                     double* d_partial, int64_t* d_chain_counts, void* stream,
                                     double* h_scalars);

/* Fold n per-process partials (each d+3 doubles, laid out back to back, in rank order) with
 * the reference's combiner (PSGD.scala:271-276) into d_out[d+3]: the cross-GPU level of the
 * treeReduce, applied after an all-gather of the partials. The _mirror form also writes the
 * folded {regVal, lossSum, count} to h_scalars[3] as psgd_run_epoch_device_mirror does. */
int32_t psgd_fold_partials_device(psgd_ctx* ctx, int32_t n, int32_t d, const double* d_partials,
                                  double* d_out, void* stream);
int32_t psgd_fold_partials_device_mirror(psgd_ctx* ctx, int32_t n, int32_t d, const double* d_partials,
                                         double* d_out, void* stream, double* h_scalars);

/* Driver-side isConverged terms (PSGD.scala:289-294, :324-336): writes
 * {sum((prev-cur)^2), sum(cur^2)} to h_out[2] (host) after synchronising `stream`. */
int32_t psgd_convergence_terms_device(psgd_ctx* ctx, int32_t d, const double* d_prev,
                                      const double* d_cur, double* h_out, void* stream);

/* Updater regVal at iteration 0 (PSGD.scala:231-233): updater.compute(w, 0, 0, 1, reg)._2 for
 * host weights w[d], computed on the context's device. */
int32_t psgd_initial_regval(psgd_ctx* ctx, const psgd_params* params, int32_t d, const double* w,
                            double* regval_out);

/* Diagnostics: which chain kernel the last epoch launched (DESIGN.md §3 has the table):
 * 100 + NV   per-sample dense chain (chain_dense), NV 16-byte row vectors per lane;
 * 200 / 201  general dense / CSR chain (chain_general);
 * 300 + NV   blocked fp32 dense chain (chain_block); 340 + NV with the per-sample break (tol > 0);
 * 400 / 410 / 420 + storage   fp32 CSR (chain_sparse / chain_sparse_spec), fp64 CSR with HBM
 *            weights (chain_sparse64); +40 with the per-sample break (440, 460);
 * 500 + layout  multinomial LogisticGradient (chain_multinomial);
 * 600 + 10 (SK = 8) + 20 (fp64) + storage   CSR with LDS-resident weights (chain_sparse_lds);
 *            +40 with the per-sample break;
 * 700 + 10 (H - 1) + NV   blocked fp64 dense chain (chain_block64, H chain waves); +40 with the
 *            per-sample break;
 * 800 + 10 H + NV   per-sample dense chain with features over H waves (chain_split).
 * storage: 1 = f32 rows, 0 = f64 rows. */
int32_t psgd_ctx_last_kernel(psgd_ctx* ctx);

/* Diagnostics: device time of the last chain-kernel launch in milliseconds, from HIP events
 * recorded around it on the launch stream (waits for that launch to finish). */
int32_t psgd_ctx_last_chain_ms(psgd_ctx* ctx, double* ms_out);

/* Diagnostics: the number of chain-kernel launches the context has made, and the device time of
 * launch `launch` (0-based, one of the last 64; waits for it to finish) -- for a caller that
 * keeps several epochs in flight and reads their times afterwards. */
int64_t psgd_ctx_chain_launches(psgd_ctx* ctx);
int32_t psgd_ctx_chain_ms(psgd_ctx* ctx, int64_t launch, double* ms_out);

/* Diagnostics (no reference counterpart): process-wide counters of the virtual-memory mappings
 * that hold the CSR chains' large weight vectors (PSGD_VMM): out4[0] chunks mapped, [1] chunks
 * unmapped, [2] bytes currently mapped, [3] failed unmap / release / address-free calls. */
int32_t psgd_vmm_stats(int64_t* out4);

/* Diagnostics (no reference counterpart): process-wide counters of the placement re-roll of the
 * CSR chains' weight-vector sets below the VMM threshold (PSGD_REROLL candidates):
 * out2[0] sets probed, [1] sets where a later candidate was kept. */
int32_t psgd_reroll_stats(int64_t* out2);

/* The device sampler of one partition, alone: RDD.sample(false, fraction, .) over a partition
 * of n rows whose PartitionwiseSampledRDD seed is `seed` (the partition's java.util.Random
 * nextLong, before hashSeed) [ext Spark 1.6.1 BernoulliSampler] -- the batch selection
 * psgd_run_epoch does for miniBatchFraction < 1 (PSGD.scala:242). Writes the kept row indices
 * in iterator order to rows_out[0..*m_out) (rows_out holds n entries). Same contract as
 * oracle/or_sample_partition. */
int32_t psgd_sample_partition(int32_t device, int64_t seed, int64_t n, double fraction, int32_t* rows_out,
                              int64_t* m_out);

/* LIBSVM text ingest (the caller side of the path: MLUtils.loadLibSVMFile(sc, path,
 * numFeatures, minPartitions) [ext Spark MLlib 1.6.1] building the RDD passed to
 * runParallelizedSGD, PSGD.scala:188). Partitions follow sc.textFile(path, minPartitions) on a
 * local file (Hadoop FileInputFormat splits, LineRecordReader line ownership); rows in file
 * order; 1-based indices become 0-based and must be strictly increasing per line;
 * num_features <= 0 infers max index + 1. Host arrays, freed by psgd_libsvm_free. */
typedef struct {
    int64_t n_rows;
    int32_t d;
    int32_t n_parts;
    int64_t* part_offsets;  /* [n_parts + 1] row offsets of the partitions */
    double* labels;         /* [n_rows] */
    int64_t* row_ptr;       /* [n_rows + 1] */
    int32_t* col;           /* [nnz] */
    double* val;            /* [nnz] */
} psgd_libsvm;

int32_t psgd_libsvm_read(const char* path, int32_t num_features, int32_t min_partitions,
                         psgd_libsvm** out);
void psgd_libsvm_free(psgd_libsvm* data);

#ifdef __cplusplus
}
#endif
#endif /* PSGD_H */
