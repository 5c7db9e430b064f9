/*
 * psgd_oracle.h -- CPU restatement of the reference's parallelized-SGD hot path.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library; the product path never does.
 *
 * Parity status: PARTIALLY PINNED. The reference (Scala 2.10/2.11 on Spark 1.6.1) cannot be
 * built or run here (no JVM, no jars, no network). The restatement is pinned against the
 * reference suite's own known-answer properties (ParallelizedSGDSuite.scala:101, :132-141, :180)
 * and cross-checked bit-for-bit against an independent pure-Python restatement
 * (oracle/psgd_ref.py). Absolute weight/loss values are otherwise unpinned.
 *
 * Semantics restated (all file:line are into /root/reference):
 *   driver loop            ParallelizedSGD.scala:188-306
 *   chain (mapPartitions)  ParallelizedSGD.scala:243-270
 *   combine (treeReduce)   ParallelizedSGD.scala:271-276
 *   isConverged            ParallelizedSGD.scala:324-336
 *   updaters               SGDUpdater.scala:86-98 (Simple), :126-148 (L1), :163-181 (SquaredL2),
 *                          :199-227 (AdaGrad), :252-285 (Adam)
 *   gradients              [ext] Spark MLlib 1.6.1 mllib/optimization/Gradient.scala
 *                          (LogisticGradient binary and multinomial, LeastSquaresGradient,
 *                          HingeGradient),
 *                          with BLAS.dot/axpy/scal on netlib-java F2J ddot/daxpy/dscal
 *                          (sequential left folds, no fused multiply-add) and
 *                          MLUtils.log1pExp.
 */
#ifndef PSGD_ORACLE_H
#define PSGD_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { OR_GRAD_LOGISTIC = 0, OR_GRAD_LEAST_SQUARES = 1, OR_GRAD_HINGE = 2 };
enum { OR_UPD_SIMPLE = 0, OR_UPD_SQUARED_L2 = 1, OR_UPD_L1 = 2, OR_UPD_ADAGRAD = 3, OR_UPD_ADAM = 4 };

/* Combine order for the per-partition results (ParallelizedSGD.scala:271-276).
 * group_offsets (nullable) splits the chains into contiguous groups: each group is
 * left-folded in chain order, then the group results are left-folded in group order
 * (a two-level tree, the order the multi-GPU build uses: chains within a GPU, then GPUs). */

/* One partition = rows [row_begin, row_end) of a global matrix, in iterator order.
 * Dense: X is row-major with leading dimension ld (>= d).
 * CSR:   row_ptr[N+1] (global), col/val indexed by row_ptr; indices strictly increasing. */
typedef struct {
    int64_t n_total;       /* N rows in the global matrix */
    int32_t d;
    int32_t is_csr;
    const double* labels;  /* [N] */
    const double* X;       /* dense [N*ld] */
    int64_t ld;
    const int64_t* row_ptr;
    const int32_t* col;
    const double* val;
} or_matrix;

typedef struct {
    int32_t gradient;
    int32_t updater;
    double step_size;
    double reg_param;
    double convergence_tol;
    double adam_beta, adam_gamma, adam_eps;
    double mini_batch_fraction;   /* RDD.sample(false, f, 42 + i) per iteration (PSGD.scala:242) */
    int32_t num_classes;          /* LogisticGradient(numClasses): <= 2 binary; > 2 multinomial,
                                     weights are (numClasses - 1) blocks of d */
} or_params;

/* Length of the weight vector: d, or (numClasses - 1) * d for the multinomial LogisticGradient. */
int32_t or_weight_dim(int32_t d, const or_params* prm);

/* One chain (ParallelizedSGD.scala:243-270) over rows [r0, r1). */
int or_chain(const or_matrix* m, int64_t r0, int64_t r1, const or_params* prm,
             const double* w_in, double* w_out, double* rv_out, double* loss_out,
             int64_t* count_out);

/* Reference pairwise combine (ParallelizedSGD.scala:271-276), in place into acc. */
void or_combine(int32_t d, double* acc_w, double* acc_rv, double* acc_loss, int64_t* acc_c,
                const double* w2, double rv2, double loss2, int64_t c2);

/* isConverged (ParallelizedSGD.scala:324-336). */
int or_is_converged(int32_t d, const double* prev, const double* cur, double tol);

/* Updater regVal at iteration 0 (ParallelizedSGD.scala:231-233). */
double or_initial_regval(int32_t d, const double* w, const or_params* prm);

/* Full driver (ParallelizedSGD.scala:188-306), prm->mini_batch_fraction sampling included.
 * part_offsets[P+1]: partition p holds rows [part_offsets[p], part_offsets[p+1]).
 * Returns number of loss-history entries in *n_hist (<= num_iterations).
 * chain_counts (nullable): [num_iterations * P], per-iteration per-chain processed counts.
 * n_threads: worker threads for the chains (results do not depend on it). */
int or_run(const or_matrix* m, int32_t P, const int64_t* part_offsets,
           const int32_t* group_offsets, int32_t n_groups,
           const or_params* prm, int32_t num_iterations, const double* w0,
           double* w_out, double* loss_hist, int32_t* n_hist, int64_t* chain_counts,
           int32_t n_threads);

/* One epoch of chains only (no combine): per-chain outputs, for the CPU baseline timer. */
int or_run_chains(const or_matrix* m, int32_t P, const int64_t* part_offsets,
                  const int64_t* part_limits, const or_params* prm, const double* w_in,
                  double* w_out /*[P*d]*/, double* rv_out, double* loss_out, int64_t* count_out,
                  int32_t n_threads);

/* Break-margin probe (test infrastructure): buf[iters * P], initialised by the caller (e.g. to
 * +inf), receives per (outer iteration, chain) the smallest |diff / (tol max(norm, 1)) - 1| over
 * the chain's isConverged tests; NULL turns it off. or_set_ratio_trace records, for one chain of
 * the first iteration, r = diff / max(norm, 1) of every sample (up to cap values). */
void or_set_margin_probe(double* buf, int32_t iters, int32_t P);
void or_set_ratio_trace(int32_t chain, double* buf, int64_t cap);
int64_t or_ratio_trace_len(void);

/* fp32 restatement switch (test infrastructure): on != 0 runs dense Simple / SquaredL2 chains
 * with binary gradients in IEEE single precision (same operations, float operands; loss and regVal
 * accumulated in double) -- the reference of what a sequential fp32 evaluation of the chain gives.
 * order 0: the dot as a left fold; 1: 64 strided partials + a pairwise tree; 2: only the weights
 * in float (dot and multiplier in double, updates rounded to float; tol = 0 only). Not thread-safe
 * across callers (one global switch); the driver and fold stay in double. */
void or_set_f32_chain(int32_t on, int32_t order);

/* RDD.sample(false, fraction, seed) [ext Spark 1.6.1]: the per-partition seeds
 * (java.util.Random(seed).nextLong() in partition order), XORShiftRandom.hashSeed, and the
 * BernoulliSampler's row selection for one partition of n rows (returns the count, writes the
 * selected row offsets 0..n-1 in iterator order). */
void or_partition_seeds(int64_t seed, int32_t P, int64_t* out);
int64_t or_xorshift_hash_seed(int64_t s);
int64_t or_sample_partition(int64_t seed, int64_t n, double fraction, int32_t* rows_out);

/* java.util.Random + StrictMath.log (fdlibm) restatements, for the suite's data generator
 * (ParallelizedSGDSuite.scala:42-62). */
double or_fdlibm_log(double x);
void or_generate_gd_input(double offset, double scale, int32_t n, int32_t seed,
                          double* x_out, double* y_out);
void or_jrandom_doubles(int64_t seed, int32_t n, double* out);
void or_jrandom_gaussians(int64_t seed, int32_t n, double* out);

#ifdef __cplusplus
}
#endif
#endif
