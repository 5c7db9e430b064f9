/*
 * psgd_oracle.c -- CPU restatement of the reference's parallelized-SGD hot path (fp64).
 *
 * TEST INFRASTRUCTURE ONLY (see psgd_oracle.h). Build with -ffp-contract=off: Java never fuses
 * a multiply into an add, and every expression below is written in the reference's evaluation
 * order (Scala/Java evaluate left to right, one rounding per operator).
 *
 * Parity status: PARTIALLY PINNED -- see psgd_oracle.h and DESIGN.md §Oracle.
 */
#include "psgd_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------------
 * Level-1 BLAS as the reference reaches it.
 * [ext] MLlib 1.6.1 BLAS.dot(dense, dense) -> netlib F2J ddot: the unit-stride loop is
 * unrolled by 5 but written `dtemp + a + b + c + d + e`, i.e. a plain left fold.
 * [ext] MLlib 1.6.1 BLAS.dot(sparse, dense): `sum += xValues(k) * yValues(xIndices(k))`.
 * ------------------------------------------------------------------------------------------ */
static double dot_dense(int32_t d, const double* x, const double* w) {
    double s = 0.0;
    for (int32_t i = 0; i < d; ++i) s = s + x[i] * w[i];
    return s;
}
static double dot_sparse(int64_t nnz, const int32_t* idx, const double* v, const double* w) {
    double s = 0.0;
    for (int64_t k = 0; k < nnz; ++k) s = s + v[k] * w[idx[k]];
    return s;
}

/* Breeze norm(v, 2.0) for a DenseVector[Double] [ext, Breeze 0.11]: sqrt of a sequential sum of
 * squares. */
static double norm2(int32_t d, const double* x) {
    double s = 0.0;
    for (int32_t i = 0; i < d; ++i) s = s + x[i] * x[i];
    return sqrt(s);
}
static double norm1(int32_t d, const double* x) {
    double s = 0.0;
    for (int32_t i = 0; i < d; ++i) s = s + fabs(x[i]);
    return s;
}

/* java.lang.Math.max(double, double): NaN if either argument is NaN. */
static double jmax(double a, double b) {
    if (a != a) return a;
    if (b != b) return b;
    return a >= b ? a : b;
}
/* java.lang.Math.signum */
static double jsignum(double x) {
    if (x != x || x == 0.0) return x;
    return x > 0.0 ? 1.0 : -1.0;
}

/* [ext] MLlib 1.6.1 MLUtils.log1pExp */
static double log1p_exp(double x) {
    if (x > 0.0) return x + log1p(exp(-x));
    return log1p(exp(x));
}

/* ------------------------------------------------------------------------------------------
 * isConverged -- ParallelizedSGD.scala:324-336.
 * ------------------------------------------------------------------------------------------ */
int or_is_converged(int32_t d, const double* prev, const double* cur, double tol) {
    double s = 0.0;
    for (int32_t i = 0; i < d; ++i) {
        double t = prev[i] - cur[i];
        s = s + t * t;
    }
    double diff = sqrt(s);
    return diff < tol * jmax(norm2(d, cur), 1.0);
}

/* ------------------------------------------------------------------------------------------
 * Break-margin probe (test infrastructure only). isConverged decides
 * `diff < tol * max(norm, 1)`; the decision flips only if `rho = diff / (tol * max(norm, 1))`
 * crosses 1. When a probe is set, every per-sample test of chain p in outer iteration i (1-based;
 * 1 for or_run_chains) lowers g_margin[(i - 1) * P + p] to |rho - 1|, the relative distance of that
 * decision from flipping; and every sample of chain g_trace_chain in iteration 1 appends the
 * tol-free r = diff / max(norm, 1) to g_trace. The decisions themselves are unchanged.
 * ------------------------------------------------------------------------------------------ */
static double* g_margin = NULL;
static int32_t g_margin_iters = 0, g_margin_P = 0, g_iter = 1;
static double* g_trace = NULL;
static int64_t g_trace_cap = 0, g_trace_n = 0;
static int32_t g_trace_chain = -1;

void or_set_margin_probe(double* buf, int32_t iters, int32_t P) {
    g_margin = buf;
    g_margin_iters = iters;
    g_margin_P = P;
}

void or_set_ratio_trace(int32_t chain, double* buf, int64_t cap) {
    g_trace_chain = buf ? chain : -1;
    g_trace = buf;
    g_trace_cap = cap;
    g_trace_n = 0;
}

int64_t or_ratio_trace_len(void) { return g_trace_n; }

/* or_is_converged with the probe's bookkeeping for chain p (p < 0: none) */
static int is_converged_probed(int32_t d, const double* prev, const double* cur, double tol, int32_t p) {
    if (p < 0 || (!g_margin && !(g_trace && p == g_trace_chain && g_iter == 1)))
        return or_is_converged(d, prev, cur, tol);
    double s = 0.0;
    for (int32_t i = 0; i < d; ++i) {
        double t = prev[i] - cur[i];
        s = s + t * t;
    }
    const double diff = sqrt(s), den = jmax(norm2(d, cur), 1.0), rhs = tol * den;
    const int conv = diff < rhs;
    if (g_margin && p < g_margin_P && g_iter >= 1 && g_iter <= g_margin_iters && rhs > 0.0) {
        double* m = &g_margin[(size_t)(g_iter - 1) * (size_t)g_margin_P + (size_t)p];
        const double dist = fabs(diff / rhs - 1.0);
        if (dist < *m) *m = dist;
    }
    if (g_trace && p == g_trace_chain && g_iter == 1 && g_trace_n < g_trace_cap) g_trace[g_trace_n++] = diff / den;
    return conv;
}

/* ------------------------------------------------------------------------------------------
 * Per-sample gradient, one row.  A gradient is either dense (g[d] valid) or sparse over the
 * row's own index set (gv[k] for idx[k]); an "empty sparse" gradient has nnz == 0.
 * ------------------------------------------------------------------------------------------ */
typedef struct {
    int is_dense;         /* dense: g[0..d) */
    int64_t nnz;          /* sparse: idx/gv */
    const int32_t* idx;
    double* gv;
    double* g;
} grad_t;

typedef struct {
    int32_t d;
    int is_csr;
    const double* x;       /* dense row */
    int64_t nnz;           /* csr row */
    const int32_t* idx;
    const double* val;
} row_t;

int32_t or_weight_dim(int32_t d, const or_params* prm) {
    if (prm->gradient == OR_GRAD_LOGISTIC && prm->num_classes > 2) return (prm->num_classes - 1) * d;
    return d;
}

/* Double.toInt (Java d2i): NaN -> 0, saturating, truncation toward zero. */
static int32_t java_d2i(double x) {
    if (x != x) return 0;
    if (x >= 2147483647.0) return 2147483647;
    if (x <= -2147483648.0) return (int32_t)(-2147483647 - 1);
    return (int32_t)x;
}

/* [ext] MLlib 1.6.1 LogisticGradient.compute(data, label, weights) for numClasses > 2: the
 * multinomial model with class 0 as pivot; weights are numClasses - 1 blocks of dataSize.
 * Margins over data.foreachActive skipping value == 0.0; the sum of exponentials shifted by
 * maxMargin when it is positive (the max class contributing exp(-maxMargin) for the pivot);
 * multiplier_i = exp(margin_i) / (sum + 1.0) - [label != 0 && label == i + 1];
 * cumGradient(i * dataSize + index) += multiplier_i * value over the non-zero values;
 * loss = log1p(sum) (- marginY when label > 0) (+ maxMargin when it is positive). The gradient
 * is dense (Vectors.zeros(weights.size)). margins holds numClasses - 1 doubles of scratch. */
static double multinomial_compute(int32_t K, const row_t* r, double label, const double* w,
                                  grad_t* out, double* margins) {
    const int32_t d = r->d, C1 = K - 1;
    const int32_t ly = java_d2i(label) - 1;   /* label.toInt - 1 */
    double marginY = 0.0, maxMargin = -INFINITY;
    int32_t maxMarginIndex = 0;
    for (int32_t i = 0; i < C1; ++i) {
        const double* wi = w + (size_t)i * (size_t)d;
        double margin = 0.0;
        if (r->is_csr) {
            for (int64_t k = 0; k < r->nnz; ++k)
                if (r->val[k] != 0.0) margin = margin + r->val[k] * wi[r->idx[k]];
        } else {
            for (int32_t j = 0; j < d; ++j)
                if (r->x[j] != 0.0) margin = margin + r->x[j] * wi[j];
        }
        if (i == ly) marginY = margin;
        if (margin > maxMargin) {
            maxMargin = margin;
            maxMarginIndex = i;
        }
        margins[i] = margin;
    }
    double sum = 0.0;
    if (maxMargin > 0) {
        for (int32_t i = 0; i < C1; ++i) {
            margins[i] = margins[i] - maxMargin;
            if (i == maxMarginIndex) sum = sum + exp(-maxMargin);
            else sum = sum + exp(margins[i]);
        }
    } else {
        for (int32_t i = 0; i < C1; ++i) sum = sum + exp(margins[i]);
    }
    out->is_dense = 1;
    memset(out->g, 0, sizeof(double) * (size_t)C1 * (size_t)d);
    for (int32_t i = 0; i < C1; ++i) {
        const double multiplier = exp(margins[i]) / (sum + 1.0) -
                                  ((label != 0.0 && label == (double)(i + 1)) ? 1.0 : 0.0);
        double* gi = out->g + (size_t)i * (size_t)d;
        if (r->is_csr) {
            for (int64_t k = 0; k < r->nnz; ++k)
                if (r->val[k] != 0.0) gi[r->idx[k]] = gi[r->idx[k]] + multiplier * r->val[k];
        } else {
            for (int32_t j = 0; j < d; ++j)
                if (r->x[j] != 0.0) gi[j] = gi[j] + multiplier * r->x[j];
        }
    }
    const double loss = label > 0.0 ? log1p(sum) - marginY : log1p(sum);
    return maxMargin > 0 ? loss + maxMargin : loss;
}

/* [ext] MLlib 1.6.1 Gradient.scala, binary LogisticGradient / LeastSquaresGradient /
 * HingeGradient compute(data, label, weights): (gradient, loss). */
static double gradient_compute(int kind, const row_t* r, double label, const double* w,
                               grad_t* out) {
    int32_t d = r->d;
    double dotv = r->is_csr ? dot_sparse(r->nnz, r->idx, r->val, w) : dot_dense(d, r->x, w);
    if (kind == OR_GRAD_LOGISTIC) {
        double margin = -1.0 * dotv;
        double multiplier = (1.0 / (1.0 + exp(margin))) - label;
        /* gradient = zeros(d); axpy(multiplier, data, gradient). F2J daxpy returns early when
         * da == 0.0 (dense); the sparse axpy has no early return. Both leave zeros. */
        out->is_dense = 1;
        memset(out->g, 0, sizeof(double) * (size_t)d);
        if (r->is_csr) {
            for (int64_t k = 0; k < r->nnz; ++k)
                out->g[r->idx[k]] = out->g[r->idx[k]] + multiplier * r->val[k];
        } else if (multiplier != 0.0) {
            for (int32_t i = 0; i < d; ++i) out->g[i] = out->g[i] + multiplier * r->x[i];
        }
        if (label > 0.0) return log1p_exp(margin);
        return log1p_exp(margin) - margin;
    }
    if (kind == OR_GRAD_LEAST_SQUARES) {
        double diff = dotv - label;
        double loss = diff * diff / 2.0;
        /* gradient = data.copy; scal(diff, gradient) */
        if (r->is_csr) {
            out->is_dense = 0;
            out->nnz = r->nnz;
            out->idx = r->idx;
            for (int64_t k = 0; k < r->nnz; ++k) out->gv[k] = diff * r->val[k];
        } else {
            out->is_dense = 1;
            for (int32_t i = 0; i < d; ++i) out->g[i] = diff * r->x[i];
        }
        return loss;
    }
    /* Hinge */
    {
        double labelScaled = 2 * label - 1.0;
        if (1.0 > labelScaled * dotv) {
            double a = -labelScaled;
            if (r->is_csr) {
                out->is_dense = 0;
                out->nnz = r->nnz;
                out->idx = r->idx;
                for (int64_t k = 0; k < r->nnz; ++k) out->gv[k] = a * r->val[k];
            } else {
                out->is_dense = 1;
                for (int32_t i = 0; i < d; ++i) out->g[i] = a * r->x[i];
            }
            return 1.0 - labelScaled * dotv;
        }
        out->is_dense = 0;   /* Vectors.sparse(weights.size, Array.empty, Array.empty) */
        out->nnz = 0;
        out->idx = NULL;
        return 0.0;
    }
}

/* Breeze axpy(a, x, y): y += a * x over x's active entries. */
static void axpy_grad(double a, const grad_t* g, int32_t d, double* w) {
    if (g->is_dense) {
        for (int32_t i = 0; i < d; ++i) w[i] = w[i] + a * g->g[i];
    } else {
        for (int64_t k = 0; k < g->nnz; ++k) w[g->idx[k]] = w[g->idx[k]] + a * g->gv[k];
    }
}

/* Expand a gradient to dense (the stateful updaters operate elementwise over all d; Breeze's
 * dense-op-sparse arithmetic gives the same numbers as operating on explicit zeros). */
static const double* dense_view(const grad_t* g, int32_t d, double* scratch) {
    if (g->is_dense) return g->g;
    memset(scratch, 0, sizeof(double) * (size_t)d);
    for (int64_t k = 0; k < g->nnz; ++k) scratch[g->idx[k]] = g->gv[k];
    return scratch;
}

typedef struct {
    int has;        /* Option defined */
    double* a;      /* AdaGrad accum / Adam v */
    double* b;      /* Adam r */
} upd_status;

/* SGDUpdater.compute(weightsOld, gradient, stepSize, iter, regParam, status) with w updated in
 * place (weightsOld.toBreeze.toDenseVector is a copy, so in place on the chain's private copy is
 * the same).  Returns regVal. */
static double updater_compute(const or_params* prm, double* w, int32_t d, const grad_t* g,
                              double stepSize, int64_t iter, upd_status* st, double* scratch) {
    double thisIterStepSize = stepSize / sqrt((double)iter);
    switch (prm->updater) {
    case OR_UPD_SIMPLE:  /* SGDUpdater.scala:86-98 */
        axpy_grad(-thisIterStepSize, g, d, w);
        return 0.0;
    case OR_UPD_SQUARED_L2: {  /* SGDUpdater.scala:163-181 */
        double c = 1.0 - thisIterStepSize * prm->reg_param;
        for (int32_t i = 0; i < d; ++i) w[i] = w[i] * c;
        axpy_grad(-thisIterStepSize, g, d, w);
        double nrm = norm2(d, w);
        return 0.5 * prm->reg_param * nrm * nrm;
    }
    case OR_UPD_L1: {  /* SGDUpdater.scala:126-148 */
        axpy_grad(-thisIterStepSize, g, d, w);
        double shrinkageVal = prm->reg_param * thisIterStepSize;
        for (int32_t i = 0; i < d; ++i) {
            double wi = w[i];
            w[i] = jsignum(wi) * jmax(0.0, fabs(wi) - shrinkageVal);
        }
        return norm1(d, w) * prm->reg_param;
    }
    case OR_UPD_ADAGRAD: {  /* SGDUpdater.scala:199-227 */
        const double* gd = dense_view(g, d, scratch);
        for (int32_t i = 0; i < d; ++i) {
            double sq = gd[i] * gd[i];
            st->a[i] = st->has ? st->a[i] + sq : sq;
        }
        st->has = 1;
        double a = -thisIterStepSize;
        /* pow(x, 0.5): fdlibm e_pow.c returns sqrt(x) for y == 0.5, x >= 0 */
        for (int32_t i = 0; i < d; ++i) w[i] = w[i] + a * (gd[i] / sqrt(st->a[i] + 1.0));
        return 0.0;
    }
    case OR_UPD_ADAM: {  /* SGDUpdater.scala:252-285 */
        const double* gd = dense_view(g, d, scratch);
        double beta = prm->adam_beta, gamma = prm->adam_gamma;
        for (int32_t i = 0; i < d; ++i) {
            double sq = gd[i] * gd[i];
            if (!st->has) {
                st->a[i] = gd[i] * (1 - beta);
                st->b[i] = sq * (1 - gamma);
            } else {
                st->a[i] = st->a[i] * beta + gd[i] * (1 - beta);
                st->b[i] = st->b[i] * gamma + sq * (1 - gamma);
            }
        }
        st->has = 1;
        double learningRate = thisIterStepSize / (1.0 - pow(beta, (double)iter));
        double a = -learningRate;
        for (int32_t i = 0; i < d; ++i) {
            double fix1 = sqrt(1.0 - pow(st->b[i], (double)iter)) + prm->adam_eps;
            w[i] = w[i] + a * (st->a[i] / fix1);
        }
        return 0.0;
    }
    default:
        return 0.0;
    }
}

double or_initial_regval(int32_t d, const double* w, const or_params* prm) {
    /* updater.compute(weights, Vectors.zeros(n), 0, 1, regParam, initStatus())._2
     * (ParallelizedSGD.scala:231-233) */
    double* tmp = (double*)malloc(sizeof(double) * (size_t)(d > 0 ? d : 1) * 4);
    double* g = tmp + d;
    double* sa = tmp + 2 * (size_t)d;
    double* sb = tmp + 3 * (size_t)d;
    memcpy(tmp, w, sizeof(double) * (size_t)d);
    memset(g, 0, sizeof(double) * (size_t)d);
    grad_t gr = {1, 0, NULL, NULL, g};
    upd_status st = {0, sa, sb};
    double rv = updater_compute(prm, tmp, d, &gr, 0.0, 1, &st, sa);
    free(tmp);
    return rv;
}

/* ------------------------------------------------------------------------------------------
 * The chain -- ParallelizedSGD.scala:243-270.
 * ------------------------------------------------------------------------------------------ */
/* The chain over rows r0 + k, k = 0..r1-r0-1, or over rows[k] (absolute row indices, the
 * partition's sampled subsequence in iterator order) when rows is not null. */
static int chain_rows(const or_matrix* m, int64_t r0, int64_t r1, const int32_t* rows,
                      const or_params* prm, const double* w_in, double* w_out, double* rv_out,
                      double* loss_out, int64_t* count_out, int32_t p) {
    const int32_t d = or_weight_dim(m->d, prm);   /* weights; rows have m->d features */
    const int32_t K = prm->gradient == OR_GRAD_LOGISTIC && prm->num_classes > 2 ? prm->num_classes : 0;
    size_t nd = (size_t)(d > 0 ? d : 1);
    int64_t max_nnz = 0;
    if (m->is_csr)
        for (int64_t q = r0; q < r1; ++q) {
            int64_t r = rows ? rows[q - r0] : q;
            int64_t z = m->row_ptr[r + 1] - m->row_ptr[r];
            if (z > max_nnz) max_nnz = z;
        }
    double* buf = (double*)malloc(sizeof(double) * (nd * 6 + (size_t)max_nnz + 1 + (size_t)K));
    if (!buf) return -1;
    double* w = buf;
    double* old = buf + nd;
    double* g = buf + 2 * nd;
    double* scratch = buf + 3 * nd;
    double* sa = buf + 4 * nd;
    double* sb = buf + 5 * nd;
    double* gv = buf + 6 * nd;
    double* margins = gv + max_nnz + 1;

    memcpy(w, w_in, sizeof(double) * (size_t)d);   /* localWeights = bcWeights.value */
    memcpy(old, w_in, sizeof(double) * (size_t)d); /* oldWeights   = bcWeights.value */
    upd_status st = {0, sa, sb};                   /* updater.initStatus() */
    double localRegVal = 0.0, localLossSum = 0.0;
    int64_t count = 0;
    int64_t j = 1;
    grad_t gr;
    gr.g = g;
    gr.gv = gv;
    row_t row;
    memset(&row, 0, sizeof(row));
    row.d = m->d;
    row.is_csr = m->is_csr;
    for (int64_t q = r0; q < r1; ++q) {
        const int64_t r = rows ? rows[q - r0] : q;
        if (m->is_csr) {
            int64_t b = m->row_ptr[r], e = m->row_ptr[r + 1];
            row.nnz = e - b;
            row.idx = m->col + b;
            row.val = m->val + b;
        } else {
            row.x = m->X + (size_t)r * (size_t)m->ld;
        }
        double loss = K ? multinomial_compute(K, &row, m->labels[r], w, &gr, margins)
                        : gradient_compute(prm->gradient, &row, m->labels[r], w, &gr);
        localRegVal = updater_compute(prm, w, d, &gr, prm->step_size, j, &st, scratch);
        localLossSum += loss;
        count += 1;
        j += 1;
        if (is_converged_probed(d, old, w, prm->convergence_tol, p)) break;
        memcpy(old, w, sizeof(double) * (size_t)d);
    }
    memcpy(w_out, w, sizeof(double) * (size_t)d);
    *rv_out = localRegVal;
    *loss_out = localLossSum;
    *count_out = count;
    free(buf);
    return 0;
}

int or_chain(const or_matrix* m, int64_t r0, int64_t r1, const or_params* prm,
             const double* w_in, double* w_out, double* rv_out, double* loss_out,
             int64_t* count_out) {
    return chain_rows(m, r0, r1, NULL, prm, w_in, w_out, rv_out, loss_out, count_out, -1);
}

/* ------------------------------------------------------------------------------------------
 * The same chain in IEEE single precision (test infrastructure: VERDICT r05 item 1, the
 * float-arithmetic restatement that separates the fp32 trajectory's own sensitivity from a
 * kernel defect). Dense rows, binary gradients, Simple / SquaredL2 only; every operation of
 * chain_rows / gradient_compute / updater_compute above in the same order with float operands
 * (w, the dot, the multiplier, the gradient and the step rounded to float), the loss and regVal
 * accumulated in double from the float quantities. g_f32_order selects the dot's summation:
 * 0 = F2J's left fold (ddot), 1 = 64 strided partial sums combined by a pairwise tree (a
 * wavefront64's order) -- two equally valid fp32 evaluations of the same chain; 2 = only the
 * weights float (dot, multiplier and step in double, each coordinate's update rounded to float
 * once; tol = 0 only) -- the error of fp32 weight storage alone.
 * ------------------------------------------------------------------------------------------ */
static int g_f32 = 0, g_f32_order = 0;

void or_set_f32_chain(int32_t on, int32_t order) {
    g_f32 = on;
    g_f32_order = order;
}

static float dot_f32(int32_t d, const float* x, const float* w) {
    if (g_f32_order == 0) {
        float s = 0.0f;
        for (int32_t i = 0; i < d; ++i) s = s + x[i] * w[i];
        return s;
    }
    float part[64];
    for (int l = 0; l < 64; ++l) part[l] = 0.0f;
    for (int32_t i = 0; i < d; ++i) part[i & 63] = part[i & 63] + x[i] * w[i];
    for (int h = 32; h >= 1; h >>= 1)
        for (int l = 0; l < h; ++l) part[l] = part[l] + part[l + h];
    return part[0];
}

static int chain_rows_f32(const or_matrix* m, int64_t r0, int64_t r1, const or_params* prm,
                          const double* w_in, double* w_out, double* rv_out, double* loss_out,
                          int64_t* count_out) {
    const int32_t d = m->d;
    size_t nd = (size_t)(d > 0 ? d : 1);
    float* buf = (float*)malloc(sizeof(float) * nd * 4);
    if (!buf) return -1;
    float *w = buf, *old = buf + nd, *x = buf + 2 * nd, *g = buf + 3 * nd;
    for (int32_t i = 0; i < d; ++i) w[i] = (float)w_in[i];
    memcpy(old, w, sizeof(float) * nd);
    double localRegVal = 0.0, localLossSum = 0.0;
    int64_t count = 0, j = 1;
    for (int64_t r = r0; r < r1; ++r) {
        const double* xr = m->X + (size_t)r * (size_t)m->ld;
        for (int32_t i = 0; i < d; ++i) x[i] = (float)xr[i];
        const float label = (float)m->labels[r];
        if (g_f32_order == 2) {
            /* order 2: only the weights are float -- dot, multiplier and step in double, each
             * coordinate's update rounded to float once (isolates the weight-storage rounding) */
            double dd = 0.0;
            for (int32_t i = 0; i < d; ++i) dd = dd + (double)x[i] * (double)w[i];
            row_t rw;
            memset(&rw, 0, sizeof rw);
            double mlt, ls;
            if (prm->gradient == OR_GRAD_LOGISTIC) {
                mlt = (1.0 / (1.0 + exp(-dd))) - m->labels[r];
                ls = m->labels[r] > 0.0 ? log1p_exp(-dd) : log1p_exp(-dd) + dd;
            } else if (prm->gradient == OR_GRAD_LEAST_SQUARES) {
                mlt = dd - m->labels[r];
                ls = mlt * mlt / 2.0;
            } else {
                const double ys = 2 * m->labels[r] - 1.0;
                mlt = 1.0 > ys * dd ? -ys : 0.0;
                ls = 1.0 > ys * dd ? 1.0 - ys * dd : 0.0;
            }
            const double st = prm->step_size / sqrt((double)j);
            const double c2 = prm->updater == OR_UPD_SQUARED_L2 ? 1.0 - st * prm->reg_param : 1.0;
            for (int32_t i = 0; i < d; ++i) w[i] = (float)((double)w[i] * c2 + (-st) * (mlt * (double)x[i]));
            localRegVal = 0.0;
            if (prm->updater == OR_UPD_SQUARED_L2) {
                double s2 = 0.0;
                for (int32_t i = 0; i < d; ++i) s2 = s2 + (double)w[i] * (double)w[i];
                localRegVal = 0.5 * prm->reg_param * s2;
            }
            localLossSum += ls;
            count += 1;
            j += 1;
            continue;   /* no per-sample test in this probe (tol = 0 only) */
        }
        const float dotv = dot_f32(d, x, w);
        float mult;
        double loss;
        int dense_grad = 1;
        if (prm->gradient == OR_GRAD_LOGISTIC) {
            const float margin = -1.0f * dotv;
            mult = (1.0f / (1.0f + expf(margin))) - label;
            loss = label > 0.0f ? log1p_exp((double)margin) : log1p_exp((double)margin) - (double)margin;
        } else if (prm->gradient == OR_GRAD_LEAST_SQUARES) {
            mult = dotv - label;
            loss = (double)mult * (double)mult / 2.0;
        } else {
            const float labelScaled = 2.0f * label - 1.0f;
            if (1.0f > labelScaled * dotv) {
                mult = -labelScaled;
                loss = 1.0 - (double)labelScaled * (double)dotv;
            } else {
                mult = 0.0f;
                loss = 0.0;
                dense_grad = 0;
            }
        }
        for (int32_t i = 0; i < d; ++i) g[i] = mult * x[i];
        const float step = (float)(prm->step_size / sqrt((double)j));
        if (prm->updater == OR_UPD_SQUARED_L2) {
            const float c = (float)(1.0 - (double)step * prm->reg_param);
            for (int32_t i = 0; i < d; ++i) w[i] = w[i] * c;
        }
        if (dense_grad)
            for (int32_t i = 0; i < d; ++i) w[i] = w[i] + (-step) * g[i];
        if (prm->updater == OR_UPD_SQUARED_L2) {
            double s = 0.0;
            for (int32_t i = 0; i < d; ++i) s = s + (double)w[i] * (double)w[i];
            localRegVal = 0.5 * prm->reg_param * s;
        } else {
            localRegVal = 0.0;
        }
        localLossSum += loss;
        count += 1;
        j += 1;
        double s = 0.0, n2 = 0.0;
        for (int32_t i = 0; i < d; ++i) {
            const double t = (double)old[i] - (double)w[i];
            s = s + t * t;
            n2 = n2 + (double)w[i] * (double)w[i];
        }
        if (sqrt(s) < prm->convergence_tol * jmax(sqrt(n2), 1.0)) break;
        memcpy(old, w, sizeof(float) * nd);
    }
    for (int32_t i = 0; i < d; ++i) w_out[i] = (double)w[i];
    *rv_out = localRegVal;
    *loss_out = localLossSum;
    *count_out = count;
    free(buf);
    return 0;
}

/* ------------------------------------------------------------------------------------------
 * Combine -- ParallelizedSGD.scala:271-276 (Breeze vector * scalar, +, / elementwise).
 * ------------------------------------------------------------------------------------------ */
void or_combine(int32_t d, double* acc_w, double* acc_rv, double* acc_loss, int64_t* acc_c,
                const double* w2, double rv2, double loss2, int64_t c2) {
    int64_t c1 = *acc_c;
    double dc1 = (double)c1, dc2 = (double)c2, dsum = (double)(c1 + c2);
    for (int32_t i = 0; i < d; ++i) acc_w[i] = (acc_w[i] * dc1 + w2[i] * dc2) / dsum;
    *acc_rv = (*acc_rv * dc1 + rv2 * dc2) / dsum;
    *acc_loss = *acc_loss + loss2;
    *acc_c = c1 + c2;
}

/* ------------------------------------------------------------------------------------------
 * Thread pool over chains.
 * ------------------------------------------------------------------------------------------ */
typedef struct {
    const or_matrix* m;
    const or_params* prm;
    int32_t P;
    const int64_t* offs;
    const int64_t* limits;
    const double* w_in;
    double* w_out;
    double* rv;
    double* loss;
    int64_t* cnt;
    int32_t tid, nthreads;
    int rc;
    int32_t* const* rows;   /* sampled epoch: rows[p][0..nrows[p]) absolute row indices */
    const int64_t* nrows;
} chain_job;

static void* chain_worker(void* arg) {
    chain_job* jb = (chain_job*)arg;
    int32_t d = or_weight_dim(jb->m->d, jb->prm);
    for (int32_t p = jb->tid; p < jb->P; p += jb->nthreads) {
        int64_t r0 = jb->offs[p], r1 = jb->offs[p + 1];
        const int32_t* rows = NULL;
        if (jb->rows) {
            rows = jb->rows[p];
            r1 = r0 + jb->nrows[p];
        }
        if (jb->limits && r1 - r0 > jb->limits[p]) r1 = r0 + jb->limits[p];
        if (g_f32 && !rows && !jb->m->is_csr && jb->prm->num_classes <= 2 &&
            (jb->prm->updater == OR_UPD_SIMPLE || jb->prm->updater == OR_UPD_SQUARED_L2)) {
            if (chain_rows_f32(jb->m, r0, r1, jb->prm, jb->w_in, jb->w_out + (size_t)p * (size_t)d,
                               &jb->rv[p], &jb->loss[p], &jb->cnt[p]) != 0)
                jb->rc = -1;
            continue;
        }
        if (chain_rows(jb->m, r0, r1, rows, jb->prm, jb->w_in, jb->w_out + (size_t)p * (size_t)d,
                       &jb->rv[p], &jb->loss[p], &jb->cnt[p], p) != 0)
            jb->rc = -1;
    }
    return NULL;
}

static int run_chains(const or_matrix* m, int32_t P, const int64_t* part_offsets,
                      const int64_t* part_limits, int32_t* const* rows, const int64_t* nrows,
                      const or_params* prm, const double* w_in, double* w_out, double* rv_out,
                      double* loss_out, int64_t* count_out, int32_t n_threads) {
    if (n_threads < 1) n_threads = 1;
    if (n_threads > P) n_threads = P > 0 ? P : 1;
    chain_job* jobs = (chain_job*)calloc((size_t)n_threads, sizeof(chain_job));
    pthread_t* th = (pthread_t*)calloc((size_t)n_threads, sizeof(pthread_t));
    int rc = 0;
    for (int32_t t = 0; t < n_threads; ++t) {
        chain_job jb = {m, prm, P, part_offsets, part_limits, w_in, w_out, rv_out, loss_out,
                        count_out, t, n_threads, 0, rows, nrows};
        jobs[t] = jb;
    }
    if (n_threads == 1) {
        chain_worker(&jobs[0]);
    } else {
        for (int32_t t = 0; t < n_threads; ++t) pthread_create(&th[t], NULL, chain_worker, &jobs[t]);
        for (int32_t t = 0; t < n_threads; ++t) pthread_join(th[t], NULL);
    }
    for (int32_t t = 0; t < n_threads; ++t) rc |= jobs[t].rc;
    free(jobs);
    free(th);
    return rc;
}

int or_run_chains(const or_matrix* m, int32_t P, const int64_t* part_offsets,
                  const int64_t* part_limits, const or_params* prm, const double* w_in,
                  double* w_out, double* rv_out, double* loss_out, int64_t* count_out,
                  int32_t n_threads) {
    g_iter = 1;
    return run_chains(m, P, part_offsets, part_limits, NULL, NULL, prm, w_in, w_out, rv_out,
                      loss_out, count_out, n_threads);
}

/* ------------------------------------------------------------------------------------------
 * Driver -- ParallelizedSGD.scala:188-306. The batch of iteration i is
 * data.sample(false, miniBatchFraction, 42 + i) (:242): or_sample_partition per partition with
 * the seeds of or_partition_seeds(42 + i) (fraction >= 1: the identity; <= 0: empty).
 * ------------------------------------------------------------------------------------------ */
int or_run(const or_matrix* m, int32_t P, const int64_t* part_offsets,
           const int32_t* group_offsets, int32_t n_groups,
           const or_params* prm, int32_t num_iterations, const double* w0,
           double* w_out, double* loss_hist, int32_t* n_hist, int64_t* chain_counts,
           int32_t n_threads) {
    int32_t d = or_weight_dim(m->d, prm);
    size_t nd = (size_t)(d > 0 ? d : 1);
    *n_hist = 0;
    int64_t numExamples = 0;
    for (int32_t p = 0; p < P; ++p) numExamples += part_offsets[p + 1] - part_offsets[p];
    if (numExamples == 0) {  /* :214-217 */
        memcpy(w_out, w0, sizeof(double) * (size_t)d);
        return 0;
    }
    int32_t one_group[2] = {0, P};
    if (!group_offsets || n_groups <= 0) {
        group_offsets = one_group;
        n_groups = 1;
    }
    double* weights = (double*)malloc(sizeof(double) * nd);
    double* prev = (double*)malloc(sizeof(double) * nd);
    double* cw = (double*)malloc(sizeof(double) * nd * (size_t)(P > 0 ? P : 1));
    double* crv = (double*)malloc(sizeof(double) * (size_t)(P > 0 ? P : 1));
    double* closs = (double*)malloc(sizeof(double) * (size_t)(P > 0 ? P : 1));
    int64_t* ccnt = (int64_t*)malloc(sizeof(int64_t) * (size_t)(P > 0 ? P : 1));
    double* gw = (double*)malloc(sizeof(double) * nd);
    double* aw = (double*)malloc(sizeof(double) * nd);
    memcpy(weights, w0, sizeof(double) * (size_t)d);  /* :224 */
    double regVal = or_initial_regval(d, weights, prm);  /* :231-233 */
    int have_cur = 0, have_prev = 0;
    int converged = 0;
    int32_t i = 1;
    int rc = 0;
    const double frac = prm->mini_batch_fraction;
    const int sampled = frac < 1.0;
    int32_t** rows = NULL;
    int64_t* nrows = NULL;
    int64_t* pseeds = NULL;
    if (sampled) {
        rows = (int32_t**)calloc((size_t)(P > 0 ? P : 1), sizeof(int32_t*));
        nrows = (int64_t*)calloc((size_t)(P > 0 ? P : 1), sizeof(int64_t));
        pseeds = (int64_t*)calloc((size_t)(P > 0 ? P : 1), sizeof(int64_t));
        for (int32_t p = 0; p < P; ++p)
            rows[p] = (int32_t*)malloc(sizeof(int32_t) * (size_t)(part_offsets[p + 1] - part_offsets[p] + 1));
    }
    while (!converged && i <= num_iterations) {  /* :237 */
        if (sampled) {  /* :242 */
            or_partition_seeds(42 + (int64_t)i, P, pseeds);
            for (int32_t p = 0; p < P; ++p) {
                const int64_t r0 = part_offsets[p];
                nrows[p] = or_sample_partition(pseeds[p], part_offsets[p + 1] - r0, frac, rows[p]);
                for (int64_t k = 0; k < nrows[p]; ++k) rows[p][k] += (int32_t)r0;
            }
        }
        g_iter = i;   /* the break-margin probe's row */
        rc = run_chains(m, P, part_offsets, NULL, rows, nrows, prm, weights, cw, crv, closs, ccnt,
                        n_threads);
        if (rc) break;
        if (chain_counts)
            for (int32_t p = 0; p < P; ++p) chain_counts[(size_t)(i - 1) * (size_t)P + p] = ccnt[p];
        /* treeReduce: left fold within each group, then across groups. */
        double arv = 0, aloss = 0;
        int64_t ac = 0;
        int have_acc = 0;
        for (int32_t gi = 0; gi < n_groups; ++gi) {
            int32_t pb = group_offsets[gi], pe = group_offsets[gi + 1];
            if (pe <= pb) continue;
            double grv = crv[pb], gloss = closs[pb];
            int64_t gc = ccnt[pb];
            memcpy(gw, cw + (size_t)pb * nd, sizeof(double) * (size_t)d);
            for (int32_t p = pb + 1; p < pe; ++p)
                or_combine(d, gw, &grv, &gloss, &gc, cw + (size_t)p * nd, crv[p], closs[p], ccnt[p]);
            if (!have_acc) {
                memcpy(aw, gw, sizeof(double) * (size_t)d);
                arv = grv;
                aloss = gloss;
                ac = gc;
                have_acc = 1;
            } else {
                or_combine(d, aw, &arv, &aloss, &ac, gw, grv, gloss, gc);
            }
        }
        if (ac > 0) {  /* :278-294 */
            double stochasticLoss = aloss / (double)ac + regVal;
            loss_hist[(*n_hist)++] = stochasticLoss;
            memcpy(weights, aw, sizeof(double) * (size_t)d);
            regVal = arv;
            have_prev = have_cur;
            if (have_cur) memcpy(prev, w_out, sizeof(double) * (size_t)d);
            memcpy(w_out, weights, sizeof(double) * (size_t)d);  /* w_out doubles as current */
            have_cur = 1;
            if (have_prev) converged = or_is_converged(d, prev, weights, prm->convergence_tol);
        }
        i += 1;
    }
    memcpy(w_out, weights, sizeof(double) * (size_t)d);
    if (sampled) {
        for (int32_t p = 0; p < P; ++p) free(rows[p]);
        free(rows);
        free(nrows);
        free(pseeds);
    }
    free(weights);
    free(prev);
    free(cw);
    free(crv);
    free(closs);
    free(ccnt);
    free(gw);
    free(aw);
    return rc;
}

/* ------------------------------------------------------------------------------------------
 * java.util.Random [ext JDK] and StrictMath.log (fdlibm 5.3 e_log.c, public algorithm),
 * for ParallelizedSGDSuite.generateGDInput (ParallelizedSGDSuite.scala:42-62).
 * ------------------------------------------------------------------------------------------ */
typedef struct {
    int64_t seed;
    int have_next;
    double next_gaussian;
} jrandom;

static void jr_init(jrandom* r, int64_t seed) {
    r->seed = (seed ^ 0x5DEECE66DLL) & ((1LL << 48) - 1);
    r->have_next = 0;
    r->next_gaussian = 0.0;
}
static int32_t jr_next(jrandom* r, int bits) {
    r->seed = (int64_t)(((uint64_t)r->seed * 0x5DEECE66DULL + 0xBULL) & ((1ULL << 48) - 1));
    return (int32_t)(uint32_t)((uint64_t)r->seed >> (48 - bits));
}
static double jr_next_double(jrandom* r) {
    int64_t a = (int64_t)jr_next(r, 26);
    int64_t b = (int64_t)jr_next(r, 27);
    return (double)((a << 27) + b) * 0x1.0p-53;
}
static double jr_next_gaussian(jrandom* r) {
    if (r->have_next) {
        r->have_next = 0;
        return r->next_gaussian;
    }
    double v1, v2, s;
    do {
        v1 = 2 * jr_next_double(r) - 1;
        v2 = 2 * jr_next_double(r) - 1;
        s = v1 * v1 + v2 * v2;
    } while (s >= 1 || s == 0);
    double multiplier = sqrt(-2 * or_fdlibm_log(s) / s);
    r->next_gaussian = v2 * multiplier;
    r->have_next = 1;
    return v1 * multiplier;
}

typedef union {
    double d;
    uint64_t u;
} dbits;
#define HI(x) ((int32_t)((x).u >> 32))
#define LO(x) ((uint32_t)((x).u & 0xffffffffu))

double or_fdlibm_log(double xin) {
    static const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
                        two54 = 1.80143985094819840000e+16, Lg1 = 6.666666666666735130e-01,
                        Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01,
                        Lg4 = 2.222219843214978396e-01, Lg5 = 1.818357216161805012e-01,
                        Lg6 = 1.531383769920937332e-01, Lg7 = 1.479819860511658591e-01;
    static volatile double zero = 0.0;
    double hfsq, f, s, z, R, w, t1, t2, dk;
    int32_t k, hx, i, j;
    uint32_t lx;
    dbits x;
    x.d = xin;
    hx = HI(x);
    lx = LO(x);
    k = 0;
    if (hx < 0x00100000) {
        if (((hx & 0x7fffffff) | (int32_t)lx) == 0) return -two54 / zero;
        if (hx < 0) return (x.d - x.d) / zero;
        k -= 54;
        x.d *= two54;
        hx = HI(x);
    }
    if (hx >= 0x7ff00000) return x.d + x.d;
    k += (hx >> 20) - 1023;
    hx &= 0x000fffff;
    i = (hx + 0x95f64) & 0x100000;
    x.u = ((uint64_t)(uint32_t)(hx | (i ^ 0x3ff00000)) << 32) | (x.u & 0xffffffffull);
    k += (i >> 20);
    f = x.d - 1.0;
    if ((0x000fffff & (2 + hx)) < 3) {
        if (f == 0.0) {
            if (k == 0) return 0.0;
            dk = (double)k;
            return dk * ln2_hi + dk * ln2_lo;
        }
        R = f * f * (0.5 - 0.33333333333333333 * f);
        if (k == 0) return f - R;
        dk = (double)k;
        return dk * ln2_hi - ((R - dk * ln2_lo) - f);
    }
    s = f / (2.0 + f);
    dk = (double)k;
    z = s * s;
    i = hx - 0x6147a;
    w = z * z;
    j = 0x6b851 - hx;
    t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    i |= j;
    R = t2 + t1;
    if (i > 0) {
        hfsq = 0.5 * f * f;
        if (k == 0) return f - (hfsq - s * (hfsq + R));
        return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
    }
    if (k == 0) return f - s * (f - R);
    return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

/* ------------------------------------------------------------------------------------------
 * RDD.sample(withReplacement = false, fraction, seed) [ext Spark 1.6.1, restated from its
 * published source]: PartitionwiseSampledRDD.getPartitions draws one seed per partition,
 * in partition order, from java.util.Random(seed).nextLong(); compute() runs a clone of
 * BernoulliSampler(fraction) with setSeed(that seed). Its RNG is XORShiftRandom, whose seed
 * is hashSeed(s) = MurmurHash3.bytesHash(ByteBuffer.allocate(java.lang.Long.SIZE).putLong(s)
 * .array()) [scala.util.hashing.MurmurHash3, Scala 2.10]: 64 bytes (Long.SIZE is in bits),
 * s big-endian in the first 8, sign-extended from Int to Long. fraction <= 0: no rows;
 * >= 1: every row; <= 0.4 (defaultMaxGapSamplingFraction): GapSamplingIterator (geometric
 * skips, u = max(nextDouble, 5e-11), k = (int)(log(u) / log1p(-f)), one skip before the first
 * row and one after every returned row); else the filter nextDouble() <= fraction per row.
 * ------------------------------------------------------------------------------------------ */
static int64_t jr_next_long(jrandom* r) {
    int64_t hi = (int64_t)jr_next(r, 32);
    int64_t lo = (int64_t)jr_next(r, 32);
    return (int64_t)((uint64_t)hi << 32) + lo;
}
void or_partition_seeds(int64_t seed, int32_t P, int64_t* out) {
    jrandom r;
    jr_init(&r, seed);
    for (int32_t p = 0; p < P; ++p) out[p] = jr_next_long(&r);
}
static uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
static uint32_t mm3_mix_last(uint32_t h, uint32_t k) {
    k *= 0xcc9e2d51u;
    k = rotl32(k, 15);
    k *= 0x1b873593u;
    return h ^ k;
}
int64_t or_xorshift_hash_seed(int64_t s) {
    uint8_t bytes[64];
    memset(bytes, 0, sizeof bytes);
    for (int b = 0; b < 8; ++b) bytes[b] = (uint8_t)((uint64_t)s >> (56 - 8 * b));
    uint32_t h = 0x3c074a61u;                     /* MurmurHash3.arraySeed */
    for (int i = 0; i < 64; i += 4) {             /* no tail: 64 is a multiple of 4 */
        uint32_t k = (uint32_t)bytes[i] | ((uint32_t)bytes[i + 1] << 8) |
                     ((uint32_t)bytes[i + 2] << 16) | ((uint32_t)bytes[i + 3] << 24);
        h = mm3_mix_last(h, k);
        h = rotl32(h, 13);
        h = h * 5u + 0xe6546b64u;
    }
    h ^= 64u;                                     /* finalizeHash(h, data.length) */
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return (int64_t)(int32_t)h;
}
static int32_t xs_next(uint64_t* st, int bits) {
    uint64_t x = *st;
    x ^= x << 21;
    x ^= x >> 35;   /* >>> on the Long */
    x ^= x << 4;
    *st = x;
    return (int32_t)(x & ((1ULL << bits) - 1));
}
static double xs_next_double(uint64_t* st) {
    int64_t a = (int64_t)xs_next(st, 26);
    int64_t b = (int64_t)xs_next(st, 27);
    return (double)((a << 27) + b) * 0x1.0p-53;
}
int64_t or_sample_partition(int64_t seed, int64_t n, double fraction, int32_t* rows_out) {
    if (fraction <= 0.0) return 0;
    int64_t m = 0;
    if (fraction >= 1.0) {
        for (int64_t t = 0; t < n; ++t) rows_out[m++] = (int32_t)t;
        return m;
    }
    uint64_t st = (uint64_t)or_xorshift_hash_seed(seed);
    if (fraction <= 0.4) {
        const double lnq = log1p(-fraction);
        int64_t pos = 0;
        for (;;) {
            double u = xs_next_double(&st);
            if (u < 5e-11) u = 5e-11;          /* math.max(rng.nextDouble(), epsilon) */
            const double q = log(u) / lnq;
            const int64_t k = q >= 2147483647.0 ? 2147483647 : (int64_t)q;   /* Double.toInt */
            pos += k;
            if (pos >= n) break;
            rows_out[m++] = (int32_t)pos;
            pos += 1;
        }
    } else {
        for (int64_t t = 0; t < n; ++t)
            if (xs_next_double(&st) <= fraction) rows_out[m++] = (int32_t)t;
    }
    return m;
}

void or_jrandom_doubles(int64_t seed, int32_t n, double* out) {
    jrandom r;
    jr_init(&r, seed);
    for (int32_t i = 0; i < n; ++i) out[i] = jr_next_double(&r);
}
void or_jrandom_gaussians(int64_t seed, int32_t n, double* out) {
    jrandom r;
    jr_init(&r, seed);
    for (int32_t i = 0; i < n; ++i) out[i] = jr_next_gaussian(&r);
}

void or_generate_gd_input(double offset, double scale, int32_t n, int32_t seed, double* x_out,
                          double* y_out) {
    jrandom rnd, unif;
    jr_init(&rnd, (int64_t)seed);
    for (int32_t i = 0; i < n; ++i) x_out[i] = jr_next_gaussian(&rnd);
    jr_init(&unif, 45);
    for (int32_t i = 0; i < n; ++i) {
        double u = jr_next_double(&unif);
        /* math.log (java.lang.Math.log) -- restated with the fdlibm algorithm as well */
        double rl = or_fdlibm_log(u) - or_fdlibm_log(1.0 - u);
        double yv = offset + scale * x_out[i] + rl;
        y_out[i] = yv > 0 ? 1.0 : 0.0;
    }
}
