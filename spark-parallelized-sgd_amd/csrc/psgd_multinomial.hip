// psgd_multinomial.hip -- the chain with the multinomial LogisticGradient (numClasses = K > 2),
// fp64 compute (parity path), dense or CSR rows, every updater (gfx950).
//
// Reference: ParallelizedSGD.scala:243-270 (the chain); [ext] MLlib 1.6.1 Gradient.scala
// LogisticGradient.compute for numClasses > 2 (restated in oracle/psgd_oracle.c
// multinomial_compute); SGDUpdater.scala:86-98, :126-148, :163-181, :199-227, :252-285.
//
// Weights are K-1 class blocks of d (class 0 is the pivot): W[c*d + i]. Per sample:
//   margin_c = sum over the row's non-zero values x_i of x_i * W[c*d + i]   (c = 0..K-2)
//   M = max margin (first index on ties); if M > 0 every margin is shifted by -M and the max
//   class contributes exp(-M) to sum instead of exp(0); else sum = sum_c exp(margin_c)
//   mult_c = exp(margin_c) / (sum + 1) - [label != 0 && label == c + 1]
//   gradient block c = mult_c * x (over x's non-zero values; dense over (K-1)*d)
//   loss = log1p(sum) - marginY (label > 0; marginY = unshifted margin of class label.toInt-1)
//          + M (if M > 0)
// One wave per chain, as chain_general: the K-1 margins are wave reductions, the scalar softmax
// bookkeeping runs redundantly on every lane in class order (the reference's order), the
// multipliers go to LDS. The updater pass covers all (K-1)*d coordinates for dense rows; for
// CSR rows Simple/AdaGrad touch only the row's coordinates in each block (their update is the
// identity where the gradient is zero), SquaredL2/L1/Adam run elementwise over all coordinates
// with the gradient staged in a per-chain scratch G (zero outside the row, reset after use).
// Per-chain status (L.state): [SA | SB | G], (K-1)*d doubles each.
#include "psgd_device.h"

namespace psgd {

namespace {

__device__ __forceinline__ void mn_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }

// Double.toInt
__device__ __forceinline__ int java_d2i(double x) {
    if (x != x) return 0;
    if (x >= 2147483647.0) return 2147483647;
    if (x <= -2147483648.0) return (-2147483647 - 1);
    return (int)x;
}

}  // namespace

template <typename S, int LAYOUT, int UPD, bool CONV>
__global__ __launch_bounds__(64) void chain_multinomial(ChainLaunch L, KParams kp) {
    extern __shared__ double mn_lds[];   // [margins | multipliers], K-1 each
    const int lane = threadIdx.x;
    const int chain = blockIdx.x;
    const ChainDesc dsc = L.descs[chain];
    const int d = kp.d;
    const int C1 = kp.nc;                 // K - 1 class blocks
    const int64_t D = (int64_t)C1 * d;    // weights
    const int64_t n = dsc.n_rows;
    double* marg = mn_lds;
    double* mult = mn_lds + C1;
    const gptr<S> X = as_global(reinterpret_cast<const S*>(dsc.x));
    const gptr<double> Y = as_global(dsc.y);
    const gptr<double> STEPS = as_global(L.steps);
    const gptr<int64_t> ROWP = as_global(dsc.row_ptr);
    const gptr<int32_t> COL = as_global(dsc.col);
    const gmut<double> W = as_global_mut(L.w_out + (int64_t)chain * D);
    const gmut<double> SA = L.state ? as_global_mut(L.state + (int64_t)chain * 3 * D) : nullptr;
    const gmut<double> SB = L.state ? SA + D : nullptr;
    const gmut<double> G = L.state ? SA + 2 * D : nullptr;
    // CSR rows: which updaters run elementwise over every coordinate (gradient staged in G)
    constexpr bool kStaged = LAYOUT == kCsr && (UPD == U_SQUARED_L2 || UPD == U_L1 || UPD == U_ADAM);

    for (int64_t i = lane; i < D; i += 64) W[i] = as_global(L.w_in)[i];
    if constexpr (kStaged)
        for (int64_t i = lane; i < D; i += 64) G[i] = 0.0;
    mn_fence();

    double loss_sum = 0.0;
    int64_t count = 0;
    double rv = 0.0;
    for (int64_t t = 0; t < n; ++t) {
        const double y = Y[t];
        const double s = STEPS[t];   // stepSize / math.sqrt(iter), iter = t + 1
        const int64_t ri = dsc.rows ? (int64_t)as_global(dsc.rows)[t] : t;   // sampled epoch
        gptr<S> xr = nullptr;
        int64_t kb = 0, ke = 0;
        if constexpr (LAYOUT == kDense) {
            xr = X + ri * dsc.ld;
        } else {
            kb = ROWP[ri];
            ke = ROWP[ri + 1];
        }
        // margins (data.foreachActive, zero values skipped)
        for (int c = 0; c < C1; ++c) {
            const gmut<double> Wc = W + (int64_t)c * d;
            double acc = 0.0;
            if constexpr (LAYOUT == kDense) {
                for (int i = lane; i < d; i += 64) {
                    const double x = double(xr[i]);
                    if (x != 0.0) acc = m_fma(x, Wc[i], acc);
                }
            } else {
                for (int64_t k = kb + lane; k < ke; k += 64) {
                    const double x = double(X[k]);
                    if (x != 0.0) acc = m_fma(x, Wc[COL[k]], acc);
                }
            }
            const double m = wave_sum(acc);
            if (lane == 0) marg[c] = m;
        }
        __syncthreads();
        // the softmax bookkeeping, in class order, on every lane
        const int ly = java_d2i(y) - 1;
        double marginY = 0.0, maxMargin = -__builtin_inf();
        int maxIdx = 0;
        for (int c = 0; c < C1; ++c) {
            const double m = marg[c];
            if (c == ly) marginY = m;
            if (m > maxMargin) {
                maxMargin = m;
                maxIdx = c;
            }
        }
        const bool shift = maxMargin > 0;
        double sum = 0.0;
        for (int c = 0; c < C1; ++c) {
            if (shift) sum = sum + (c == maxIdx ? exp(-maxMargin) : exp(marg[c] - maxMargin));
            else sum = sum + exp(marg[c]);
        }
        for (int c = lane; c < C1; c += 64) {
            const double m = shift ? marg[c] - maxMargin : marg[c];
            mult[c] = exp(m) / (sum + 1.0) - ((y != 0.0 && y == double(c + 1)) ? 1.0 : 0.0);
        }
        double loss = y > 0.0 ? log1p(sum) - marginY : log1p(sum);
        if (shift) loss = loss + maxMargin;
        __syncthreads();
        loss_sum += loss;
        count += 1;
        const double a = -s;
        double dsq = 0.0, nsq = 0.0;

        if constexpr (LAYOUT == kCsr && !kStaged) {
            // Simple / AdaGrad at the row's coordinates of every block
            if constexpr (UPD == U_ADAGRAD) {
                if (t == 0) {
                    for (int64_t i = lane; i < D; i += 64) SA[i] = 0.0;
                    mn_fence();
                }
            }
            for (int c = 0; c < C1; ++c) {
                const double mc = mult[c];
                const gmut<double> Wc = W + (int64_t)c * d;
                for (int64_t k = kb + lane; k < ke; k += 64) {
                    const double x = double(X[k]);
                    const double g = x != 0.0 ? 0.0 + mc * x : 0.0;
                    const int64_t i = COL[k];
                    const double old = Wc[i];
                    double nw;
                    if constexpr (UPD == U_SIMPLE) {
                        nw = old + a * g;
                    } else {
                        const double acc2 = SA[(int64_t)c * d + i] + g * g;
                        SA[(int64_t)c * d + i] = acc2;
                        nw = old + a * (g / sqrt(acc2 + 1.0));
                    }
                    Wc[i] = nw;
                    if constexpr (CONV) { const double df = old - nw; dsq += df * df; }
                }
            }
            if constexpr (CONV) {
                mn_fence();
                for (int64_t i = lane; i < D; i += 64) nsq += W[i] * W[i];
            }
        } else {
            if constexpr (kStaged) {
                for (int c = 0; c < C1; ++c) {
                    const double mc = mult[c];
                    for (int64_t k = kb + lane; k < ke; k += 64) {
                        const double x = double(X[k]);
                        G[(int64_t)c * d + COL[k]] = x != 0.0 ? 0.0 + mc * x : 0.0;
                    }
                }
                mn_fence();
            }
            const bool first = (t == 0);
            const double c2 = 1.0 - s * kp.reg;   // SquaredL2
            const double shrink = kp.reg * s;     // L1
            const double iter = double(t + 1);
            const double al = (UPD == U_ADAM) ? -(s / (1.0 - pow(kp.beta, iter))) : 0.0;
            for (int c = 0; c < C1; ++c) {
                const double mc = mult[c];
                for (int i = lane; i < d; i += 64) {
                    const int64_t j = (int64_t)c * d + i;
                    double g;
                    if constexpr (kStaged) {
                        g = G[j];
                    } else {
                        const double x = double(xr[i]);
                        g = x != 0.0 ? 0.0 + mc * x : 0.0;
                    }
                    const double old = W[j];
                    double nw;
                    if constexpr (UPD == U_SIMPLE) {
                        nw = old + a * g;
                    } else if constexpr (UPD == U_SQUARED_L2) {
                        nw = old * c2;
                        nw = nw + a * g;
                    } else if constexpr (UPD == U_L1) {
                        nw = old + a * g;
                        nw = jsignum(nw) * jmax(0.0, fabs(nw) - shrink);
                    } else if constexpr (UPD == U_ADAGRAD) {
                        const double sq = g * g;
                        const double acc2 = first ? sq : SA[j] + sq;
                        SA[j] = acc2;
                        nw = old + a * (g / sqrt(acc2 + 1.0));
                    } else {   // Adam, UPD.scala:252-285 (reproduced literally)
                        const double sq = g * g;
                        double v, r;
                        if (first) { v = g * (1 - kp.beta); r = sq * (1 - kp.gamma); }
                        else { v = SA[j] * kp.beta + g * (1 - kp.beta); r = SB[j] * kp.gamma + sq * (1 - kp.gamma); }
                        SA[j] = v;
                        SB[j] = r;
                        const double fix1 = sqrt(1.0 - pow(r, iter)) + kp.eps;
                        nw = old + al * (v / fix1);
                    }
                    W[j] = nw;
                    if constexpr (CONV) { const double df = old - nw; dsq += df * df; nsq += nw * nw; }
                }
            }
            if constexpr (kStaged) {
                mn_fence();
                for (int c = 0; c < C1; ++c)
                    for (int64_t k = kb + lane; k < ke; k += 64) G[(int64_t)c * d + COL[k]] = 0.0;
            }
        }
        mn_fence();
        if constexpr (CONV) {
            wave_sum2(dsq, nsq);
            if (sqrt(dsq) < kp.tol * jmax(sqrt(nsq), 1.0)) break;
        }
    }

    if constexpr (UPD == U_SQUARED_L2 || UPD == U_L1) {
        double acc = 0.0;
        for (int64_t i = lane; i < D; i += 64) acc += (UPD == U_SQUARED_L2) ? W[i] * W[i] : fabs(W[i]);
        acc = wave_sum(acc);
        if (count > 0) {
            if constexpr (UPD == U_SQUARED_L2) {
                const double nrm = sqrt(acc);
                rv = 0.5 * kp.reg * nrm * nrm;
            } else {
                rv = acc * kp.reg;
            }
        }
    }
    if (lane == 0) {
        L.rv[chain] = rv;
        L.loss[chain] = loss_sum;
        L.cnt[chain] = count;
        L.cnt_d[chain] = double(count);
    }
}

template <typename S, int LAYOUT, int UPD>
static int mn_launch(const ChainLaunch& L, const KParams& kp, bool conv, hipStream_t st, int* variant) {
    if (variant) *variant = 500 + LAYOUT;
    const size_t lds = (size_t)2 * (size_t)kp.nc * sizeof(double);
    if (conv)
        hipLaunchKernelGGL((chain_multinomial<S, LAYOUT, UPD, true>), dim3(kp.n_chains), dim3(64), lds, st, L, kp);
    else
        hipLaunchKernelGGL((chain_multinomial<S, LAYOUT, UPD, false>), dim3(kp.n_chains), dim3(64), lds, st, L, kp);
    return (int)hipGetLastError();
}

template <typename S, int LAYOUT>
static int mn_upd(const ChainLaunch& L, const KParams& kp, int upd, bool conv, hipStream_t st, int* variant) {
    switch (upd) {
    case U_SIMPLE: return mn_launch<S, LAYOUT, U_SIMPLE>(L, kp, conv, st, variant);
    case U_SQUARED_L2: return mn_launch<S, LAYOUT, U_SQUARED_L2>(L, kp, conv, st, variant);
    case U_L1: return mn_launch<S, LAYOUT, U_L1>(L, kp, conv, st, variant);
    case U_ADAGRAD: return mn_launch<S, LAYOUT, U_ADAGRAD>(L, kp, conv, st, variant);
    case U_ADAM: return mn_launch<S, LAYOUT, U_ADAM>(L, kp, conv, st, variant);
    default: return -1;
    }
}

int launch_multinomial_chains(const ChainLaunch& L, const KParams& kp, int layout, int storage, int updater,
                              bool check_conv, hipStream_t stream, int* kernel_variant) {
    if (kp.n_chains <= 0) return 0;
    if (kp.nc < 2 || kp.nc > kMultinomialMaxBlocks || !L.state) return (int)hipErrorInvalidValue;
    if (storage == 1) {
        if (layout == kDense) return mn_upd<float, kDense>(L, kp, updater, check_conv, stream, kernel_variant);
        return mn_upd<float, kCsr>(L, kp, updater, check_conv, stream, kernel_variant);
    }
    if (layout == kDense) return mn_upd<double, kDense>(L, kp, updater, check_conv, stream, kernel_variant);
    return mn_upd<double, kCsr>(L, kp, updater, check_conv, stream, kernel_variant);
}

}  // namespace psgd
