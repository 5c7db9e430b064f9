// psgd_kernels.hip -- CDNA4 (gfx950) kernels for the parallelized-SGD hot path.
//
// Reference (paths under /root/reference, src/main/scala/org/apache/spark/mllib/optimization/):
//   chain loop      ParallelizedSGD.scala:243-270   -> chain_dense_reg / chain_general
//   gradients       [ext] MLlib 1.6.1 Gradient.scala (called at ParallelizedSGD.scala:254)
//   updaters        SGDUpdater.scala:86-98, :126-148, :163-181, :199-227, :252-285
//   isConverged     ParallelizedSGD.scala:324-336 (per-sample form at :262)
//   combine         ParallelizedSGD.scala:271-276   -> fold_kernel
//
// Mapping: one wavefront64 = one chain (= one RDD partition). The chain is sequential in its
// samples; parallelism comes from the chains (one per CU) and, inside a chain, from the feature
// dimension spread over the 64 lanes. Per sample: a d-long dot reduced across the wave with
// DPP row ops + gfx950 permlane16/32 swaps (all lanes end with the bit-identical sum), the
// gradient's scalar multiplier, and the updater's elementwise update, all in registers.
// No MFMA: per-sample GEMV + axpy is not a dense contraction.
//
// Arithmetic follows the reference operator by operator (this file is compiled with
// -ffp-contract=off): grad_i = mult * x_i, then w_i = w_i + (-s) * grad_i (Breeze axpy over
// the MLlib gradient), L2 scaling w_i * (1 - s*lambda) before it. Only the dot product and the
// norms are reassociated (wave tree instead of the F2J left fold), so fp64 mode agrees with the
// reference to rounding, not bitwise.
#include "psgd_device.h"

#include <string.h>
#include "psgd_split.h"

#include <stdlib.h>

namespace psgd {

template <typename S, typename T, int GRAD, int UPD, bool CONV, int NV, bool FULL>
__global__ __launch_bounds__(128) void chain_dense(ChainLaunch L, KParams kp, RingGeom geom) {
    using V = typename Vec16<S>::type;
    constexpr int VEC = Vec16<S>::N;
    constexpr int E = NV * VEC;
    constexpr int ROW_BYTES = NV * 1024;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // LDS: [header 16 B][meta ring MB x 256 B][row ring R x ROW_BYTES]
    RingHeader* hdr = reinterpret_cast<RingHeader*>(smem);
    char* meta_ring = smem + sizeof(RingHeader);
    char* ring = meta_ring + geom.meta_blocks * kMetaBlockBytes;

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int chain = blockIdx.x;
    const ChainDesc dsc = L.descs[chain];
    const int d = kp.d;
    const int64_t n = dsc.n_rows;
    const int R = geom.rows;
    const int MB = geom.meta_blocks;

    if (threadIdx.x == 0) {
        hdr->ready = 0;
        hdr->consumed = 0;
        hdr->stop = 0;
    }
    __syncthreads();

    if (wave == 1) {
        ring_loader<S, NV, FULL, 4>(L, dsc, hdr, meta_ring, ring, geom, lane);
        return;
    }

    // ---------------- compute ----------------
    // Weights and rows are held as pairs (T2) so that fp32 runs on packed VALU ops
    // (v_pk_fma/mul/add_f32: two IEEE-rounded lanes per instruction).
    using T2 = T __attribute__((ext_vector_type(2)));
    constexpr int E2 = E / 2;
    T2 w[E2];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const int base = (v * 64 + lane) * VEC;
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            const int f = base + k;
            const double wv = as_global(L.w_in)[f < d ? f : 0];  // unconditional, clamped
            w[(v * VEC + k) / 2][(v * VEC + k) % 2] = f < d ? T(wv) : T(0);
        }
    }

    // AdaGrad / Adam status (UPD.scala:193-286) in registers beside the weights, laid out as w:
    // ua = the squared-gradient accumulator (AdaGrad) or v (Adam), ub = r (Adam). The reference
    // starts each chain's status at None (`updater.initStatus`, PSGD.scala:246): the first sample
    // takes the `None` branch.
    constexpr bool STATE_A = UPD == U_ADAGRAD || UPD == U_ADAM;
    constexpr bool STATE_B = UPD == U_ADAM;
    T2 ua[STATE_A ? E2 : 1], ub[STATE_B ? E2 : 1];
#pragma unroll
    for (int e = 0; e < (STATE_A ? E2 : 1); ++e) ua[e] = T2{T(0), T(0)};
#pragma unroll
    for (int e = 0; e < (STATE_B ? E2 : 1); ++e) ub[e] = T2{T(0), T(0)};

    // Row buffers: two register copies (ping-pong) so row t+1's LDS reads are in flight while
    // sample t computes.
    T2 xb[2][E2];
    double yb[2], sb[2];
    int meta_blk = 0;
    auto read_row = [&](auto pc, const char* src, int64_t t) __attribute__((always_inline)) {
        constexpr int p = decltype(pc)::value;
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            V xv = *reinterpret_cast<const V*>(src + v * 1024 + lane * 16);
            if constexpr (!FULL) {
                // vectors past the row end were not loaded: their LDS bytes are stale
                if ((v * 64 + lane) * VEC >= dsc.ld) xv = V(0);
            }
            T tmp[VEC];
            unpack<S, T>(xv, tmp);
#pragma unroll
            for (int k = 0; k < VEC; k += 2) xb[p][(v * VEC + k) / 2] = T2{tmp[k], tmp[k + 1]};
        }
        // rows are read in order: the meta block advances every kMetaRows rows
        if (t > 0 && (t & (kMetaRows - 1)) == 0) meta_blk = (meta_blk + 1 == MB) ? 0 : meta_blk + 1;
        const f64x2 meta = *reinterpret_cast<const f64x2*>(
            meta_ring + meta_blk * kMetaBlockBytes + (int)(t & (kMetaRows - 1)) * 16);
        yb[p] = meta.x;
        sb[p] = meta.y;
    };

    unsigned ready = 0;
    bool stop = false;
    // Wait until `rows` rows have landed; false (and the watchdog flag) if the loader makes no
    // progress for kWatchdogTicks.
    auto wait_rows = [&](int64_t rows) __attribute__((always_inline)) -> bool {
        if (rows > (int64_t)ready) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            for (;;) {
                ready = __hip_atomic_load(&hdr->ready, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (rows <= (int64_t)ready) break;
                if (__builtin_amdgcn_s_memrealtime() - t0 > kWatchdogTicks) {
                    __hip_atomic_fetch_or(L.watchdog, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(&hdr->stop, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    return false;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        return true;
    };

    double loss_sum = 0.0;
    T loss_blk = T(0);          // fp32 mode: block partial, flushed to the fp64 sum every 32 rows
    // fp64 Logistic: the per-row dots go to L.zbuf64, the losses are summed after the chain
    constexpr bool ZEXT = GRAD == G_LOGISTIC && sizeof(T) == 8;
    double* zout = ZEXT ? L.zbuf64 + (int64_t)chain * L.zstride : nullptr;
    int64_t count = 0;
    const char* slot_ptr = ring;                       // slot of row t
    const char* const ring_end = ring + R * ROW_BYTES;

    auto sample = [&](auto pc, int64_t t) __attribute__((always_inline)) {
        constexpr int p = decltype(pc)::value;
        const char* next_ptr = slot_ptr + ROW_BYTES;
        if (next_ptr == ring_end) next_ptr = ring;
        if (t + 1 < n) {   // prefetch row t+1 into the other buffer
            if (!wait_rows(t + 2)) { stop = true; return; }
            read_row(std::integral_constant<int, 1 - p>{}, next_ptr, t + 1);
        }
        const T y = T(yb[p]);
        const T s = T(sb[p]);
        const T2* x = xb[p];

        // dot(data, weights): two packed partial sums; four in the fp32 mode (shorter dependent
        // chains: the next sample's dot waits on this sample's updates)
        T2 acc;
        if constexpr (sizeof(T) == 4) {
            T2 d0 = T2{T(0), T(0)}, d1 = T2{T(0), T(0)}, d2 = T2{T(0), T(0)}, d3 = T2{T(0), T(0)};
#pragma unroll
            for (int e = 0; e < E2; e += 4) {
                d0 = __builtin_elementwise_fma(x[e], w[e], d0);
                if (e + 1 < E2) d1 = __builtin_elementwise_fma(x[e + 1], w[e + 1], d1);
                if (e + 2 < E2) d2 = __builtin_elementwise_fma(x[e + 2], w[e + 2], d2);
                if (e + 3 < E2) d3 = __builtin_elementwise_fma(x[e + 3], w[e + 3], d3);
            }
            acc = (d0 + d1) + (d2 + d3);
        } else {
            T2 acc0 = T2{T(0), T(0)}, acc1 = T2{T(0), T(0)};
#pragma unroll
            for (int e = 0; e < E2; e += 2) {
                acc0 = __builtin_elementwise_fma(x[e], w[e], acc0);
                if (e + 1 < E2) acc1 = __builtin_elementwise_fma(x[e + 1], w[e + 1], acc1);
            }
            acc = acc0 + acc1;
        }
        const T z = wave_sum_uniform(acc.x + acc.y);
        if ((t & 1) == 1 || t + 1 == n) {
            // rows <= t have been read into registers: hand their slots back to the loader
            __hip_atomic_store(&hdr->consumed, (unsigned)(t + 1), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
        }

        T mult, loss;
        if constexpr (ZEXT) {
            // mult as gradient_scalar; the row's loss (log1pExp: a second exp and a log1p on
            // the sequential wave) is summed after the chain by logistic_loss64_kernel from z
            mult = (T(1) / (T(1) + m_exp(-z))) - y;
            loss = T(0);
            if (lane == 0) zout[t] = z;
        } else if constexpr (GRAD == G_LEAST_SQUARES) {
            // loss = diff*diff/2.0: the halving is exact, so the chain accumulates diff*diff and
            // halves the sum (identical to summing the halves)
            mult = z - y;
            loss = mult * mult;
        } else {
            loss = gradient_scalar<GRAD, T>(z, y, mult);
        }
        if constexpr (sizeof(T) == 4) {
            loss_blk += loss;
            if ((t & 31) == 31) { loss_sum += double(loss_blk); loss_blk = T(0); }
        } else {
            loss_sum += loss;
        }
        count += 1;

        const T a = -s;
        T2 dsq2 = T2{T(0), T(0)}, nsq2 = T2{T(0), T(0)};
        // Adam's per-sample scalars (UPD.scala:258-262): iter = j, lr = s / (1 - beta^iter)
        const bool first = t == 0;
        const T iter = T(t + 1);
        T al = T(0);
        if constexpr (UPD == U_ADAM) {
            // fp32 mode: beta^iter by the hardware log2 / exp2, as r^iter below
            if constexpr (sizeof(T) == 4) al = -(s / (T(1) - pow_fast(T(kp.beta), iter)));
            // fp64: 1 - beta^iter as 1.0 once beta^iter <= 2^-54 (bit-identical, no library pow
            // per sample on the chain) and the division by rcp + one Newton step
            else al = -(s * recip_newton(one_minus_pow_iter(T(kp.beta), iter)));
        }
#pragma unroll
        for (int e = 0; e < E2; ++e) {
            const T2 old = w[e];
            T2 nw;
            if constexpr (UPD == U_ADAGRAD) {
                // accum = None ? g*g : accum + g*g; w += -s * (g / sqrt(accum + 1.0))
                const T2 g = mult * x[e];
                const T2 acc2 = first ? g * g : ua[e] + g * g;
                ua[e] = acc2;
                if constexpr (sizeof(T) == 4) {
                    // fp32 mode: g * rsqrt(accum + 1) (one v_rsq_f32, ~1 ulp) for g / sqrt(accum + 1)
                    nw.x = old.x + a * (g.x * __builtin_amdgcn_rsqf(acc2.x + T(1)));
                    nw.y = old.y + a * (g.y * __builtin_amdgcn_rsqf(acc2.y + T(1)));
                } else {
                    // g / pow(accum + 1.0, 0.5) (UPD.scala:209) as g * rsqrt(accum + 1): v_rsq_f64
                    // and one Newton step (4.3e-15 relative, tools/newton_check; the library sqrt + division were
                    // ~20 dependent f64 operations per coordinate and sample)
                    nw.x = old.x + a * (g.x * rsqrt_newton(acc2.x + T(1)));
                    nw.y = old.y + a * (g.y * rsqrt_newton(acc2.y + T(1)));
                }
            } else if constexpr (UPD == U_ADAM) {
                // the reference's variant, literally: v = beta v + (1-beta) g,
                // r = gamma r + (1-gamma) g^2, fix1 = sqrt(1 - r^iter) + eps, w += -lr * v / fix1
                const T beta = T(kp.beta), gamma = T(kp.gamma);
                const T2 g = mult * x[e];
                const T2 sq = g * g;
                T2 v, r;
                if (first) { v = g * (T(1) - beta); r = sq * (T(1) - gamma); }
                else { v = ua[e] * beta + g * (T(1) - beta); r = ub[e] * gamma + sq * (T(1) - gamma); }
                ua[e] = v;
                ub[e] = r;
                // fp32 mode: r^iter = exp2(iter * log2 r) (v_log_f32 / v_exp_f32; r = 0 gives 0,
                // r > 1 overflows to inf and fix1 to NaN, as pow does)
                // and v / fix1 as v * rcp(fix1), sqrt by v_sqrt_f32 (~1 ulp each; a negative
                // 1 - r^iter still gives NaN)
                if constexpr (sizeof(T) == 4) {
                    const T fx = __builtin_amdgcn_sqrtf(T(1) - pow_fast(r.x, iter)) + T(kp.eps);
                    const T fy = __builtin_amdgcn_sqrtf(T(1) - pow_fast(r.y, iter)) + T(kp.eps);
                    nw.x = old.x + al * (v.x * __builtin_amdgcn_rcpf(fx));
                    nw.y = old.y + al * (v.y * __builtin_amdgcn_rcpf(fy));
                } else {
                    // sqrt and v / fix1 by the hardware estimates + one Newton step (~1e-14)
                    const T fx = sqrt_newton(one_minus_pow_iter(r.x, iter)) + T(kp.eps);
                    const T fy = sqrt_newton(one_minus_pow_iter(r.y, iter)) + T(kp.eps);
                    nw.x = old.x + al * (v.x * recip_newton(fx));
                    nw.y = old.y + al * (v.y * recip_newton(fy));
                }
            } else if constexpr (UPD == U_SQUARED_L2) {
                const T c = T(1) - s * T(kp.reg);
                nw = old * c;                       // brzWeights :*= (1 - s*lambda)
                nw = nw + a * (mult * x[e]);        // axpy(-s, grad, w)
            } else if constexpr (UPD == U_L1) {
                const T shrink = T(kp.reg) * s;
                nw = old + a * (mult * x[e]);
                nw.x = jsignum(nw.x) * jmax(T(0), m_fabs(nw.x) - shrink);
                nw.y = jsignum(nw.y) * jmax(T(0), m_fabs(nw.y) - shrink);
            } else if constexpr (sizeof(T) == 4) {
                // fp32 throughput mode: one fused update per pair, w + (-s*mult) * x
                nw = __builtin_elementwise_fma(T2{a * mult, a * mult}, x[e], old);
            } else {
                nw = old + a * (mult * x[e]);   // the reference's two roundings (fp64 mode)
            }
            w[e] = nw;
            if constexpr (CONV) { const T2 df = old - nw; dsq2 += df * df; nsq2 += nw * nw; }
        }
        slot_ptr = next_ptr;
        if constexpr (CONV) {
            T dsq = dsq2.x + dsq2.y, nsq = nsq2.x + nsq2.y;
            wave_sum2(dsq, nsq);
            // ||old - new|| < tol * max(||new||, 1.0)   (PSGD.scala:262, :333-335)
            if (m_sqrt(dsq) < T(kp.tol) * jmax(m_sqrt(nsq), T(1))) {
                __hip_atomic_store(&hdr->stop, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                stop = true;
            }
        }
    };

    if (n > 0) {
        if (wait_rows(1)) read_row(std::integral_constant<int, 0>{}, ring, 0);
        else stop = true;
    }
    int64_t t = 0;
    for (; t + 2 <= n && !stop; t += 2) {
        sample(std::integral_constant<int, 0>{}, t);
        if (stop) break;
        sample(std::integral_constant<int, 1>{}, t + 1);
    }
    if (t < n && !stop) sample(std::integral_constant<int, 0>{}, t);
    if constexpr (sizeof(T) == 4) loss_sum += double(loss_blk);
    if constexpr (GRAD == G_LEAST_SQUARES) loss_sum = loss_sum / 2.0;

    // regVal of the chain's last update (PSGD.scala:257; 0.0 if no sample, :247)
    double rv = 0.0;
    if constexpr (UPD == U_SQUARED_L2 || UPD == U_L1) {
        T acc = T(0);
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const T we = w[e / 2][e % 2];
            if constexpr (UPD == U_SQUARED_L2) acc += we * we;
            else acc += m_fabs(we);
        }
        acc = wave_sum(acc);
        if (count > 0) {
            if constexpr (UPD == U_SQUARED_L2) {
                const double nrm = sqrt(double(acc));
                rv = 0.5 * kp.reg * nrm * nrm;
            } else {
                rv = double(acc) * kp.reg;
            }
        }
    }

    double* wo = L.w_out + (int64_t)chain * d;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const int base = (v * 64 + lane) * VEC;
#pragma unroll
        for (int k = 0; k < VEC; ++k)
            if (base + k < d) wo[base + k] = double(w[(v * VEC + k) / 2][(v * VEC + k) % 2]);
    }
    if (lane == 0) {
        L.rv[chain] = rv;
        if constexpr (!ZEXT) L.loss[chain] = loss_sum;
        L.cnt[chain] = count;
        L.cnt_d[chain] = double(count);
    }
}

// ------------------------------------------------------------------------------------------
// chain_general: any d, dense or CSR rows, every updater. Parity path, fp64 compute.
// The chain's working weights live in its own slice of w_out (global memory, L2-resident for
// moderate d); stateful updaters keep their status in `state`. One wave per chain.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void wave_mem_fence() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
}

template <typename S, int LAYOUT, int GRAD, int UPD, bool CONV>
__global__ __launch_bounds__(64) void chain_general(ChainLaunch L, KParams kp) {
    const int lane = threadIdx.x;
    const int chain = blockIdx.x;
    const ChainDesc dsc = L.descs[chain];
    const int d = kp.d;
    const int64_t n = dsc.n_rows;
    const gptr<S> X = as_global(reinterpret_cast<const S*>(dsc.x));
    const gptr<double> Y = as_global(dsc.y);
    const gptr<double> STEPS = as_global(L.steps);
    const gptr<int64_t> ROWP = as_global(dsc.row_ptr);
    const gptr<int32_t> COL = as_global(dsc.col);
    const gmut<double> W = as_global_mut(L.w_out + (int64_t)chain * d);
    // per-chain status: dense rows [SA | SB] (2d), CSR rows [SA | SB | SC] (3d; SC: the sample's
    // dense gradient for Adam, zero outside the row's indices between samples)
    constexpr int NS = LAYOUT == kCsr ? 3 : 2;
    const gmut<double> SA = L.state ? as_global_mut(L.state + (int64_t)chain * NS * d) : nullptr;
    const gmut<double> SB = L.state ? SA + d : nullptr;
    const gmut<double> SC = (L.state && LAYOUT == kCsr) ? SA + 2 * d : nullptr;

    // CSR rows with Simple / SquaredL2 / AdaGrad and the per-sample break: ||w||^2 is carried from
    // sample to sample (O(nnz) per sample instead of a pass over all d): Simple and AdaGrad (which
    // change only the row's coordinates) add each changed coordinate's nw^2 - old^2; SquaredL2 (lazy form below) the recurrence of chain_block64,
    // ||w'||^2 = a (a ||w||^2 + 2 c z) + c^2 q, ||w - w'||^2 = b (b ||w||^2 - 2 c z) + c^2 q
    // (a = 1 - s lambda, b = 1 - a, c = -s mult, z = x . w, q = x . x). Starts from ||w_in||^2.
    constexpr bool NORMS = CONV && LAYOUT == kCsr && (UPD == U_SIMPLE || UPD == U_SQUARED_L2 || UPD == U_ADAGRAD);
    double wn = 0.0;
    for (int i = lane; i < d; i += 64) {
        const double v = as_global(L.w_in)[i];
        W[i] = v;
        if constexpr (NORMS) wn += v * v;
    }
    if constexpr (LAYOUT == kCsr && UPD == U_ADAM)
        for (int i = lane; i < d; i += 64) SC[i] = 0.0;
    wave_mem_fence();
    if constexpr (NORMS) wn = wave_sum(wn);

    // CSR rows with SquaredL2: the alpha-scaled lazy form. The chain keeps
    // w = alpha * v, so the reference's O(d) scale w *= 1 - s*lambda (UPD.scala:169) is one
    // multiply of alpha and the gradient step adds (-s g_j) / alpha to v_j at the row's indices;
    // alpha is folded back into v (O(d)) when it leaves [2^-400, 2^400] or becomes 0, and at the
    // chain's end. Equal to the reference's arithmetic up to rounding (the 1e-9 fp64 bar).
    constexpr bool LAZY = LAYOUT == kCsr && UPD == U_SQUARED_L2;
    double alpha = 1.0;
    double loss_sum = 0.0;
    int64_t count = 0;
    double rv = 0.0;
    for (int64_t t = 0; t < n; ++t) {
        const double y = Y[t];
        const double s = STEPS[t];           // stepSize / math.sqrt(iter), iter = t + 1
        gptr<S> xr = nullptr;
        int64_t kb = 0, ke = 0;
        // dot(data, weights)
        double acc = 0.0;
        [[maybe_unused]] double qacc = 0.0;   // NORMS + SquaredL2: x . x
        const int64_t ri = dsc.rows ? (int64_t)as_global(dsc.rows)[t] : t;   // sampled epoch
        if constexpr (LAYOUT == kDense) {
            xr = X + ri * dsc.ld;
            for (int i = lane; i < d; i += 64) acc = m_fma(double(xr[i]), W[i], acc);
        } else {
            kb = ROWP[ri];
            ke = ROWP[ri + 1];
            for (int64_t k = kb + lane; k < ke; k += 64) {
                acc = m_fma(double(X[k]), W[COL[k]], acc);
                if constexpr (NORMS && UPD == U_SQUARED_L2) qacc = m_fma(double(X[k]), double(X[k]), qacc);
            }
        }
        double z;
        if constexpr (NORMS && UPD == U_SQUARED_L2) {
            wave_sum2(acc, qacc);
            z = acc;
        } else {
            z = wave_sum(acc);
        }
        if constexpr (LAZY) z = alpha * z;   // dot(x, w) with w = alpha * v
        double mult;
        const double loss = gradient_scalar<GRAD, double>(z, y, mult);
        loss_sum += loss;
        count += 1;
        const double a = -s;
        double dsq = 0.0, nsq = 0.0;

        if constexpr (UPD == U_SIMPLE && LAYOUT == kCsr) {
            // Breeze axpy over the gradient's active entries only.
            for (int64_t k = kb + lane; k < ke; k += 64) {
                const int i = COL[k];
                const double old = W[i];
                const double nw = old + a * (mult * double(X[k]));
                W[i] = nw;
                if constexpr (CONV) {
                    const double df = old - nw;
                    dsq += df * df;
                    nsq += nw * nw - old * old;   // the change of ||w||^2 (NORMS)
                }
            }
        } else {
            if constexpr (LAYOUT == kCsr) {
                // Updaters that touch every coordinate: run the elementwise part over all d,
                // with the gradient applied at the row's indices in a second pass (ordered as
                // the reference: L2 scales before the axpy, L1 thresholds after it).
                if constexpr (LAZY) {
                    const double c = 1.0 - s * kp.reg;
                    if constexpr (NORMS) {
                        // ||w'||^2 and ||w - w'||^2 from the recurrence (header of this branch)
                        const double cc = a * mult, b = 1.0 - c, cq = cc * cc * qacc;
                        const double nn = c * __builtin_fma(c, wn, 2.0 * cc * z) + cq;
                        dsq = b * __builtin_fma(b, wn, -2.0 * cc * z) + cq;
                        nsq = nn > 0.0 ? nn : 0.0;
                    }
                    const double na = alpha * c;
                    if (!(__builtin_fabs(na) >= 0x1p-400 && __builtin_fabs(na) <= 0x1p400)) {
                        for (int i = lane; i < d; i += 64) W[i] = (alpha * W[i]) * c;
                        alpha = 1.0;
                        wave_mem_fence();
                    } else {
                        alpha = na;
                    }
                    for (int64_t k = kb + lane; k < ke; k += 64) {
                        const int i = COL[k];
                        W[i] = W[i] + (a * (mult * double(X[k]))) / alpha;
                    }
                } else if constexpr (UPD == U_SQUARED_L2) {
                    const double c = 1.0 - s * kp.reg;
                    for (int i = lane; i < d; i += 64) {
                        const double old = W[i];
                        const double nw = old * c;
                        W[i] = nw;
                        if constexpr (CONV) SB[i] = old;   // keep old for the convergence test
                    }
                    wave_mem_fence();
                    for (int64_t k = kb + lane; k < ke; k += 64) {
                        const int i = COL[k];
                        W[i] = W[i] + a * (mult * double(X[k]));
                    }
                } else if constexpr (UPD == U_L1) {
                    if constexpr (CONV)
                        for (int i = lane; i < d; i += 64) SB[i] = W[i];
                    wave_mem_fence();
                    for (int64_t k = kb + lane; k < ke; k += 64) {
                        const int i = COL[k];
                        W[i] = W[i] + a * (mult * double(X[k]));
                    }
                    wave_mem_fence();
                    const double shrink = kp.reg * s;
                    for (int i = lane; i < d; i += 64) {
                        const double v = W[i];
                        W[i] = jsignum(v) * jmax(0.0, fabs(v) - shrink);
                    }
                } else if constexpr (UPD == U_ADAGRAD) {
                    // UPD.scala:199-227 on a gradient that is zero outside the row's indices:
                    // the accumulator (None -> squaredGrad, i.e. zero there at the first sample)
                    // and the weights change only at the row's indices (w + a*(0/..) == w)
                    if (t == 0) {
                        for (int i = lane; i < d; i += 64) SA[i] = 0.0;
                        wave_mem_fence();
                    }
                    for (int64_t k = kb + lane; k < ke; k += 64) {
                        const int i = COL[k];
                        const double g = mult * double(X[k]);
                        const double acc2 = SA[i] + g * g;
                        SA[i] = acc2;
                        const double old = W[i];
                        const double nw = old + a * (g / sqrt(acc2 + 1.0));
                        W[i] = nw;
                        if constexpr (CONV) {
                            const double df = old - nw;
                            dsq += df * df;
                            nsq += nw * nw - old * old;   // the change of ||w||^2 (NORMS)
                        }
                    }
                } else {  // U_ADAM, UPD.scala:252-285: v and r decay at every coordinate
                    for (int64_t k = kb + lane; k < ke; k += 64) SC[COL[k]] = mult * double(X[k]);
                    wave_mem_fence();
                    const bool first = (t == 0);
                    const double beta = kp.beta, gamma = kp.gamma;
                    const double iter = double(t + 1);
                    const double lr = s / (1.0 - pow(beta, iter));
                    const double al = -lr;
                    for (int i = lane; i < d; i += 64) {
                        const double g = SC[i];
                        const double sq = g * g;
                        double v, r;
                        if (first) { v = g * (1 - beta); r = sq * (1 - gamma); }
                        else { v = SA[i] * beta + g * (1 - beta); r = SB[i] * gamma + sq * (1 - gamma); }
                        SA[i] = v;
                        SB[i] = r;
                        const double fix1 = sqrt(1.0 - pow(r, iter)) + kp.eps;
                        const double old = W[i];
                        const double nw = old + al * (v / fix1);
                        W[i] = nw;
                        if constexpr (CONV) { const double df = old - nw; dsq += df * df; nsq += nw * nw; }
                    }
                    wave_mem_fence();
                    for (int64_t k = kb + lane; k < ke; k += 64) SC[COL[k]] = 0.0;
                }
                if constexpr (CONV && UPD == U_L1) {   // (SquaredL2: the lazy form's recurrence)
                    wave_mem_fence();
                    for (int i = lane; i < d; i += 64) {
                        const double nw = W[i];
                        const double df = SB[i] - nw;
                        dsq += df * df;
                        nsq += nw * nw;
                    }
                }
            } else {
                if constexpr (UPD == U_SIMPLE) {
                    for (int i = lane; i < d; i += 64) {
                        const double old = W[i];
                        const double nw = old + a * (mult * double(xr[i]));
                        W[i] = nw;
                        if constexpr (CONV) { const double df = old - nw; dsq += df * df; nsq += nw * nw; }
                    }
                } else if constexpr (UPD == U_SQUARED_L2) {
                    const double c = 1.0 - s * kp.reg;
                    for (int i = lane; i < d; i += 64) {
                        const double old = W[i];
                        double nw = old * c;
                        nw = nw + a * (mult * double(xr[i]));
                        W[i] = nw;
                        if constexpr (CONV) { const double df = old - nw; dsq += df * df; nsq += nw * nw; }
                    }
                } else if constexpr (UPD == U_L1) {
                    const double shrink = kp.reg * s;
                    for (int i = lane; i < d; i += 64) {
                        const double old = W[i];
                        double nw = old + a * (mult * double(xr[i]));
                        nw = jsignum(nw) * jmax(0.0, fabs(nw) - shrink);
                        W[i] = nw;
                        if constexpr (CONV) { const double df = old - nw; dsq += df * df; nsq += nw * nw; }
                    }
                } else if constexpr (UPD == U_ADAGRAD) {
                    // accum = (first ? g*g : accum + g*g); w += -s * (g / sqrt(accum + 1.0))
                    const bool first = (t == 0);
                    for (int i = lane; i < d; i += 64) {
                        const double g = mult * double(xr[i]);
                        const double sq = g * g;
                        const double acc2 = first ? sq : SA[i] + sq;
                        SA[i] = acc2;
                        const double old = W[i];
                        const double nw = old + a * (g / sqrt(acc2 + 1.0));
                        W[i] = nw;
                        if constexpr (CONV) { const double df = old - nw; dsq += df * df; nsq += nw * nw; }
                    }
                } else {  // U_ADAM, UPD.scala:252-285 (reproduced literally)
                    const bool first = (t == 0);
                    const double beta = kp.beta, gamma = kp.gamma;
                    const double iter = double(t + 1);
                    const double lr = s / (1.0 - pow(beta, iter));
                    const double al = -lr;
                    for (int i = lane; i < d; i += 64) {
                        const double g = mult * double(xr[i]);
                        const double sq = g * g;
                        double v, r;
                        if (first) { v = g * (1 - beta); r = sq * (1 - gamma); }
                        else { v = SA[i] * beta + g * (1 - beta); r = SB[i] * gamma + sq * (1 - gamma); }
                        SA[i] = v;
                        SB[i] = r;
                        const double fix1 = sqrt(1.0 - pow(r, iter)) + kp.eps;
                        const double old = W[i];
                        const double nw = old + al * (v / fix1);
                        W[i] = nw;
                        if constexpr (CONV) { const double df = old - nw; dsq += df * df; nsq += nw * nw; }
                    }
                }
            }
        }
        wave_mem_fence();
        if constexpr (NORMS && UPD == U_SQUARED_L2) {
            // dsq and nsq are the recurrence's (wave-uniform)
            wn = nsq;
            if (sqrt(dsq > 0.0 ? dsq : 0.0) < kp.tol * jmax(sqrt(nsq), 1.0)) break;
        } else if constexpr (NORMS) {
            wave_sum2(dsq, nsq);
            wn = wn + nsq;
            if (sqrt(dsq) < kp.tol * jmax(sqrt(wn), 1.0)) break;
        } else if constexpr (CONV) {
            wave_sum2(dsq, nsq);
            if (sqrt(dsq) < kp.tol * jmax(sqrt(nsq), 1.0)) break;
        }
    }

    if constexpr (LAZY) {
        for (int i = lane; i < d; i += 64) W[i] = alpha * W[i];
        wave_mem_fence();
    }
    if constexpr (UPD == U_SQUARED_L2 || UPD == U_L1) {
        double acc = 0.0;
        for (int i = lane; i < d; i += 64) acc += (UPD == U_SQUARED_L2) ? W[i] * W[i] : fabs(W[i]);
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

// ------------------------------------------------------------------------------------------
// The reference combiner (PSGD.scala:271-276) as a left fold over n items in index order, one
// thread per coordinate; the thread with i == d folds the scalars.
//   w = (w1*c1 + w2*c2) / (c1 + c2);  rv likewise;  loss = l1 + l2;  c = c1 + c2
// out[0..d) = w, out[d] = regVal, out[d+1] = lossSum, out[d+2] = count.
//
// Each step is one dependent f64 multiply, add and IEEE division on the coordinate's running
// value; the item loads are not on that chain. Loading item p at its step (before round 6)
// left the steps waiting on memory round trips: 40 us per c2 epoch (256 chains, d = 512). The
// block stages the per-item scalars (counts, and regVal, loss, alpha as needed) in LDS,
// kFoldStage items at a time, and every coordinate thread keeps its next kFoldAhead weights in
// flight while it folds the current ones. Same operations in the same order: bit-identical
// results. (Measured and not kept: the division with its denominator-only part -- the refined
// reciprocal of c1 + c2 -- taken off the running value's dependent path, bit-identical by
// construction where v_div_scale scales nothing and checked over the whole f64 range: 33 us
// against 28 per c2 epoch, the extra reciprocal work per step costs more than the shorter path.)
// ------------------------------------------------------------------------------------------
constexpr int kFoldStage = 512;    // items staged in LDS at a time
constexpr int kFoldAhead = 16;     // weight loads in flight per coordinate thread
constexpr int kFoldThreads = 256;

// WLOAD(p, a) -> item p's weight for this thread's coordinate (a = item p's alpha, if staged)
template <bool ALPHA, typename WLoad>
__device__ __forceinline__ void fold_items(WLoad wload, const double* __restrict__ alpha,
                                           const double* __restrict__ rv, const double* __restrict__ loss,
                                           const double* __restrict__ cnt, int64_t s_stride, int n, int d,
                                           double* __restrict__ out, int* __restrict__ watchdog,
                                           double* __restrict__ mirror) {
    __shared__ double sc[kFoldStage], sr[kFoldStage], sl[kFoldStage], sa[ALPHA ? kFoldStage : 1];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool wt = i < d;                                   // a weight coordinate
    const bool st = i == d;                                  // the scalars
    const bool blk_st = (int)(blockIdx.x * blockDim.x) <= d && d < (int)((blockIdx.x + 1) * blockDim.x);
    double acc = 0.0, r = 0.0, l = 0.0, c1 = 0.0;
    for (int s0 = 0; s0 < n; s0 += kFoldStage) {
        const int m = n - s0 < kFoldStage ? n - s0 : kFoldStage;
        __syncthreads();   // the previous stage's items are folded
        for (int k = threadIdx.x; k < m; k += blockDim.x) {
            const int64_t q = (int64_t)(s0 + k) * s_stride;
            sc[k] = cnt[q];
            if (blk_st) {
                sr[k] = rv[q];
                sl[k] = loss[q];
            }
            if constexpr (ALPHA) sa[k] = alpha[s0 + k];
        }
        __syncthreads();
        const int k0 = s0 == 0 ? 1 : 0;   // item 0 starts the fold
        if (s0 == 0) {
            c1 = sc[0];
            if (wt) acc = wload(0, ALPHA ? sa[0] : 1.0);
            if (st) {
                r = sr[0];
                l = sl[0];
            }
        }
        if (wt) {
            // items [k0, m) of the stage, kFoldAhead at a time, the next group's loads issued
            // before the current group's steps (indices clamped to the stage: a group past its
            // end loads item m - 1 again and folds nothing)
            double cur[kFoldAhead], nxt[kFoldAhead];
            auto fetch = [&](double (&v)[kFoldAhead], int g0) __attribute__((always_inline)) {
#pragma unroll
                for (int j = 0; j < kFoldAhead; ++j) {
                    const int k = g0 + j < m ? g0 + j : m - 1;
                    v[j] = wload(s0 + k, ALPHA ? sa[k] : 1.0);
                }
            };
            fetch(cur, k0);
            for (int g0 = k0; g0 < m; g0 += kFoldAhead) {
                fetch(nxt, g0 + kFoldAhead);
#pragma unroll
                for (int j = 0; j < kFoldAhead; ++j) {
                    if (g0 + j < m) {
                        const double c2 = sc[g0 + j];
                        acc = (acc * c1 + cur[j] * c2) / (c1 + c2);
                        c1 = c1 + c2;
                    }
                }
#pragma unroll
                for (int j = 0; j < kFoldAhead; ++j) cur[j] = nxt[j];
            }
        } else if (st) {
            for (int k = k0; k < m; ++k) {
                const double c2 = sc[k];
                r = (r * c1 + sr[k] * c2) / (c1 + c2);
                l = l + sl[k];
                c1 = c1 + c2;
            }
        }
    }
    if (wt) {
        out[i] = acc;
    } else if (st) {
        // a chain kernel that tripped its watchdog poisons the count: the host raises. The
        // flags are cleared here for the next epoch (every epoch's chains end in one fold), so
        // the epoch enqueues no memset of its own
        bool fired = false;
        if (watchdog) {
            fired = watchdog[0] != 0;   // (the chains' flags are OR-ed into word 0)
            watchdog[0] = watchdog[1] = watchdog[2] = watchdog[3] = 0;
        }
        const double cnt_out = fired ? __builtin_nan("") : c1;
        out[d] = r;
        out[d + 1] = l;
        out[d + 2] = cnt_out;
        if (mirror) {
            // the host's copy, system-scope stores; the count last, with release order, so a
            // host that polls it (for a value other than the one it left there) then reads the
            // other two finds them written
            __hip_atomic_store(reinterpret_cast<unsigned long long*>(mirror), (unsigned long long)__double_as_longlong(r),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(reinterpret_cast<unsigned long long*>(mirror) + 1, (unsigned long long)__double_as_longlong(l),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(reinterpret_cast<unsigned long long*>(mirror) + 2,
                               (unsigned long long)__double_as_longlong(cnt_out), __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

__global__ __launch_bounds__(kFoldThreads) void fold_kernel(const double* __restrict__ w, int64_t w_stride,
                            const double* __restrict__ rv, const double* __restrict__ loss,
                            const double* __restrict__ cnt, int64_t s_stride, int n, int d,
                            double* __restrict__ out, int* __restrict__ watchdog, double* __restrict__ mirror) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    fold_items<false>([&](int p, double) { return w[(int64_t)p * w_stride + i]; }, nullptr, rv, loss, cnt,
                      s_stride, n, d, out, watchdog, mirror);
}

// The same combiner over the fp32 CSR chains' weights, w_p = walpha[p] * double(v_p[i]) -- the
// value those chains once wrote to w_out, so the fold's arithmetic is unchanged; reading the
// fp32 vectors directly saves the O(P d) f64 write and re-read (C5: 2^22 features x 1024 chains).
// (V = double: chain_sparse64's vectors, the same combiner with w_p = walpha[p] * v_p[i] -- the
// value chain_general's W[i] = alpha * W[i] writes at the chain's end.)
template <typename V>
__global__ __launch_bounds__(kFoldThreads) void fold_scaled_kernel(const V* __restrict__ v, int64_t v_stride,
                                const double* __restrict__ alpha, const double* __restrict__ rv,
                                const double* __restrict__ loss, const double* __restrict__ cnt,
                                int n, int d, double* __restrict__ out, int* __restrict__ watchdog,
                                double* __restrict__ mirror) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    fold_items<true>([&](int p, double a) { return a * double(v[(int64_t)p * v_stride + i]); }, alpha, rv, loss,
                     cnt, 1, n, d, out, watchdog, mirror);
}

int launch_fold_f32(const float* wf32, int64_t wstride, const double* walpha, const double* rv,
                    const double* loss, const double* cnt, int n, int d, double* out,
                    int* watchdog, hipStream_t stream, double* mirror) {
    if (n <= 0) return -1;
    const int threads = kFoldThreads;
    const int blocks = (d + 1 + threads - 1) / threads;
    hipLaunchKernelGGL(fold_scaled_kernel<float>, dim3(blocks), dim3(threads), 0, stream, wf32, wstride, walpha,
                       rv, loss, cnt, n, d, out, watchdog, mirror);
    return (int)hipGetLastError();
}

int launch_fold_f64(const double* wv, int64_t wstride_d, const double* walpha, const double* rv,
                    const double* loss, const double* cnt, int n, int d, double* out,
                    int* watchdog, hipStream_t stream, double* mirror) {
    if (n <= 0) return -1;
    const int threads = kFoldThreads;
    const int blocks = (d + 1 + threads - 1) / threads;
    hipLaunchKernelGGL(fold_scaled_kernel<double>, dim3(blocks), dim3(threads), 0, stream, wv, wstride_d, walpha,
                       rv, loss, cnt, n, d, out, watchdog, mirror);
    return (int)hipGetLastError();
}

// sum((a-b)^2) and sum(b^2) (a may be null: then sum(b^2) and sum(|b|)) -- one block, fixed
// reduction tree, deterministic.
__global__ __launch_bounds__(256) void sq_terms_kernel(const double* __restrict__ a,
                                                       const double* __restrict__ b, int d,
                                                       double* __restrict__ out) {
    __shared__ double s0[256], s1[256];
    double t0 = 0.0, t1 = 0.0;
    for (int i = threadIdx.x; i < d; i += 256) {
        const double bv = b[i];
        if (a) { const double df = a[i] - bv; t0 += df * df; t1 += bv * bv; }
        else { t0 += bv * bv; t1 += fabs(bv); }
    }
    s0[threadIdx.x] = t0;
    s1[threadIdx.x] = t1;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
        if (threadIdx.x < h) {
            s0[threadIdx.x] += s0[threadIdx.x + h];
            s1[threadIdx.x] += s1[threadIdx.x + h];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) { out[0] = s0[0]; out[1] = s1[0]; }
}

// The fp64 Logistic chain's lossSum (PSGD.scala:254/:259; [ext] MLlib 1.6.1 LogisticGradient:
// margin = -z, loss = y > 0 ? log1pExp(margin) : log1pExp(margin) - margin) from the dots z_t
// chain_dense stored, one 1024-thread workgroup per chain. Every row's loss is the reference's
// arithmetic on the chain's own z_t; only the sum is a tree instead of the sequential `+=`
// (within the fp64 1e-9 bar).
__global__ __launch_bounds__(1024) void logistic_loss64_kernel(ChainLaunch L) {
    const int chain = blockIdx.x;
    const int64_t n = L.cnt[chain];
    const double* y = L.descs[chain].y;
    const double* z = L.zbuf64 + (int64_t)chain * L.zstride;
    double acc = 0.0;
    for (int64_t t = threadIdx.x; t < n; t += blockDim.x) {
        double mult;
        acc += gradient_scalar<G_LOGISTIC, double>(as_global(z)[t], as_global(y)[t], mult);
    }
    acc = wave_sum(acc);
    __shared__ double part[16];
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double s = 0.0;
        for (int k = 0; k < 16; ++k) s += part[k];
        L.loss[chain] = s;
    }
}

// stepSize / math.sqrt(iter) for iter = 1..n (SGDUpdater.scala:93, :133, :174, :210, :261).
__global__ void steps_kernel(double step, int64_t n, double* __restrict__ steps) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n) steps[j] = step / sqrt(double(j + 1));
}

// ------------------------------------------------------------------------------------------
// Launchers / dispatch.
// ------------------------------------------------------------------------------------------
template <typename S, typename T, int GRAD, int UPD, bool CONV, int NV>
static int launch_reg(const ChainLaunch& L, const KParams& kp, bool full, size_t lds, hipStream_t st) {
    // Ring geometry from the per-workgroup LDS budget (`lds`: chosen by the host so that the
    // chains spread evenly over the CUs). D rows stay in flight beyond the newest published row
    // (vmcnt holds at most 63 instructions, NV per row); R - D >= 8 slots stay published or
    // free so neither wave can wait on the other forever.
    constexpr int ROW = NV * 1024;
    // Ring geometry from the per-workgroup LDS budget (`lds`: chosen by the host so that the
    // chains spread evenly over the CUs); the consumer reads rows t and t+1, the loader keeps
    // loader_depth rows in flight and drains before it blocks on a full ring.
    const size_t budget = lds > 0 ? lds : (size_t)64 * 1024;
    const int D = loader_depth<NV>();
    int R = (int)((budget - sizeof(RingHeader) - 3 * kMetaBlockBytes) / ROW);
    int MB = (R + kMetaRows - 1) / kMetaRows + 2;
    while (R > 0 && sizeof(RingHeader) + (size_t)MB * kMetaBlockBytes + (size_t)R * ROW > budget) {
        --R;
        MB = (R + kMetaRows - 1) / kMetaRows + 2;
    }
    if (R < 6) return (int)hipErrorInvalidValue;  // LDS budget too small for this d (R >= PUB + 2)
    RingGeom g{R, MB, D, 0};
    const size_t bytes = sizeof(RingHeader) + (size_t)MB * kMetaBlockBytes + (size_t)R * ROW;
    if (full) {
        auto k = chain_dense<S, T, GRAD, UPD, CONV, NV, true>;
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
        hipLaunchKernelGGL(k, dim3(kp.n_chains), dim3(128), bytes, st, L, kp, g);
    } else {
        auto k = chain_dense<S, T, GRAD, UPD, CONV, NV, false>;
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
        hipLaunchKernelGGL(k, dim3(kp.n_chains), dim3(128), bytes, st, L, kp, g);
    }
    if constexpr (GRAD == G_LOGISTIC && sizeof(T) == 8) {
        if (!L.zbuf64) return (int)hipErrorInvalidValue;
        hipLaunchKernelGGL(logistic_loss64_kernel, dim3(kp.n_chains), dim3(1024), 0, st, L);
    }
    return (int)hipGetLastError();
}

int launch_logistic_loss64(const ChainLaunch& L, int n_chains, hipStream_t st) {
    if (!L.zbuf64) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(logistic_loss64_kernel, dim3(n_chains), dim3(1024), 0, st, L);
    return (int)hipGetLastError();
}

template <typename S, typename T, int GRAD, int UPD, bool CONV>
static int dispatch_nv(const ChainLaunch& L, const KParams& kp, int64_t min_ld, int64_t max_ld,
                       size_t lds, hipStream_t st, int* variant) {
    constexpr int VEC = 16 / sizeof(S);
    int nv = 1;
    while (nv * 64 * VEC < max_ld) nv *= 2;
    // FULL: every lane's every vector is inside every row (no exec masking on the loads).
    const bool full = min_ld >= (int64_t)nv * 64 * VEC;
    if (variant) *variant = 100 + nv;
    // fp64 AdaGrad / Adam hold at most 16 doubles per lane (dispatch_layout): no NV past that
    constexpr int NVMAX = (sizeof(T) == 8 && UPD >= U_ADAGRAD) ? 16 / VEC : 8;
    switch (nv) {
    case 1: return launch_reg<S, T, GRAD, UPD, CONV, 1>(L, kp, full, lds, st);
    case 2: return launch_reg<S, T, GRAD, UPD, CONV, 2>(L, kp, full, lds, st);
    case 4: return launch_reg<S, T, GRAD, UPD, CONV, 4>(L, kp, full, lds, st);
    case 8:
        if constexpr (NVMAX >= 8) return launch_reg<S, T, GRAD, UPD, CONV, 8>(L, kp, full, lds, st);
        return -1;
    default: return -1;
    }
}

template <typename S, int LAYOUT, int GRAD, int UPD, bool CONV>
static int launch_gen(const ChainLaunch& L, const KParams& kp, hipStream_t st, int* variant) {
    if (variant) *variant = 200 + LAYOUT;
    hipLaunchKernelGGL((chain_general<S, LAYOUT, GRAD, UPD, CONV>), dim3(kp.n_chains), dim3(64), 0,
                       st, L, kp);
    return (int)hipGetLastError();
}

template <typename S, int GRAD, int UPD, bool CONV>
static int dispatch_layout(const ChainLaunch& L, const KParams& kp, int layout, int compute,
                           int64_t min_ld, int64_t max_ld, size_t lds, hipStream_t st, int* variant) {
    constexpr int VEC = 16 / sizeof(S);
    if constexpr (UPD <= U_L1) {
        if (layout == kDense && max_ld <= 8 * 64 * VEC) {
            if (compute == 1) return dispatch_nv<S, float, GRAD, UPD, CONV>(L, kp, min_ld, max_ld, lds, st, variant);
            return dispatch_nv<S, double, GRAD, UPD, CONV>(L, kp, min_ld, max_ld, lds, st, variant);
        }
    } else {
        // AdaGrad / Adam: weights and status in registers. fp32: up to 8 row vectors per lane;
        // fp64 (the parity mode): up to 16 doubles per lane (weights, status and two row buffers
        // are 5 x 16 doubles = 160 VGPRs), d <= 1,024; past that chain_general, status in HBM
        if (layout == kDense && compute == 1 && max_ld <= 8 * 64 * VEC)
            return dispatch_nv<S, float, GRAD, UPD, CONV>(L, kp, min_ld, max_ld, lds, st, variant);
        if (layout == kDense && compute == 0 && max_ld <= 16 * 64)
            return dispatch_nv<S, double, GRAD, UPD, CONV>(L, kp, min_ld, max_ld, lds, st, variant);
    }
    if (layout == kDense) return launch_gen<S, kDense, GRAD, UPD, CONV>(L, kp, st, variant);
    return launch_gen<S, kCsr, GRAD, UPD, CONV>(L, kp, st, variant);
}

template <typename S, int GRAD, int UPD>
static int dispatch_conv(const ChainLaunch& L, const KParams& kp, int layout, int compute,
                         bool conv, int64_t min_ld, int64_t max_ld, size_t lds, hipStream_t st, int* variant) {
    if (conv) return dispatch_layout<S, GRAD, UPD, true>(L, kp, layout, compute, min_ld, max_ld, lds, st, variant);
    return dispatch_layout<S, GRAD, UPD, false>(L, kp, layout, compute, min_ld, max_ld, lds, st, variant);
}

template <typename S, int GRAD>
static int dispatch_upd(const ChainLaunch& L, const KParams& kp, int layout, int compute, int upd,
                        bool conv, int64_t min_ld, int64_t max_ld, size_t lds, hipStream_t st, int* variant) {
    switch (upd) {
    case U_SIMPLE: return dispatch_conv<S, GRAD, U_SIMPLE>(L, kp, layout, compute, conv, min_ld, max_ld, lds, st, variant);
    case U_SQUARED_L2: return dispatch_conv<S, GRAD, U_SQUARED_L2>(L, kp, layout, compute, conv, min_ld, max_ld, lds, st, variant);
    case U_L1: return dispatch_conv<S, GRAD, U_L1>(L, kp, layout, compute, conv, min_ld, max_ld, lds, st, variant);
    case U_ADAGRAD: return dispatch_conv<S, GRAD, U_ADAGRAD>(L, kp, layout, compute, conv, min_ld, max_ld, lds, st, variant);
    case U_ADAM: return dispatch_conv<S, GRAD, U_ADAM>(L, kp, layout, compute, conv, min_ld, max_ld, lds, st, variant);
    default: return -1;
    }
}

template <typename S>
static int dispatch_grad(const ChainLaunch& L, const KParams& kp, int layout, int compute, int grad,
                         int upd, bool conv, int64_t min_ld, int64_t max_ld, size_t lds,
                         hipStream_t st, int* variant) {
    switch (grad) {
    case G_LOGISTIC: return dispatch_upd<S, G_LOGISTIC>(L, kp, layout, compute, upd, conv, min_ld, max_ld, lds, st, variant);
    case G_LEAST_SQUARES: return dispatch_upd<S, G_LEAST_SQUARES>(L, kp, layout, compute, upd, conv, min_ld, max_ld, lds, st, variant);
    case G_HINGE: return dispatch_upd<S, G_HINGE>(L, kp, layout, compute, upd, conv, min_ld, max_ld, lds, st, variant);
    default: return -1;
    }
}

// PSGD_PER_SAMPLE=1 keeps the per-sample kernels (A/B measurements, tests; read at every launch)
bool per_sample_forced() {
    const char* e = getenv("PSGD_PER_SAMPLE");
    return e && *e && *e != '0';
}

int launch_chains(const ChainLaunch& L, const KParams& kp, int layout, int storage, int compute,
                  int gradient, int updater, bool check_conv, int64_t min_ld, int64_t max_ld,
                  int lds_spread, hipStream_t stream, int* kernel_variant, int64_t max_nnz,
                  int* weights_in) {
    if (weights_in) *weights_in = kWeightsOut;
    if (kp.n_chains <= 0) return 0;
    if (kp.nc > 0)   // LogisticGradient(numClasses > 2)
        return launch_multinomial_chains(L, kp, layout, storage, updater, check_conv, stream, kernel_variant);
    const bool per_sample = per_sample_forced();
    if (!per_sample && block64_path_applies(layout, compute, updater, check_conv, storage, max_ld))
        return launch_block64_chains(L, kp, storage, gradient, updater, min_ld, max_ld, lds_spread,
                                     stream, kernel_variant);
    if (!per_sample && block_path_applies(layout, compute, updater, check_conv, storage, max_ld))
        return launch_block_chains(L, kp, storage, gradient, updater, min_ld, max_ld, lds_spread,
                                   stream, kernel_variant);
    if (!per_sample && sparse_path_applies(layout, compute, updater, check_conv)) {
        if (weights_in) *weights_in = kWeightsF32;
        const int e = launch_sparse_chains(L, kp, storage, gradient, updater, max_nnz, stream, kernel_variant);
        if (e != -3) return e;
        if (weights_in) *weights_in = kWeightsOut;   // tol > 0 past the LDS kernel's range
    }
    // PSGD_SPARSE_KERNEL=hbm64 keeps fp64 CSR epochs off the LDS kernel (tests, A/B measurements;
    // read at every launch)
    const char* force = getenv("PSGD_SPARSE_KERNEL");
    const bool hbm64 = force && strcmp(force, "hbm64") == 0;
    if (!per_sample && !hbm64 && layout == kCsr && compute == 0 &&
        sparse_lds64_applies(kp.d, max_nnz, updater, check_conv, kp.alpha_ok != 0, kp.n_max) && L.wf32)
        return launch_sparse_lds64_chains(L, kp, storage, gradient, updater, max_nnz, stream, kernel_variant);
    // fp64 CSR beyond the LDS kernel's d (C5): the chain's weights as a double vector in HBM
    if (!per_sample && sparse64_path_applies(layout, compute, updater, check_conv, kp.alpha_ok != 0) && L.wf32 &&
        L.walpha) {
        if (weights_in) *weights_in = kWeightsF64;
        return launch_sparse64_chains(L, kp, storage, gradient, updater, stream, kernel_variant);
    }
    if (!per_sample && split_path_applies(layout, updater, check_conv, storage, max_ld)) {
        const int e = launch_split_chains(L, kp, storage, compute, gradient, updater, min_ld, max_ld,
                                          lds_spread, stream, kernel_variant);
        if (e != -3) return e;
    }
    const size_t lds = (size_t)(lds_spread > 0 ? lds_spread : 0);
    if (storage == 1)
        return dispatch_grad<float>(L, kp, layout, compute, gradient, updater, check_conv, min_ld,
                                    max_ld, lds, stream, kernel_variant);
    return dispatch_grad<double>(L, kp, layout, compute, gradient, updater, check_conv, min_ld,
                                 max_ld, lds, stream, kernel_variant);
}

int launch_fold(const double* w, int64_t w_stride, const double* rv, const double* loss,
                const double* cnt, int64_t s_stride, int n, int d, double* out,
                int* watchdog, hipStream_t stream, double* mirror) {
    if (n <= 0) return -1;
    const int threads = kFoldThreads;
    const int blocks = (d + 1 + threads - 1) / threads;
    hipLaunchKernelGGL(fold_kernel, dim3(blocks), dim3(threads), 0, stream, w, w_stride, rv, loss,
                       cnt, s_stride, n, d, out, watchdog, mirror);
    return (int)hipGetLastError();
}

int launch_sq_terms(const double* a, const double* b, int d, double* out2, hipStream_t stream) {
    hipLaunchKernelGGL(sq_terms_kernel, dim3(1), dim3(256), 0, stream, a, b, d, out2);
    return (int)hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// Bernoulli sampling of one epoch's batch ([ext] Spark 1.6.1 BernoulliSampler on an
// XORShiftRandom, restated in oracle/psgd_oracle.c or_sample_partition). fraction <= 0.4:
// GapSamplingIterator (geometric skips, u = max(nextDouble, 5e-11), k = (int)(log(u) /
// log1p(-f)), a skip before the first row and after every returned row); else the filter
// nextDouble() <= fraction per row, in iterator order.
//
// The reference walks one XORShift sequence per partition; a lane doing the same is bound by
// one dependent label load per row (~20 ms for 40k-row partitions). Both samplers consume
// exactly two XORShift steps per draw (one nextDouble), and XORShift is linear over GF(2), so
// draw j's state is D^j s0 with D the 64x64 bit matrix of two steps. One workgroup per
// partition: thread i owns draws [r + 64 i, r + 64 i + 64) of round r (16384 draws a round),
// reaching its first state through the jump matrices D^(64 * 2^k) (built at compile time),
// and an exclusive scan over threads places its output: the filter's kept-row counts, or
// the gap sampler's positions (pos_j = sum_{i<=j} k_i + j, strictly increasing, so the
// emitted rows are exactly the draws with pos_j < n_rows and row j lands at index j).
// ------------------------------------------------------------------------------------------
namespace {
struct Gf2Mat {
    uint64_t c[64];   // column b = D * e_b
};
constexpr uint64_t xs_step(uint64_t x) {
    x ^= x << 21;
    x ^= x >> 35;
    x ^= x << 4;
    return x;
}
constexpr uint64_t gf2_apply_c(const Gf2Mat& m, uint64_t s) {
    uint64_t r = 0;
    for (int b = 0; b < 64; ++b)
        if ((s >> b) & 1) r ^= m.c[b];
    return r;
}
constexpr Gf2Mat gf2_square(const Gf2Mat& m) {
    Gf2Mat r{};
    for (int b = 0; b < 64; ++b) r.c[b] = gf2_apply_c(m, m.c[b]);
    return r;
}
constexpr int kSampThreads = 256;
constexpr int kSampDraws = 64;   // draws per thread per round (a power of two: D^64 by squaring)
struct SampleJumps {
    Gf2Mat j[9];   // j[k] = D^(64 * 2^k): k < 8 place thread i, j[8] advances a round
};
constexpr SampleJumps make_sample_jumps() {
    Gf2Mat d{};
    for (int b = 0; b < 64; ++b) d.c[b] = xs_step(xs_step(1ull << b));
    for (int i = 0; i < 6; ++i) d = gf2_square(d);
    SampleJumps s{};
    s.j[0] = d;
    for (int k = 1; k < 9; ++k) s.j[k] = gf2_square(s.j[k - 1]);
    return s;
}
static_assert(kSampThreads == 256 && kSampDraws == 64, "jump table is built for 256 x 64 draws");
}  // namespace

__constant__ SampleJumps kSampleJumps = make_sample_jumps();

__device__ __forceinline__ uint64_t gf2_apply(const Gf2Mat& m, uint64_t s) {
    uint64_t r = 0;
#pragma unroll 16
    for (int b = 0; b < 64; ++b) r ^= m.c[b] & (0ull - ((s >> b) & 1));
    return r;
}

__device__ __forceinline__ int32_t xs_next(uint64_t& st, int bits) {
    const uint64_t x = xs_step(st);
    st = x;
    return (int32_t)(x & ((1ull << bits) - 1));
}
__device__ __forceinline__ double xs_next_double(uint64_t& st) {
    const int64_t a = xs_next(st, 26);
    const int64_t b = xs_next(st, 27);
    return (double)((a << 27) + b) * 0x1.0p-53;
}
// GapSamplingIterator's skip for one draw
__device__ __forceinline__ int64_t gap_skip(uint64_t& st, double lnq) {
    double u = xs_next_double(st);
    if (u < 5e-11) u = 5e-11;
    const double q = log(u) / lnq;
    return q >= 2147483647.0 ? 2147483647 : (int64_t)q;
}

// Exclusive scan of v over the workgroup; *total gets the sum. sh holds kSampThreads entries.
__device__ __forceinline__ int64_t block_excl_scan(int64_t v, int64_t* sh, int64_t* total) {
    const int tid = threadIdx.x;
    sh[tid] = v;
    __syncthreads();
    for (int off = 1; off < kSampThreads; off <<= 1) {
        const int64_t t = tid >= off ? sh[tid - off] : 0;
        __syncthreads();
        sh[tid] += t;
        __syncthreads();
    }
    const int64_t incl = sh[tid];
    *total = sh[kSampThreads - 1];
    __syncthreads();
    return incl - v;
}

__global__ __launch_bounds__(kSampThreads) void sample_kernel(const ChainDesc* __restrict__ base,
                                                              ChainDesc* __restrict__ out,
                                                              const uint64_t* __restrict__ xs_state,
                                                              double fraction, int32_t* __restrict__ rows,
                                                              double* __restrict__ ys, int64_t stride) {
    __shared__ int64_t sh[kSampThreads];
    __shared__ int sh_emit;
    const int c = blockIdx.x;
    const int tid = threadIdx.x;
    ChainDesc dsc = base[c];
    int32_t* r = rows + (int64_t)c * stride;
    double* yo = ys ? ys + (int64_t)c * stride : nullptr;
    const double* Y = dsc.y;
    const int64_t nr = dsc.n_rows;
    uint64_t st = xs_state[c];
#pragma unroll 1
    for (int k = 0; k < 8; ++k)
        if ((tid >> k) & 1) st = gf2_apply(kSampleJumps.j[k], st);
    constexpr int64_t kRound = (int64_t)kSampThreads * kSampDraws;
    int64_t m = 0;
    if (fraction <= 0.4) {
        const double lnq = log1p(-fraction);
        int64_t pos_round = 0;   // the position before the round's first draw
        for (int64_t draw0 = 0;; draw0 += kRound) {
            uint64_t s = st;
            int64_t adv = 0;
            for (int j = 0; j < kSampDraws; ++j) adv += gap_skip(s, lnq) + 1;
            int64_t total;
            int64_t pos = pos_round + block_excl_scan(adv, sh, &total);
            if (tid == 0) sh_emit = 0;
            __syncthreads();
            s = st;
            int emitted = 0;
            const int64_t j0 = draw0 + (int64_t)tid * kSampDraws;
            for (int j = 0; j < kSampDraws; ++j) {
                pos += gap_skip(s, lnq);
                if (pos >= nr) break;
                r[j0 + j] = (int32_t)pos;
                if (yo) yo[j0 + j] = Y[pos];
                ++emitted;
                pos += 1;
            }
            atomicAdd(&sh_emit, emitted);
            __syncthreads();
            const int64_t e = sh_emit;
            pos_round += total;
            if (e < kRound) {   // a draw reached n_rows: the emitted draws are a prefix
                m = draw0 + e;
                break;
            }
            st = gf2_apply(kSampleJumps.j[8], st);
            __syncthreads();   // sh_emit is reset next round
        }
    } else {
        for (int64_t draw0 = 0; draw0 < nr; draw0 += kRound) {
            uint64_t s = st;
            uint64_t keep = 0;
            const int64_t t0 = draw0 + (int64_t)tid * kSampDraws;
            for (int j = 0; j < kSampDraws; ++j)
                if (xs_next_double(s) <= fraction && t0 + j < nr) keep |= 1ull << j;
            int64_t total;
            int64_t o = m + block_excl_scan(__popcll(keep), sh, &total);
            while (keep) {
                const int j = __ffsll((unsigned long long)keep) - 1;
                keep &= keep - 1;
                r[o] = (int32_t)(t0 + j);
                if (yo) yo[o] = Y[t0 + j];
                ++o;
            }
            m += total;
            st = gf2_apply(kSampleJumps.j[8], st);
        }
    }
    if (tid == 0) {
        dsc.rows = r;
        if (yo) dsc.y = yo;
        dsc.n_rows = m;
        out[c] = dsc;
    }
}

int launch_sample(const ChainDesc* base, ChainDesc* out, const uint64_t* xs_state, double fraction,
                  int32_t* rows, double* ys, int64_t stride, int n_chains, hipStream_t stream) {
    if (n_chains <= 0) return 0;
    hipLaunchKernelGGL(sample_kernel, dim3((unsigned)n_chains), dim3(kSampThreads), 0, stream, base, out,
                       xs_state, fraction, rows, ys, stride);
    return (int)hipGetLastError();
}

int launch_steps(double step, int64_t n, double* steps, hipStream_t stream) {
    if (n <= 0) return 0;
    const int threads = 256;
    const int64_t blocks = (n + threads - 1) / threads;
    hipLaunchKernelGGL(steps_kernel, dim3((unsigned)blocks), dim3(threads), 0, stream, step, n, steps);
    return (int)hipGetLastError();
}

}  // namespace psgd
