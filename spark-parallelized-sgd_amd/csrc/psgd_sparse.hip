// psgd_sparse.hip -- the fp32 throughput-mode chain for CSR rows (gfx950).
//
// Reference: ParallelizedSGD.scala:243-270 (the chain), [ext] MLlib 1.6.1 Gradient.scala
// (Logistic / LeastSquares / Hinge on SparseVector rows: the gradient is mult * x, non-zero only
// at the row's indices), SGDUpdater.scala:86-98 (Simple) and :163-181 (SquaredL2).
//
// Wide sparse models (rcv1: 47,236 features; 2^22 in BASELINE config 5) do not fit a CU's LDS,
// so each chain keeps its weights as an fp32 vector in HBM (P x d floats: 48 MB at rcv1 shape,
// L2/MALL-resident) and one wave walks the partition:
//   * lane l owns the row's entries l, l+64, ... (two per lane for rows of <= 128 non-zeros);
//   * the weights at those indices are gathered with L1-bypassing (sc1) loads, which the same
//     wave's earlier plain stores to the same addresses precede in L2: consecutive rows that
//     share a feature see the updated value;
//   * the next row's (col, val), label and step, and the row pointers of the row after it, are
//     loaded while the current row's gather is in flight, so a sample costs one gather round
//     trip plus the wave reduction;
//   * the update touches only the row's indices (w_j += c x_j); Hinge rows inside the margin
//     (c = 0) store nothing.
// SquaredL2 scales every coordinate by a_t = 1 - s_t*lambda each sample (UPD.scala:169): the
// chain keeps w = alpha * v (alpha in f64), so the scale is one multiply of alpha and an update
// adds c x_j / alpha to v_j (the alpha-scaled lazy form). regVal needs ||w|| after
// the chain's last sample only (PSGD.scala:257): 0.5 * lambda * alpha^2 * ||v||^2.
// No MFMA, no LDS: the work per sample is a 94-long gather-dot and scatter.
// The per-sample break (tol > 0, CONV; PSGD.scala:262, :324-336), here and in chain_sparse64: the
// wave tests isConverged after every sample from z, q = x . x (a second wave sum), c and an f64
// ||w||^2 recurrence from ||w_in||^2 (L.wnsq0), as chain_sparse_lds does (its header), and leaves
// the walk after the first passing sample.
#include "psgd_device.h"

#include <stdlib.h>
#include <string.h>

namespace psgd {

// isConverged(w, w') with w' = a w + c x from z = x . w, q = x . x and nsq = ||w||^2 (updated to
// ||w'||^2): D < tol^2 max(N, 1) with N = a (a nsq + 2 c z) + c^2 q, D = b (b nsq - 2 c z) + c^2 q
__device__ __forceinline__ bool conv_step(double a, double c, double z, double q, double tol2, double& nsq) {
    const double b = 1.0 - a, cq = c * c * q;
    const double nn = a * __builtin_fma(a, nsq, 2.0 * c * z) + cq;
    const double dd = b * __builtin_fma(b, nsq, -2.0 * c * z) + cq;
    nsq = nn > 0.0 ? nn : 0.0;
    return dd < tol2 * (nn > 1.0 ? nn : 1.0);
}

template <typename S, int GRAD, int UPD, bool CONV = false>
__global__ __launch_bounds__(64) void chain_sparse(ChainLaunch L, KParams kp) {
    constexpr bool L2 = UPD == U_SQUARED_L2;
    const int lane = threadIdx.x;
    const int chain = blockIdx.x;
    const ChainDesc dsc = L.descs[chain];
    const int64_t n = dsc.n_rows;
    const gptr<S> X = as_global(reinterpret_cast<const S*>(dsc.x));
    const gptr<int32_t> COL = as_global(dsc.col);
    const gptr<int64_t> RP = as_global(dsc.row_ptr);
    const gptr<double> Y = as_global(dsc.y);
    const gptr<double> STEPS = as_global(L.steps);
    const gptr<int32_t> RIDX = dsc.rows ? as_global(dsc.rows) : nullptr;   // sampled epoch
    float* V = L.wf32 + (int64_t)chain * L.wstride;   // = float(w_in) (wf32_init_kernel)
    const gmut<float> VW = as_global_mut(V);

    double alpha = 1.0;      // SquaredL2: w = alpha * v
    double dnsq = 0.0;       // SquaredL2: this lane's part of ||v||^2 - ||v_0||^2
    double loss_sum = 0.0;
    float loss_blk = 0.0f;
    int64_t count = 0;
    double wn = CONV ? *L.wnsq0 : 0.0;   // CONV: ||w||^2
    const double tol2 = kp.tol * kp.tol;

    // Software pipeline: row t+2's entry range is loaded during sample t, row t+1's entries,
    // label and step during sample t (their range is known by then), so the only round trip a
    // sample waits for is its own gather.
    auto row_of = [&](int64_t t) __attribute__((always_inline)) -> int64_t {
        return RIDX ? (int64_t)RIDX[t] : t;
    };
    auto range_of = [&](int64_t t, int64_t& b, int64_t& e) __attribute__((always_inline)) {
        if (t < n) {
            const int64_t r = row_of(t);
            b = RP[r];
            e = RP[r + 1];
        } else {
            b = e = 0;
        }
    };
    auto entries_of = [&](int64_t t, int64_t b, int64_t e, double& yy, double& ss, int32_t& ca,
                          int32_t& cb, float& xa, float& xb) __attribute__((always_inline)) {
        yy = t < n ? Y[t] : 0.0;
        ss = t < n ? STEPS[t] : 0.0;
        const int64_t ka = b + lane, kc = b + 64 + lane;
        ca = ka < e ? COL[ka] : 0;
        xa = ka < e ? float(X[ka]) : 0.0f;
        cb = kc < e ? COL[kc] : 0;
        xb = kc < e ? float(X[kc]) : 0.0f;
    };
    int64_t kb = 0, ke = 0, kb1 = 0, ke1 = 0;     // ranges of rows t and t+1
    double y = 0.0, s = 0.0;
    int32_t c0 = 0, c1 = 0;
    float x0 = 0.0f, x1 = 0.0f;
    range_of(0, kb, ke);
    range_of(1, kb1, ke1);
    entries_of(0, kb, ke, y, s, c0, c1, x0, x1);

    for (int64_t t = 0; t < n; ++t) {
        const int64_t nnz = ke - kb;
        const bool a0 = lane < nnz, a1 = lane + 64 < nnz;
        // gather (sc1: served by L2, after this wave's earlier stores to the same lines)
        float w0 = a0 ? __hip_atomic_load(&V[c0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0f;
        float w1 = a1 ? __hip_atomic_load(&V[c1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0f;
        // under the gather: row t+1's entries (its range is known), row t+2's range
        double ny = 0.0, ns = 0.0;
        int32_t n0 = 0, n1 = 0;
        float nx0 = 0.0f, nx1 = 0.0f;
        entries_of(t + 1, kb1, ke1, ny, ns, n0, n1, nx0, nx1);
        int64_t kb2, ke2;
        range_of(t + 2, kb2, ke2);

        float acc = x0 * w0;
        acc = __builtin_fmaf(x1, w1, acc);
        [[maybe_unused]] float qa = CONV ? __builtin_fmaf(x1, x1, x0 * x0) : 0.0f;
        // entries past the first 128 (rows wider than two per lane)
        for (int64_t k = kb + 128 + lane; k < ke; k += 64) {
            const float xk = float(X[k]);
            acc = __builtin_fmaf(xk, __hip_atomic_load(&V[COL[k]], __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT), acc);
            if constexpr (CONV) qa = __builtin_fmaf(xk, xk, qa);
        }
        float z = wave_sum_uniform(acc);
        [[maybe_unused]] const float qx = CONV ? wave_sum_uniform(qa) : 0.0f;
        const float sf = float(s);
        if constexpr (L2) {
            // w <- a w + c x: alpha absorbs a; the dot was taken against w = alpha v
            z = float(alpha * double(z));
            alpha *= 1.0 - s * kp.reg;
        }
        float loss;
        const float c = sparse_coef<GRAD>(z, float(y), sf, loss);
        bool conv = false;
        if constexpr (CONV)
            conv = conv_step(L2 ? 1.0 - s * kp.reg : 1.0, double(c), double(z), double(qx), tol2, wn);
        loss_blk += loss;
        if ((t & 31) == 31) { loss_sum += double(loss_blk); loss_blk = 0.0f; }
        count += 1;
        if (c != 0.0f) {
            const float cv = L2 ? float(double(c) / alpha) : c;
            const float nv0 = __builtin_fmaf(cv, x0, w0), nv1 = __builtin_fmaf(cv, x1, w1);
            if (a0) VW[c0] = nv0;
            if (a1) VW[c1] = nv1;
            if constexpr (L2) dnsq += nsq_delta(w0, nv0) + nsq_delta(w1, nv1);
            for (int64_t k = kb + 128 + lane; k < ke; k += 64) {
                const int32_t j = COL[k];
                const float wj = __hip_atomic_load(&V[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const float nj = __builtin_fmaf(cv, float(X[k]), wj);
                VW[j] = nj;
                if constexpr (L2) dnsq += nsq_delta(wj, nj);
            }
        }
        if (conv) break;   // CONV: sample t passed isConverged (it is taken)
        kb = kb1; ke = ke1; kb1 = kb2; ke1 = ke2;
        y = ny; s = ns; c0 = n0; c1 = n1; x0 = nx0; x1 = nx1;
    }
    loss_sum += double(loss_blk);
    if constexpr (GRAD == G_LEAST_SQUARES) loss_sum = loss_sum / 2.0;

    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    sparse_chain_out<L2>(L, kp, chain, lane, alpha, dnsq, loss_sum, count);
}

// ------------------------------------------------------------------------------------------
// chain_sparse64: the same walk in fp64 compute -- the parity mode's CSR chain for models whose
// weights cannot live on chip (C5: 2^22 features), i.e. the reference's own arithmetic
// (ParallelizedSGD.scala:253-268 on Double, SGDUpdater.scala:86-98 / :163-181).
//   * the chain's weights are a double vector in HBM (its slice of L.wf32, 2 (d + 1152) floats;
//     34 GB for C5's 1,024 chains), = w_in at the start (w64_init_kernel);
//   * per sample: gathers of the row's weights (global_load_dwordx2 sc1, after this wave's earlier
//     stores in L2), dot = per-lane fma over entries l, l + 64 and the wave tree (chain_general's
//     order), Gradient.compute in Double (gradient_scalar<GRAD, double>), and the row's stores
//     w_j + (-s) (mult x_j) (global_store_dwordx2); rows with mult = 0 (Hinge inside the margin)
//     store nothing -- the reference's update adds a zero there;
//   * SquaredL2 in the alpha-scaled form w = alpha v of chain_general (alpha *= 1 - s lambda, then
//     v_j += ((-s)(mult x_j)) / alpha), valid without renormalisation only while every prefix
//     product of the epoch stays in [2^-400, 2^400]: the host checks that (kp.alpha_ok) and runs
//     chain_general otherwise;
//   * regVal = 0.5 lambda ||alpha v||^2 after the last sample by one O(d) pass in chain_general's
//     lane order; the fold reads w = alpha v straight from the vectors (fold_f64_kernel).
// Everything but the dot's wave tree is chain_general's arithmetic operator for operator.
// ------------------------------------------------------------------------------------------
template <typename S, int GRAD, int UPD, bool CONV = false>
__global__ __launch_bounds__(64) void chain_sparse64(ChainLaunch L, KParams kp) {
    constexpr bool L2 = UPD == U_SQUARED_L2;
    const int lane = threadIdx.x;
    const int chain = blockIdx.x;
    const ChainDesc dsc = L.descs[chain];
    const int64_t n = dsc.n_rows;
    const int d = kp.d;
    const gptr<S> X = as_global(reinterpret_cast<const S*>(dsc.x));
    const gptr<int32_t> COL = as_global(dsc.col);
    const gptr<int64_t> RP = as_global(dsc.row_ptr);
    const gptr<double> Y = as_global(dsc.y);
    const gptr<double> STEPS = as_global(L.steps);
    const gptr<int32_t> RIDX = dsc.rows ? as_global(dsc.rows) : nullptr;   // sampled epoch
    double* V = reinterpret_cast<double*>(L.wf32 + (int64_t)chain * L.wstride);   // = w_in
    const gmut<double> VW = as_global_mut(V);
    // gathers: relaxed agent-scope loads (global_load_dwordx2 ... sc1, served by L2 after this
    // wave's earlier stores to the same lines, as in chain_sparse); the compiler counts them
    auto gather = [&](int32_t j) __attribute__((always_inline)) -> double {
        return __hip_atomic_load(&V[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };

    double alpha = 1.0;      // SquaredL2: w = alpha * v
    double loss_sum = 0.0;
    int64_t count = 0;
    double wn = CONV ? *L.wnsq0 : 0.0;   // CONV: ||w||^2
    const double tol2 = kp.tol * kp.tol;

    // software pipeline as chain_sparse: row t+1's entries, label and step and row t+2's range
    // load under row t's gather
    auto range_of = [&](int64_t t, int64_t& b, int64_t& e) __attribute__((always_inline)) {
        if (t < n) {
            const int64_t r = RIDX ? (int64_t)RIDX[t] : t;
            b = RP[r];
            e = RP[r + 1];
        } else {
            b = e = 0;
        }
    };
    auto entries_of = [&](int64_t t, int64_t b, int64_t e, double& yy, double& ss, int32_t& ca,
                          int32_t& cb, double& xa, double& xb) __attribute__((always_inline)) {
        yy = t < n ? Y[t] : 0.0;
        ss = t < n ? STEPS[t] : 0.0;
        const int64_t ka = b + lane, kc = b + 64 + lane;
        ca = ka < e ? COL[ka] : 0;
        xa = ka < e ? double(X[ka]) : 0.0;
        cb = kc < e ? COL[kc] : 0;
        xb = kc < e ? double(X[kc]) : 0.0;
    };
    int64_t kb = 0, ke = 0, kb1 = 0, ke1 = 0;
    double y = 0.0, s = 0.0;
    int32_t c0 = 0, c1 = 0;
    double x0 = 0.0, x1 = 0.0;
    range_of(0, kb, ke);
    range_of(1, kb1, ke1);
    entries_of(0, kb, ke, y, s, c0, c1, x0, x1);

    for (int64_t t = 0; t < n; ++t) {
        const int64_t nnz = ke - kb;
        const bool a0 = lane < nnz, a1 = lane + 64 < nnz;
        const double w0 = a0 ? gather(c0) : 0.0;
        const double w1 = a1 ? gather(c1) : 0.0;
        double ny = 0.0, ns = 0.0;
        int32_t n0 = 0, n1 = 0;
        double nx0 = 0.0, nx1 = 0.0;
        entries_of(t + 1, kb1, ke1, ny, ns, n0, n1, nx0, nx1);
        int64_t kb2, ke2;
        range_of(t + 2, kb2, ke2);

        // dot(x, v): chain_general's per-lane fma order over entries lane, lane + 64, lane + 128, ...
        double acc = m_fma(x0, w0, 0.0);
        acc = m_fma(x1, w1, acc);
        [[maybe_unused]] double qa = CONV ? m_fma(x1, x1, x0 * x0) : 0.0;
        for (int64_t k = kb + 128 + lane; k < ke; k += 64) {
            const double xk = double(X[k]);
            acc = m_fma(xk, gather(COL[k]), acc);
            if constexpr (CONV) qa = m_fma(xk, xk, qa);
        }
        double z;
        if constexpr (CONV) {
            wave_sum2(acc, qa);
            z = acc;
        } else {
            z = wave_sum(acc);
        }
        if constexpr (L2) z = alpha * z;      // dot(x, w) with w = alpha v
        double mult;
        loss_sum += gradient_scalar<GRAD, double>(z, y, mult);
        count += 1;
        const double a = -s;
        bool conv = false;
        if constexpr (CONV) conv = conv_step(L2 ? 1.0 - s * kp.reg : 1.0, a * mult, z, qa, tol2, wn);
        if constexpr (L2) alpha = alpha * (1.0 - s * kp.reg);
        if (mult != 0.0) {
            // v_j + (a * (mult * x_j)) [/ alpha] at the row's indices
            double u0 = a * (mult * x0), u1 = a * (mult * x1);
            if constexpr (L2) { u0 = u0 / alpha; u1 = u1 / alpha; }
            if (a0) VW[c0] = w0 + u0;
            if (a1) VW[c1] = w1 + u1;
            for (int64_t k = kb + 128 + lane; k < ke; k += 64) {
                const int32_t j = COL[k];
                double u = a * (mult * double(X[k]));
                if constexpr (L2) u = u / alpha;
                VW[j] = gather(j) + u;
            }
        }
        if (conv) break;   // CONV: sample t passed isConverged (it is taken)
        kb = kb1; ke = ke1; kb1 = kb2; ke1 = ke2;
        y = ny; s = ns; c0 = n0; c1 = n1; x0 = nx0; x1 = nx1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    double rv = 0.0;
    if constexpr (L2) {
        // regVal = 0.5 lambda ||w||^2 of the last update (UPD.scala:176-180), w_i = alpha v_i, in
        // chain_general's lane order (its W[i] = alpha * W[i]; acc += W[i] * W[i])
        double nsq = 0.0;
#pragma unroll 8
        for (int i = lane; i < d; i += 64) {
            const double wi = alpha * gather(i);
            nsq += wi * wi;
        }
        nsq = wave_sum(nsq);
        if (count > 0) {
            const double nrm = sqrt(nsq);
            rv = 0.5 * kp.reg * nrm * nrm;
        }
    }
    if (lane == 0) {
        L.walpha[chain] = alpha;
        L.rv[chain] = rv;
        L.loss[chain] = loss_sum;
        L.cnt[chain] = count;
        L.cnt_d[chain] = double(count);
    }
}

// ------------------------------------------------------------------------------------------
// chain_sparse_spec: the same chain with the gathers issued SK samples ahead (rows of <= 128
// non-zeros).
//
// A gather for row u issued during sample u-SK does not see the stores of rows u-SK .. u-1
// (issued after it). A helper wave finds, for every entry of row u, the latest of those rows
// that has the same feature: it keeps tagpos[j] = (row & 255) << 8 | entry of the last row that
// touched feature j (2 bytes per feature in LDS: d up to ~58k); an entry from outside the
// window is ignored, and a row's tags are cleared before its LDS slot is reused (so an 8-bit
// row tag never aliases). The chain wave replaces such a gathered value by that row's new value (kept in LDS) --
// exactly the value the reference's sequential update would read. Waves:
//   wave 0 (chain)  per sample t: waits for row t's gather (issued SK samples earlier; a fixed
//                   count of VMEM instructions per sample makes it s_waitcnt vmcnt(4 SK - 2)),
//                   corrects it, dot + wave reduction + coefficient, issues the gather of row
//                   t + SK, stores the row's new weights (to HBM and to its LDS slot);
//   wave 1 (helper) loads the rows (64 row pointers / labels / steps per batch, entries of 8
//                   rows per round trip) into an SR-slot LDS ring with their correction entries.
// The chain's weights start as float(w_in) (wf32_init_kernel) and stay in L.wf32.
// ------------------------------------------------------------------------------------------
constexpr int SCAP = 128;         // entries per row (two per lane)
// The chain at sample t needs row t + SK staged; the helper stages 8-row groups and may reuse
// the slot of row u - SR once the chain is done with row u - SR + SK: it can always stage the
// group holding row t + SK if SR >= 2 SK + 8.
template <int SK, int SR>
constexpr bool spec_ring_ok() { return SR >= 2 * SK + 8 && (SR & (SR - 1)) == 0 && 4 * SK - 2 <= 63; }

struct SpecHeader {
    unsigned ready;   // rows staged by the helper
    unsigned done;    // rows finished by the chain
    unsigned stop;
    unsigned pad;
};
struct SpecSlot {
    int32_t col[SCAP];
    float val[SCAP];
    int16_t prev[SCAP];    // -1, or (row delta 1..SK) << 8 | entry of the latest earlier row
    float nv[SCAP];        // the row's new weights (chain)
    int32_t nnz;
    int32_t pad;
    double y, s;
};

template <typename S, int GRAD, int UPD, int SK, int SR>
__global__ __launch_bounds__(128) void chain_sparse_spec(ChainLaunch L, KParams kp) {
    static_assert(spec_ring_ok<SK, SR>(), "ring too small for the speculation depth");
    constexpr bool L2 = UPD == U_SQUARED_L2;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    SpecHeader* hdr = reinterpret_cast<SpecHeader*>(smem);
    SpecSlot* slots = reinterpret_cast<SpecSlot*>(smem + sizeof(SpecHeader));
    uint16_t* tagpos = reinterpret_cast<uint16_t*>(smem + sizeof(SpecHeader) + SR * sizeof(SpecSlot));
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int chain = blockIdx.x;
    const ChainDesc dsc = L.descs[chain];
    const int d = kp.d;
    const int64_t n = dsc.n_rows;
    float* V = L.wf32 + (int64_t)chain * L.wstride;   // [d] weights + [128] dummy targets

    for (int i = threadIdx.x; i < d; i += blockDim.x) tagpos[i] = 0xFFFF;
    if (threadIdx.x == 0) { hdr->ready = 0; hdr->done = 0; hdr->stop = 0; }
    __syncthreads();

    uint64_t st_wait = 0;                     // diagnostic: cycles spent waiting on the other wave
    const uint64_t st_begin = __builtin_amdgcn_s_memtime();
    auto spin = [&](const unsigned* flag, int64_t need, int code) __attribute__((always_inline)) -> bool {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        const uint64_t c0 = __builtin_amdgcn_s_memtime();
        for (;;) {
            // relaxed: the flags and the slots are LDS, which one wave reads and writes in order
            if ((int64_t)__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= need) {
                __atomic_signal_fence(__ATOMIC_SEQ_CST);
                st_wait += __builtin_amdgcn_s_memtime() - c0;
                return true;
            }
            if (__hip_atomic_load(&hdr->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return false;
            if (__builtin_amdgcn_s_memrealtime() - t0 > kWatchdogTicks) {
                __hip_atomic_fetch_or(L.watchdog, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&hdr->stop, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                return false;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    };

    if (wave == 1) {
        // ---------------- helper: stage rows with their correction entries ----------------
        const gptr<S> X = as_global(reinterpret_cast<const S*>(dsc.x));
        const gptr<int32_t> COL = as_global(dsc.col);
        const gptr<int64_t> RP = as_global(dsc.row_ptr);
        const gptr<double> Y = as_global(dsc.y);
        const gptr<double> STEPS = as_global(L.steps);
        const gptr<int32_t> RIDX = dsc.rows ? as_global(dsc.rows) : nullptr;
        unsigned done = 0;
        const void* dummy_i = (const void*)(V + d + lane);            // valid, never used
        const void* dummy_s = (const void*)(V + d + 2 * lane);
        // Software pipeline: the row ranges / labels / steps of the next 64-row batch and the
        // entries of the next 8-row group are in flight while the current group is staged.
        struct Batch { int64_t rb, re; double y, s; };
        auto load_batch = [&](int64_t g) __attribute__((always_inline)) -> Batch {
            Batch bt{0, 0, 0.0, 0.0};
            const int64_t ti = g + lane;
            if (ti < n) {
                const int64_t r = RIDX ? (int64_t)RIDX[ti] : ti;
                bt.rb = RP[r];
                bt.re = RP[r + 1];
                bt.y = Y[ti];
                bt.s = STEPS[ti];
            }
            return bt;
        };
        struct Group { int32_t ca[8], cb[8]; float xa[8], xb[8]; int64_t b[8], e[8]; };
        auto rl64 = [&](int64_t v, int i) __attribute__((always_inline)) -> int64_t {
            return (int64_t)(uint32_t)__builtin_amdgcn_readlane((int)(v & 0xffffffff), i) |
                   ((int64_t)__builtin_amdgcn_readlane((int)(v >> 32), i) << 32);
        };
        // entries of rows g + i0 .. g + i0 + 7 of batch bt (rows past n: empty)
        auto load_group = [&](const Batch& bt, int64_t g, int i0, Group& G) __attribute__((always_inline)) {
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const bool live = g + i0 + q < n;
                G.b[q] = live ? rl64(bt.rb, i0 + q) : 0;
                G.e[q] = live ? rl64(bt.re, i0 + q) : 0;
                // unconditional loads (masked-off entries read the chain's dummy floats), so the
                // compiler can count them instead of draining vmcnt around branches
                const int64_t ka = G.b[q] + lane, kc = G.b[q] + 64 + lane;
                const bool ia = ka < G.e[q], ic = kc < G.e[q];
                const int32_t va = *(ia ? &COL[ka] : (gptr<int32_t>)dummy_i);
                const S sa = *(ia ? &X[ka] : (gptr<S>)dummy_s);
                const int32_t vc = *(ic ? &COL[kc] : (gptr<int32_t>)dummy_i);
                const S sc = *(ic ? &X[kc] : (gptr<S>)dummy_s);
                G.ca[q] = ia ? va : 0;
                G.xa[q] = ia ? float(sa) : 0.0f;
                G.cb[q] = ic ? vc : 0;
                G.xb[q] = ic ? float(sc) : 0.0f;
            }
        };
        // Stage rows g + i0 .. + 7 (those < n) from G, in phases so that the LDS round trips of
        // the eight rows overlap (one wave's LDS operations execute in program order, so a later
        // row's tag read still sees an earlier row's tag write without waiting for it):
        //   D: clear the tags rows u - SR + 1 still own (their slots are reused by rows u + 1);
        //   A: each row's tag lookups and tag writes;
        //   B: wait until the chain is done with the slots being reused;
        //   C: write the rows' slots (entries, correction entries, label, step), publish.
        auto stage_group = [&](const Batch& bt, int64_t g, int i0, const Group& G) __attribute__((always_inline)) -> bool {
            const int64_t u0 = g + i0;
            int nq = (int)(n - u0 < 8 ? n - u0 : 8);
            // D
            {
                int32_t oa[8], ob[8], on[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const int64_t o = u0 + q - SR + 1;
                    const bool live = q < nq && o >= 0;
                    const SpecSlot& so = slots[(o + SR) % SR];
                    on[q] = live ? so.nnz : 0;
                    oa[q] = so.col[lane];
                    ob[q] = so.col[lane + 64];
                }
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const int64_t o = u0 + q - SR + 1;
                    const unsigned otag = (unsigned)(o & 255) << 8;
                    if (lane < on[q] && tagpos[oa[q]] == (otag | (unsigned)lane)) tagpos[oa[q]] = 0xFFFF;
                    if (lane + 64 < on[q] && tagpos[ob[q]] == (otag | (unsigned)(lane + 64))) tagpos[ob[q]] = 0xFFFF;
                }
            }
            // A
            unsigned ta[8], tc[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int64_t u = u0 + q;
                const int nnz = q < nq ? (int)(G.e[q] - G.b[q]) : 0;
                const unsigned tag = (unsigned)(u & 255) << 8;
                ta[q] = 0xFFFF;
                tc[q] = 0xFFFF;
                if (lane < nnz) {
                    ta[q] = tagpos[G.ca[q]];
                    tagpos[G.ca[q]] = (uint16_t)(tag | (unsigned)lane);
                }
                if (lane + 64 < nnz) {
                    tc[q] = tagpos[G.cb[q]];
                    tagpos[G.cb[q]] = (uint16_t)(tag | (unsigned)(lane + 64));
                }
            }
            // B: slot u % SR last held row u - SR, read by the chain up to row u - SR + SK
            const int64_t need = u0 + nq - 1 - SR + SK + 1;
            if ((int64_t)done < need) {
                if (!spin(&hdr->done, need, 16)) return false;
                done = __hip_atomic_load(&hdr->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            // C
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                if (q < nq) {
                    const int64_t u = u0 + q;
                    SpecSlot& sl = slots[u % SR];
                    const unsigned dla = ((unsigned)u - (ta[q] >> 8)) & 255;
                    const unsigned dlc = ((unsigned)u - (tc[q] >> 8)) & 255;
                    const int32_t pa = (ta[q] != 0xFFFF && dla >= 1 && dla <= SK) ? (int32_t)(dla << 8 | (ta[q] & 255)) : -1;
                    const int32_t pb = (tc[q] != 0xFFFF && dlc >= 1 && dlc <= SK) ? (int32_t)(dlc << 8 | (tc[q] & 255)) : -1;
                    sl.col[lane] = G.ca[q];
                    sl.col[lane + 64] = G.cb[q];
                    sl.val[lane] = G.xa[q];
                    sl.val[lane + 64] = G.xb[q];
                    sl.prev[lane] = (int16_t)pa;
                    sl.prev[lane + 64] = (int16_t)pb;
                    if (lane == 0) {
                        sl.nnz = (int)(G.e[q] - G.b[q]);
                        sl.y = readlane_d(bt.y, i0 + q);
                        sl.s = readlane_d(bt.s, i0 + q);
                    }
                }
            }
            __atomic_signal_fence(__ATOMIC_SEQ_CST);
            if (nq > 0)
                __hip_atomic_store(&hdr->ready, (unsigned)(u0 + nq), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            return true;
        };
        Batch cur = load_batch(0), nxt = load_batch(64);
        Group GA, GB;
        load_group(cur, 0, 0, GA);
        for (int64_t g = 0; g < n; g += 64) {
            bool ok = true;
            static_for<4>([&](auto kc) {
                // group i0 is in GA; fetch group i0 + 8 into GB, stage GA; then the same the other way
                constexpr int i0 = 16 * decltype(kc)::value;
                if (!ok) return;
                load_group(cur, g, i0 + 8, GB);
                ok = stage_group(cur, g, i0, GA);
                if constexpr (i0 + 16 < 64) load_group(cur, g, i0 + 16, GA);
                else load_group(nxt, g + 64, 0, GA);
                if (ok) ok = stage_group(cur, g, i0 + 8, GB);
            });
            if (!ok) break;
            cur = nxt;
            nxt = load_batch(g + 128);
        }
        if (L.stamps && lane == 0) {
            L.stamps[(size_t)chain * 4 + 2] = __builtin_amdgcn_s_memtime() - st_begin;
            L.stamps[(size_t)chain * 4 + 3] = st_wait;
        }
        return;
    }

    // ---------------- chain ----------------
    double alpha = 1.0;
    double dnsq = 0.0;                        // SquaredL2: ||v||^2 - ||v_0||^2 (this lane)
    double loss_sum = 0.0;
    float loss_blk = 0.0f;
    int64_t count = 0;
    unsigned ready = 0;
    float* dummy = V + d + lane;              // target of masked-off gathers / stores
    float gr[SK][2];                          // gathered weights of rows t .. t + SK - 1
    // prologue: gathers of rows 0 .. SK-1, each followed by two (dummy) stores, the same
    // VMEM pattern as a sample of the loop
    auto issue_gather = [&](int64_t u, float (&g)[2]) __attribute__((always_inline)) -> bool {
        const float* pa = dummy;
        const float* pb = dummy;
        if (u < n) {
            if ((int64_t)ready < u + 1) {
                if (!spin(&hdr->ready, u + 1, 2)) return false;
                ready = __hip_atomic_load(&hdr->ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            const SpecSlot& sl = slots[u % SR];
            const int nnz = sl.nnz;
            if (lane < nnz) pa = V + sl.col[lane];
            if (lane + 64 < nnz) pb = V + sl.col[lane + 64];
        }
        g[0] = gather_sc1(pa);
        g[1] = gather_sc1(pb);
        return true;
    };
    bool ok = true;
    static_for<SK>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        if (ok) ok = issue_gather(q, gr[q]);
        store_f32(dummy, 0.0f);
        store_f32(dummy, 0.0f);
    });
    // one sample; Q = t % SK (compile-time in the unrolled loop)
    auto sample = [&](auto qc, int64_t t) __attribute__((always_inline)) -> bool {
        constexpr int Q = decltype(qc)::value;
        // row t's gather: issued SK samples ago, followed by 4 SK - 2 VMEM instructions
        asm volatile("s_waitcnt vmcnt(%2)" : "+v"(gr[Q][0]), "+v"(gr[Q][1]) : "i"(4 * SK - 2) : "memory");
        const SpecSlot& sl = slots[t % SR];
        const int nnz = sl.nnz;
        float w0 = gr[Q][0], w1 = gr[Q][1];
        const float x0 = sl.val[lane], x1 = sl.val[lane + 64];
        const int32_t p0 = sl.prev[lane], p1 = sl.prev[lane + 64];   // sign-extended
        // features also in rows t-SK .. t-1: their stores came after this gather
        if (p0 >= 0) w0 = slots[(t - (p0 >> 8)) % SR].nv[p0 & 255];
        if (p1 >= 0) w1 = slots[(t - (p1 >> 8)) % SR].nv[p1 & 255];
        if (lane >= nnz) { w0 = 0.0f; }
        if (lane + 64 >= nnz) { w1 = 0.0f; }
        float acc = x0 * w0;
        acc = __builtin_fmaf(x1, w1, acc);
        float z = wave_sum_uniform(acc);
        const double s = sl.s;
        if constexpr (L2) {
            z = float(alpha * double(z));
            alpha *= 1.0 - s * kp.reg;
        }
        float loss;
        const float c = sparse_coef<GRAD>(z, float(sl.y), float(s), loss);
        loss_blk += loss;
        if ((t & 31) == 31) { loss_sum += double(loss_blk); loss_blk = 0.0f; }
        count += 1;
        const float cv = L2 ? float(double(c) / alpha) : c;
        const float nv0 = __builtin_fmaf(cv, x0, w0);
        const float nv1 = __builtin_fmaf(cv, x1, w1);
        if constexpr (L2) dnsq += nsq_delta(w0, nv0) + nsq_delta(w1, nv1);
        SpecSlot& slw = slots[t % SR];
        slw.nv[lane] = nv0;
        slw.nv[lane + 64] = nv1;
        const int32_t c0 = sl.col[lane], c1 = sl.col[lane + 64];
        // the gather of row t + SK, then this row's stores (2 + 2 VMEM instructions)
        if (!issue_gather(t + SK, gr[Q])) return false;
        store_f32(lane < nnz ? V + c0 : dummy, nv0);
        store_f32(lane + 64 < nnz ? V + c1 : dummy, nv1);
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        __hip_atomic_store(&hdr->done, (unsigned)(t + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return true;
    };
    for (int64_t t = 0; ok && t < n; t += SK) {
        static_for<SK>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            if (ok && t + q < n) ok = sample(qc, t + q);
        });
    }
    __hip_atomic_store(&hdr->stop, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (L.stamps && lane == 0) {
        L.stamps[(size_t)chain * 4 + 0] = __builtin_amdgcn_s_memtime() - st_begin;
        L.stamps[(size_t)chain * 4 + 1] = st_wait;
    }
    loss_sum += double(loss_blk);
    if constexpr (GRAD == G_LEAST_SQUARES) loss_sum = loss_sum / 2.0;
    sparse_chain_out<L2>(L, kp, chain, lane, alpha, dnsq, loss_sum, count);
}

template <int SK, int SR>
size_t spec_lds_bytes(int d) {
    return sizeof(SpecHeader) + SR * sizeof(SpecSlot) + (((size_t)d * 2 + 15) / 16) * 16;
}

// any tol: with the per-sample break (tol > 0) chain_sparse_lds or chain_sparse runs it
bool sparse_path_applies(int layout, int compute, int updater, bool check_conv) {
    (void)check_conv;
    return layout == kCsr && compute == 1 && (updater == U_SIMPLE || updater == U_SQUARED_L2);
}

template <typename S, int GRAD>
static int sparse_upd(const ChainLaunch& L, const KParams& kp, int upd, hipStream_t st) {
    const bool conv = kp.tol > 0.0;   // the per-sample break: instances of their own
    auto k = upd == U_SIMPLE ? (conv ? chain_sparse<S, GRAD, U_SIMPLE, true> : chain_sparse<S, GRAD, U_SIMPLE, false>)
                             : (conv ? chain_sparse<S, GRAD, U_SQUARED_L2, true>
                                     : chain_sparse<S, GRAD, U_SQUARED_L2, false>);
    hipLaunchKernelGGL(k, dim3(kp.n_chains), dim3(64), 0, st, L, kp);
    return (int)hipGetLastError();
}

template <typename S>
static int sparse_grad(const ChainLaunch& L, const KParams& kp, int grad, int upd, hipStream_t st) {
    switch (grad) {
    case G_LOGISTIC: return sparse_upd<S, G_LOGISTIC>(L, kp, upd, st);
    case G_LEAST_SQUARES: return sparse_upd<S, G_LEAST_SQUARES>(L, kp, upd, st);
    case G_HINGE: return sparse_upd<S, G_HINGE>(L, kp, upd, st);
    default: return -3;
    }
}

template <typename S, int GRAD, int SK, int SR>
static int spec_upd(const ChainLaunch& L, const KParams& kp, int upd, hipStream_t st) {
    const size_t lds = spec_lds_bytes<SK, SR>(kp.d);
    auto k = upd == U_SIMPLE ? chain_sparse_spec<S, GRAD, U_SIMPLE, SK, SR>
                             : chain_sparse_spec<S, GRAD, U_SQUARED_L2, SK, SR>;
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k, dim3(kp.n_chains), dim3(128), lds, st, L, kp);
    return (int)hipGetLastError();
}

template <typename S, int SK, int SR>
static int spec_grad(const ChainLaunch& L, const KParams& kp, int grad, int upd, hipStream_t st) {
    switch (grad) {
    case G_LOGISTIC: return spec_upd<S, G_LOGISTIC, SK, SR>(L, kp, upd, st);
    case G_LEAST_SQUARES: return spec_upd<S, G_LEAST_SQUARES, SK, SR>(L, kp, upd, st);
    case G_HINGE: return spec_upd<S, G_HINGE, SK, SR>(L, kp, upd, st);
    default: return -3;
    }
}

template <int SK, int SR>
static int spec_launch(const ChainLaunch& L, const KParams& kp, int storage, int grad, int upd, hipStream_t st) {
    if (storage == 1) return spec_grad<float, SK, SR>(L, kp, grad, upd, st);
    return spec_grad<double, SK, SR>(L, kp, grad, upd, st);
}

// ------------------------------------------------------------------------------------------
// Epoch set-up of the fp32 CSR chains: every chain's fp32 weights = float(w_in), written by the
// whole GPU (a slice of w_in is read once per block and stored to a range of chains), instead of
// by each chain's one wave before its first sample (2^22 features x 1024 chains = 17 GB);
// wnsq0 = ||float(w_in)||^2 in f64 (SquaredL2 and the per-sample break; one block, fixed tree:
// deterministic; the fp64 kernels' break takes ||w_in||^2 itself, round_f32 = false).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void wf32_init_kernel(float* __restrict__ wf, int64_t wstride,
                                                        const double* __restrict__ w_in, int d,
                                                        int n_chains, int chains_per_block) {
    const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
    if (i >= d) return;
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = i + k < d ? float(w_in[i + k]) : 0.0f;
    const int p0 = blockIdx.y * chains_per_block;
    const int p1 = p0 + chains_per_block < n_chains ? p0 + chains_per_block : n_chains;
    const bool full = i + 4 <= d;
    for (int p = p0; p < p1; ++p) {
        float* dst = wf + (int64_t)p * wstride + i;
        if (full) {
            *reinterpret_cast<f32x4*>(dst) = f32x4{v[0], v[1], v[2], v[3]};
        } else {
            for (int k = 0; k < 4 && i + k < d; ++k) dst[k] = v[k];
        }
    }
}

__global__ __launch_bounds__(1024) void wnsq0_kernel(const double* __restrict__ w_in, int d,
                                                     double* __restrict__ out, bool round_f32) {
    __shared__ double s[1024];
    double t = 0.0;
    for (int i = threadIdx.x; i < d; i += 1024) {
        const double v = round_f32 ? double(float(w_in[i])) : w_in[i];
        t += v * v;
    }
    s[threadIdx.x] = t;
    __syncthreads();
    for (int h = 512; h > 0; h >>= 1) {
        if ((int)threadIdx.x < h) s[threadIdx.x] += s[threadIdx.x + h];
        __syncthreads();
    }
    if (threadIdx.x == 0) *out = s[0];
}

int launch_wnsq0(const ChainLaunch& L, int d, bool round_f32, hipStream_t st) {
    hipLaunchKernelGGL(wnsq0_kernel, dim3(1), dim3(1024), 0, st, L.w_in, d, L.wnsq0, round_f32);
    return (int)hipGetLastError();
}

static int sparse_epoch_init(const ChainLaunch& L, const KParams& kp, int updater, hipStream_t st) {
    const int bx = (kp.d + 1023) / 1024;
    int by = (2048 + bx - 1) / bx;          // >= 2048 blocks in all
    by = by < kp.n_chains ? by : kp.n_chains;
    const int per = (kp.n_chains + by - 1) / by;
    by = (kp.n_chains + per - 1) / per;
    hipLaunchKernelGGL(wf32_init_kernel, dim3(bx, by), dim3(256), 0, st, L.wf32, L.wstride, L.w_in,
                       kp.d, kp.n_chains, per);
    if (updater == U_SQUARED_L2 || kp.tol > 0.0) return launch_wnsq0(L, kp.d, true, st);
    return (int)hipGetLastError();
}

// Epoch set-up of the fp64 CSR chains: every chain's double vector = w_in (GPU-wide, as
// wf32_init_kernel; C5: 34 GB in ~5 ms).
__global__ __launch_bounds__(256) void w64_init_kernel(double* __restrict__ wv, int64_t wstride_d,
                                                       const double* __restrict__ w_in, int d,
                                                       int n_chains, int chains_per_block) {
    const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 2;
    if (i >= d) return;
    const bool full = i + 2 <= d;
    const f64x2 v = full ? *reinterpret_cast<const f64x2*>(w_in + i) : f64x2{w_in[i], 0.0};
    const int p0 = blockIdx.y * chains_per_block;
    const int p1 = p0 + chains_per_block < n_chains ? p0 + chains_per_block : n_chains;
    for (int p = p0; p < p1; ++p) {
        double* dst = wv + (int64_t)p * wstride_d + i;
        if (full) *reinterpret_cast<f64x2*>(dst) = v;
        else dst[0] = v.x;
    }
}

bool sparse64_path_applies(int layout, int compute, int updater, bool check_conv, bool alpha_ok) {
    (void)check_conv;   // any tol: the per-sample break is a CONV instance (kp.tol > 0)
    return layout == kCsr && compute == 0 &&
           (updater == U_SIMPLE || (updater == U_SQUARED_L2 && alpha_ok));
}

template <typename S, int GRAD>
static int sparse64_upd(const ChainLaunch& L, const KParams& kp, int upd, hipStream_t st) {
    const bool conv = kp.tol > 0.0;   // the per-sample break: instances of their own
    auto k = upd == U_SIMPLE ? (conv ? chain_sparse64<S, GRAD, U_SIMPLE, true> : chain_sparse64<S, GRAD, U_SIMPLE, false>)
                             : (conv ? chain_sparse64<S, GRAD, U_SQUARED_L2, true>
                                     : chain_sparse64<S, GRAD, U_SQUARED_L2, false>);
    hipLaunchKernelGGL(k, dim3(kp.n_chains), dim3(64), 0, st, L, kp);
    return (int)hipGetLastError();
}

template <typename S>
static int sparse64_grad(const ChainLaunch& L, const KParams& kp, int grad, int upd, hipStream_t st) {
    switch (grad) {
    case G_LOGISTIC: return sparse64_upd<S, G_LOGISTIC>(L, kp, upd, st);
    case G_LEAST_SQUARES: return sparse64_upd<S, G_LEAST_SQUARES>(L, kp, upd, st);
    case G_HINGE: return sparse64_upd<S, G_HINGE>(L, kp, upd, st);
    default: return -3;
    }
}

int launch_sparse64_chains(const ChainLaunch& L, const KParams& kp, int storage, int gradient,
                           int updater, hipStream_t stream, int* kernel_variant) {
    if (kp.n_chains <= 0) return 0;
    if (!sparse64_path_applies(kCsr, 0, updater, false, kp.alpha_ok != 0)) return -3;
    // the chain's f64 vector: [d] + [128] + [1024] doubles inside its slice of L.wf32
    if (!L.wf32 || L.wstride < 2 * ((int64_t)kp.d + 128 + 1024) || (L.wstride & 3) || !L.walpha)
        return (int)hipErrorInvalidValue;
    const int bx = (kp.d + 511) / 512;
    int by = (2048 + bx - 1) / bx;
    by = by < kp.n_chains ? by : kp.n_chains;
    const int per = (kp.n_chains + by - 1) / by;
    by = (kp.n_chains + per - 1) / per;
    hipLaunchKernelGGL(w64_init_kernel, dim3(bx, by), dim3(256), 0, stream, reinterpret_cast<double*>(L.wf32),
                       L.wstride / 2, L.w_in, kp.d, kp.n_chains, per);
    if (kp.tol > 0.0) {
        // ||w_in||^2 for the per-sample break's norm recurrence
        if (!L.wnsq0) return (int)hipErrorInvalidValue;
        const int e = launch_wnsq0(L, kp.d, false, stream);
        if (e) return e;
    }
    // variant 420 + 40 (the per-sample break) + storage
    if (kernel_variant) *kernel_variant = 420 + (kp.tol > 0.0 ? 40 : 0) + storage;
    if (storage == 1) return sparse64_grad<float>(L, kp, gradient, updater, stream);
    return sparse64_grad<double>(L, kp, gradient, updater, stream);
}

int launch_sparse_chains(const ChainLaunch& L, const KParams& kp, int storage, int gradient,
                         int updater, int64_t max_nnz, hipStream_t stream, int* kernel_variant) {
    if (kp.n_chains <= 0) return 0;
    if (!L.wf32 || L.wstride < (int64_t)kp.d + 128 + 1024 || (L.wstride & 3) || !L.walpha || !L.wnsq0)
        return (int)hipErrorInvalidValue;
    int rc = sparse_epoch_init(L, kp, updater, stream);
    if (rc) return rc;
    // PSGD_SPARSE_KERNEL = lds | spec | plain forces a variant (tests, A/B measurements; read at
    // every launch); default: the first that applies in that order
    const char* force = getenv("PSGD_SPARSE_KERNEL");
    const bool any = !force || !*force;
    const bool no_lds = !any && strcmp(force, "lds") != 0;
    const bool no_spec = !any && strcmp(force, "spec") != 0;
    // first choice: the chain's weights in LDS (psgd_sparse_lds.hip), for rows of <= 128
    // non-zeros and d up to ~65k features
    if (!no_lds) {
        rc = launch_sparse_lds_chains(L, kp, storage, gradient, updater, max_nnz, stream, kernel_variant);
        if (rc != -3) return rc;
    }
    // chain_sparse_spec has no per-sample break; chain_sparse has (variant 440 + storage)
    if (!no_spec && kp.tol <= 0.0 && max_nnz <= SCAP && spec_lds_bytes<8, 32>(kp.d) <= 160 * 1024) {
        if (kernel_variant) *kernel_variant = 410 + storage;
        return spec_launch<8, 32>(L, kp, storage, gradient, updater, stream);
    }
    if (kernel_variant) *kernel_variant = 400 + (kp.tol > 0.0 ? 40 : 0) + storage;
    if (storage == 1) return sparse_grad<float>(L, kp, gradient, updater, stream);
    return sparse_grad<double>(L, kp, gradient, updater, stream);
}

// Longest row of a CSR partition (registration of device-resident rows).
__global__ void max_nnz_kernel(const int64_t* __restrict__ rp, int64_t n, unsigned long long* out) {
    unsigned long long m = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const unsigned long long z = (unsigned long long)(rp[i + 1] - rp[i]);
        m = z > m ? z : m;
    }
    if (m) atomicMax(out, m);
}

int csr_max_nnz(const int64_t* d_row_ptr, int64_t n, int64_t* out, hipStream_t st) {
    *out = 0;
    if (n <= 0) return 0;
    unsigned long long* d = nullptr;
    hipError_t e = hipMallocAsync((void**)&d, sizeof(unsigned long long), st);
    if (e) return (int)e;
    (void)hipMemsetAsync(d, 0, sizeof(unsigned long long), st);
    hipLaunchKernelGGL(max_nnz_kernel, dim3(256), dim3(256), 0, st, d_row_ptr, n, d);
    unsigned long long h = 0;
    (void)hipMemcpyAsync(&h, d, sizeof h, hipMemcpyDeviceToHost, st);
    e = hipStreamSynchronize(st);
    (void)hipFreeAsync(d, st);
    *out = (int64_t)h;
    return (int)e;
}

}  // namespace psgd
