// psgd_device.h -- device-side helpers shared by the chain kernels (psgd_kernels.hip: per-sample
// kernels; psgd_block.hip: the blocked fp32 kernel): wave reductions, scalar math in the
// reference's operator order, the MLlib gradient multipliers, and the LDS-DMA row loader.
#pragma once
#include "psgd_internal.h"

#include <hip/hip_runtime.h>
#include <math.h>

#include <utility>

namespace psgd {

enum { G_LOGISTIC = 0, G_LEAST_SQUARES = 1, G_HINGE = 2 };
enum { U_SIMPLE = 0, U_SQUARED_L2 = 1, U_L1 = 2, U_ADAGRAD = 3, U_ADAM = 4 };

// ------------------------------------------------------------------------------------------
// Wave-wide all-reduce. Every step adds a lane's value to its partner's (partners swap), so
// each lane computes the same two operands in the same order and ends with the same bits.
// ------------------------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
// (64-bit adds take no DPP operand: two v_mov_b32_dpp; bound_ctrl writes 0 for a lane without a
// source, as the old value 0 would, without the two v_mov 0 that an old operand costs)
template <int CTRL>
__device__ __forceinline__ double dpp_mov(double v) {
    long long b = __double_as_longlong(v);
    int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffffll), CTRL, 0xF, 0xF, true);
    int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, true);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// v_permlane16_swap / v_permlane32_swap (gfx950): with both operands = v, the pair returned
// holds {value of the even partner, value of the odd partner} in every lane.
__device__ __forceinline__ float swap_sum16(float v) {
    auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(p[0]) + __uint_as_float(p[1]);
}
__device__ __forceinline__ float swap_sum32(float v) {
    auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(p[0]) + __uint_as_float(p[1]);
}
__device__ __forceinline__ double swap_sum16(double v) {
    unsigned long long b = (unsigned long long)__double_as_longlong(v);
    unsigned lo = (unsigned)b, hi = (unsigned)(b >> 32);
    auto pl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    auto ph = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    double e = __longlong_as_double((long long)(((unsigned long long)ph[0] << 32) | pl[0]));
    double o = __longlong_as_double((long long)(((unsigned long long)ph[1] << 32) | pl[1]));
    return e + o;
}
__device__ __forceinline__ double swap_sum32(double v) {
    unsigned long long b = (unsigned long long)__double_as_longlong(v);
    unsigned lo = (unsigned)b, hi = (unsigned)(b >> 32);
    auto pl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    auto ph = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    double e = __longlong_as_double((long long)(((unsigned long long)ph[0] << 32) | pl[0]));
    double o = __longlong_as_double((long long)(((unsigned long long)ph[1] << 32) | pl[1]));
    return e + o;
}

// The k-ordered butterfly over a block's 8 rows where the blocked kernels' transposed reductions
// leave them (lane l carries row k(l) = l5 | l4<<1 | l3<<2): level J pairs the lanes that differ
// in k's bit J -- lane bit 5 (permlane32_swap), 4 (permlane16_swap), 3 (DPP row_ror 8) -- and
// returns the pair's values in k order (lo: the member with the bit clear), the same in both.
struct PairD { double lo, hi; };
template <int J>
__device__ __forceinline__ PairD kpair(double v, int lane) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)b, hi = (unsigned)(b >> 32);
    auto mk = [](unsigned l, unsigned h) __attribute__((always_inline)) {
        return __longlong_as_double((long long)(((unsigned long long)h << 32) | l));
    };
    if constexpr (J == 0) {
        auto pl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
        auto ph = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
        return {mk(pl[0], ph[0]), mk(pl[1], ph[1])};
    } else if constexpr (J == 1) {
        auto pl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
        auto ph = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
        return {mk(pl[0], ph[0]), mk(pl[1], ph[1])};
    } else {
        const double p = dpp_mov<0x128>(v);   // row_ror 8: lane l ^ 8
        return (lane & 8) ? PairD{p, v} : PairD{v, p};
    }
}
// the lane bit of k's bit J
template <int J>
constexpr int kbit() { return J == 0 ? 32 : J == 1 ? 16 : 8; }
// the rows (bit k) of a ballot over lanes 8g (lane 8g carries row g2 | g1<<1 | g0<<2)
__device__ __forceinline__ unsigned ballot_rows(unsigned long long m) {
    unsigned rows = 0;
#pragma unroll
    for (int g = 0; g < 8; ++g)
        if ((m >> (8 * g)) & 1ull) rows |= 1u << (((g >> 2) & 1) | (((g >> 1) & 1) << 1) | ((g & 1) << 2));
    return rows;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
    v = v + dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
    v = v + dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
    v = v + dpp_mov<0x141>(v);  // row_half_mirror
    v = v + dpp_mov<0x140>(v);  // row_mirror
    v = swap_sum16(v);
    v = swap_sum32(v);
    return v;
}

// Wave sum delivered as a wave-uniform value: four DPP row steps, then row_bcast:15 / :31 fold
// the four row sums into lane 63 ((r3 + r2) + (r1 + r0)), which v_readlane broadcasts. Two
// fewer instructions than the swap form and the result lands in SGPRs for the scalar math.
template <int CTRL, int ROWS>
__device__ __forceinline__ float dpp_mov_rows(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROWS, 0xF, false));
}
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_mov_rows(double v) {
    long long b = __double_as_longlong(v);
    int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffll), CTRL, ROWS, 0xF, false);
    int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, ROWS, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ float readlane63(float v) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
__device__ __forceinline__ double readlane63(double v) {
    long long b = __double_as_longlong(v);
    int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), 63);
    int hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
template <typename T>
__device__ __forceinline__ T wave_sum_uniform(T v) {
    v = v + dpp_mov<0xB1>(v);            // quad_perm [1,0,3,2]
    v = v + dpp_mov<0x4E>(v);            // quad_perm [2,3,0,1]
    v = v + dpp_mov<0x141>(v);           // row_half_mirror
    v = v + dpp_mov<0x140>(v);           // row_mirror: every lane holds its row's sum
    v = v + dpp_mov_rows<0x142, 0xA>(v); // row_bcast:15 -> rows 1, 3 hold r0+r1, r2+r3
    v = v + dpp_mov_rows<0x143, 0xC>(v); // row_bcast:31 -> row 3 holds the total
    return readlane63(v);
}

// Two independent sums reduced together (ILP for the convergence terms).
template <typename T>
__device__ __forceinline__ void wave_sum2(T& a, T& b) {
    a = a + dpp_mov<0xB1>(a);  b = b + dpp_mov<0xB1>(b);
    a = a + dpp_mov<0x4E>(a);  b = b + dpp_mov<0x4E>(b);
    a = a + dpp_mov<0x141>(a); b = b + dpp_mov<0x141>(b);
    a = a + dpp_mov<0x140>(a); b = b + dpp_mov<0x140>(b);
    a = swap_sum16(a);         b = swap_sum16(b);
    a = swap_sum32(a);         b = swap_sum32(b);
}

__device__ __forceinline__ double readlane_d(double v, int lane) {
    long long b = __double_as_longlong(v);
    int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), lane);
    int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// Global-address-space views: loads through them are global_load_* (in-order vmcnt) instead of
// flat_load_* (which also count on lgkmcnt and force full drains before every use).
template <typename T>
using gptr = const T __attribute__((address_space(1)))*;
template <typename T>
using gmut = T __attribute__((address_space(1)))*;
template <typename T>
__device__ __forceinline__ gptr<T> as_global(const T* p) { return (gptr<T>)(p); }
template <typename T>
__device__ __forceinline__ gmut<T> as_global_mut(T* p) { return (gmut<T>)(p); }

// ------------------------------------------------------------------------------------------
// Scalar math per precision.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ double m_exp(double x) { return exp(x); }
__device__ __forceinline__ float m_exp(float x) { return expf(x); }
__device__ __forceinline__ double m_log1p(double x) { return log1p(x); }
__device__ __forceinline__ float m_log1p(float x) { return log1pf(x); }
__device__ __forceinline__ double m_sqrt(double x) { return sqrt(x); }
__device__ __forceinline__ double m_fabs(double x) { return __builtin_fabs(x); }
__device__ __forceinline__ float m_fabs(float x) { return __builtin_fabsf(x); }
__device__ __forceinline__ float m_sqrt(float x) { return sqrtf(x); }
__device__ __forceinline__ double m_fma(double a, double b, double c) { return __builtin_fma(a, b, c); }
__device__ __forceinline__ double m_pow(double a, double b) { return pow(a, b); }
__device__ __forceinline__ float m_pow(float a, float b) { return powf(a, b); }
// a^b for a >= 0 in the fp32 throughput mode: the hardware log2 / exp2 (a few ulp)
__device__ __forceinline__ float pow_fast(float a, float b) {
    return __builtin_amdgcn_exp2f(b * __builtin_amdgcn_logf(a));
}
__device__ __forceinline__ float m_fma(float a, float b, float c) { return __builtin_fmaf(a, b, c); }

// The fp64 kernels' reciprocals and square roots sit on per-sample dependent chains: the
// hardware estimate and ONE Newton step. Measured on gfx950 (tools/newton_check, 4M inputs in
// [1, 1e6)): v_rcp_f64 alone 4.6e-8 relative, + 1 Newton step 2.2e-15 (2 steps: exact);
// v_rsq_f64 5.2e-8, + 1 step 4.3e-15 (2 steps: 2.6e-16) -- ~10-20 ulp, six orders of magnitude
// inside the fp64 mode's 1e-9 bar, for two fewer dependent f64 operations (four for rsq).
// 1/sqrt(x) for x >= 1 (x = inf gives 0, NaN stays NaN).
__device__ __forceinline__ double rsqrt_newton(double x) {
    double y = __builtin_amdgcn_rsq(x);
    const double e = __builtin_fma(-(x * y), y, 1.0);
    y = __builtin_fma(0.5 * y, e, y);
    return x == __builtin_inf() ? 0.0 : y;
}
// 1/x for finite x != 0 (NaN stays NaN).
__device__ __forceinline__ double recip_newton(double x) {
    const double y = __builtin_amdgcn_rcp(x);
    return __builtin_fma(y, __builtin_fma(-x, y, 1.0), y);
}
// sqrt(x) for x >= 0 as x * rsq(x) with one Newton step (sqrt(0) = 0, x < 0 or NaN gives NaN,
// sqrt(inf) = inf).
__device__ __forceinline__ double sqrt_newton(double x) {
    double y = __builtin_amdgcn_rsq(x);
    const double e = __builtin_fma(-(x * y), y, 1.0);
    y = __builtin_fma(0.5 * y, e, y);
    return (x == 0.0 || x == __builtin_inf()) ? x : x * y;
}

// 1.0 - pow(r, iter), the inside of AdamSGDUpdater's fix1 (UPD.scala:262), iter = j >= 1,
// bit for bit: when pow(r, iter) <= 2^-54 the f64 subtraction rounds 1 - p to exactly 1.0 (the
// double below 1 is 1 - 2^-53), so the ~100-instruction f64 pow is needed only while
// iter * log2(r) >= -60. The hardware f32 log2 (relative error ~1e-7: 6e-6 binades at 60) decides
// that; the wave runs the pow only while one of its coordinates still needs it, i.e. for its
// first few tens of samples (r is an average of squared gradients, well below 1).
__device__ __forceinline__ double one_minus_pow_iter(double r, double iter) {
    const float l2 = __builtin_amdgcn_logf((float)r);
    double q = 1.0;
    if (!((float)iter * l2 < -60.0f)) q = 1.0 - pow(r, iter);
    return q;
}

// 1 / (1 + exp(m)) in f64 with a short dependent chain: the chains evaluate it once per row on
// their critical path, where the library exp (Horner) and IEEE division (div_scale / div_fmas /
// div_fixup) are ~30 dependent f64 operations. Here: exp(m) = 2^k e^r, k = rint(m log2 e),
// r = m - k ln2 (two-part ln2, |r| <= ln2/2), e^r by its Taylor polynomial of degree 11
// (truncation < 1e-14 relative; degree 13 until round 4, two more FMAs on every row's critical
// path for digits the 1e-9 bar does not use) evaluated Estrin-style (depth 4), 2^k by ldexp;
// the reciprocal by v_rcp_f64 and one Newton step (above). Within ~1e-14 relative of the
// reference's 1.0 / (1.0 + exp(margin)) (the fp64 mode's bar is 1e-9 relative). m is clamped to
// [-746, 709] (exp(-746) is 0 in f64; beyond 709 the result is ~1e-308 instead of 0); a NaN
// stays NaN.
__device__ __forceinline__ double recip_one_plus_exp(double m) {
    m = m > 709.0 ? 709.0 : m;
    m = m < -746.0 ? -746.0 : m;
    const double kd = __builtin_rint(m * 1.4426950408889634);
    double r = __builtin_fma(-kd, 6.93147180369123816490e-01, m);   // ln2 high part
    r = __builtin_fma(-kd, 1.90821492927058770002e-10, r);          // ln2 low part
    const double r2 = r * r, r4 = r2 * r2, r8 = r4 * r4;
    const double p01 = __builtin_fma(r, 1.0, 1.0);
    const double p23 = __builtin_fma(r, 1.0 / 6, 0.5);
    const double p45 = __builtin_fma(r, 1.0 / 120, 1.0 / 24);
    const double p67 = __builtin_fma(r, 1.0 / 5040, 1.0 / 720);
    const double p89 = __builtin_fma(r, 1.0 / 362880, 1.0 / 40320);
    const double pab = __builtin_fma(r, 1.0 / 39916800, 1.0 / 3628800);
    const double q03 = __builtin_fma(r2, p23, p01);
    const double q47 = __builtin_fma(r2, p67, p45);
    const double q8b = __builtin_fma(r2, pab, p89);
    const double q07 = __builtin_fma(r4, q47, q03);
    const double er = __builtin_fma(r8, q8b, q07);
    return recip_newton(1.0 + __builtin_amdgcn_ldexp(er, (int)kd));
}

// java.lang.Math.max(a, b): NaN if either is NaN.
template <typename T>
__device__ __forceinline__ T jmax(T a, T b) {
    return (a != a) ? a : ((b != b) ? b : (a >= b ? a : b));
}
// java.lang.Math.signum
template <typename T>
__device__ __forceinline__ T jsignum(T x) {
    return (x != x || x == T(0)) ? x : (x > T(0) ? T(1) : T(-1));
}

// [ext] MLlib 1.6.1 MLUtils.log1pExp
template <typename T>
__device__ __forceinline__ T log1p_exp(T x) {
    return x > T(0) ? x + m_log1p(m_exp(-x)) : m_log1p(m_exp(x));
}

// [ext] MLlib 1.6.1 Gradient.compute: the gradient is mult * x (Logistic: axpy(mult, x, 0);
// LeastSquares: scal(diff, x.copy); Hinge: scal(-labelScaled, x.copy) or the empty vector,
// which adds nothing -- mult = 0 gives the same weights). Returns loss.
template <int GRAD, typename T>
__device__ __forceinline__ T gradient_scalar(T z, T y, T& mult) {
    if constexpr (GRAD == G_LOGISTIC) {
        T margin = -z;                                    // -1.0 * dot(data, weights)
        mult = (T(1) / (T(1) + m_exp(margin))) - y;
        T l = log1p_exp(margin);
        return y > T(0) ? l : l - margin;
    } else if constexpr (GRAD == G_LEAST_SQUARES) {
        T diff = z - y;
        mult = diff;
        return diff * diff / T(2);
    } else {
        T ls = T(2) * y - T(1);
        T lz = ls * z;
        bool on = T(1) > lz;
        mult = on ? -ls : T(0);
        return on ? T(1) - lz : T(0);
    }
}

// fp32 CSR chains (psgd_sparse*.hip): the sample's update coefficient c = -s * mult (the row's
// new weights are w_j + c x_j) and its loss, in fp32 (LeastSquares loss is halved by the caller).
template <int GRAD>
__device__ __forceinline__ float sparse_coef(float z, float y, float s, float& loss) {
    if constexpr (GRAD == G_LEAST_SQUARES) {
        const float diff = z - y;
        loss = diff * diff;                      // halved once at the end
        return -s * diff;
    } else if constexpr (GRAD == G_LOGISTIC) {
        const float margin = -z;
        const float e = __expf(margin);
        const float sig = __builtin_amdgcn_rcpf(1.0f + e);
        const float ax = __builtin_fabsf(margin);
        const float l = __logf(1.0f + __expf(-ax)) + (margin > 0.0f ? margin : 0.0f);
        loss = y > 0.0f ? l : l - margin;
        return -s * (sig - y);
    } else {
        const float ls = 2.0f * y - 1.0f;
        const float lz = ls * z;
        const bool on = 1.0f > lz;
        loss = on ? 1.0f - lz : 0.0f;
        return on ? s * ls : 0.0f;
    }
}

// fp32 CSR chains: the chain's VMEM instructions are inline asm: their count per sample is what its vmcnt waits
// rely on, so the compiler must neither merge nor drop any of them.
__device__ __forceinline__ float gather_sc1(const float* p) {
    float v;
    asm volatile("global_load_dword %0, %1, off sc1" : "=v"(v) : "v"(p) : "memory");
    return v;
}
__device__ __forceinline__ void store_f32(float* p, float v) {
    asm volatile("global_store_dword %0, %1, off" : : "v"(p), "v"(v) : "memory");
}

// fp32 CSR chains with SquaredL2 track ||v||^2 as they update (regVal needs ||w|| after the
// chain's last sample, PSGD.scala:257, and an O(d) pass per chain over 2^22 features is what the
// sample stream cannot afford): the change of one coordinate, exact products of floats in f64.
__device__ __forceinline__ double nsq_delta(float w_old, float w_new) {
    const double a = double(w_old), b = double(w_new);
    return b * b - a * a;
}

// The end of an fp32 CSR chain: its weights stay in L.wf32 (w = alpha v, folded by
// launch_fold_f32), regVal = 0.5 lambda ||alpha v||^2 (UPD.scala:176-180) from the tracked norm.
template <bool L2>
__device__ __forceinline__ void sparse_chain_out(const ChainLaunch& L, const KParams& kp, int chain,
                                                 int lane, double alpha, double dnsq, double loss_sum,
                                                 int64_t count) {
    double rv = 0.0;
    if constexpr (L2) {
        const double nsq = *L.wnsq0 + wave_sum(dnsq);
        if (count > 0) {
            const double nrm = sqrt(alpha * alpha * nsq);
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

template <int... Is, typename F>
__device__ __forceinline__ void static_for_impl(std::integer_sequence<int, Is...>, F&& f) {
    (f(std::integral_constant<int, Is>{}), ...);
}
// Calls f(std::integral_constant<int, i>) for i = 0..N-1: a guaranteed compile-time unroll.
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    static_for_impl(std::make_integer_sequence<int, N>{}, f);
}

template <typename S> struct Vec16;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));
template <> struct Vec16<float> { using type = f32x4; static constexpr int N = 4; };
template <> struct Vec16<double> { using type = f64x2; static constexpr int N = 2; };

template <typename S, typename T>
__device__ __forceinline__ void unpack(const typename Vec16<S>::type& v, T* out) {
    if constexpr (Vec16<S>::N == 4) {
        out[0] = T(v.x); out[1] = T(v.y); out[2] = T(v.z); out[3] = T(v.w);
    } else {
        out[0] = T(v.x); out[1] = T(v.y);
    }
}

// ------------------------------------------------------------------------------------------
// chain_dense: dense rows, weights in VGPRs, rows streamed through an LDS ring.
//
// One workgroup = one chain = two waves on two SIMDs:
//   wave 1 (loader)  streams the partition's rows, in iterator order, into an R-slot LDS ring
//                    with global_load_lds (LDS DMA, 1 KiB per instruction, up to ~60 KiB in
//                    flight), plus each row's label and stepSize/sqrt(j) (the "meta" bytes), and
//                    publishes `ready` = number of rows that have landed;
//   wave 0 (compute) owns the weights in registers and runs the sequential chain:
//                    lane l, vector v (0..NV-1) owns features (v*64 + l)*VEC .. +VEC-1, so a
//                    row slot is read with NV ds_read_b128 per lane; it publishes `consumed`.
// Only the loader issues VMEM, so the compute wave never waits on vmcnt; the loader's LDS
// accesses are inline asm so that the compiler does not drain its DMA before them.
// ------------------------------------------------------------------------------------------
struct RingHeader {
    unsigned ready;     // rows landed in the ring (loader -> compute)
    unsigned consumed;  // rows whose slot may be refilled (compute -> loader)
    unsigned stop;      // compute wave left the chain early (per-sample convergence break)
    unsigned consumed1; // a second consumer's `consumed` (chain_block64 with two chain waves)
};
// Labels and steps travel in 256-byte meta blocks, one per 16 rows: {y, stepSize/sqrt(j)} x 16.
constexpr int kMetaRows = 16;
constexpr int kMetaBlockBytes = 256;
// s_memrealtime runs at 100 MHz: a wave that sees no progress from its partner for 4 s sets the
// launch's watchdog word and leaves (the host then raises instead of hanging).
constexpr uint64_t kWatchdogTicks = 400000000ull;

// s_waitcnt vmcnt(k) for a runtime k (the immediate must be a constant).
__device__ __forceinline__ void wait_vmcnt_le(int k) {
#define PSGD_VMCNT_CASE(K) case K: asm volatile("s_waitcnt vmcnt(" #K ")" ::: "memory"); break;
    switch (k) {
        PSGD_VMCNT_CASE(0) PSGD_VMCNT_CASE(1) PSGD_VMCNT_CASE(2) PSGD_VMCNT_CASE(3)
        PSGD_VMCNT_CASE(4) PSGD_VMCNT_CASE(5) PSGD_VMCNT_CASE(6) PSGD_VMCNT_CASE(7)
        PSGD_VMCNT_CASE(8) PSGD_VMCNT_CASE(10) PSGD_VMCNT_CASE(12) PSGD_VMCNT_CASE(14)
        PSGD_VMCNT_CASE(16) PSGD_VMCNT_CASE(20) PSGD_VMCNT_CASE(24) PSGD_VMCNT_CASE(28)
        PSGD_VMCNT_CASE(32) PSGD_VMCNT_CASE(36) PSGD_VMCNT_CASE(40) PSGD_VMCNT_CASE(44)
        PSGD_VMCNT_CASE(48) PSGD_VMCNT_CASE(52) PSGD_VMCNT_CASE(56) PSGD_VMCNT_CASE(60)
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
#undef PSGD_VMCNT_CASE
}

// Ring geometry chosen by the launcher (psgd_kernels.hip, launch_reg).
struct RingGeom {
    int rows;         // R row slots
    int meta_blocks;  // MB meta blocks (16 rows each)
    int depth;        // D: rows the loader keeps in flight past the oldest unpublished one
    int gslots;       // Gram slots (chain_block only)
};

__device__ __forceinline__ unsigned lds_load_u32_asm(const unsigned* p) {
    unsigned v;
    const unsigned addr = (unsigned)(uintptr_t)p;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
    return v;
}
__device__ __forceinline__ void lds_store_u32_asm(unsigned* p, unsigned v) {
    const unsigned addr = (unsigned)(uintptr_t)p;
    asm volatile("ds_write_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : : "v"(addr), "v"(v) : "memory");
}

// ------------------------------------------------------------------------------------------
// The row loader wave (shared by chain_dense and chain_block): streams the partition's rows, in
// iterator order, into an R-slot LDS ring with global_load_lds (LDS DMA, 1 KiB per instruction,
// loader_depth(NV) rows in flight), plus each row's label and stepSize/sqrt(j) in 256-byte meta
// blocks (one per 16 rows), and publishes hdr->ready = number of rows that have landed, every
// PUB rows. It refills the slot of row t only once hdr->consumed > t - R; before it blocks on a
// full ring it drains its DMA and publishes every row it has issued, so a consumer that waits
// for any row inside the ring always makes progress. Its LDS accesses are inline asm so that
// the compiler does not drain the DMA before them; the depth is a compile-time constant (a
// runtime s_waitcnt needs a branch tree that costs more than the row).
// ------------------------------------------------------------------------------------------
// Cache policy of the row stream's LDS-DMA loads (the aux operand of global_load_lds): nt (2).
// Every row is read once per epoch and an epoch's rows (GBs) do not fit the caches, so nothing
// is lost by not keeping them; measured on the c2 workload (tools/chain_bench, 256 chains, d 512):
// 83.7-84.7 ns/row nt vs 85.7-87.2 default policy (LeastSquares), 93.4-93.7 vs 95.0-96.3 (Logistic).
#ifndef PSGD_LOAD_AUX
#define PSGD_LOAD_AUX 2
#endif

template <int NV>
__host__ __device__ constexpr int loader_depth() {
    return NV == 1 ? 56 : NV == 2 ? 28 : NV == 4 ? 14 : 7;   // <= 56 instructions in vmcnt
}

__device__ __forceinline__ void lds_store_u32_nowait(unsigned* p, unsigned v) {
    const unsigned addr = (unsigned)(uintptr_t)p;
    asm volatile("ds_write_b32 %0, %1" : : "v"(addr), "v"(v) : "memory");
}

// GB > 0: rows are also read by two helper waves that take alternate blocks of GB rows and
// count their finished blocks in gdone[0] (even blocks) / gdone[1] (odd blocks); a slot is free
// only once both the consumer and its helper are done with it. GALL: both helpers read every
// block (each a share of its features) and count in gdone[0] / gdone[1]; a block is free once
// both have passed it. CONS = 2: two consumers, the second counting in hdr->consumed1; a slot is
// free once both have passed it.
template <typename S, int NV, bool FULL, int PUB, int GB = 0, int CONS = 1, bool GALL = false>
__device__ __forceinline__ void ring_loader(const ChainLaunch& L, const ChainDesc& dsc, RingHeader* hdr,
                                            char* meta_ring, char* ring, const RingGeom& geom,
                                            int lane, const unsigned* gdone = nullptr) {
    using V = typename Vec16<S>::type;
    constexpr int VEC = Vec16<S>::N;
    constexpr int ROW_BYTES = NV * 1024;
    constexpr int D = loader_depth<NV>();
    static_assert(kMetaRows % PUB == 0, "a meta block covers whole groups");
    const int64_t n = dsc.n_rows;
    const int R = geom.rows;
    const int MB = geom.meta_blocks;
    const S* X = reinterpret_cast<const S*>(dsc.x);
    const int64_t ld = dsc.ld;
    // meta DMA lane l: row 16k + l/4, dword l%4 of {y lo, y hi, step lo, step hi}
    const unsigned* msrc = reinterpret_cast<const unsigned*>((lane & 2) ? L.steps : dsc.y) + (lane & 1);
    const int mrow = lane >> 2;
    int64_t limit = R;            // rows < limit have a free slot
    int64_t pub = 0;              // rows published in hdr->ready (never decreases)
    int slot = 0, mslot = 0;
    // sampled epoch: sample t is row rows[t], read with scalar loads (constant address space)
    const int32_t __attribute__((address_space(4)))* RIDX =
        (const int32_t __attribute__((address_space(4)))*)dsc.rows;
    auto issue_row = [&](int64_t r) __attribute__((always_inline)) {   // r: partition row
        char* dst = ring + slot * ROW_BYTES;
        const V* row = reinterpret_cast<const V*>(X + r * ld);
        // every lane issues (past the row end it re-reads the row's first vector, bytes the
        // consumers ignore): each row is exactly NV vmcnt entries, which the counted waits need
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            const V* src = (FULL || (v * 64 + lane) * VEC < ld) ? row + v * 64 + lane : row;
            __builtin_amdgcn_global_load_lds(
                (const void*)(as_global(src)),
                (__attribute__((address_space(3))) void*)(dst + v * 1024), 16, 0, PSGD_LOAD_AUX);
        }
        slot = (slot + 1 == R) ? 0 : slot + 1;
    };
    // Rows go out in groups of PUB: one ring-space check, at most one meta DMA and one publish
    // per group, no branch per row.
    PSGD_STAMP(const uint64_t st_begin = __builtin_amdgcn_s_memtime(); uint64_t st_full = 0, st_vm = 0;)
    for (int64_t t = 0; t < n; t += PUB) {
        const int64_t te = (t + PUB < n) ? t + PUB : n;
        if (te > limit) {
            PSGD_STAMP(const uint64_t st_w = __builtin_amdgcn_s_memtime();)
            // ring full: wait for the consumer to free slots. A ring deeper than the loader's
            // depth plus two groups always leaves the consumer published rows to work on; a
            // shallower one publishes everything issued first (drains the DMA).
            // (the helper waves' next blocks, GB rows each, must be published too)
            if (R < D + 2 * PUB + 2 * GB) {
                asm volatile("s_waitcnt vmcnt(0)" : : : "memory");
                lds_store_u32_nowait(&hdr->ready, (unsigned)t);
                pub = t;
            }
            // rows issued but not published yet (the youngest D: see the publish below)
            int inflight = (int)(t - pub);
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            for (;;) {
                unsigned c = __builtin_amdgcn_readfirstlane(lds_load_u32_asm(&hdr->consumed));
                if constexpr (CONS == 2) {
                    const unsigned c1 = __builtin_amdgcn_readfirstlane(lds_load_u32_asm(&hdr->consumed1));
                    c = c < c1 ? c : c1;
                }
                if constexpr (GB > 0) {
                    const unsigned g0 = __builtin_amdgcn_readfirstlane(lds_load_u32_asm(&gdone[0]));
                    const unsigned g1 = __builtin_amdgcn_readfirstlane(lds_load_u32_asm(&gdone[1]));
                    // blocks 0 .. min(2 g0, 2 g1 + 1) - 1 are all done by their helper
                    // (GALL: blocks 0 .. min(g0, g1) - 1 by both)
                    const unsigned gb = GALL ? (g0 < g1 ? g0 : g1) : 2 * g0 < 2 * g1 + 1 ? 2 * g0 : 2 * g1 + 1;
                    c = c < gb * GB ? c : gb * GB;
                }
                limit = (int64_t)c + R;
                if (te <= limit) break;
                if (inflight > 0) {
                    // while the ring is full, publish the in-flight rows as they land (PUB at a
                    // time) rather than only after the next group: the consumers see the whole
                    // ring, not R - D rows of it
                    inflight = inflight > PUB ? inflight - PUB : 0;
                    wait_vmcnt_le(inflight * NV);
                    pub = t - inflight;
                    lds_store_u32_nowait(&hdr->ready, (unsigned)pub);
                    continue;
                }
                if (__builtin_amdgcn_readfirstlane(lds_load_u32_asm(&hdr->stop))) goto drain;
                if (__builtin_amdgcn_s_memrealtime() - t0 > kWatchdogTicks) {
                    __hip_atomic_fetch_or(L.watchdog, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    lds_store_u32_asm(&hdr->stop, 1u);
                    goto drain;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            PSGD_STAMP(st_full += __builtin_amdgcn_s_memtime() - st_w;)
        }
        if ((t & (kMetaRows - 1)) == 0) {
            int64_t r = t + mrow;
            if (r >= n) r = n - 1;
            __builtin_amdgcn_global_load_lds(
                (const void*)(as_global(msrc + 2 * r)),
                (__attribute__((address_space(3))) void*)(meta_ring + mslot * kMetaBlockBytes), 4, 0, 0);
            mslot = (mslot + 1 == MB) ? 0 : mslot + 1;
        }
        if (te - t == PUB) {
            if (RIDX) {
#pragma unroll
                for (int k = 0; k < PUB; ++k) issue_row(RIDX[t + k]);
            } else {
#pragma unroll
                for (int k = 0; k < PUB; ++k) issue_row(t + k);
            }
        } else {
            for (int64_t u = t; u < te; ++u) issue_row(RIDX ? (int64_t)RIDX[u] : u);
        }
        if (te > D) {
            // all but the youngest D rows' instructions are done: rows < te - D have landed
            PSGD_STAMP(const uint64_t st_v = __builtin_amdgcn_s_memtime();)
            wait_vmcnt_le(D * NV);
            PSGD_STAMP(st_vm += __builtin_amdgcn_s_memtime() - st_v;)
            if (te - D > pub) {
                pub = te - D;
                lds_store_u32_nowait(&hdr->ready, (unsigned)pub);
            }
        }
    }
drain:
    asm volatile("s_waitcnt vmcnt(0)" : : : "memory");
    lds_store_u32_asm(&hdr->ready, (unsigned)n);
    PSGD_STAMP(if (L.stamps && lane == 0) {
        unsigned long long* o = L.stamps + (size_t)blockIdx.x * 16 + 4;
        o[0] = __builtin_amdgcn_s_memtime() - st_begin; o[1] = st_full; o[2] = st_vm;
    })
}
}  // namespace psgd
