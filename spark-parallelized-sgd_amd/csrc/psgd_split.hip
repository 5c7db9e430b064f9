// psgd_split.hip -- the per-sample dense chain with the feature dimension split over H compute
// waves (gfx950): the throughput kernel of the updaters the blocked kernels do not take
// (AdaGrad, Adam, L1).
//
// Reference (paths under /root/reference, src/main/scala/org/apache/spark/mllib/optimization/):
//   chain loop      ParallelizedSGD.scala:243-270 (one chain per partition, per-sample updates)
//   AdaGrad         SGDUpdater.scala:193-227  (status r += g*g; w += -s/sqrt(j) * g / (r + 1)^0.5)
//   Adam            SGDUpdater.scala:238-286  (v, r; fix1 = (1 - r^iter)^0.5 + eps; lr = s / (1 - beta^iter))
//   L1              SGDUpdater.scala:120-148  (soft thresholding: per coordinate, not a rank-1 step)
//   gradients       [ext] MLlib 1.6.1 Gradient.scala (mult * x), as in psgd_kernels.hip
//
// AdaGrad / Adam keep per-feature status that depends non-linearly on each sample's gradient, so
// the blocked Gram form of chain_block / chain_block64 does not apply: the chain is sequential
// per sample. chain_dense runs it on one wave, whose per-sample path (a d-long dot, the wave
// reduction, the multiplier, d status + weight updates with a reciprocal square root or a power
// each) is ~2,000 cycles at d = 1,024 in fp32. Here the features are split over H compute waves,
// one per SIMD: wave h owns the row vectors [h NV/H, (h+1) NV/H) of W, of the status and of every
// row. Per sample each wave takes its partial dot, reduces it across its lanes and publishes it
// in LDS as tagged 64-bit words ({32 bits of the partial, sample number + 1}: one word per fp32
// partial, two per fp64 one), so a reader needs no separate flag: it polls the H words of the
// sample's parity slot until every tag is the sample's. All waves add the partials in one fixed
// order -- (p0 + p1) + (p2 + p3) by DPP across lane groups when a sample carries one value,
// ((p0 + p1) + p2) + p3 by readlane with the convergence terms -- bit-identical in every wave,
// run the identical scalar multiplier, and update only their own features. A parity slot is
// rewritten two samples later, only after every wave has published the sample in between (which
// it does after reading this one).
//
// Rows stream through the LDS ring of chain_dense (ring_loader, one loader wave); compute wave 0
// hands slots back: when it has every partial of sample t, all waves have read row t + 1.
// The per-element arithmetic is chain_dense's (this file is compiled with -ffp-contract=off)
// except that AdaGrad's and Adam's status and weight updates are fused where a multiply feeds an
// add (v = fma(g, 1 - beta, beta v), accum = fma(g, g, accum), w = fma(-lr', u, w), round 4: one
// rounding fewer each), and the dot is reassociated (per-wave partials, wave trees, the fixed
// order above) -- all inside the fp64 mode's 1e-9 relative bar. Logistic's multiplier is on every
// sample's critical path: fp64 takes the shared recip_one_plus_exp (psgd_device.h: a degree-11 exp core, truncation < 1e-14,
// v_rcp_f64 + one Newton step; DESIGN.md §4 lists every fp64 divergence),
// fp32 the hardware exp2 / reciprocal (as chain_block); the row losses (log1pExp) are summed
// after the chain from the stored margins, off the sequential path.
#include "psgd_device.h"
#include "psgd_split.h"

#include <stdlib.h>

#include <type_traits>

// compute waves per chain: min(NV, PSGD_SPLIT_HMAX), one per SIMD
#ifndef PSGD_SPLIT_HMAX
#define PSGD_SPLIT_HMAX 4
#endif

namespace psgd {

namespace {

// The SIMD a wave runs on (HW_REG_HW_ID bits 5:4).
__device__ __forceinline__ unsigned split_simd() {
    unsigned id;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(id));
    return (id >> 4) & 3;
}

// Roles of the H + 1 waves from their SIMDs (the same answer in every wave): compute waves 0 ..
// H-1 on distinct SIMDs where the dispatcher allows it, the remaining wave is the loader (H).
template <int H>
__device__ __forceinline__ int split_role(const unsigned* simd, int w) {
    constexpr int NW = H + 1;
    int role[NW];
    bool used[4] = {false, false, false, false};
    int nc = 0;
    for (int i = 0; i < NW; ++i) role[i] = -1;
    for (int i = 0; i < NW; ++i)
        if (!used[simd[i] & 3] && nc < H) { used[simd[i] & 3] = true; role[i] = nc++; }
    for (int i = 0; i < NW; ++i)
        if (role[i] < 0 && nc < H) role[i] = nc++;
    for (int i = 0; i < NW; ++i)
        if (role[i] < 0) role[i] = H;
    return role[w];
}

__device__ __forceinline__ void lds_write_u64(uint64_t* p, uint64_t v) {
    asm volatile("ds_write_b64 %0, %1" : : "v"((unsigned)(uintptr_t)p), "v"(v) : "memory");
}
__device__ __forceinline__ uint64_t lds_read_u64(const uint64_t* p) {
    uint64_t v;
    asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"((unsigned)(uintptr_t)p) : "memory");
    return v;
}
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u32x4 lds_read_b128(const uint64_t* p) {
    u32x4 v;
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"((unsigned)(uintptr_t)p) : "memory");
    return v;
}

// RingHeader::stop values: the loader stops on any non-zero one; the compute waves' spins give up
// only on an error (a watchdog), not on a per-sample convergence break, which every wave takes
// at the same sample by itself.
constexpr unsigned kStopError = 1u, kStopConverged = 2u;

// fixed LDS area: [RingHeader 16 B][exchange 2 x H x W u64 (W words per wave and sample)]
// [SIMD ids of the H + 1 waves]
template <int H, int PC>
constexpr size_t split_fixed_bytes() {
    return (sizeof(RingHeader) + 2 * H * PC * 8 + (H + 1) * 4 + 15) / 16 * 16;
}

}  // namespace

template <typename S, typename T, int GRAD, int UPD, bool CONV, int NV, bool FULL, int H>
__global__ __launch_bounds__(64 * (H + 1)) void chain_split(ChainLaunch L, KParams kp, RingGeom geom) {
    using V = typename Vec16<S>::type;
    constexpr int VEC = Vec16<S>::N;
    constexpr int NVH = NV / H;              // row vectors of one compute wave
    constexpr int E = NVH * VEC;             // features per lane of one compute wave
    constexpr int E2 = E / 2;
    constexpr int ROW_BYTES = NV * 1024;
    constexpr int PC = sizeof(T) / 4;        // 32-bit pieces of a partial
    // values a wave publishes per sample: its partial dot; with the per-sample convergence test
    // (CONV, PSGD.scala:262) also its partial ||w_old - w_new||^2 and ||w_new||^2 of the previous
    // sample, so the test of sample t - 1 rides on the exchange of sample t
    constexpr int KV = CONV ? 3 : 1;
    constexpr int XW = H * PC * KV;          // exchange words per sample
    static_assert(NV % H == 0 && E % 2 == 0, "the compute waves split the row vectors evenly");
    static_assert(XW <= 64, "one lane per exchange word");
    // Logistic: the per-row dots go to L.zbuf64 / L.zbuf, the losses are summed after the chain
    constexpr bool ZOUT = GRAD == G_LOGISTIC;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    RingHeader* hdr = reinterpret_cast<RingHeader*>(smem);
    uint64_t* xw = reinterpret_cast<uint64_t*>(smem + sizeof(RingHeader));
    unsigned* simd_of = reinterpret_cast<unsigned*>(xw + 2 * XW);
    char* meta_ring = smem + split_fixed_bytes<H, PC * KV>();
    char* ring = meta_ring + geom.meta_blocks * kMetaBlockBytes;

    const int lane = threadIdx.x & 63;
    const int chain = blockIdx.x;
    const ChainDesc dsc = L.descs[chain];
    const int d = kp.d;
    // a chain's rows live in HBM at >= 1 KiB each (two row vectors on), so n < 2^31: the
    // per-sample bookkeeping runs in 32-bit (one SALU op per step, v_cvt_f32/f64_i32 for iter)
    const int32_t n = (int32_t)dsc.n_rows;
    const int MB = geom.meta_blocks;

    if (threadIdx.x == 0) {
        hdr->ready = 0;
        hdr->consumed = 0;
        hdr->stop = 0;
        hdr->consumed1 = 0;
    }
    for (int i = threadIdx.x; i < 2 * XW; i += blockDim.x) xw[i] = 0;   // tag 0: no sample yet
    // every wave's SIMD, for the roles
    if (lane == 0) simd_of[threadIdx.x >> 6] = split_simd();
    __syncthreads();
    const int h = __builtin_amdgcn_readfirstlane(split_role<H>(simd_of, threadIdx.x >> 6));
    __syncthreads();

    if (h == H) {
        ring_loader<S, NV, FULL, 4>(L, dsc, hdr, meta_ring, ring, geom, lane);
        return;
    }

    // ---------------- compute wave h ----------------
    using T2 = T __attribute__((ext_vector_type(2)));
    T2 w[E2];
#pragma unroll
    for (int u = 0; u < NVH; ++u) {
        const int base = ((h * NVH + u) * 64 + lane) * VEC;
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            const int f = base + k;
            const double wv = as_global(L.w_in)[f < d ? f : 0];   // unconditional, clamped
            w[(u * VEC + k) / 2][(u * VEC + k) % 2] = f < d ? T(wv) : T(0);
        }
    }
    // status (UPD.scala:193-286) in registers beside the weights: ua = AdaGrad's accumulator or
    // Adam's v, ub = Adam's r; the chain's first sample takes the reference's `None` branch
    constexpr bool STATE_B = UPD == U_ADAM;
    T2 ua[E2], ub[STATE_B ? E2 : 1];
#pragma unroll
    for (int e = 0; e < E2; ++e) ua[e] = T2{T(0), T(0)};
#pragma unroll
    for (int e = 0; e < (STATE_B ? E2 : 1); ++e) ub[e] = T2{T(0), T(0)};

    // this wave's slice of rows t and t+1 (ping-pong), read from the ring
    T2 xb[2][E2];
    double yb[2], sb[2];
    int meta_blk = 0;
    // the LDS reads of row t's slice and meta into buffer p (issued here, waited for at first use)
    auto read_row = [&](auto pc, const char* src, int32_t t) __attribute__((always_inline)) {
        constexpr int p = decltype(pc)::value;
#pragma unroll
        for (int u = 0; u < NVH; ++u) {
            const int v = h * NVH + u;
            V xv = *reinterpret_cast<const V*>(src + v * 1024 + lane * 16);
            if constexpr (!FULL) {
                // vectors past the row end were not loaded: their LDS bytes are stale
                if ((v * 64 + lane) * VEC >= dsc.ld) xv = V(0);
            }
            T tmp[VEC];
            unpack<S, T>(xv, tmp);
#pragma unroll
            for (int k = 0; k < VEC; k += 2) xb[p][(u * VEC + k) / 2] = T2{tmp[k], tmp[k + 1]};
        }
        if (t > 0 && (t & (kMetaRows - 1)) == 0) meta_blk = (meta_blk + 1 == MB) ? 0 : meta_blk + 1;
        const f64x2 meta = *reinterpret_cast<const f64x2*>(
            meta_ring + meta_blk * kMetaBlockBytes + (int)(t & (kMetaRows - 1)) * 16);
        yb[p] = meta.x;
        sb[p] = meta.y;
    };

    // Spin until `rows` rows have landed (rare: the loader runs a ring ahead). Only `ready`
    // leaves the branch, so no LDS read waits at its join. false: the chain stopped.
    unsigned ready = 0;
    bool stop = false;
    auto wait_rows = [&](int32_t rows) __attribute__((always_inline)) {
        if (rows > (int32_t)ready) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            for (;;) {
                ready = __hip_atomic_load(&hdr->ready, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (rows <= (int32_t)ready) break;
                if (__hip_atomic_load(&hdr->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) { stop = true; break; }
                if (__builtin_amdgcn_s_memrealtime() - t0 > kWatchdogTicks) {
                    __hip_atomic_fetch_or(L.watchdog, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(&hdr->stop, kStopError, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    stop = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
    };

    // The exchange of sample t: publish writes this wave's KV values (lane l < PC KV writes word
    // l: value l / PC, 32-bit piece l % PC); collect polls the XW words of the parity slot (lane l
    // reads word l) until all carry the sample's tag and returns each value summed over the waves
    // in wave order. A stopped chain leaves collect with whatever it read (the host raises on the
    // watchdog word).
    constexpr uint64_t kMask = XW == 64 ? ~0ull : ((1ull << XW) - 1);
    // H = 1 (the diagnostic PSGD_SPLIT_HMAX=1 builds only: the product runs H = min(NV, 4) >= 2 --
    // one-vector rows take chain_dense): one wave holds every partial, so there is no exchange;
    // publish keeps the values and collect returns them (round 6: the per-H table's H = 1 row
    // without the wave's LDS round trip to itself)
    T xown[KV];
    // Every lane writes (no EXEC juggling on the per-sample path): lanes past the wave's PC * KV
    // words write its last word again, with the same value (the partials are wave-uniform).
    auto publish = [&](const T (&val)[KV], int32_t t) __attribute__((always_inline)) {
        if constexpr (H == 1) {
#pragma unroll
            for (int q = 0; q < KV; ++q) xown[q] = val[q];
            return;
        }
        const int l = lane < PC * KV ? lane : PC * KV - 1;
        const int k = l / PC;
        T vk = val[0];
#pragma unroll
        for (int q = 1; q < KV; ++q) vk = k == q ? val[q] : vk;
        uint32_t piece;
        if constexpr (PC == 1) {
            piece = __float_as_uint(vk);
        } else {
            const uint64_t b = (uint64_t)__double_as_longlong(vk);
            piece = (l & 1) == 0 ? (uint32_t)b : (uint32_t)(b >> 32);
        }
        lds_write_u64(xw + (int)(t & 1) * XW + h * PC * KV + l, ((uint64_t)(uint32_t)(t + 1) << 32) | piece);
    };
    // One partial per sample (KV = 1, H = 2 or 4): every lane reads wave (lane % H)'s partial (fp64:
    // both of its words in one 16-byte read) and the H partials are added across each group of H
    // lanes by DPP, (p0 + p1) + (p2 + p3) in every lane of every wave (a + b and b + a are the same
    // bits) -- no readlane and no SGPR round trip on the sample's path.
    constexpr bool kLaneSum = KV == 1 && (H == 2 || H == 4);
    auto collect = [&](int32_t t, T (&sum)[KV]) __attribute__((always_inline)) {
        if constexpr (H == 1) {
#pragma unroll
            for (int q = 0; q < KV; ++q) sum[q] = xown[q];
            return;
        }
        const uint32_t tag = (uint32_t)(t + 1);
        const uint64_t* src = xw + (int)(t & 1) * XW + (kLaneSum ? PC * (lane & (H - 1)) : (lane < XW ? lane : 0));
        constexpr uint64_t kNeed = kLaneSum ? ~0ull : kMask;
        u32x4 v;   // {piece, tag} (kLaneSum fp64: {low piece, tag, high piece, tag})
        auto poll = [&]() __attribute__((always_inline)) -> bool {
            if constexpr (kLaneSum && PC == 2) {
                v = lds_read_b128(src);
                return __ballot(v[1] == tag && v[3] == tag) == kNeed;
            } else {
                const uint64_t q = lds_read_u64(src);
                v[0] = (uint32_t)q;
                v[1] = (uint32_t)(q >> 32);
                return (__ballot(v[1] == tag) & kNeed) == kNeed;
            }
        };
        if (!poll()) {
            // spin on the LDS words alone (s_memrealtime is a scalar-memory round trip that the
            // next LDS wait would also wait for); the stop flag and the clock every 1024 polls
            uint64_t t0 = 0;
            for (unsigned spin = 1;; ++spin) {
                if (poll()) break;
                if ((spin & 1023) == 0) {
                    if (__hip_atomic_load(&hdr->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == kStopError) { stop = true; break; }
                    const uint64_t now = __builtin_amdgcn_s_memrealtime();
                    if (t0 == 0) t0 = now;
                    if (now - t0 > kWatchdogTicks) {
                        __hip_atomic_fetch_or(L.watchdog, 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store(&hdr->stop, kStopError, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        stop = true;
                        break;
                    }
                }
            }
        }
        if constexpr (kLaneSum) {
            T pg;
            if constexpr (PC == 1) pg = __uint_as_float(v[0]);
            else pg = __longlong_as_double((long long)(((uint64_t)v[2] << 32) | v[0]));
            T s = pg + dpp_mov<0xB1>(pg);                 // quad_perm [1,0,3,2]
            if constexpr (H == 4) s = s + dpp_mov<0x4E>(s);   // quad_perm [2,3,0,1]
            sum[0] = s;
            return;
        }
        const int lo = (int)v[0];
#pragma unroll
        for (int q = 0; q < KV; ++q) {
            T acc = T(0);
#pragma unroll
            for (int g = 0; g < H; ++g) {
                const int wd = g * PC * KV + q * PC;
                T pg;
                if constexpr (PC == 1) {
                    pg = __int_as_float(__builtin_amdgcn_readlane(lo, wd));
                } else {
                    const uint32_t a = (uint32_t)__builtin_amdgcn_readlane(lo, wd);
                    const uint32_t b = (uint32_t)__builtin_amdgcn_readlane(lo, wd + 1);
                    pg = __longlong_as_double((long long)(((uint64_t)b << 32) | a));
                }
                acc = g == 0 ? pg : acc + pg;
            }
            sum[q] = acc;
        }
    };

    double loss_sum = 0.0;
    T loss_blk = T(0);          // fp32 mode: block partial, flushed to the fp64 sum every 32 rows
    T* zout = nullptr;
    if constexpr (ZOUT) {
        if constexpr (sizeof(T) == 8) zout = L.zbuf64 + (int64_t)chain * L.zstride;
        else zout = L.zbuf + (int64_t)chain * L.zstride;
    }
    T zprev = T(0);             // Logistic: the last sample's dot, stored during the next exchange
    const char* slot_ptr = ring;
    const char* const ring_end = ring + geom.rows * ROW_BYTES;
    // CONV: this wave's ||w_old - w_new||^2, ||w_new||^2 of the last update (wave-reduced), the
    // sample at which the test of its predecessor broke the chain (n: no break)
    T pdsq = T(0), pnsq = T(0);
    int32_t conv_at = n;

    // diagnostic builds (-DPSGD_STAMPS): cycles per phase of this wave's samples
    PSGD_STAMP(uint64_t st_dot = 0, st_x = 0, st_upd = 0; const uint64_t st_begin = __builtin_amdgcn_s_memtime();
               uint64_t st_mark = st_begin;)
#define SPLIT_STAMP(acc) PSGD_STAMP({ const uint64_t now_ = __builtin_amdgcn_s_memtime(); acc += now_ - st_mark; st_mark = now_; })

    // Sample t (row t in xb[p]): the partial dot and its wave reduction, publish; the reads of
    // row t + 1 go out before the poll so that their LDS latency overlaps the exchange's; then
    // the multiplier and this wave's updates. Straight-line: the only branches spin.
    auto sample = [&](auto pc, int32_t t) __attribute__((always_inline)) {
        constexpr int p = decltype(pc)::value;
        const T y = T(yb[p]);
        const T s = T(sb[p]);
        const T2* x = xb[p];
        T2 a0 = T2{T(0), T(0)}, a1 = T2{T(0), T(0)};
#pragma unroll
        for (int e = 0; e < E2; e += 2) {
            a0 = __builtin_elementwise_fma(x[e], w[e], a0);
            if (e + 1 < E2) a1 = __builtin_elementwise_fma(x[e + 1], w[e + 1], a1);
        }
        const T2 a = a0 + a1;
        {
            // the partial in every lane (permlane swaps, the same bits as wave_sum_uniform's lane
            // 63): it is stored from VGPRs, so no readlane / v_mov round trip through an SGPR
            T val[KV];
            val[0] = wave_sum(a.x + a.y);
            if constexpr (CONV) { val[1] = pdsq; val[2] = pnsq; }
            publish(val, t);
        }
        SPLIT_STAMP(st_dot);
        // the sample's scalars that do not depend on its dot, before the exchange's wait (the spin
        // is a branch: nothing after it is moved above it)
        const T a_s = -s;
        const T iter = T(t + 1);
        T al = T(0);
        if constexpr (UPD == U_ADAM) {
            // lr = s / (1 - beta^iter); once 1 - beta^iter is exactly 1.0 (after a few tens of
            // samples) the quotient is s itself: a wave-uniform branch skips the division
            // (fp32: IEEE division, ~10 instructions; fp64: rcp + one Newton step, which gives
            // exactly 1 for 1.0)
            if constexpr (sizeof(T) == 4) {
                const T q = T(1) - pow_fast(T(kp.beta), iter);
                al = q == T(1) ? -s : -(s / q);
            } else {
                // 1 - beta^iter as 1.0 once beta^iter <= 2^-54 (bit-identical, no library pow per
                // sample on the chain)
                const T q = one_minus_pow_iter(T(kp.beta), iter);
                al = q == T(1) ? -s : -(s * recip_newton(q));
            }
        }
        [[maybe_unused]] const T shrink = T(kp.reg) * s;          // L1 (UPD.scala:133)
        [[maybe_unused]] const T l2c = T(1) - s * T(kp.reg);      // SquaredL2 (UPD.scala:169)

        const char* next_ptr = slot_ptr + ROW_BYTES;
        if (next_ptr == ring_end) next_ptr = ring;
        wait_rows(t + 2 < n ? t + 2 : n);
        read_row(std::integral_constant<int, 1 - p>{}, next_ptr, t + 1);   // past the end: unused
        slot_ptr = next_ptr;

        // the previous sample's dot goes out under this exchange's LDS latency, not between the
        // exchange and the multiplier (wave 0's extra work delays every wave at the next exchange)
        if constexpr (ZOUT) { if (h == 0 && lane == 0 && t > 0) zout[t - 1] = zprev; }
        T sums[KV];
        collect(t, sums);
        const T z = sums[0];
        SPLIT_STAMP(st_x);
        if constexpr (CONV) {
            // isConverged(old, new, tol) of sample t - 1 (PSGD.scala:262, :333-335): the chain
            // breaks after it -- sample t is not taken (no update, loss or count)
            if (t > 0 && m_sqrt(sums[1]) < T(kp.tol) * jmax(m_sqrt(sums[2]), T(1))) {
                conv_at = t;
                // the loader stops refilling (kStopConverged: not an error -- the waves' spins
                // give up only on kStopError)
                if (h == 0) __hip_atomic_store(&hdr->stop, kStopConverged, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                return;
            }
        }
        if (h == 0 && ((t & 1) == 1 || t + 1 == n)) {
            // every wave has published sample t, so every wave has read rows <= t + 1
            __hip_atomic_store(&hdr->consumed, (unsigned)(t + 1), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
        }

        T mult;
        if constexpr (ZOUT) {
            // 1/(1 + exp(margin)) - y, margin = -z; the row's loss from z after the chain
            if constexpr (sizeof(T) == 8) mult = recip_one_plus_exp(-z) - y;
            else mult = __builtin_amdgcn_rcpf(1.0f + __expf(-z)) - y;
            zprev = z;
        } else {
            T loss;
            if constexpr (GRAD == G_LEAST_SQUARES) {
                mult = z - y;
                loss = mult * mult;   // halved once at the end (chain_dense)
            } else {
                loss = gradient_scalar<GRAD, T>(z, y, mult);
            }
            if constexpr (sizeof(T) == 4) {
                loss_blk += loss;
                if ((t & 31) == 31) { loss_sum += double(loss_blk); loss_blk = T(0); }
            } else {
                loss_sum += loss;
            }
        }

        T2 dsq2 = T2{T(0), T(0)}, nsq2 = T2{T(0), T(0)};
        if constexpr (UPD == U_ADAM) {
            // Adam, the reference's variant: v = beta v + (1-beta) g, r = gamma r + (1-gamma) g^2,
            // fix1 = sqrt(1 - r^iter) + eps, w += -lr * v / fix1. The status first; then, when
            // 1 - r^iter rounds to exactly 1 for every coordinate of the wave (r^iter below half
            // an ulp of 1 -- after a few tens of samples for an average of squared gradients
            // below 1), fix1 is the constant 1 + eps and v / fix1 one multiply by its reciprocal:
            // the same operations as the general path (whose sqrt of 1 is exactly 1), hoisted.
            const T beta = T(kp.beta), gamma = T(kp.gamma);
            const T2 omb = T2{T(1) - beta, T(1) - beta}, omg = T2{T(1) - gamma, T(1) - gamma};
            T2 vv[E2], rr[E2];
            // The test runs once per lane, on an upper bound of the lane's r values: with gamma in
            // [0, 1] every r is +0 or more, +inf or a NaN, and such floats order as their bit
            // patterns (a NaN of either sign compares above +inf), so the largest pattern is the
            // largest r, or a NaN when any r is one (fp64: the high words, completed with all-ones
            // low words: a bound >= every r). The threshold has half a unit of margin over the per-coordinate test below, so
            // the bound passing implies every coordinate passing (v_log_f32 need not be strictly
            // monotone); gamma outside [0, 1] takes the general path.
            uint32_t rbits = 0;
            auto rmax = [&](T r) __attribute__((always_inline)) {
                uint32_t b;
                if constexpr (sizeof(T) == 4) b = __float_as_uint(r);
                else b = (uint32_t)((uint64_t)__double_as_longlong(r) >> 32);
                rbits = b > rbits ? b : rbits;
            };
#pragma unroll
            for (int e = 0; e < E2; ++e) {
                // v = beta v + (1 - beta) g, r = gamma r + (1 - gamma) g^2, fused; the status starts at
                // +0, so the first sample's None branch (v = (1 - beta) g) is the same expression
                const T2 g = mult * x[e];
                const T2 v = __builtin_elementwise_fma(g, omb, ua[e] * beta);
                const T2 r = __builtin_elementwise_fma(g * g, omg, ub[e] * gamma);
                ua[e] = v;
                ub[e] = r;
                vv[e] = v;
                rr[e] = r;
                rmax(r.x);
                rmax(r.y);
            }
            bool general = !(kp.gamma >= 0.0 && kp.gamma <= 1.0);
            if constexpr (sizeof(T) == 4) {
                // pow_fast(r, iter) = exp2(iter log2 r) < 2^-26: 1 - r^iter == 1.0f
                general |= !(iter * __builtin_amdgcn_logf(__uint_as_float(rbits)) < -26.5f);
            } else {
                // one_minus_pow_iter's own test (it returns exactly 1.0 then)
                const double rb = __longlong_as_double((long long)(((uint64_t)rbits << 32) | 0xFFFFFFFFull));
                general |= !((float)iter * __builtin_amdgcn_logf((float)rb) < -60.5f);
            }
            if (__builtin_amdgcn_ballot_w64(general) != 0) {
#pragma unroll
                for (int e = 0; e < E2; ++e) {
                    const T2 old = w[e], v = vv[e], r = rr[e];
                    T2 nw;
                    // w + (-lr) (v / fix1) as fma((-lr) / fix1, v, w)
                    if constexpr (sizeof(T) == 4) {
                        const T fx = __builtin_amdgcn_sqrtf(T(1) - pow_fast(r.x, iter)) + T(kp.eps);
                        const T fy = __builtin_amdgcn_sqrtf(T(1) - pow_fast(r.y, iter)) + T(kp.eps);
                        nw = __builtin_elementwise_fma(T2{al * __builtin_amdgcn_rcpf(fx), al * __builtin_amdgcn_rcpf(fy)}, v, old);
                    } else {
                        // sqrt and v / fix1 by the hardware estimates + one Newton step (~1e-14)
                        const T fx = sqrt_newton(one_minus_pow_iter(r.x, iter)) + T(kp.eps);
                        const T fy = sqrt_newton(one_minus_pow_iter(r.y, iter)) + T(kp.eps);
                        nw = __builtin_elementwise_fma(T2{al * recip_newton(fx), al * recip_newton(fy)}, v, old);
                    }
                    w[e] = nw;
                    if constexpr (CONV) { const T2 df = old - nw; dsq2 += df * df; nsq2 += nw * nw; }
                }
            } else {
                T rfix;
                if constexpr (sizeof(T) == 4) rfix = __builtin_amdgcn_rcpf(T(1) + T(kp.eps));
                else rfix = recip_newton(T(1) + T(kp.eps));
                const T alr = al * rfix;   // the general path's al * (1 / fix1) at fix1 = 1 + eps
#pragma unroll
                for (int e = 0; e < E2; ++e) {
                    const T2 old = w[e], v = vv[e];
                    const T2 nw = __builtin_elementwise_fma(T2{alr, alr}, v, old);
                    w[e] = nw;
                    if constexpr (CONV) { const T2 df = old - nw; dsq2 += df * df; nsq2 += nw * nw; }
                }
            }
        } else {
#pragma unroll
            for (int e = 0; e < E2; ++e) {
                const T2 old = w[e];
                T2 nw;
                if constexpr (UPD == U_ADAGRAD) {
                    // accum = None ? g*g : accum + g*g; w += -s * (g / sqrt(accum + 1.0))
                    // (the status starts at +0, and +0 + g*g is g*g: the first sample's None
                    // branch without a select)
                    const T2 g = mult * x[e];
                    const T2 acc2 = __builtin_elementwise_fma(g, g, ua[e]);
                    ua[e] = acc2;
                    T2 q;   // g / sqrt(accum + 1)
                    if constexpr (sizeof(T) == 4) {
                        q = g * T2{__builtin_amdgcn_rsqf(acc2.x + T(1)), __builtin_amdgcn_rsqf(acc2.y + T(1))};
                    } else {
                        q = g * T2{rsqrt_newton(acc2.x + T(1)), rsqrt_newton(acc2.y + T(1))};
                    }
                    nw = __builtin_elementwise_fma(T2{a_s, a_s}, q, old);
                } else if constexpr (UPD == U_SQUARED_L2) {
                    nw = old * l2c;                     // brzWeights :*= (1 - s*lambda) (UPD.scala:172)
                    nw = nw + a_s * (mult * x[e]);      // axpy(-s, grad, w)
                } else if constexpr (UPD == U_SIMPLE) {
                    if constexpr (sizeof(T) == 4) nw = __builtin_elementwise_fma(T2{a_s * mult, a_s * mult}, x[e], old);
                    else nw = old + a_s * (mult * x[e]);   // the reference's two roundings (UPD.scala:95)
                } else if constexpr (UPD == U_L1) {
                    // axpy(-s, grad, w), then soft thresholding by regParam * s (UPD.scala:133-146)
                    nw = old + a_s * (mult * x[e]);
                    nw.x = jsignum(nw.x) * jmax(T(0), m_fabs(nw.x) - shrink);
                    nw.y = jsignum(nw.y) * jmax(T(0), m_fabs(nw.y) - shrink);
                }
                w[e] = nw;
                if constexpr (CONV) { const T2 df = old - nw; dsq2 += df * df; nsq2 += nw * nw; }
            }
        }
        if constexpr (CONV) {
            pdsq = wave_sum_uniform(dsq2.x + dsq2.y);
            pnsq = wave_sum_uniform(nsq2.x + nsq2.y);
        }
        SPLIT_STAMP(st_upd);
    };

    if (n > 0) {
        wait_rows(1);
        read_row(std::integral_constant<int, 0>{}, ring, 0);
    }
    int32_t t = 0;
    for (; t + 2 <= n && !stop && conv_at == n; t += 2) {
        sample(std::integral_constant<int, 0>{}, t);
        if (conv_at < n) break;
        sample(std::integral_constant<int, 1>{}, t + 1);
    }
    if (t < n && !stop && conv_at == n) sample(std::integral_constant<int, 0>{}, t++);
    // the samples taken: n, or up to the per-sample break (a stopped chain: the host raises)
    const int64_t count = conv_at < n ? conv_at : t;
    // (after a break at sample t, sample t - 1's dot went out during sample t's exchange)
    if constexpr (ZOUT) { if (h == 0 && lane == 0 && conv_at == n && count > 0) zout[count - 1] = zprev; }
    if constexpr (sizeof(T) == 4) loss_sum += double(loss_blk);
    // regVal of the chain's last update (PSGD.scala:257): Simple / AdaGrad / Adam 0.0
    // (UPD.scala:97, :221, :266), L1 regParam * ||w||_1 (:147), SquaredL2 0.5 regParam ||w||^2
    // (:180): the waves' partial norms through one more exchange
    double rv = 0.0;
    if constexpr (UPD == U_L1 || UPD == U_SQUARED_L2) {
        if (n > 0) {
            T acc = T(0);
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const T we = w[e / 2][e % 2];
                if constexpr (UPD == U_L1) acc += m_fabs(we);
                else acc += we * we;
            }
            T val[KV], nrm[KV];
            val[0] = wave_sum_uniform(acc);
            if constexpr (CONV) { val[1] = T(0); val[2] = T(0); }
            // exchange index: n, or after a break at sample t, t + 1 -- its parity slot last held
            // sample t - 1, which every wave has read (each published t after reading it); slot
            // t & 1 may still be being polled for sample t by a slower wave
            const int32_t fx = conv_at < n ? conv_at + 1 : n;
            publish(val, fx);
            collect(fx, nrm);
            if (count > 0) {
                if constexpr (UPD == U_L1) {
                    rv = double(nrm[0]) * kp.reg;
                } else {
                    const double r2 = sqrt(double(nrm[0]));
                    rv = 0.5 * kp.reg * r2 * r2;
                }
            }
        }
    }
    PSGD_STAMP(if (L.stamps && lane == 0) {
        unsigned long long* o = L.stamps + (size_t)chain * 16 + 4 * h;
        o[0] = st_mark - st_begin;
        o[1] = st_dot;
        o[2] = st_x;
        o[3] = st_upd;
    })
#undef SPLIT_STAMP

    // weights of this wave's features
    double* wo = L.w_out + (int64_t)chain * d;
#pragma unroll
    for (int u = 0; u < NVH; ++u) {
        const int base = ((h * NVH + u) * 64 + lane) * VEC;
#pragma unroll
        for (int k = 0; k < VEC; ++k)
            if (base + k < d) wo[base + k] = double(w[(u * VEC + k) / 2][(u * VEC + k) % 2]);
    }
    if (h > 0) return;
    if constexpr (GRAD == G_LEAST_SQUARES) loss_sum = loss_sum / 2.0;
    if (lane == 0) {
        L.rv[chain] = rv;
        if constexpr (!ZOUT) L.loss[chain] = loss_sum;
        L.cnt[chain] = count;
        L.cnt_d[chain] = double(count);
    }
}

// ------------------------------------------------------------------------------------------
// Launcher (left out of single-kernel ISA probes, tools/isa_probe.sh).
// ------------------------------------------------------------------------------------------
#ifndef PSGD_NO_DISPATCH
namespace {

template <typename S>
int split_nv(int64_t max_ld) {
    constexpr int VEC = 16 / sizeof(S);
    int nv = 1;
    while (nv * 64 * VEC < max_ld) nv *= 2;
    return nv;
}

template <typename S, typename T, int GRAD, int UPD, bool CONV, int NV>
int launch_split(const ChainLaunch& L, const KParams& kp, bool full, size_t lds, hipStream_t st) {
    constexpr int H = NV < PSGD_SPLIT_HMAX ? NV : PSGD_SPLIT_HMAX;
    constexpr int PC = sizeof(T) / 4 * (CONV ? 3 : 1);   // 32-bit words per wave and sample
    constexpr int ROW = NV * 1024;
    constexpr size_t FIX = split_fixed_bytes<H, PC>();
    const size_t budget = lds > 0 ? lds : (size_t)64 * 1024;
    const int D = loader_depth<NV>();
    int R = (int)((budget - FIX - 3 * kMetaBlockBytes) / ROW);
    int MB = (R + kMetaRows - 1) / kMetaRows + 2;
    while (R > 0 && FIX + (size_t)MB * kMetaBlockBytes + (size_t)R * ROW > budget) {
        --R;
        MB = (R + kMetaRows - 1) / kMetaRows + 2;
    }
    if (R < 6) return (int)hipErrorInvalidValue;   // the ring needs >= PUB + 2 slots
    if constexpr (GRAD == G_LOGISTIC) {
        // the rows' margins / dots, summed into the loss after the chain
        if (sizeof(T) == 8 ? !L.zbuf64 : !L.zbuf) return (int)hipErrorInvalidValue;
    }
    RingGeom g{R, MB, D, 0};
    const size_t bytes = FIX + (size_t)MB * kMetaBlockBytes + (size_t)R * ROW;
    auto k = full ? chain_split<S, T, GRAD, UPD, CONV, NV, true, H> : chain_split<S, T, GRAD, UPD, CONV, NV, false, H>;
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    hipLaunchKernelGGL(k, dim3(kp.n_chains), dim3(64 * (H + 1)), bytes, st, L, kp, g);
    if constexpr (GRAD == G_LOGISTIC) {
        const int e = (int)hipGetLastError();
        if (e) return e;
        if constexpr (sizeof(T) == 8) return launch_logistic_loss64(L, kp.n_chains, st);
        else return launch_margin_loss(L, kp.n_chains, st);
    }
    return (int)hipGetLastError();
}

template <typename S, typename T, int GRAD, int UPD, bool CONV>
int split_dispatch_nv(const ChainLaunch& L, const KParams& kp, int64_t min_ld, int64_t max_ld, size_t lds,
                      hipStream_t st, int* variant) {
    constexpr int VEC = 16 / sizeof(S);
    const int nv = split_nv<S>(max_ld);
    const bool full = min_ld >= (int64_t)nv * 64 * VEC;
    if (variant) *variant = 800 + 10 * (nv < PSGD_SPLIT_HMAX ? nv : PSGD_SPLIT_HMAX) + nv;
    switch (nv) {
    case 2: return launch_split<S, T, GRAD, UPD, CONV, 2>(L, kp, full, lds, st);
    case 4: return launch_split<S, T, GRAD, UPD, CONV, 4>(L, kp, full, lds, st);
    case 8: return launch_split<S, T, GRAD, UPD, CONV, 8>(L, kp, full, lds, st);
    default: return -3;
    }
}

template <typename S, typename T, int GRAD, bool CONV>
int split_dispatch_conv(const ChainLaunch& L, const KParams& kp, int updater, int64_t min_ld, int64_t max_ld,
                        size_t lds, hipStream_t st, int* variant) {
    switch (updater) {
    case U_ADAGRAD: return split_dispatch_nv<S, T, GRAD, U_ADAGRAD, CONV>(L, kp, min_ld, max_ld, lds, st, variant);
    case U_ADAM: return split_dispatch_nv<S, T, GRAD, U_ADAM, CONV>(L, kp, min_ld, max_ld, lds, st, variant);
    case U_L1: return split_dispatch_nv<S, T, GRAD, U_L1, CONV>(L, kp, min_ld, max_ld, lds, st, variant);
    default: break;
    }
    if constexpr (CONV) {   // tol = 0 keeps the blocked kernels for these two
        if (updater == U_SIMPLE) return split_dispatch_nv<S, T, GRAD, U_SIMPLE, true>(L, kp, min_ld, max_ld, lds, st, variant);
        if (updater == U_SQUARED_L2) return split_dispatch_nv<S, T, GRAD, U_SQUARED_L2, true>(L, kp, min_ld, max_ld, lds, st, variant);
    }
    return -3;
}

template <typename S, typename T, int GRAD>
int split_dispatch_upd(const ChainLaunch& L, const KParams& kp, int updater, int64_t min_ld, int64_t max_ld,
                       size_t lds, hipStream_t st, int* variant) {
    // the per-sample convergence test runs exactly when tol > 0 (psgd_capi.cpp: check_conv)
    if (kp.tol > 0.0) return split_dispatch_conv<S, T, GRAD, true>(L, kp, updater, min_ld, max_ld, lds, st, variant);
    return split_dispatch_conv<S, T, GRAD, false>(L, kp, updater, min_ld, max_ld, lds, st, variant);
}

template <typename S, typename T>
int split_dispatch_grad(const ChainLaunch& L, const KParams& kp, int gradient, int updater, int64_t min_ld,
                        int64_t max_ld, size_t lds, hipStream_t st, int* variant) {
    switch (gradient) {
    case G_LOGISTIC: return split_dispatch_upd<S, T, G_LOGISTIC>(L, kp, updater, min_ld, max_ld, lds, st, variant);
    case G_LEAST_SQUARES: return split_dispatch_upd<S, T, G_LEAST_SQUARES>(L, kp, updater, min_ld, max_ld, lds, st, variant);
    case G_HINGE: return split_dispatch_upd<S, T, G_HINGE>(L, kp, updater, min_ld, max_ld, lds, st, variant);
    default: return -3;
    }
}

}  // namespace

bool split_path_applies(int layout, int updater, bool check_conv, int storage, int64_t max_ld) {
    if (layout != kDense) return false;
    // AdaGrad / Adam / L1 always; Simple / SquaredL2 with the per-sample convergence test (at
    // tol = 0 the blocked kernels take them)
    if (updater != U_ADAGRAD && updater != U_ADAM && updater != U_L1 && !check_conv) return false;
    // PSGD_SPLIT=0 keeps chain_dense (A/B measurements)
    static const bool off = [] {
        const char* e = getenv("PSGD_SPLIT");
        return e && *e == '0';
    }();
    if (off) return false;
    const int nv = storage == 1 ? split_nv<float>(max_ld) : split_nv<double>(max_ld);
    return nv >= 2 && nv <= 8;
}

int launch_split_chains(const ChainLaunch& L, const KParams& kp, int storage, int compute, int gradient,
                        int updater, int64_t min_ld, int64_t max_ld, int lds_spread, hipStream_t st,
                        int* variant) {
    if (!split_path_applies(kDense, updater, kp.tol > 0.0, storage, max_ld)) return -3;
    const size_t lds = (size_t)(lds_spread > 0 ? lds_spread : 0);
    if (storage == 1) {
        if (compute == 1) return split_dispatch_grad<float, float>(L, kp, gradient, updater, min_ld, max_ld, lds, st, variant);
        return split_dispatch_grad<float, double>(L, kp, gradient, updater, min_ld, max_ld, lds, st, variant);
    }
    if (compute == 1) return split_dispatch_grad<double, float>(L, kp, gradient, updater, min_ld, max_ld, lds, st, variant);
    return split_dispatch_grad<double, double>(L, kp, gradient, updater, min_ld, max_ld, lds, st, variant);
}

#endif  // PSGD_NO_DISPATCH

}  // namespace psgd
