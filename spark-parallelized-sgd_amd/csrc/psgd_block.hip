// psgd_block.hip -- the blocked chain kernel of the fp32 throughput mode (gfx950).
//
// Reference: ParallelizedSGD.scala:243-270 (the chain), [ext] MLlib 1.6.1 Gradient.scala
// (Logistic / LeastSquares / Hinge multipliers, called at ParallelizedSGD.scala:254),
// SGDUpdater.scala:86-98 (SimpleSGDUpdater) and :163-181 (SquaredL2SGDUpdater).
//
// The chain is sequential: w_{t+1} = a_t w_t + c_t x_t with c_t = -s_t * mult(x_t . w_t, y_t),
// s_t = stepSize/sqrt(t+1), a_t = 1 (Simple) or 1 - s_t*lambda (SquaredL2). Done sample by sample
// the critical path of every sample is a 512-long dot, a cross-lane reduction and the update
// (~100 dependent cycles), which caps one chain per CU well below the HBM rate. Over a block of
// K = 8 consecutive rows with weights W at its start the same recurrence is exactly
//
//     p_k = x_k . W                       (K independent dots against one W)
//     G[k][i] = x_k . x_i, i < k          (the block's Gram triangle, independent of W)
//     z_0 = p_0;  acc_k <- a_i acc_k + c_i G[k][i]  after step i;  z_k = acc_k after step k-1
//     W'  = a_{K-1}(...(a_0 W + c_0 x_0)...) + c_{K-1} x_{K-1}
//
// so the only sequential work left per sample is scalar (c_i from z_i, one FMA per lane). The
// rounding differs from the per-sample form (dot products reassociated, updates fused), which
// is the fp32 throughput mode's stated tolerance; the fp64 parity mode runs the
// same blocked recurrence in doubles (chain_block64, psgd_block64.hip).
//
// One workgroup = one chain = four waves, one per SIMD:
//   wave 0 (chain)   owns W in VGPRs (lane l: features (v*64+l)*VEC ..), per block: reads the K
//                    rows from the LDS ring, the K dots (packed FMAs + one transposed reduction
//                    of 8 values), the scalar recurrence with the Gram row of its lane, the loss,
//                    and the K updates;
//   wave 1 (loader)  LDS-DMA row ring (ring_loader, shared with chain_dense);
//   waves 2, 3 (Gram) alternate blocks: the 28 pair dots of a block (packed FMAs + a transposed
//                    reduction of 32 values), written as an 8x8 lower-triangular matrix into a
//                    Gram ring slot in LDS.
// No MFMA: the Gram triangle is 3.5 dots per row; a 16x16 f32 MFMA tile would spend 16.
//
// The per-sample break (tol > 0, CONV; PSGD.scala:262, :324-336) is decided inside the block as in
// chain_block64 (psgd_block64.hip): with w' = a w + c x, z = x . w and q = x . x (the Gram
// diagonal, added to the Gram slot), ||w'||^2 = a (a ||w||^2 + 2 c z) + c^2 q and
// ||w - w'||^2 = b (b ||w||^2 - 2 c z) + c^2 q (b = 1 - a); isConverged is D < tol^2 max(N, 1).
// ||w||^2 is taken exactly from the registers at every block start (one more wave sum under the
// dots), so the fp32 recurrence runs over at most 8 rows. The first passing row ends the chain.
#include "psgd_device.h"

#include <stdlib.h>

namespace psgd {

constexpr int kBlk = 8;           // rows per block
constexpr int kPairs = 28;        // kBlk*(kBlk-1)/2 Gram entries below the diagonal
constexpr float kNegLog2e = -1.44269504088896341f;   // u = -log2(e) * z
constexpr float kLn2Neg = -0.693147180559945309f;    // z = -ln(2) * u
static_assert(kMetaRows == 2 * kBlk, "a meta block holds two row blocks");

struct GramHeader {
    unsigned gdone[2];   // blocks finished by Gram wave 0 (even blocks) / 1 (odd blocks)
    unsigned gread[2];   // blocks whose rows Gram wave 0 / 1 holds in registers (ring slots free)
};

// --- transposed wave reductions -----------------------------------------------------------
// Several per-lane partial sums are reduced at once: every stage halves the number of values a
// lane carries and doubles the lanes each value is summed over. permlane32_swap(x, y) leaves
// {x.lo|y.lo} and {x.hi|y.hi}: their sum holds x's total over the two halves in lanes 0-31 and
// y's in lanes 32-63. permlane16_swap does the same for odd/even rows of 16 lanes.
__device__ __forceinline__ float pair32(float x, float y) {
    auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(y), false, false);
    return __uint_as_float(p[0]) + __uint_as_float(p[1]);
}
__device__ __forceinline__ float pair16(float x, float y) {
    auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(y), false, false);
    return __uint_as_float(p[0]) + __uint_as_float(p[1]);
}
// Inside a row: lanes with `bit` clear keep x, the others y; each adds its DPP partner's copy.
template <int CTRL, int BIT>
__device__ __forceinline__ float pair_dpp(float x, float y, int lane) {
    const bool hi = (lane & BIT) != 0;
    const float keep = hi ? y : x;
    const float send = hi ? x : y;
    return keep + dpp_mov<CTRL>(send);
}

// 8 values -> lane l holds the total of value k(l) = l5 | l4<<1 | l3<<2 (lane bits).
__device__ __forceinline__ float reduce8(const float (&v)[8], int lane) {
    const float a0 = pair32(v[0], v[1]), a1 = pair32(v[2], v[3]);
    const float a2 = pair32(v[4], v[5]), a3 = pair32(v[6], v[7]);
    const float b0 = pair16(a0, a1), b1 = pair16(a2, a3);
    float r = pair_dpp<0x140, 8>(b0, b1, lane);   // row_mirror: partner l^15
    r = r + dpp_mov<0xB1>(r);                      // quad_perm [1,0,3,2]: l^1
    r = r + dpp_mov<0x4E>(r);                      // quad_perm [2,3,0,1]: l^2
    r = r + dpp_mov<0x141>(r);                     // row_half_mirror: l^7
    return r;
}
// 32 values -> lane l holds the total of value j(l) = l5 | l4<<1 | l3<<2 | l2<<3 | l1<<4.
__device__ __forceinline__ float reduce32(const float (&v)[32], int lane) {
    float a[16], b[8], c[4], e[2];
#pragma unroll
    for (int m = 0; m < 16; ++m) a[m] = pair32(v[2 * m], v[2 * m + 1]);
#pragma unroll
    for (int m = 0; m < 8; ++m) b[m] = pair16(a[2 * m], a[2 * m + 1]);
#pragma unroll
    for (int m = 0; m < 4; ++m) c[m] = pair_dpp<0x140, 8>(b[2 * m], b[2 * m + 1], lane);   // l^15
#pragma unroll
    for (int m = 0; m < 2; ++m) e[m] = pair_dpp<0x141, 4>(c[2 * m], c[2 * m + 1], lane);   // l^7
    float r = pair_dpp<0x4E, 2>(e[0], e[1], lane);                                           // l^2
    return r + dpp_mov<0xB1>(r);                                                             // l^1
}

// Lane that carries row i of a block after reduce8 (any lane with k(l) = i; this one has l&7 = 0).
__host__ __device__ constexpr int row_lane(int i) {
    return 32 * (i & 1) + 16 * ((i >> 1) & 1) + 8 * ((i >> 2) & 1);
}

__device__ __forceinline__ float readlane_f(float v, int lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

// Lane `addr / 4`'s double (ds_bpermute on both halves); a double of the lane `sh` below in a row
// of 16 (DPP row_shr, 0 past the row's start).
__device__ __forceinline__ double bperm_d32(double v, int addr) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const int lo = __builtin_amdgcn_ds_bpermute(addr, (int)(unsigned)b);
    const int hi = __builtin_amdgcn_ds_bpermute(addr, (int)(unsigned)(b >> 32));
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
__device__ __forceinline__ double dpp_shr_d(double v, int sh) {
    return sh == 1 ? dpp_mov<0x111>(v) : sh == 2 ? dpp_mov<0x112>(v) : dpp_mov<0x114>(v);
}

// c = -s * mult(z, y) for the gradient (vector form; only lane row_lane(i) matters at step i).
//   Logistic: mult = 1/(1+exp(-z)) - y;  LeastSquares: mult = z - y;  Hinge: mult = 1 > ls*z ? -ls : 0
template <int GRAD>
__device__ __forceinline__ float coef(float z, float y, float s, float ns, float aux) {
    if constexpr (GRAD == G_LEAST_SQUARES) {
        return __builtin_fmaf(ns, z, aux);            // aux = s*y: -s*z + s*y
    } else if constexpr (GRAD == G_LOGISTIC) {
        // z is u = -log2(e) * dot: 1/(1+exp(-dot)) = 1/(1+2^u); aux = s*y
        const float sig = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(z));
        return __builtin_fmaf(ns, sig, aux);
    } else {
        return (aux * z < 1.0f) ? s * aux : 0.0f;     // aux = ls = 2y - 1: -s * (-ls)
    }
}

// MLUtils.log1pExp with the hardware exp2/log2 (fp32 throughput mode: ~1e-7 absolute)
__device__ __forceinline__ float fast_log1p_exp(float x) {
    const float ax = __builtin_fabsf(x);
    const float l = __logf(1.0f + __expf(-ax));
    return x > 0.0f ? x + l : l;
}

template <int GRAD>
__device__ __forceinline__ float row_loss(float z, float y, float aux) {
    if constexpr (GRAD == G_LEAST_SQUARES) {
        const float m = z - y;
        return m * m;                                  // halved once at the end (exact)
    } else if constexpr (GRAD == G_LOGISTIC) {
        const float margin = -z;
        const float l = fast_log1p_exp(margin);
        return y > 0.0f ? l : l - margin;
    } else {
        const float lz = aux * z;
        return (1.0f > lz) ? 1.0f - lz : 0.0f;
    }
}

// floats per Gram ring slot: the 8x8 triangle, and with the per-sample break the 8 row norms
template <bool CONV>
constexpr int gram_slot32() { return kBlk * kBlk + (CONV ? kBlk : 0); }

template <typename S, int GRAD, int UPD, int NV, bool FULL, bool CONV = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void chain_block(ChainLaunch L, KParams kp, RingGeom geom) {
    using V = typename Vec16<S>::type;
    using T2 = float __attribute__((ext_vector_type(2)));
    constexpr int VEC = Vec16<S>::N;
    constexpr int E = NV * VEC;            // features per lane
    constexpr int E2 = E / 2;
    constexpr int H = VEC / 2;             // pairs per 16-byte vector
    constexpr int ROW_BYTES = NV * 1024;
    constexpr bool KEEP = E2 * kBlk <= 64; // the chain wave keeps a block's rows in registers
    constexpr int GSZ = gram_slot32<CONV>();
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // LDS: [RingHeader 16 B][GramHeader 16 B][meta ring MB x 256 B][Gram ring GS x 256 B]
    //      [row ring R x ROW_BYTES]
    RingHeader* hdr = reinterpret_cast<RingHeader*>(smem);
    GramHeader* ghdr = reinterpret_cast<GramHeader*>(smem + sizeof(RingHeader));
    char* meta_ring = smem + sizeof(RingHeader) + sizeof(GramHeader);
    float* gring = reinterpret_cast<float*>(meta_ring + geom.meta_blocks * kMetaBlockBytes);
    const int GS = geom.gslots;
    char* ring = reinterpret_cast<char*>(gring + GS * GSZ);

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int chain = blockIdx.x;
    const ChainDesc dsc = L.descs[chain];
    const int d = kp.d;
    const int64_t n = dsc.n_rows;
    const int R = geom.rows;               // multiple of kBlk: a block never wraps
    const int MB = geom.meta_blocks;
    const int64_t nblk = (n + kBlk - 1) / kBlk;

    if (threadIdx.x == 0) {
        hdr->ready = 0;
        hdr->consumed = 0;
        hdr->stop = 0;
        ghdr->gdone[0] = 0;
        ghdr->gdone[1] = 0;
        ghdr->gread[0] = 0;
        ghdr->gread[1] = 0;
    }
    // entries on and above the diagonal stay zero (the Gram waves write only i < k)
    for (int i = threadIdx.x; i < GS * GSZ; i += blockDim.x) gring[i] = 0.0f;
    __syncthreads();

    if (wave == 1) {
        ring_loader<S, NV, FULL, kBlk, kBlk>(L, dsc, hdr, meta_ring, ring, geom, lane, ghdr->gread);
        return;
    }

    // Wait until `rows` rows have landed. false (and the watchdog) if nothing moves for 4 s.
    auto wait_ready = [&](unsigned& ready, int64_t rows, int code) __attribute__((always_inline)) -> bool {
        if (rows <= (int64_t)ready) return true;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        for (;;) {
            ready = __hip_atomic_load(&hdr->ready, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (rows <= (int64_t)ready) return true;
            if (__hip_atomic_load(&hdr->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return false;
            if (__builtin_amdgcn_s_memrealtime() - t0 > kWatchdogTicks) {
                __hip_atomic_fetch_or(L.watchdog, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&hdr->stop, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                return false;
            }
            if (code != 2) __builtin_amdgcn_s_sleep(1);   // the chain wave polls without sleeping
        }
    };
    // One 16-byte vector of a row slot, zero past the row end (those LDS bytes are stale).
    auto read_vec = [&](const char* slot, int v) __attribute__((always_inline)) -> V {
        V xv = *reinterpret_cast<const V*>(slot + v * 1024 + lane * 16);
        if constexpr (!FULL) {
            if ((v * 64 + lane) * VEC >= dsc.ld) xv = V(0);
        }
        return xv;
    };
    auto to_pairs = [&](const V& xv, T2* out) __attribute__((always_inline)) {
        float tmp[VEC];
        unpack<S, float>(xv, tmp);
#pragma unroll
        for (int h = 0; h < H; ++h) out[h] = T2{tmp[2 * h], tmp[2 * h + 1]};
    };

    if (wave >= 2) {
        // ---------------- Gram waves ----------------
        const int gw = wave - 2;
        // this lane's (k, i) after reduce32, as an offset into an 8x8 slot (-1: padding / odd lane)
        const int j = ((lane >> 5) & 1) | (((lane >> 4) & 1) << 1) | (((lane >> 3) & 1) << 2) |
                      (((lane >> 2) & 1) << 3) | (((lane >> 1) & 1) << 4);
        int goff = -1;
        {
            int jj = 0;
            for (int k = 1; k < kBlk; ++k)
                for (int i = 0; i < k; ++i, ++jj)
                    if (jj == j) goff = k * kBlk + i;
            if (lane & 1) goff = -1;
        }
        unsigned ready = 0;
        unsigned done = 0;
        int rs = gw * kBlk;          // ring slot of the block's first row (R is a multiple of 16)
        int gs = gw;                 // Gram slot of the block
        PSGD_STAMP(const uint64_t st_begin = __builtin_amdgcn_s_memtime(); uint64_t st_rd = 0;)
        for (int64_t b = gw; b < nblk; b += 2) {
            const int64_t t0 = b * kBlk;
            const int64_t kk = (n - t0) < kBlk ? (n - t0) : kBlk;
            PSGD_STAMP(const uint64_t st_w = __builtin_amdgcn_s_memtime();)
            if (!wait_ready(ready, t0 + kk, 4)) break;
            PSGD_STAMP(st_rd += __builtin_amdgcn_s_memtime() - st_w;)
            const char* base = ring + rs * ROW_BYTES;
            rs += 2 * kBlk;
            if (rs >= R) rs -= R;
            // NV >= 4: the whole block into registers first, then hand its ring slots back: the
            // loader refills them while the pair dots run (with a 4-block ring at d = 1,024 the
            // slots held for the Gram's ~2,000 cycles are what the row stream waits for; c3
            // 3-5 % faster). At NV = 2 (9-block ring) the early hand-back measured 1-2 % slower.
            constexpr bool EARLY = NV >= 4;
            T2 xall[NV][kBlk][H];
#pragma unroll
            for (int v = 0; v < NV; ++v)
#pragma unroll
                for (int k = 0; k < kBlk; ++k) to_pairs(read_vec(base + k * ROW_BYTES, v), xall[v][k]);
            if constexpr (EARLY) {
                asm volatile("s_waitcnt lgkmcnt(0)" : : : "memory");
                __hip_atomic_store(&ghdr->gread[gw], done + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            T2 acc[kPairs];
#pragma unroll
            for (int q = 0; q < kPairs; ++q) acc[q] = T2{0.0f, 0.0f};
            T2 dg[CONV ? kBlk : 1];   // CONV: the rows' squared norms (the Gram diagonal)
#pragma unroll
            for (int k = 0; k < (CONV ? kBlk : 1); ++k) dg[k] = T2{0.0f, 0.0f};
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                auto& xc = xall[v];
                int q = 0;
#pragma unroll
                for (int k = 1; k < kBlk; ++k)
#pragma unroll
                    for (int i = 0; i < k; ++i, ++q)
#pragma unroll
                        for (int h = 0; h < H; ++h)
                            acc[q] = __builtin_elementwise_fma(xc[k][h], xc[i][h], acc[q]);
                if constexpr (CONV) {
#pragma unroll
                    for (int k = 0; k < kBlk; ++k)
#pragma unroll
                        for (int h = 0; h < H; ++h) dg[k] = __builtin_elementwise_fma(xc[k][h], xc[k][h], dg[k]);
                }
            }
            float g[32];
#pragma unroll
            for (int q = 0; q < kPairs; ++q) g[q] = acc[q].x + acc[q].y;
#pragma unroll
            for (int q = kPairs; q < 32; ++q) g[q] = 0.0f;
            float val = reduce32(g, lane);
            if constexpr (GRAD == G_LOGISTIC) val *= kNegLog2e;   // the chain works on u
            float* slot = gring + gs * GSZ;
            gs += 2;
            if (gs >= GS) gs -= GS;
            if (goff >= 0) slot[goff] = val;
            if constexpr (CONV) {
                // unscaled (the break test uses the real norms); reduce8's layout, one lane per row
                float dv[kBlk];
#pragma unroll
                for (int k = 0; k < kBlk; ++k) dv[k] = dg[k].x + dg[k].y;
                const float qn = reduce8(dv, lane);
                const int kq = ((lane >> 5) & 1) | (((lane >> 4) & 1) << 1) | (((lane >> 3) & 1) << 2);
                if ((lane & 7) == 0) slot[kBlk * kBlk + kq] = qn;
            }
            ++done;
            __hip_atomic_store(&ghdr->gdone[gw], done, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            if constexpr (!EARLY)
                __hip_atomic_store(&ghdr->gread[gw], done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        PSGD_STAMP(if (L.stamps && lane == 0) {
            unsigned long long* o = L.stamps + (size_t)chain * 16 + 8 + 4 * gw;
            o[0] = __builtin_amdgcn_s_memtime() - st_begin; o[1] = st_rd;
        })
        return;
    }

    // ---------------- chain wave ----------------
    T2 w[E2];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const int base = (v * 64 + lane) * VEC;
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            const int f = base + k;
            const double wv = as_global(L.w_in)[f < d ? f : 0];
            w[(v * VEC + k) / 2][(v * VEC + k) % 2] = f < d ? float(wv) : 0.0f;
        }
    }
    const int krow = ((lane >> 5) & 1) | (((lane >> 4) & 1) << 1) | (((lane >> 3) & 1) << 2);
    const bool loss_lane = (lane & 7) == 0;   // one copy of every row's loss
    // Logistic: the rows' margins go to L.zbuf and margin_loss_kernel sums their losses after
    // the chain (log1pExp costs the sequential wave ~60 cycles per row; off its critical path)
    constexpr bool LOSS_EXT = GRAD == G_LOGISTIC;
    gmut<float> zout = as_global_mut(L.zbuf + (LOSS_EXT ? (int64_t)chain * L.zstride : 0));
    const float lam = float(kp.reg);
    double loss_sum = 0.0;
    float loss_blk = 0.0f;
    int64_t count = 0;
    unsigned ready = 0;
    int rs = 0, gs = 0, ms = 0;      // ring slot, Gram slot and meta block of the current block
    const int64_t nfull = n / kBlk;
    const int ntail = (int)(n - nfull * kBlk);
    bool conv_stop = false;   // CONV: a row passed isConverged, the chain has ended
    PSGD_STAMP(const uint64_t st_begin = __builtin_amdgcn_s_memtime(); uint64_t st_rd = 0, st_gr = 0, st_p = 0, st_rec = 0, st_upd = 0;)

    auto wait_rows = [&](int64_t rows) __attribute__((always_inline)) -> bool {
        PSGD_STAMP(const uint64_t st_w = __builtin_amdgcn_s_memtime();)
        const bool ok = wait_ready(ready, rows, 2);
        PSGD_STAMP(st_rd += __builtin_amdgcn_s_memtime() - st_w;)
        return ok;
    };
    // A block's rows from the ring into registers; rows >= kk (a tail block) read as zero.
    auto load_rows = [&](auto tail_c, T2 (&xr)[kBlk][E2], const char* base, int kk) __attribute__((always_inline)) {
        constexpr bool TAIL = decltype(tail_c)::value;
#pragma unroll
        for (int k = 0; k < kBlk; ++k) {
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                T2 xv[H];
                to_pairs(read_vec(base + k * ROW_BYTES, v), xv);
#pragma unroll
                for (int h = 0; h < H; ++h) xr[k][v * H + h] = (TAIL && k >= kk) ? T2{0.0f, 0.0f} : xv[h];
            }
        }
    };

    // One block: rows in xr (KEEP) or in the ring at `base`; kk rows (kBlk unless TAIL).
    auto block = [&](auto tail_c, T2 (&xr)[kBlk][E2], int64_t b, int kk, const char* base)
                     __attribute__((always_inline)) -> bool {
        constexpr bool TAIL = decltype(tail_c)::value;
        const int64_t t0 = b * kBlk;
        // this lane's row: label and step
        const f64x2 meta = *reinterpret_cast<const f64x2*>(
            meta_ring + ms * kMetaBlockBytes + ((int)(b & 1) * kBlk + krow) * 16);
        if constexpr (KEEP) {
            // the block's rows are in registers (its Gram and meta slots are reused only after
            // the next block is handed back): free its ring slots (the loader also waits for the
            // block's Gram wave to be done with them)
            __hip_atomic_store(&hdr->consumed, (unsigned)(t0 + kk), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        // The flags this block will test, read now: one wave per SIMD hides no LDS latency, so a
        // flag read where it is tested costs a full LDS round trip per block (~30 cycles per row
        // at c2); read here it lands under the dots. (Relaxed: LDS accesses of a workgroup are
        // performed in order, and the data they guard is read only after the test.)
        const unsigned gpre = __hip_atomic_load(&ghdr->gdone[b & 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const unsigned rpre = __hip_atomic_load(&hdr->ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        // p_k = x_k . W (one packed accumulator per row; eight rows interleave)
        PSGD_STAMP(const uint64_t st_a = __builtin_amdgcn_s_memtime();)
        float pk[kBlk];
#pragma unroll
        for (int k = 0; k < kBlk; ++k) {
            T2 a;
            if constexpr (KEEP) {
                a = xr[k][0] * w[0];
#pragma unroll
                for (int e = 1; e < E2; ++e) a = __builtin_elementwise_fma(xr[k][e], w[e], a);
            } else {
                a = T2{0.0f, 0.0f};
#pragma unroll
                for (int v = 0; v < NV; ++v) {
                    T2 xv[H];
                    to_pairs(read_vec(base + k * ROW_BYTES, v), xv);
#pragma unroll
                    for (int h = 0; h < H; ++h) a = __builtin_elementwise_fma(xv[h], w[v * H + h], a);
                }
            }
            pk[k] = a.x + a.y;
        }
        // CONV: ||W||^2 at the block start, exact from the registers (the recurrence below then
        // spans at most this block's 8 rows)
        float nsq = 0.0f;
        if constexpr (CONV) {
            T2 a = w[0] * w[0];
#pragma unroll
            for (int e = 1; e < E2; ++e) a = __builtin_elementwise_fma(w[e], w[e], a);
            nsq = wave_sum(a.x + a.y);
        }
        const float yv = float(meta.x), sv = float(meta.y);
        const float nsv = -sv;
        float aux;
        if constexpr (GRAD == G_HINGE) aux = 2.0f * yv - 1.0f;
        else aux = sv * yv;
        const float alpha = 1.0f - sv * lam;      // SquaredL2 shrink of this lane's row
        float z = reduce8(pk, lane);
        // Logistic runs the recurrence on u = -log2(e) z (its Gram triangle is scaled the same
        // way by the Gram waves): exp(-z) is then one v_exp_f32 of u
        if constexpr (GRAD == G_LOGISTIC) z *= kNegLog2e;
        PSGD_STAMP(const uint64_t st_b = __builtin_amdgcn_s_memtime(); st_p += st_b - st_a;)
        // the block's Gram triangle (Gram wave b&1 publishes blocks in order), waited for only
        // now so that the dots above overlap its computation
        PSGD_STAMP(const uint64_t st_g = __builtin_amdgcn_s_memtime();)
        {
            const unsigned need = (unsigned)(b >> 1) + 1;
            unsigned* gd = &ghdr->gdone[b & 1];
            if (gpre < need) {
                const uint64_t tw = __builtin_amdgcn_s_memrealtime();
                while (__hip_atomic_load(gd, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < need) {
                    if (__builtin_amdgcn_s_memrealtime() - tw > kWatchdogTicks) {
                        __hip_atomic_fetch_or(L.watchdog, 8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store(&hdr->stop, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        return false;
                    }
                }
            }
        }
        PSGD_STAMP(st_gr += __builtin_amdgcn_s_memtime() - st_g;)
        const float* grow = gring + gs * GSZ + krow * kBlk;
        const f32x4 g0 = *reinterpret_cast<const f32x4*>(grow);
        const f32x4 g1 = *reinterpret_cast<const f32x4*>(grow + 4);
        const float G[kBlk] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
        float q = 0.0f;   // CONV: the squared norm of this lane's row
        if constexpr (CONV) q = gring[gs * GSZ + kBlk * kBlk + krow];

        // the scalar recurrence: c_i from z_i, then every later row's dot moves by c_i G[k][i]
        // (SquaredL2 also shrinks the finished rows' z: zf keeps z_k for the loss)
        float c[kBlk], al[kBlk];
        float zf = z;
        bool brk = false;   // CONV: a row of this block passed isConverged
        int keff = kk;      // the rows taken
        float ck = 0.0f;    // CONV: this lane's row's coefficient (lane row_lane(k) computed c_k at step k)
#pragma unroll
        for (int i = 0; i < kBlk; ++i) {
            const float cv = coef<GRAD>(z, yv, sv, nsv, aux);
            c[i] = readlane_f(cv, row_lane(i));
            if constexpr (TAIL) c[i] = i < kk ? c[i] : 0.0f;
            if constexpr (UPD == U_SQUARED_L2) {
                al[i] = readlane_f(alpha, row_lane(i));
                if constexpr (TAIL) al[i] = i < kk ? al[i] : 1.0f;
            }
            if constexpr (UPD == U_SQUARED_L2) {
                if (krow == i) zf = z;
                if (i + 1 < kBlk) z = __builtin_fmaf(c[i], G[i], al[i] * z);
            } else {
                if (i + 1 < kBlk) z = __builtin_fmaf(c[i], G[i], z);
            }
        }
        if constexpr (UPD != U_SQUARED_L2) zf = z;
        // CONV: this lane's row's coefficient, recomputed once from its final z (a lane's z stops
        // moving after its row's step: G[k][i] = 0 for i >= k; SquaredL2's zf keeps it through
        // the later rows' shrinks) -- the value row_lane(k) computed at step k, for ~3 operations
        // instead of a select at each of the 8 steps
        if constexpr (CONV) ck = coef<GRAD>(zf, yv, sv, nsv, aux);
        // W <- a_i W + c_i x_i for the block's rows in sample order (CONV: every row, as if no
        // row passes; W at the block start is kept for the rare block where one does)
        auto update_rows = [&](int last) __attribute__((always_inline)) {
#pragma unroll
            for (int i = 0; i < kBlk; ++i) {
                if (i > last) break;
                const T2 ci = T2{c[i], c[i]};
                if constexpr (KEEP) {
#pragma unroll
                    for (int e = 0; e < E2; ++e) {
                        if constexpr (UPD == U_SQUARED_L2)
                            w[e] = __builtin_elementwise_fma(ci, xr[i][e], w[e] * T2{al[i], al[i]});
                        else
                            w[e] = __builtin_elementwise_fma(ci, xr[i][e], w[e]);
                    }
                } else if (!TAIL || i < kk) {
#pragma unroll
                    for (int v = 0; v < NV; ++v) {
                        T2 xv[H];
                        to_pairs(read_vec(base + i * ROW_BYTES, v), xv);
#pragma unroll
                        for (int h = 0; h < H; ++h) {
                            const int e = v * H + h;
                            if constexpr (UPD == U_SQUARED_L2)
                                w[e] = __builtin_elementwise_fma(ci, xv[h], w[e] * T2{al[i], al[i]});
                            else
                                w[e] = __builtin_elementwise_fma(ci, xv[h], w[e]);
                        }
                    }
                }
            }
        };
        if constexpr (CONV) {
            // isConverged(w_k, w_{k+1}) (PSGD.scala:262, :324-336) for the block's rows at once, in
            // f64 (as the CSR kernels' conv_step): with w' = a w + c x, z = x . w and
            // q = x . x, ||w_{k+1}||^2 = a^2 ||w_k||^2 + c (2 a z + c q) and
            // ||w_k - w_{k+1}||^2 = b^2 ||w_k||^2 + c (c q - 2 b z) with b = s lambda taken directly
            // (1 - a is 0 in fp32 once s lambda < 2^-25). The rows' terms move to lanes 8m + k
            // (ds_bpermute) and a segmented DPP scan from the block start's exact ||W||^2 gives
            // every row's norms; the first row with D_k < tol^2 max(N_{k+1}, 1) ends the chain.
            // The block's updates run between the bpermutes and the scan (their latency), as if no
            // row passed; on a pass (once per chain) W is restored and the taken rows replayed.
            const bool live = !TAIL || krow < kk;
            const double c_ = live ? double(ck) : 0.0;
            double zd = double(zf);
            if constexpr (GRAD == G_LOGISTIC) zd *= double(kLn2Neg);   // u -> the dot
            const double cq1 = c_ * double(q);
            const int kl = lane & 7;
            const int src = row_lane(kl) * 4;
            const double n0 = double(nsq);
            double A = 1.0, B, b2 = 0.0, E;
            if constexpr (UPD == U_SQUARED_L2) {
                const double a_ = live ? double(alpha) : 1.0, b_ = meta.y * kp.reg;
                A = bperm_d32(a_ * a_, src);
                B = bperm_d32(c_ * __builtin_fma(2.0 * a_, zd, cq1), src);
                b2 = bperm_d32(b_ * b_, src);
                E = bperm_d32(c_ * __builtin_fma(-2.0 * b_, zd, cq1), src);
            } else {
                B = bperm_d32(c_ * __builtin_fma(2.0, zd, cq1), src);
                E = bperm_d32(c_ * cq1, src);
            }
            T2 wsave[E2];
#pragma unroll
            for (int e = 0; e < E2; ++e) wsave[e] = w[e];
            update_rows(kBlk - 1);
            double Nn, dd;
            if constexpr (UPD == U_SQUARED_L2) {
#pragma unroll
                for (int sh = 1; sh < kBlk; sh *= 2) {   // (this after the earlier one)
                    const double oA = dpp_shr_d(A, sh), oB = dpp_shr_d(B, sh);
                    const bool take = kl >= sh;
                    const double nB = __builtin_fma(A, oB, B);
                    A = take ? A * oA : A;
                    B = take ? nB : B;
                }
                Nn = __builtin_fma(A, n0, B);
                double Nk = dpp_shr_d(Nn, 1);
                Nk = kl == 0 ? n0 : Nk;
                dd = __builtin_fma(b2, Nk, E);
            } else {
#pragma unroll
                for (int sh = 1; sh < kBlk; sh *= 2) {
                    const double oB = dpp_shr_d(B, sh);
                    B = kl >= sh ? oB + B : B;
                }
                Nn = n0 + B;
                dd = E;
            }
            const double tol2d = kp.tol * kp.tol;
            const bool pass = (lane < kBlk) & (!TAIL || kl < kk) & (dd < tol2d * (Nn > 1.0 ? Nn : 1.0));   // branch-free
            // the updates stay ahead of the test (not sunk into its no-pass branch)
#pragma unroll
            for (int e = 0; e < E2; ++e) asm volatile("" : "+v"(w[e]));
            const unsigned long long m = __builtin_amdgcn_ballot_w64(pass);
            if (m != 0ull) {   // the first passing row ends the chain (once per chain)
                const int kstar = __builtin_ctzll(m);
                brk = true;
                keff = kstar + 1;
#pragma unroll
                for (int e = 0; e < E2; ++e) w[e] = wsave[e];
                update_rows(kstar);
            }
        }
        PSGD_STAMP(const uint64_t st_c = __builtin_amdgcn_s_memtime(); st_rec += st_c - st_b;)
        if constexpr (LOSS_EXT) {
            if (loss_lane && ((!TAIL && !CONV) || krow < keff)) zout[t0 + krow] = zf * kLn2Neg;   // u -> dot
        } else {
            const float l = row_loss<GRAD>(zf, yv, aux);
            if (loss_lane && ((!TAIL && !CONV) || krow < keff)) loss_blk += l;
            if ((b & 3) == 3) { loss_sum += double(loss_blk); loss_blk = 0.0f; }
        }
        count += keff;
        if constexpr (CONV) conv_stop = brk;
        if (rpre > ready) ready = rpre;   // the next block's wait_rows rarely reads the flag again
        if constexpr (!CONV) update_rows(kBlk - 1);
        if constexpr (!KEEP) {
            __hip_atomic_store(&hdr->consumed, (unsigned)(t0 + kk), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        PSGD_STAMP(st_upd += __builtin_amdgcn_s_memtime() - st_c;)
        rs += kBlk;
        if (rs == R) rs = 0;
        if (++gs == GS) gs = 0;
        if ((b & 1) && ++ms == MB) ms = 0;
        return true;
    };

    using Full = std::integral_constant<bool, false>;
    using Tail = std::integral_constant<bool, true>;
    T2 xr[kBlk][E2];
    bool ok = true;
    for (int64_t b = 0; ok && !conv_stop && b < nfull; ++b) {
        ok = wait_rows((b + 1) * kBlk);
        if (!ok) break;
        const char* base = ring + rs * ROW_BYTES;
        if constexpr (KEEP) load_rows(Full{}, xr, base, kBlk);
        ok = block(Full{}, xr, b, kBlk, base);
    }
    if (ok && !conv_stop && ntail > 0 && wait_rows(n)) {
        const char* base = ring + rs * ROW_BYTES;
        if constexpr (KEEP) load_rows(Tail{}, xr, base, ntail);
        block(Tail{}, xr, nfull, ntail, base);
    }
    // a wave that stopped early leaves the others blocked on it: wake them
    __hip_atomic_store(&hdr->stop, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    PSGD_STAMP(if (L.stamps && lane == 0) {
        unsigned long long* o = L.stamps + (size_t)chain * 16;
        o[0] = __builtin_amdgcn_s_memtime() - st_begin; o[1] = st_rd; o[2] = st_gr;
        o[3] = st_p; o[12 + 2] = st_rec; o[12 + 3] = st_upd;
    })
    loss_sum += double(loss_blk);
    // the loss partials of the 8 loss lanes
    {
        double ls = loss_sum;
        ls = wave_sum(ls);
        loss_sum = ls;
    }
    if constexpr (GRAD == G_LEAST_SQUARES) loss_sum = loss_sum / 2.0;

    // regVal of the chain's last update (PSGD.scala:257; 0.0 if no sample, :247)
    double rv = 0.0;
    if constexpr (UPD == U_SQUARED_L2) {
        float acc = 0.0f;
#pragma unroll
        for (int e = 0; e < E2; ++e) acc += w[e].x * w[e].x + w[e].y * w[e].y;
        acc = wave_sum(acc);
        if (count > 0) {
            const double nrm = sqrt(double(acc));
            rv = 0.5 * kp.reg * nrm * nrm;
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
        if constexpr (!LOSS_EXT) L.loss[chain] = loss_sum;
        L.cnt[chain] = count;
        L.cnt_d[chain] = double(count);
    }
}

// The Logistic loss of the chain's rows from their margins (PSGD.scala:254's lossSum; [ext] MLlib
// 1.6.1 LogisticGradient: margin = -z, loss = y > 0 ? log1pExp(margin) : log1pExp(margin) - margin),
// in f64, one 1024-thread workgroup per chain (16 waves per CU: the f64 log1p/exp chains are
// latency-bound per thread). z_t is the fp32 chain's dot for row t before its update.
__global__ __launch_bounds__(1024) void margin_loss_kernel(ChainLaunch L) {
    const int chain = blockIdx.x;
    const int64_t n = L.cnt[chain];
    const double* y = L.descs[chain].y;
    const float* z = L.zbuf + (int64_t)chain * L.zstride;
    double acc = 0.0;
    for (int64_t t = threadIdx.x; t < n; t += blockDim.x) {
        const double margin = -double(as_global(z)[t]);
        const double l = log1p_exp(margin);
        acc += as_global(y)[t] > 0.0 ? l : l - margin;
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

int launch_margin_loss(const ChainLaunch& L, int n_chains, hipStream_t st) {
    if (!L.zbuf) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(margin_loss_kernel, dim3(n_chains), dim3(1024), 0, st, L);
    return (int)hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// Launcher.
// ------------------------------------------------------------------------------------------
template <typename S, int GRAD, int UPD, int NV, bool CONV>
static int launch_block(const ChainLaunch& L, const KParams& kp, bool full, size_t lds, hipStream_t st) {
    constexpr int ROW = NV * 1024;
    const size_t budget = lds > 0 ? lds : (size_t)64 * 1024;
    const size_t fixed = sizeof(RingHeader) + sizeof(GramHeader);
    const int D = loader_depth<NV>();
    int R = 0, MB = 0, GS = 0;
    auto bytes_for = [&](int r) {
        const int mb = (r + kMetaRows - 1) / kMetaRows + 2;
        const int gs = r / kBlk + 1;
        return fixed + (size_t)mb * kMetaBlockBytes + (size_t)gs * gram_slot32<CONV>() * 4 + (size_t)r * ROW;
    };
    // a block never wraps (R multiple of kBlk); one block beyond the loader's depth keeps the
    // stream going while the chain wave holds a block
    R = (int)((budget - fixed) / ROW) / kBlk * kBlk;
    while (R > 0 && bytes_for(R) > budget) R -= kBlk;
    if (R < 2 * kBlk) return (int)hipErrorInvalidValue;  // LDS budget too small for this d
    MB = (R + kMetaRows - 1) / kMetaRows + 2;
    GS = R / kBlk + 1;
    RingGeom g{R, MB, D, GS};
    const size_t bytes = bytes_for(R);
    if (full) {
        auto k = chain_block<S, GRAD, UPD, NV, true, CONV>;
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
        hipLaunchKernelGGL(k, dim3(kp.n_chains), dim3(256), bytes, st, L, kp, g);
    } else {
        auto k = chain_block<S, GRAD, UPD, NV, false, CONV>;
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
        hipLaunchKernelGGL(k, dim3(kp.n_chains), dim3(256), bytes, st, L, kp, g);
    }
    if constexpr (GRAD == G_LOGISTIC) {
        if (!L.zbuf) return (int)hipErrorInvalidValue;
        hipLaunchKernelGGL(margin_loss_kernel, dim3(kp.n_chains), dim3(1024), 0, st, L);
    }
    return (int)hipGetLastError();
}

// The dispatch over every instantiation (left out of the diagnostic build, tools/chain_bench.hip).
#ifndef PSGD_NO_DISPATCH
// Variant 300 + 40 (the per-sample break, tol > 0) + NV.
template <typename S, int GRAD, int UPD, bool CONV>
static int block_nv(const ChainLaunch& L, const KParams& kp, int64_t min_ld, int64_t max_ld,
                    size_t lds, hipStream_t st, int* variant) {
    constexpr int VEC = 16 / sizeof(S);
    int nv = 1;
    while (nv * 64 * VEC < max_ld) nv *= 2;
    const bool full = min_ld >= (int64_t)nv * 64 * VEC;
    if (variant) *variant = 300 + (CONV ? 40 : 0) + nv;
    switch (nv) {
    case 1: return launch_block<S, GRAD, UPD, 1, CONV>(L, kp, full, lds, st);
    case 2: return launch_block<S, GRAD, UPD, 2, CONV>(L, kp, full, lds, st);
    case 4: return launch_block<S, GRAD, UPD, 4, CONV>(L, kp, full, lds, st);
    case 8: return launch_block<S, GRAD, UPD, 8, CONV>(L, kp, full, lds, st);
    default: return -3;
    }
}

template <typename S, int GRAD>
static int block_upd(const ChainLaunch& L, const KParams& kp, int upd, int64_t min_ld,
                     int64_t max_ld, size_t lds, hipStream_t st, int* variant) {
    const bool conv = kp.tol > 0.0;   // the per-sample break: a template instance of its own
    if (upd == U_SIMPLE)
        return conv ? block_nv<S, GRAD, U_SIMPLE, true>(L, kp, min_ld, max_ld, lds, st, variant)
                    : block_nv<S, GRAD, U_SIMPLE, false>(L, kp, min_ld, max_ld, lds, st, variant);
    if (upd == U_SQUARED_L2)
        return conv ? block_nv<S, GRAD, U_SQUARED_L2, true>(L, kp, min_ld, max_ld, lds, st, variant)
                    : block_nv<S, GRAD, U_SQUARED_L2, false>(L, kp, min_ld, max_ld, lds, st, variant);
    return -3;
}

template <typename S>
static int block_grad(const ChainLaunch& L, const KParams& kp, int grad, int upd, int64_t min_ld,
                      int64_t max_ld, size_t lds, hipStream_t st, int* variant) {
    switch (grad) {
    case G_LOGISTIC: return block_upd<S, G_LOGISTIC>(L, kp, upd, min_ld, max_ld, lds, st, variant);
    case G_LEAST_SQUARES: return block_upd<S, G_LEAST_SQUARES>(L, kp, upd, min_ld, max_ld, lds, st, variant);
    case G_HINGE: return block_upd<S, G_HINGE>(L, kp, upd, min_ld, max_ld, lds, st, variant);
    default: return -3;
    }
}

bool block_path_applies(int layout, int compute, int updater, bool check_conv, int storage,
                        int64_t max_ld) {
    // any tol (CONV instances when kp.tol > 0); PSGD_B64_CONV=0 keeps tol > 0 on the per-sample
    // kernels, as for chain_block64 (read at every launch)
    if (check_conv) {
        const char* e = getenv("PSGD_B64_CONV");
        if (e && e[0] == '0') return false;
    }
    const int vec = storage == 1 ? 4 : 2;
    return layout == kDense && compute == 1 &&
           (updater == U_SIMPLE || updater == U_SQUARED_L2) && max_ld <= 8 * 64 * vec;
}

int launch_block_chains(const ChainLaunch& L, const KParams& kp, int storage, int gradient,
                        int updater, int64_t min_ld, int64_t max_ld, int lds_spread,
                        hipStream_t stream, int* kernel_variant) {
    if (kp.n_chains <= 0) return 0;
    const size_t lds = (size_t)(lds_spread > 0 ? lds_spread : 0);
    if (storage == 1)
        return block_grad<float>(L, kp, gradient, updater, min_ld, max_ld, lds, stream, kernel_variant);
    return block_grad<double>(L, kp, gradient, updater, min_ld, max_ld, lds, stream, kernel_variant);
}

#endif  // PSGD_NO_DISPATCH

}  // namespace psgd
