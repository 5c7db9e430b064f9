// psgd_block64.hip -- the blocked chain kernel of the fp64 parity mode (gfx950).
//
// Reference: ParallelizedSGD.scala:243-270 (the chain), [ext] MLlib 1.6.1 Gradient.scala
// (Logistic / LeastSquares / Hinge, called at ParallelizedSGD.scala:254), SGDUpdater.scala:86-98
// (SimpleSGDUpdater) and :163-181 (SquaredL2SGDUpdater); all in Double, as here.
//
// Same recurrence as the fp32 chain_block (psgd_block.hip): over a block of K = 8 consecutive
// rows with weights W at its start,
//
//     z_k = x_k . W + sum_{i<k} c_i (x_k . x_i)          (SquaredL2: z <- a_i z + c_i G[k][i])
//     W'  = a_{K-1}(...(a_0 W + c_0 x_0)...) + c_{K-1} x_{K-1}
//
// with c_i = -s_i * mult(z_i, y_i), s_i = stepSize/sqrt(j), a_i = 1 - s_i*lambda. Every quantity is
// a double: the K dots against W, the Gram triangle (products of the stored values are exact in
// f64 for f32 rows), the scalar recurrence with the reference's multipliers (exp and the division
// of LogisticGradient in f64), the updates. Only sums are reassociated (the wave tree of each dot,
// the Gram identity above, the fused c*x + w update), which is the fp64 mode's 1e-9 relative bar
// (DESIGN.md §4). L1/AdaGrad/Adam run on the per-sample kernels (psgd_split.hip, psgd_kernels.hip).
//
// The per-sample break (tol > 0, CONV; PSGD.scala:262, :324-336): isConverged(w_i, w_{i+1}) after
// row i's update needs ||w_i - w_{i+1}|| and ||w_{i+1}||, and both follow from scalars the block
// already has. With w' = a w + c x (a = 1 for Simple), z = x . w (the row's dot) and q = x . x
// (the Gram diagonal, which the Gram waves add to their slot):
//     ||w'||^2       = a^2 ||w||^2 + c (2 a z + c q)
//     ||w - w'||^2   = b^2 ||w||^2 + c (c q - 2 b z),   b = s lambda (= 1 - a)
// and the test sqrt(D) < tol max(sqrt(N), 1) is D < tol^2 max(N, 1). ||w||^2 starts exact (the
// chain waves' partial norms of w_in) and follows these affine maps in the chain's sample order:
// round 5 evaluates a block's 8 tests at once after its recurrence (a scan over the rows' maps
// in lane registers, block64's CONV section), not row by row on the recurrence's dependent path. Every
// fp64 kernel decides as the oracle down to tol = r (1 +- 1e-13) (tests/test_gpu_break_margin.py).
// The first row that passes ends the chain: the updates of the block's later rows, issued
// interleaved with the recurrence, are undone (W restored from the block start, the taken rows
// replayed: once per chain), their loss and count dropped, and no later block runs.
//
// Why blocks in fp64: the per-sample kernel (chain_dense) has the dot's wave reduction, an f64
// exp and a division and the update on one dependent path per sample (~400 ns at d = 100). Here
// only the scalar recurrence is sequential per sample; the dots, the Gram triangle and the
// updates are batched over 8 rows and spread over three waves on three SIMDs.
//
// One workgroup = one chain = four waves, one per SIMD:
//   wave 0 (chain)   owns W (doubles in VGPRs: lane l holds features (v*64+l)*VEC ..), per block:
//                    the 8 dots, one transposed 8-value reduction, the recurrence, the loss terms,
//                    the 8 updates;
//   wave 1 (loader)  the LDS-DMA row ring of chain_dense/chain_block (ring_loader);
//   waves 2, 3 (Gram) alternate blocks: the 28 pair dots of a block in f64 (rows converted from
//                    the storage type), one transposed 32-value reduction, an 8x8 lower-triangular
//                    f64 slot in LDS.
// No MFMA: the triangle is 3.5 dots per row (an f64 16x16x4 MFMA tile would spend 16).
#include "psgd_device.h"

#include <type_traits>


namespace psgd {

namespace {

constexpr int kB = 8;            // rows per block
constexpr int kPairs = 28;       // kB*(kB-1)/2
static_assert(kMetaRows == 2 * kB, "a meta block holds two row blocks");

struct GramHeader64 {
    unsigned gdone[2];   // blocks finished by Gram wave 0 (even blocks) / 1 (odd blocks)
    unsigned gread[2];   // blocks whose rows Gram wave 0 / 1 has read (their ring slots are free)
};

__device__ __forceinline__ unsigned lo32(double v) { return (unsigned)(unsigned long long)__double_as_longlong(v); }
__device__ __forceinline__ unsigned hi32(double v) { return (unsigned)((unsigned long long)__double_as_longlong(v) >> 32); }
__device__ __forceinline__ double mk64(unsigned lo, unsigned hi) {
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// Transposed wave reductions on doubles (both 32-bit halves permuted alike), as reduce8 /
// reduce32 of psgd_block.hip: each stage halves the values a lane carries.
__device__ __forceinline__ double pair32d(double x, double y) {
    auto pl = __builtin_amdgcn_permlane32_swap(lo32(x), lo32(y), false, false);
    auto ph = __builtin_amdgcn_permlane32_swap(hi32(x), hi32(y), false, false);
    return mk64(pl[0], ph[0]) + mk64(pl[1], ph[1]);
}
__device__ __forceinline__ double pair16d(double x, double y) {
    auto pl = __builtin_amdgcn_permlane16_swap(lo32(x), lo32(y), false, false);
    auto ph = __builtin_amdgcn_permlane16_swap(hi32(x), hi32(y), false, false);
    return mk64(pl[0], ph[0]) + mk64(pl[1], ph[1]);
}
template <int CTRL, int BIT>
__device__ __forceinline__ double pair_dppd(double x, double y, int lane) {
    const bool hi = (lane & BIT) != 0;
    const double keep = hi ? y : x;
    const double send = hi ? x : y;
    return keep + dpp_mov<CTRL>(send);
}

// 8 values -> lane l holds the total of value k(l) = l5 | l4<<1 | l3<<2.
__device__ __forceinline__ double reduce8d(const double (&v)[8], int lane) {
    const double a0 = pair32d(v[0], v[1]), a1 = pair32d(v[2], v[3]);
    const double a2 = pair32d(v[4], v[5]), a3 = pair32d(v[6], v[7]);
    const double b0 = pair16d(a0, a1), b1 = pair16d(a2, a3);
    double r = pair_dppd<0x140, 8>(b0, b1, lane);   // row_mirror: partner l^15
    r = r + dpp_mov<0xB1>(r);                        // quad_perm [1,0,3,2]: l^1
    r = r + dpp_mov<0x4E>(r);                        // quad_perm [2,3,0,1]: l^2
    r = r + dpp_mov<0x141>(r);                       // row_half_mirror: l^7
    return r;
}
// 32 values -> lane l holds the total of value j(l) = l5 | l4<<1 | l3<<2 | l2<<3 | l1<<4.
__device__ __forceinline__ double reduce32d(const double (&v)[32], int lane) {
    double a[16], b[8], c[4], e[2];
#pragma unroll
    for (int m = 0; m < 16; ++m) a[m] = pair32d(v[2 * m], v[2 * m + 1]);
#pragma unroll
    for (int m = 0; m < 8; ++m) b[m] = pair16d(a[2 * m], a[2 * m + 1]);
#pragma unroll
    for (int m = 0; m < 4; ++m) c[m] = pair_dppd<0x140, 8>(b[2 * m], b[2 * m + 1], lane);   // l^15
#pragma unroll
    for (int m = 0; m < 2; ++m) e[m] = pair_dppd<0x141, 4>(c[2 * m], c[2 * m + 1], lane);   // l^7
    double r = pair_dppd<0x4E, 2>(e[0], e[1], lane);                                          // l^2
    return r + dpp_mov<0xB1>(r);                                                              // l^1
}

// Lane that carries row i of a block after reduce8d (one with k(l) = i and l&7 = 0).
__host__ __device__ constexpr int row_lane64(int i) {
    return 32 * (i & 1) + 16 * ((i >> 1) & 1) + 8 * ((i >> 2) & 1);
}


#ifndef PSGD_B64_FAST_SIGMOID
#define PSGD_B64_FAST_SIGMOID 1
#endif

// c = (-s) * mult(z, y): the step the row's gradient takes ([ext] MLlib 1.6.1 Gradient.compute,
// SGDUpdater.scala:95 / :178 axpy(-thisIterStepSize, gradient, w)).
//   Logistic: mult = 1/(1 + exp(-z)) - y;  LeastSquares: mult = z - y;
//   Hinge: mult = 1 > ls*z ? -ls : 0 (ls = 2y - 1; the empty gradient adds nothing)
template <int GRAD>
__device__ __forceinline__ double coef64(double z, double y, double ns) {
    if constexpr (GRAD == G_LEAST_SQUARES) {
        return ns * (z - y);
    } else if constexpr (GRAD == G_LOGISTIC) {
        const double margin = -z;
#if PSGD_B64_FAST_SIGMOID
        return ns * (recip_one_plus_exp(margin) - y);
#else
        return ns * ((1.0 / (1.0 + exp(margin))) - y);
#endif
    } else {
        const double ls = 2.0 * y - 1.0;
        return (1.0 > ls * z) ? ns * (-ls) : 0.0;
    }
}

// The row's loss ([ext] MLlib 1.6.1): LeastSquares diff*diff/2.0; Hinge 1 - ls*z or 0.
// (Logistic's loss is evaluated after the chain from the stored z, logistic_loss64_kernel.)
template <int GRAD>
__device__ __forceinline__ double row_loss64(double z, double y) {
    if constexpr (GRAD == G_LEAST_SQUARES) {
        const double diff = z - y;
        return diff * diff / 2.0;
    } else {
        const double ls = 2.0 * y - 1.0;
        const double lz = ls * z;
        return (1.0 > lz) ? 1.0 - lz : 0.0;
    }
}

}  // namespace

// The SIMD a wave runs on (HW_REG_HW_ID bits 5:4).
__device__ __forceinline__ unsigned wave_simd() {
    unsigned id;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(id));
    return (id >> 4) & 3;
}

// Role of wave w given every wave's SIMD (3 + H waves; the same answer in every wave). Roles:
// 0 .. H-1 chain waves, then (H = 1) 1 loader, 2, 3 Gram waves / (H = 2) 2, 3 Gram waves,
// 4 loader. The dispatcher does not promise which SIMD a wave of a workgroup lands on, and the
// chain waves are the critical path: the first chain wave is wave 0, the second the first wave on
// another SIMD (one it has to itself if there is one); the loader (it mostly sleeps on the
// ring) takes a SIMD a chain wave is on if any remaining wave is, so the Gram waves do not.
template <int H>
__device__ __forceinline__ int role_of_wave(const unsigned* simd, int w) {
    constexpr int NW = 3 + H;
    int count[4] = {0, 0, 0, 0};
    for (int i = 0; i < NW; ++i) ++count[simd[i] & 3];
    int role[NW];
    for (int i = 0; i < NW; ++i) role[i] = -1;
    role[0] = 0;
    int c1 = -1;
    if constexpr (H == 2) {
        for (int i = 1; i < NW && c1 < 0; ++i)
            if (simd[i] != simd[0] && count[simd[i] & 3] == 1) c1 = i;
        for (int i = 1; i < NW && c1 < 0; ++i)
            if (simd[i] != simd[0]) c1 = i;
        if (c1 < 0) c1 = 1;
        role[c1] = 1;
    }
    int ld = -1;
    for (int i = 1; i < NW && ld < 0; ++i)
        if (role[i] < 0 && (simd[i] == simd[0] || (c1 >= 0 && simd[i] == simd[c1]))) ld = i;
    for (int i = NW - 1; i >= 1 && ld < 0; --i)
        if (role[i] < 0) ld = i;
    role[ld] = H == 1 ? 1 : 4;
    int g = 2;
    for (int i = 1; i < NW; ++i)
        if (role[i] < 0) role[i] = g++;
    return role[w];
}

// The chain waves of one chain (H = 2) exchange their partial dots through LDS once per block:
// per block parity and chain wave, one partial per row; at the chain's end, the partial ||w||^2.
struct XchgHeader64 {
    unsigned xdone[2];   // blocks whose partial dots chain wave 0 / 1 has published
    unsigned fin[2];     // chain wave 0 / 1 has published its partial ||w||^2
    unsigned start[2];   // CONV: chain wave 0 / 1 has published its partial ||w_in||^2
    unsigned pad[2];
};
constexpr int kXchgDoubles = 2 * 2 * kB + 2 + 2;
constexpr size_t kFixed64 = sizeof(RingHeader) + sizeof(GramHeader64) + sizeof(XchgHeader64) +
                            kXchgDoubles * sizeof(double);
static_assert(kFixed64 % 16 == 0, "the meta and row rings start 16-byte aligned");

// f32 rows: a chain wave that owns at most 8 features per lane converts its share of a block to
// doubles once (64 VGPRs of rows become 128); 0 converts at every use (dot and update).
#ifndef PSGD_B64_CONV1
#define PSGD_B64_CONV1 1
#endif
#ifndef PSGD_B64_INTERLEAVE
#define PSGD_B64_INTERLEAVE 1
#endif
// the next block's row reads under this block's recurrence (PREF in chain_block64; 0 for A/B)
#ifndef PSGD_B64_PREFETCH
#define PSGD_B64_PREFETCH 1
#endif
// cost probes (tools/chain_bench64 builds only; wrong results): 1 the recurrence without its
// dependency (z not moved by the Gram terms), 2 no wait for the other chain wave's partials
#ifndef PSGD_B64_EXP
#define PSGD_B64_EXP 0
#endif

// doubles per Gram ring slot: the 8x8 triangle, and with the per-sample break the block's 8
// squared row norms
template <bool CONV>
constexpr int gram_slot64() { return kB * kB + (CONV ? kB : 0); }

// The Gram work split by features (round 5): from PSGD_B64_FSPLIT_NV row vectors on (c3 with the
// reference's f64 rows: NV = 8, 2 blocks of 8 KiB rows in the LDS ring), both Gram waves take every
// block, each over half of the row's vectors, into a sub-slot of their own; the chain waves add the
// halves. A Gram wave's half of a block fits its registers, so it reads it first and hands the
// ring slots back before the pair dots (the undivided Gram read one vector of every row at a time
// and held the slots for its whole ~2,300 cycles: at c3 f64 rows the chain waited ~300 cycles per
// row for it, the loader was blocked on the full ring half the time; tools/chain_bench64 stamps).
#ifndef PSGD_B64_FSPLIT_NV
#define PSGD_B64_FSPLIT_NV 8
#endif
template <int NV>
constexpr bool gram_fsplit64() { return PSGD_B64_FSPLIT_NV > 0 && NV >= PSGD_B64_FSPLIT_NV && NV >= 2; }

template <typename S, int GRAD, int UPD, int NV, bool FULL, int H, bool CONV>
__global__ __launch_bounds__(64 * (3 + H)) __attribute__((amdgpu_waves_per_eu(H, H)))
void chain_block64(ChainLaunch L, KParams kp, RingGeom geom) {
    using V = typename Vec16<S>::type;
    constexpr int VEC = Vec16<S>::N;
    constexpr bool F32 = std::is_same<S, float>::value;
    constexpr int NVH = NV / H;            // 1 KiB row slices owned by one chain wave
    constexpr int EH = NVH * VEC;          // features per lane of one chain wave
    constexpr int ROW_BYTES = NV * 1024;
    static_assert(H == 1 || H == 2, "one or two chain waves");
    static_assert(NV % H == 0, "the chain waves split the row slices evenly");
    static_assert(EH <= (F32 ? 16 : 8), "a chain wave keeps its share of a block's rows in registers");
    constexpr bool CONV1 = F32 && H == 2 && EH <= 8 && PSGD_B64_CONV1;
    // wave roles (role_of_waves): chain waves 0 .. H-1, Gram waves 2 and 3, the loader
    constexpr int kRoleLoader = H == 1 ? 1 : 4;
    constexpr int GSZ = gram_slot64<CONV>();
    constexpr bool FS = gram_fsplit64<NV>();
    constexpr int GSL = FS ? 2 * GSZ : GSZ;   // doubles per block in the Gram ring
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // LDS: [RingHeader 16 B][GramHeader64 16 B][XchgHeader64 32 B][exchange 36 doubles]
    //      [meta ring MB x 256 B][Gram ring GS x GSZ doubles][row ring R x ROW_BYTES]
    RingHeader* hdr = reinterpret_cast<RingHeader*>(smem);
    GramHeader64* ghdr = reinterpret_cast<GramHeader64*>(smem + sizeof(RingHeader));
    XchgHeader64* xhdr = reinterpret_cast<XchgHeader64*>(smem + sizeof(RingHeader) + sizeof(GramHeader64));
    double* xchg = reinterpret_cast<double*>(smem + sizeof(RingHeader) + sizeof(GramHeader64) + sizeof(XchgHeader64));
    char* meta_ring = smem + kFixed64;
    double* gring = reinterpret_cast<double*>(meta_ring + geom.meta_blocks * kMetaBlockBytes);
    const int GS = geom.gslots;
    char* ring = reinterpret_cast<char*>(gring + GS * GSL);

    const int lane = threadIdx.x & 63;
    const int chain = blockIdx.x;
    const ChainDesc dsc = L.descs[chain];
    const int d = kp.d;
    const int64_t n = dsc.n_rows;
    const int R = geom.rows;               // multiple of kB: a block never wraps
    const int MB = geom.meta_blocks;
    const int64_t nblk = (n + kB - 1) / kB;

    if (threadIdx.x == 0) {
        hdr->ready = 0;
        hdr->consumed = 0;
        hdr->stop = 0;
        hdr->consumed1 = 0;
        ghdr->gdone[0] = 0;
        ghdr->gdone[1] = 0;
        ghdr->gread[0] = 0;
        ghdr->gread[1] = 0;
        xhdr->xdone[0] = 0;
        xhdr->xdone[1] = 0;
        xhdr->fin[0] = 0;
        xhdr->fin[1] = 0;
        xhdr->start[0] = 0;
        xhdr->start[1] = 0;
    }
    // entries on and above the diagonal stay zero (the Gram waves write only i < k)
    for (int i = threadIdx.x; i < GS * GSL; i += blockDim.x) gring[i] = 0.0;
    // every wave's SIMD, for the role assignment (the exchange area is free until the chain starts)
    unsigned* simd_of = reinterpret_cast<unsigned*>(xchg);
    if (lane == 0) simd_of[threadIdx.x >> 6] = wave_simd();
    __syncthreads();
    const int wave = __builtin_amdgcn_readfirstlane(role_of_wave<H>(simd_of, threadIdx.x >> 6));
    __syncthreads();   // the SIMD table is read by every wave before the exchange area is used

    if (wave == kRoleLoader) {
        ring_loader<S, NV, FULL, kB, kB, H, FS>(L, dsc, hdr, meta_ring, ring, geom, lane, ghdr->gread);
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
            if (code != 2) __builtin_amdgcn_s_sleep(1);   // the chain waves poll without sleeping
        }
    };
    // One 16-byte vector of a row slot as doubles, zero past the row end (stale LDS bytes).
    auto read_vec = [&](const char* slot, int v, double* out) __attribute__((always_inline)) {
        V xv = *reinterpret_cast<const V*>(slot + v * 1024 + lane * 16);
        if constexpr (!FULL) {
            if ((v * 64 + lane) * VEC >= dsc.ld) xv = V(0);
        }
        unpack<S, double>(xv, out);
    };

    if (wave >= 2) {
        // ---------------- Gram waves ----------------
        const int gw = wave - 2;
        const int j = ((lane >> 5) & 1) | (((lane >> 4) & 1) << 1) | (((lane >> 3) & 1) << 2) |
                      (((lane >> 2) & 1) << 3) | (((lane >> 1) & 1) << 4);
        int goff = -1;   // this lane's (k, i) after reduce32d, as an offset into an 8x8 slot
        {
            int jj = 0;
            for (int k = 1; k < kB; ++k)
                for (int i = 0; i < k; ++i, ++jj)
                    if (jj == j) goff = k * kB + i;
            if (lane & 1) goff = -1;
        }
        unsigned ready = 0;
        unsigned done = 0;
        PSGD_STAMP(const uint64_t st_begin = __builtin_amdgcn_s_memtime(); uint64_t st_rd = 0;)
        // FS: every block, vectors [v0, v0 + NVG) of its rows; else alternate blocks, every vector
        constexpr int BSTEP = FS ? 1 : 2;
        constexpr int NVG = FS ? NV / 2 : NV;
        const int v0 = FS ? gw * NVG : 0;
        int rs = FS ? 0 : gw * kB;   // ring slot of the block's first row (R is a multiple of 16)
        int gs = FS ? 0 : gw;        // Gram slot of the block
        for (int64_t b = FS ? 0 : gw; b < nblk; b += BSTEP) {
            const int64_t t0 = b * kB;
            const int64_t kk = (n - t0) < kB ? (n - t0) : kB;
            PSGD_STAMP(const uint64_t st_w = __builtin_amdgcn_s_memtime();)
            if (!wait_ready(ready, t0 + kk, 4)) break;
            PSGD_STAMP(st_rd += __builtin_amdgcn_s_memtime() - st_w;)
            const char* base = ring + rs * ROW_BYTES;
            rs += BSTEP * kB;
            if (rs >= R) rs -= R;
            double acc[kPairs];
#pragma unroll
            for (int q = 0; q < kPairs; ++q) acc[q] = 0.0;
            double dg[kB];   // CONV: the rows' squared norms (the Gram diagonal)
#pragma unroll
            for (int k = 0; k < kB; ++k) dg[k] = 0.0;
            if constexpr (FS) {
                // this wave's half of the block into registers, the slots back, then the dots
                double xa[NVG][kB][VEC];
#pragma unroll
                for (int v = 0; v < NVG; ++v)
#pragma unroll
                    for (int k = 0; k < kB; ++k) read_vec(base + k * ROW_BYTES, v0 + v, xa[v][k]);
                asm volatile("s_waitcnt lgkmcnt(0)" : : : "memory");
                __hip_atomic_store(&ghdr->gread[gw], done + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
                for (int v = 0; v < NVG; ++v) {
                    int q = 0;
#pragma unroll
                    for (int k = 1; k < kB; ++k)
#pragma unroll
                        for (int i = 0; i < k; ++i, ++q)
#pragma unroll
                            for (int hh = 0; hh < VEC; ++hh) acc[q] = __builtin_fma(xa[v][k][hh], xa[v][i][hh], acc[q]);
                    if constexpr (CONV) {
#pragma unroll
                        for (int k = 0; k < kB; ++k)
#pragma unroll
                            for (int hh = 0; hh < VEC; ++hh) dg[k] = __builtin_fma(xa[v][k][hh], xa[v][k][hh], dg[k]);
                    }
                }
            } else {
            // one 16-byte vector of every row at a time (f64 rows of a whole block would not
            // fit the registers at NV >= 4)
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                double xc[kB][VEC];
#pragma unroll
                for (int k = 0; k < kB; ++k) read_vec(base + k * ROW_BYTES, v, xc[k]);
                int q = 0;
#pragma unroll
                for (int k = 1; k < kB; ++k)
#pragma unroll
                    for (int i = 0; i < k; ++i, ++q)
#pragma unroll
                        for (int h = 0; h < VEC; ++h) acc[q] = __builtin_fma(xc[k][h], xc[i][h], acc[q]);
            }
            if constexpr (CONV) {
                // the diagonal in a pass of its own, one row vector at a time (in the pair pass
                // its 8 accumulators beside the 28 pushed the wave past its registers; the rows are
                // read again -- the compiler barrier keeps it from reusing the pair pass's loads)
                asm volatile("" : : : "memory");
#pragma unroll
                for (int k = 0; k < kB; ++k)
#pragma unroll
                    for (int v = 0; v < NV; ++v) {
                        double xk[VEC];
                        read_vec(base + k * ROW_BYTES, v, xk);
#pragma unroll
                        for (int h = 0; h < VEC; ++h) dg[k] = __builtin_fma(xk[h], xk[h], dg[k]);
                    }
            }
            // every row of the block has been read: hand its ring slots back
            asm volatile("s_waitcnt lgkmcnt(0)" : : : "memory");
            __hip_atomic_store(&ghdr->gread[gw], done + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            double g[32];
#pragma unroll
            for (int q = 0; q < kPairs; ++q) g[q] = acc[q];
#pragma unroll
            for (int q = kPairs; q < 32; ++q) g[q] = 0.0;
            const double val = reduce32d(g, lane);
            double* slot = gring + gs * GSL + (FS ? gw * GSZ : 0);
            gs += BSTEP;
            if (gs >= GS) gs -= GS;
            if (goff >= 0) slot[goff] = val;
            if constexpr (CONV) {
                // lane l holds row k(l)'s norm (reduce8d's layout); one lane per row writes it
                const double qn = reduce8d(dg, lane);
                const int kq = ((lane >> 5) & 1) | (((lane >> 4) & 1) << 1) | (((lane >> 3) & 1) << 2);
                if ((lane & 7) == 0) slot[kB * kB + kq] = qn;
            }
            ++done;
            __hip_atomic_store(&ghdr->gdone[gw], done, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        PSGD_STAMP(if (L.stamps && lane == 0) {
            unsigned long long* o = L.stamps + (size_t)chain * 16 + 8 + 4 * gw;
            o[0] = __builtin_amdgcn_s_memtime() - st_begin; o[1] = st_rd;
        })
        return;
    }

    // ---------------- chain waves ----------------
    // Chain wave h owns the row slices [h*NVH, (h+1)*NVH): lane l holds features
    // ((h*NVH + u)*64 + l)*VEC .. +VEC-1 of W, u < NVH. With H = 2 each wave takes the partial
    // dots of a block over its features; the two partials of row k are added as p0 + p1 in both
    // waves, so both run the identical scalar recurrence and update their own features.
    const int h = wave;
    const bool lead = h == 0;                 // the loss terms, count and regVal
    double w[EH];
#pragma unroll
    for (int u = 0; u < NVH; ++u) {
        const int base = ((h * NVH + u) * 64 + lane) * VEC;
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            const int f = base + k;
            const double wv = as_global(L.w_in)[f < d ? f : 0];
            w[u * VEC + k] = f < d ? wv : 0.0;
        }
    }
    // CONV: ||w||^2 of the chain's current weights (the same value in both chain waves), from the
    // exact partial norms of w_in; tol2 = tol^2
    double nsq = 0.0;
    const double tol2 = kp.tol * kp.tol;
    bool conv_stop = false;   // CONV: a row passed isConverged, the chain has ended
    if constexpr (CONV) {
        double a = 0.0;
#pragma unroll
        for (int e = 0; e < EH; ++e) a = __builtin_fma(w[e], w[e], a);
        a = wave_sum(a);
        if constexpr (H == 2) {
            if (lane == 0) xchg[2 * 2 * kB + 2 + h] = a;
            asm volatile("s_waitcnt lgkmcnt(0)" : : : "memory");
            __hip_atomic_store(&xhdr->start[h], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            const uint64_t tw = __builtin_amdgcn_s_memrealtime();
            while (!__hip_atomic_load(&xhdr->start[h ^ 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
                if (__builtin_amdgcn_s_memrealtime() - tw > kWatchdogTicks) {
                    __hip_atomic_fetch_or(L.watchdog, 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(&hdr->stop, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    break;
                }
            }
            asm volatile("" : : : "memory");   // the partial is read after its flag
            const double other = xchg[2 * 2 * kB + 2 + (h ^ 1)];
            a = h == 0 ? a + other : other + a;
        }
        nsq = a;
    }
    const int krow = ((lane >> 5) & 1) | (((lane >> 4) & 1) << 1) | (((lane >> 3) & 1) << 2);
    const bool loss_lane = (lane & 7) == 0;   // one copy of every row's loss
    // Logistic: the rows' dots go to L.zbuf64 and logistic_loss64_kernel sums their losses after
    // the chain (log1pExp is a second exp and a log1p; off the sequential wave)
    constexpr bool LOSS_EXT = GRAD == G_LOGISTIC;
    gmut<double> zout = as_global_mut(L.zbuf64 + (LOSS_EXT ? (int64_t)chain * L.zstride : 0));
    unsigned* const my_consumed = (H == 2 && h == 1) ? &hdr->consumed1 : &hdr->consumed;
    const double lam = kp.reg;
    double loss_sum = 0.0;
    int64_t count = 0;
    unsigned ready = 0;
    int rs = 0, gs = 0, ms = 0;      // ring slot, Gram slot and meta block of the current block
    const int64_t nfull = n / kB;
    const int ntail = (int)(n - nfull * kB);
    PSGD_STAMP(const uint64_t st_begin = __builtin_amdgcn_s_memtime(); uint64_t st_rd = 0, st_gr = 0, st_p = 0, st_rec = 0, st_upd = 0, st_x = 0;)

    auto wait_rows = [&](int64_t rows) __attribute__((always_inline)) -> bool {
        return wait_ready(ready, rows, 2);
    };
    // This wave's share of a block's rows, from the ring into registers (as stored, or as
    // doubles with CONV1); rows >= kk (a tail block) are zero.
    V xraw[kB][NVH];
    double xcv[CONV1 ? kB : 1][CONV1 ? EH : 1];
    // the reads of a block's rows into xraw, as stored (no use of the loaded values: a prefetch
    // must not wait for them here)
    auto issue_rows = [&](const char* base) __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < kB; ++k)
#pragma unroll
            for (int u = 0; u < NVH; ++u)
                xraw[k][u] = *reinterpret_cast<const V*>(base + k * ROW_BYTES + (h * NVH + u) * 1024 + lane * 16);
    };
    // zero past the row end (stale LDS bytes) and, in a tail block, the rows >= kk; CONV1: convert
    auto finish_rows = [&](auto tail_c, int kk) __attribute__((always_inline)) {
        constexpr bool TAIL = decltype(tail_c)::value;
#pragma unroll
        for (int k = 0; k < kB; ++k) {
#pragma unroll
            for (int u = 0; u < NVH; ++u) {
                if constexpr (!FULL) {
                    if (((h * NVH + u) * 64 + lane) * VEC >= dsc.ld) xraw[k][u] = V(0);
                }
                if (TAIL && k >= kk) xraw[k][u] = V(0);
            }
        }
        if constexpr (CONV1) {
            // every read is issued before the first conversion: converting as each read lands
            // made the compiler reuse one register quad and wait for every read in turn
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int k = 0; k < kB; ++k)
#pragma unroll
                for (int u = 0; u < NVH; ++u) unpack<S, double>(xraw[k][u], &xcv[k][u * VEC]);
        }
    };
    // PREF (round 6): with CONV1 xraw is dead once converted, so the next block's row reads are
    // issued into it under this block's recurrence and break test (block(); `pre` says they were)
    // instead of at the next block's start. Measured in tools/chain_bench64 (c2 shape, f32 rows,
    // profiles/r06_block64_prefetch_ab.log): LeastSquares with the break on 5.16 -> 4.85 ms, at
    // tol = 0 -1 %; Logistic +8 % at c2 and, at NV = 4, 64 more live VGPRs spill (c3 +58 %) -- so
    // only the break-on instances of the cheap multipliers at NV <= 2.
    constexpr bool PREF = CONV1 && CONV && GRAD != G_LOGISTIC && NV <= 2 && PSGD_B64_PREFETCH;
    bool pre = false;
    // VEC doubles of row k, slice u
    auto xrow = [&](int k, int u, double* out) __attribute__((always_inline)) {
        if constexpr (CONV1) {
#pragma unroll
            for (int q = 0; q < VEC; ++q) out[q] = xcv[k][u * VEC + q];
        } else {
            unpack<S, double>(xraw[k][u], out);
        }
    };
    // CONV: isConverged(w_k, w_{k+1}) (PSGD.scala:262, :333-335) for a block's rows at once:
    // with w' = a w + c x, z = x . w (zf: the row's dot before its step) and q = x . x,
    // ||w_{k+1}||^2 = a^2 ||w_k||^2 + c (2 a z + c q) is an affine map of ||w_k||^2 per row and
    // D_k = ||w_k - w_{k+1}||^2 = b^2 N_k + c (c q - 2 b z) with b = s lambda. A scan over the rows'
    // maps in k order gives N_k and N_{k+1} from the block start's norm n0, and the first row with
    // D_k < tol^2 max(N_{k+1}, 1) ends the chain. Every lane has its own row's terms (krow): the
    // scan is the kpair butterfly across the rows' lane groups, in registers. (Round 4 ran the test
    // per row, ~10 dependent f64 operations on the chain waves: c2 fp64 +51 % over tol 0; the first
    // round-5 form moved the rows' terms with ds_bpermute for a DPP segmented scan.) Returns the
    // ballot of the passing rows (lanes 8g, ballot_rows) and sets nsq_out to N after the block.
    auto conv_test = [&](double c_, double zf, double q, double a_, double b_, bool live, double n0,
                         double& nsq_out) __attribute__((always_inline)) -> unsigned long long {
        const double cq1 = c_ * q;
        double Nn, dd;
        if constexpr (UPD == U_SQUARED_L2) {
            // row k's map N -> A N + B; the exclusive prefix map (eA, eB) of the rows before it
            // gives N_k, then N_{k+1} = A N_k + B and D_k = b^2 N_k + E
            const double A = a_ * a_;
            const double B = c_ * __builtin_fma(2.0 * a_, zf, cq1);
            const double E = c_ * __builtin_fma(-2.0 * b_, zf, cq1);
            double eA = 1.0, eB = 0.0, tA = A, tB = B;
            static_for<3>([&](auto jc) {
                constexpr int J = decltype(jc)::value;
                const PairD pA = kpair<J>(tA, lane), pB = kpair<J>(tB, lane);
                const bool up = (lane & kbit<J>()) != 0;   // the lower half's rows come first
                const double nA = eA * pA.lo, nB = __builtin_fma(eA, pB.lo, eB);
                eA = up ? nA : eA;
                eB = up ? nB : eB;
                if constexpr (J < 2) {
                    tA = pA.hi * pA.lo;
                    tB = __builtin_fma(pA.hi, pB.lo, pB.hi);
                }
            });
            const double Nk = __builtin_fma(eA, n0, eB);
            Nn = __builtin_fma(A, Nk, B);
            dd = __builtin_fma(b_ * b_, Nk, E);
        } else {
            // N_{k+1} = n0 + the inclusive sum of B over the rows up to k
            double incl = c_ * __builtin_fma(2.0, zf, cq1), tot = incl;
            dd = c_ * cq1;
            static_for<3>([&](auto jc) {
                constexpr int J = decltype(jc)::value;
                const PairD p = kpair<J>(tot, lane);
                incl = (lane & kbit<J>()) ? p.lo + incl : incl;
                if constexpr (J < 2) tot = p.lo + p.hi;
            });
            Nn = n0 + incl;
        }
        // one lane per row (l & 7 == 0) decides it; rows >= kk carry no step and never pass
        const bool pass = ((lane & 7) == 0) & live & (dd < tol2 * (Nn > 1.0 ? Nn : 1.0));   // branch-free
        const double nb = readlane_d(Nn, row_lane64(kB - 1));   // rows >= kk are identities
        nsq_out = nb > 0.0 ? nb : 0.0;
        return __builtin_amdgcn_ballot_w64(pass);
    };
    double wsave[CONV ? EH : 1];   // CONV: W at the block start (a pass restores it)
    // One block of kk rows (kB unless TAIL), rows in registers.
    auto block = [&](auto tail_c, int64_t b, int kk) __attribute__((always_inline)) -> bool {
        constexpr bool TAIL = decltype(tail_c)::value;
        const int64_t t0 = b * kB;
        // this lane's row: label and stepSize/sqrt(j)
        const f64x2 meta = *reinterpret_cast<const f64x2*>(
            meta_ring + ms * kMetaBlockBytes + ((int)(b & 1) * kB + krow) * 16);
        // the rows are in registers (the Gram and meta slots are reused only after the next
        // block is handed back): free the ring slots (the loader also waits for the Gram)
        __hip_atomic_store(my_consumed, (unsigned)(t0 + kk), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        // flags this block tests, read now so that their LDS round trip lands under the dots
        unsigned gpre = __hip_atomic_load(&ghdr->gdone[FS ? 0 : (b & 1)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if constexpr (FS) {
            const unsigned g1 = __hip_atomic_load(&ghdr->gdone[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            gpre = g1 < gpre ? g1 : gpre;
        }
        const unsigned rpre = __hip_atomic_load(&hdr->ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        PSGD_STAMP(const uint64_t st_a = __builtin_amdgcn_s_memtime();)
        // p_k = x_k . W over this wave's features
        double pk[kB];
#pragma unroll
        for (int k = 0; k < kB; ++k) {
            double a = 0.0;
#pragma unroll
            for (int u = 0; u < NVH; ++u) {
                double xv[VEC];
                xrow(k, u, xv);
#pragma unroll
                for (int q = 0; q < VEC; ++q) a = __builtin_fma(xv[q], w[u * VEC + q], a);
            }
            pk[k] = a;
        }
        const double yv = meta.x, sv = meta.y;
        const double nsv = -sv;
        const double alpha = 1.0 - sv * lam;      // SquaredL2 shrink of this lane's row (UPD:169)
        double z = reduce8d(pk, lane);
        if constexpr (H == 2) {
            // publish this wave's partial of every row (one lane per row), then the block count
            double* xs = xchg + ((int)(b & 1) * 2 + h) * kB;
            if (loss_lane) xs[krow] = z;
            asm volatile("s_waitcnt lgkmcnt(0)" : : : "memory");
            __hip_atomic_store(&xhdr->xdone[h], (unsigned)(b + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        PSGD_STAMP(const uint64_t st_b = __builtin_amdgcn_s_memtime(); st_p += st_b - st_a;)
        // the block's Gram triangle (Gram wave b&1 publishes its blocks in order; FS: both halves)
        {
            const unsigned need = FS ? (unsigned)b + 1 : (unsigned)(b >> 1) + 1;
            unsigned* gd = &ghdr->gdone[FS ? 0 : (b & 1)];
            auto gdone_now = [&]() __attribute__((always_inline)) -> unsigned {
                unsigned g = __hip_atomic_load(gd, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                if constexpr (FS) {
                    const unsigned g1 = __hip_atomic_load(&ghdr->gdone[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    g = g1 < g ? g1 : g;
                }
                return g;
            };
            if (gpre < need) {
                const uint64_t tw = __builtin_amdgcn_s_memrealtime();
                while (gdone_now() < need) {
                    if (__builtin_amdgcn_s_memrealtime() - tw > kWatchdogTicks) {
                        __hip_atomic_fetch_or(L.watchdog, 8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store(&hdr->stop, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        return false;
                    }
                }
            }
        }
        PSGD_STAMP(const uint64_t st_g = __builtin_amdgcn_s_memtime(); st_gr += st_g - st_b;)
        const double* grow = gring + gs * GSL + krow * kB;
        double G[kB];
#pragma unroll
        for (int q = 0; q < kB / 2; ++q) {
            const f64x2 g2 = *reinterpret_cast<const f64x2*>(grow + 2 * q);
            G[2 * q] = g2.x;
            G[2 * q + 1] = g2.y;
            if constexpr (FS) {   // the second Gram wave's half of the features
                const f64x2 h2 = *reinterpret_cast<const f64x2*>(grow + GSZ + 2 * q);
                G[2 * q] += h2.x;
                G[2 * q + 1] += h2.y;
            }
        }
        double q = 0.0;   // CONV: the squared norm of this lane's row
        if constexpr (CONV) {
            q = gring[gs * GSL + kB * kB + krow];
            if constexpr (FS) q += gring[gs * GSL + GSZ + kB * kB + krow];
        }
        if constexpr (H == 2 && (PSGD_B64_EXP & 2)) {
            z = z + z;
        } else if constexpr (H == 2) {
            // the other chain wave's partial of this lane's row: z = p0 + p1 in both waves
            const unsigned need = (unsigned)(b + 1);
            unsigned* xo = &xhdr->xdone[h ^ 1];
            if (__hip_atomic_load(xo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < need) {
                const uint64_t tw = __builtin_amdgcn_s_memrealtime();
                for (;;) {
                    if (__hip_atomic_load(xo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= need) break;
                    if (__hip_atomic_load(&hdr->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
                        if (__hip_atomic_load(xo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= need) break;
                        return false;
                    }
                    if (__builtin_amdgcn_s_memrealtime() - tw > kWatchdogTicks) {
                        __hip_atomic_fetch_or(L.watchdog, 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store(&hdr->stop, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        return false;
                    }
                }
            }
            asm volatile("" : : : "memory");   // the partial is read after its count
            const double other = xchg[((int)(b & 1) * 2 + (h ^ 1)) * kB + krow];
            z = h == 0 ? z + other : other + z;
        }
        if constexpr (PREF && !TAIL) {
            // the next full block's rows, if they have landed (the count read at this block's
            // start), into xraw: their LDS round trip runs under the recurrence and the test.
            // After the exchange's read (LDS returns in order: issued earlier, they would delay
            // it); the memory clobber keeps the compiler from hoisting them above it or above
            // the count they follow (LDS executes one wave's operations in order)
            asm volatile("" : "+v"(z) : : "memory");
            const unsigned rr = rpre > ready ? rpre : ready;
            pre = b + 1 < nfull && (int64_t)rr >= (b + 2) * kB;
            if (pre) issue_rows(ring + (rs + kB == R ? 0 : rs + kB) * ROW_BYTES);
        }
        PSGD_STAMP(const uint64_t st_xe = __builtin_amdgcn_s_memtime(); st_x += st_xe - st_g;)

        // the scalar recurrence: c_i from z_i, then every later row's dot moves by c_i G[k][i]
        // (SquaredL2 also shrinks the finished rows' z: zf keeps z_k for the loss)
        double c[kB], al[kB];
        double zf = z;
        // W <- a_i W + c_i x_i for row i (a tail block's missing rows are zero with c_i = 0,
        // a_i = 1: they leave W as it is)
        auto update_row = [&](int i) __attribute__((always_inline)) {
#pragma unroll
            for (int u = 0; u < NVH; ++u) {
                double xv[VEC];
                xrow(i, u, xv);
#pragma unroll
                for (int q = 0; q < VEC; ++q) {
                    const int e = u * VEC + q;
                    if constexpr (UPD == U_SQUARED_L2) w[e] = __builtin_fma(c[i], xv[q], w[e] * al[i]);
                    else w[e] = __builtin_fma(c[i], xv[q], w[e]);
                }
            }
        };
        bool brk = false;   // CONV: a row of this block passed isConverged
        int keff = kk;      // the rows taken
        // CONV: this lane's row's coefficient (lane row_lane64(k) computes c_k at step k), and W
        // at the block start (the updates run interleaved with the recurrence, before the block's
        // break test; a break -- once per chain -- restores W and replays the rows it takes)
        double ck = 0.0;
        if constexpr (CONV && PSGD_B64_INTERLEAVE) {
#pragma unroll
            for (int e = 0; e < EH; ++e) wsave[e] = w[e];
        }
#pragma unroll
        for (int i = 0; i < kB; ++i) {
            const double cv = coef64<GRAD>(z, yv, nsv);
            c[i] = readlane_d(cv, row_lane64(i));
            if constexpr (TAIL) c[i] = i < kk ? c[i] : 0.0;
            // (Logistic: this lane's coefficient as computed at its row's step; the cheap
            // multipliers are recomputed once after the recurrence from the same z)
            if constexpr (CONV && GRAD == G_LOGISTIC) ck = krow == i ? cv : ck;
            if constexpr (UPD == U_SQUARED_L2) {
                al[i] = readlane_d(alpha, row_lane64(i));
                if constexpr (TAIL) al[i] = i < kk ? al[i] : 1.0;
            }
            if constexpr (UPD == U_SQUARED_L2) {
                if (krow == i) zf = z;
                if (i + 1 < kB) z = __builtin_fma(c[i], G[i], al[i] * z);
            } else if constexpr (PSGD_B64_EXP & 1) {
                if (i + 1 < kB) zf = __builtin_fma(c[i], G[i], zf);
            } else {
                if (i + 1 < kB) z = __builtin_fma(c[i], G[i], z);
            }
            // row i's update is independent of the next coefficient's dependent chain: issued
            // here, it fills that chain's latency (PSGD_B64_INTERLEAVE=0: after the recurrence;
            // pinning each row's update before the next step with an empty asm measured no gain,
            // r05: c3 Logistic f32 rows 488 -> 492 cycles per row, c2 LeastSquares 239 -> 242)
            if constexpr (PSGD_B64_INTERLEAVE) update_row(i);
        }
        if constexpr (UPD != U_SQUARED_L2 && !(PSGD_B64_EXP & 1)) zf = z;
        // (a lane's z stops moving after its row's step: G[k][i] = 0 for i >= k; SquaredL2's zf
        // keeps it through the later rows' shrinks)
        if constexpr (CONV && GRAD != G_LOGISTIC) ck = coef64<GRAD>(zf, yv, nsv);
        if constexpr (CONV) {
            // isConverged for the block's rows at once (conv_test)
            const bool live = !TAIL || krow < kk;
            const double c_ = live ? ck : 0.0;
            const double a_ = (UPD == U_SQUARED_L2 && live) ? alpha : 1.0, b_ = sv * lam;
            double nb;
            const unsigned long long m = conv_test(c_, zf, q, a_, b_, live, nsq, nb);
            if constexpr (PSGD_B64_INTERLEAVE) {
                // the interleaved updates stay ahead of the test (the compiler would otherwise
                // sink them into the no-break branch, off the recurrence they are there to fill)
#pragma unroll
                for (int e = 0; e < EH; ++e) asm volatile("" : "+v"(w[e]));
            }
            if (m != 0ull) {   // a row passed: the first one ends the chain (once per chain)
                const int kstar = __builtin_ctz(ballot_rows(m));   // the first passing row
                brk = true;
                keff = kstar + 1;
                if constexpr (PSGD_B64_INTERLEAVE) {
#pragma unroll
                    for (int e = 0; e < EH; ++e) w[e] = wsave[e];
#pragma unroll
                    for (int i = 0; i < kB; ++i)
                        if (i <= kstar) update_row(i);
                }
            } else {
                nsq = nb;
            }
        }
        if (lead) {
            if constexpr (LOSS_EXT) {
                if (loss_lane && ((!TAIL && !CONV) || krow < keff)) zout[t0 + krow] = zf;
            } else {
                const double l = row_loss64<GRAD>(zf, yv);
                if (loss_lane && ((!TAIL && !CONV) || krow < keff)) loss_sum += l;
            }
        }
        count += keff;
        if constexpr (CONV) conv_stop = brk;
        if (rpre > ready) ready = rpre;
        PSGD_STAMP(const uint64_t st_c = __builtin_amdgcn_s_memtime(); st_rec += st_c - st_xe;)

        // W <- a_i W + c_i x_i, i = 0..kB-1, in sample order
        if constexpr (!PSGD_B64_INTERLEAVE) {
#pragma unroll
            for (int i = 0; i < kB; ++i)
                if (i < keff) update_row(i);
        }
        PSGD_STAMP(st_upd += __builtin_amdgcn_s_memtime() - st_c;)
        rs += kB;
        if (rs == R) rs = 0;
        if (++gs == GS) gs = 0;
        if ((b & 1) && ++ms == MB) ms = 0;
        return true;
    };

    using Full = std::integral_constant<bool, false>;
    using Tail = std::integral_constant<bool, true>;
    bool ok = true;
    for (int64_t b = 0; ok && !conv_stop && b < nfull; ++b) {
        if (!pre) {   // (PREF: the previous block issued these reads)
            PSGD_STAMP(const uint64_t st_w = __builtin_amdgcn_s_memtime();)
            ok = wait_rows((b + 1) * kB);
            PSGD_STAMP(st_rd += __builtin_amdgcn_s_memtime() - st_w;)
            if (!ok) break;
            issue_rows(ring + rs * ROW_BYTES);
        }
        finish_rows(Full{}, kB);
        ok = block(Full{}, b, kB);
    }
    if (ok && !conv_stop && ntail > 0 && wait_rows(n)) {
        issue_rows(ring + rs * ROW_BYTES);
        finish_rows(Tail{}, ntail);
        block(Tail{}, nfull, ntail);
    }
    // a wave that stopped early leaves the others blocked on it: wake them
    __hip_atomic_store(&hdr->stop, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    PSGD_STAMP(if (L.stamps && lead && lane == 0) {
        unsigned long long* o = L.stamps + (size_t)chain * 16;
        o[0] = __builtin_amdgcn_s_memtime() - st_begin; o[1] = st_rd; o[2] = st_gr;
        o[3] = st_p; o[7] = st_x; o[12 + 2] = st_rec; o[12 + 3] = st_upd;
    } else if (L.stamps && H == 2 && lane == 0) {
        unsigned long long* o = L.stamps + (size_t)chain * 16;
        o[10] = st_x; o[11] = st_p;   // the second chain wave's exchange wait and dots
    })
    loss_sum = wave_sum(loss_sum);   // the 8 loss lanes' partials

    // regVal of the chain's last update (PSGD.scala:257; 0.0 if no sample, :247)
    double rv = 0.0;
    if constexpr (UPD == U_SQUARED_L2) {
        double acc = 0.0;
#pragma unroll
        for (int e = 0; e < EH; ++e) acc += w[e] * w[e];
        acc = wave_sum(acc);
        if constexpr (H == 2) {
            // ||w||^2 = n0 + n1 from the two chain waves' features
            if (lane == 0) xchg[2 * 2 * kB + h] = acc;
            asm volatile("s_waitcnt lgkmcnt(0)" : : : "memory");
            __hip_atomic_store(&xhdr->fin[h], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (lead) {
                const uint64_t tw = __builtin_amdgcn_s_memrealtime();
                while (!__hip_atomic_load(&xhdr->fin[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
                    if (__builtin_amdgcn_s_memrealtime() - tw > kWatchdogTicks) {
                        __hip_atomic_fetch_or(L.watchdog, 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                }
                asm volatile("" : : : "memory");
                acc = acc + xchg[2 * 2 * kB + 1];
            }
        }
        if (count > 0) {
            const double nrm = sqrt(acc);
            rv = 0.5 * kp.reg * nrm * nrm;
        }
    }

    double* wo = L.w_out + (int64_t)chain * d;
#pragma unroll
    for (int u = 0; u < NVH; ++u) {
        const int base = ((h * NVH + u) * 64 + lane) * VEC;
#pragma unroll
        for (int k = 0; k < VEC; ++k)
            if (base + k < d) wo[base + k] = w[u * VEC + k];
    }
    if (lead && lane == 0) {
        L.rv[chain] = rv;
        if constexpr (!LOSS_EXT) L.loss[chain] = loss_sum;
        L.cnt[chain] = count;
        L.cnt_d[chain] = double(count);
    }
}

// ------------------------------------------------------------------------------------------
// Launcher.
// ------------------------------------------------------------------------------------------
template <typename S, int GRAD, int UPD, int NV, int H, bool CONV>
static int launch_block64(const ChainLaunch& L, const KParams& kp, bool full, size_t lds, hipStream_t st) {
    constexpr int ROW = NV * 1024;
    const size_t budget = lds > 0 ? lds : (size_t)64 * 1024;
    const int D = loader_depth<NV>();
    auto bytes_for = [&](int r) {
        const int mb = (r + kMetaRows - 1) / kMetaRows + 2;
        const int gs = r / kB + 1;
        return kFixed64 + (size_t)mb * kMetaBlockBytes +
               (size_t)gs * gram_slot64<CONV>() * 8 * (gram_fsplit64<NV>() ? 2 : 1) + (size_t)r * ROW;
    };
    int R = (int)((budget - kFixed64) / ROW) / kB * kB;
    while (R > 0 && bytes_for(R) > budget) R -= kB;
    if (R < 2 * kB) return (int)hipErrorInvalidValue;   // LDS budget too small for this d
    const int MB = (R + kMetaRows - 1) / kMetaRows + 2;
    const int GS = R / kB + 1;
    RingGeom g{R, MB, D, GS};
    const size_t bytes = bytes_for(R);
    const dim3 threads(64 * (3 + H));
    if (full) {
        auto k = chain_block64<S, GRAD, UPD, NV, true, H, CONV>;
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
        hipLaunchKernelGGL(k, dim3(kp.n_chains), threads, bytes, st, L, kp, g);
    } else {
        auto k = chain_block64<S, GRAD, UPD, NV, false, H, CONV>;
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
        hipLaunchKernelGGL(k, dim3(kp.n_chains), threads, bytes, st, L, kp, g);
    }
    if constexpr (GRAD == G_LOGISTIC) {
        const int e = launch_logistic_loss64(L, kp.n_chains, st);
        if (e) return e;
    }
    return (int)hipGetLastError();
}

#ifndef PSGD_NO_DISPATCH
// Two chain waves (H = 2) from NV = 2 on; PSGD_B64_WAVES=1 keeps one where its share of a
// block fits the registers (NV <= 4; A/B measurements). Variant 700 + 40 (per-sample break) +
// 10 (H - 1) + NV.
template <typename S, int GRAD, int UPD, bool CONV>
static int block64_nv(const ChainLaunch& L, const KParams& kp, int64_t min_ld, int64_t max_ld,
                      size_t lds, hipStream_t st, int* variant) {
    constexpr int VEC = 16 / sizeof(S);
    static const bool one_wave = [] {
        const char* e = getenv("PSGD_B64_WAVES");
        return e && atoi(e) == 1;
    }();
    int nv = 1;
    while (nv * 64 * VEC < max_ld) nv *= 2;
    const bool full = min_ld >= (int64_t)nv * 64 * VEC;
    const int H = (nv >= 2 && !(one_wave && nv <= 4)) ? 2 : 1;
    if (variant) *variant = 700 + (CONV ? 40 : 0) + 10 * (H - 1) + nv;
    if (H == 1) {
        switch (nv) {
        case 1: return launch_block64<S, GRAD, UPD, 1, 1, CONV>(L, kp, full, lds, st);
        case 2: return launch_block64<S, GRAD, UPD, 2, 1, CONV>(L, kp, full, lds, st);
        case 4: return launch_block64<S, GRAD, UPD, 4, 1, CONV>(L, kp, full, lds, st);
        default: return -3;
        }
    }
    switch (nv) {
    case 2: return launch_block64<S, GRAD, UPD, 2, 2, CONV>(L, kp, full, lds, st);
    case 4: return launch_block64<S, GRAD, UPD, 4, 2, CONV>(L, kp, full, lds, st);
    case 8: return launch_block64<S, GRAD, UPD, 8, 2, CONV>(L, kp, full, lds, st);
    default: return -3;
    }
}

template <typename S, int GRAD>
static int block64_upd(const ChainLaunch& L, const KParams& kp, int upd, int64_t min_ld,
                       int64_t max_ld, size_t lds, hipStream_t st, int* variant) {
    // the per-sample break (tol > 0, PSGD.scala:262) is a template instance of its own
    const bool conv = kp.tol > 0.0;
    if (upd == U_SIMPLE)
        return conv ? block64_nv<S, GRAD, U_SIMPLE, true>(L, kp, min_ld, max_ld, lds, st, variant)
                    : block64_nv<S, GRAD, U_SIMPLE, false>(L, kp, min_ld, max_ld, lds, st, variant);
    if (upd == U_SQUARED_L2)
        return conv ? block64_nv<S, GRAD, U_SQUARED_L2, true>(L, kp, min_ld, max_ld, lds, st, variant)
                    : block64_nv<S, GRAD, U_SQUARED_L2, false>(L, kp, min_ld, max_ld, lds, st, variant);
    return -3;
}

template <typename S>
static int block64_grad(const ChainLaunch& L, const KParams& kp, int grad, int upd, int64_t min_ld,
                        int64_t max_ld, size_t lds, hipStream_t st, int* variant) {
    switch (grad) {
    case G_LOGISTIC: return block64_upd<S, G_LOGISTIC>(L, kp, upd, min_ld, max_ld, lds, st, variant);
    case G_LEAST_SQUARES: return block64_upd<S, G_LEAST_SQUARES>(L, kp, upd, min_ld, max_ld, lds, st, variant);
    case G_HINGE: return block64_upd<S, G_HINGE>(L, kp, upd, min_ld, max_ld, lds, st, variant);
    default: return -3;
    }
}

bool block64_path_applies(int layout, int compute, int updater, bool check_conv, int storage,
                          int64_t max_ld) {
    // any tol: the per-sample break runs in the block recurrence (CONV instances, kp.tol > 0);
    // PSGD_B64_CONV=0 sends tol > 0 to the per-sample kernels instead (tests of chain_split's
    // break path, A/B measurements; read at every launch)
    if (check_conv) {
        const char* e = getenv("PSGD_B64_CONV");
        if (e && e[0] == '0') return false;
    }
    const int vec = storage == 1 ? 4 : 2;
    return layout == kDense && compute == 0 &&
           (updater == U_SIMPLE || updater == U_SQUARED_L2) && max_ld <= 8 * 64 * vec;
}

int launch_block64_chains(const ChainLaunch& L, const KParams& kp, int storage, int gradient,
                          int updater, int64_t min_ld, int64_t max_ld, int lds_spread,
                          hipStream_t stream, int* kernel_variant) {
    if (kp.n_chains <= 0) return 0;
    if (gradient == G_LOGISTIC && !L.zbuf64) return (int)hipErrorInvalidValue;
    const size_t lds = (size_t)(lds_spread > 0 ? lds_spread : 0);
    if (storage == 1)
        return block64_grad<float>(L, kp, gradient, updater, min_ld, max_ld, lds, stream, kernel_variant);
    return block64_grad<double>(L, kp, gradient, updater, min_ld, max_ld, lds, stream, kernel_variant);
}

#endif  // PSGD_NO_DISPATCH

}  // namespace psgd
