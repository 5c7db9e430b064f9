// NOT BUILT: a measured negative result (DESIGN.md §3, 342 vs 573 M samples/s for
// chain_sparse_lds at c4), moved out of libpsgd.so in round 3. It compiles only against the
// round-2 tree (git history: spark-parallelized-sgd_amd/csrc/psgd_sparse_gram.hip).
// psgd_sparse_gram.hip -- the fp32 CSR chain as a batched scalar recurrence over sparse Gram
// terms (gfx950).
//
// Reference: ParallelizedSGD.scala:243-270 (the chain: Gradient.compute reads the weights at :254,
// SGDUpdater.compute writes them at :255-256), [ext] MLlib 1.6.1 Gradient.scala on SparseVector
// rows (the gradient is mult * x, non-zero only at the row's indices), SGDUpdater.scala:86-98
// (Simple) and :163-181 (SquaredL2, alpha-scaled lazy form as in psgd_sparse.hip).
//
// chain_sparse_lds keeps the per-sample weight read -> dot -> coefficient -> weight write on one
// wave: every sample waits for an LDS (or L2) round trip and a wave reduction (~1,000 cycles per
// row at rcv1 shape). Here the weights are read 8..15 rows late and the missing updates are
// added back as scalars. Over batches of 8 rows, for row t of batch b,
//
//     y_t = x_t . v_snap(b) + sum_{r in batch b-1} c_r G[t][r] + sum_{r < t in batch b} c_r G[t][r]
//
// where v_snap(b) holds the updates of batches <= b-2 and G[t][r] = x_t . x_r, non-zero only when
// the rows share features (~0.2 shared features per row pair at rcv1 density). SquaredL2 runs in
// v-space (w = alpha v): z_t = alpha_t y_t, c'_t = c_t / alpha_{t+1}. The only sequential work is
// the scalar recurrence (one FMA, a readlane and the gradient multiplier per row); the dots, the
// Gram terms and the weight updates are batched on other waves.
//
// One workgroup = one chain = one CU, four waves (one per SIMD):
//   wave 0 (chain)   per batch: P and G from LDS, the cross terms with the previous batch's c, the
//                    8-step recurrence (lane i holds row i), c of the batch into LDS;
//   wave 1 (loader)  CSR entries into a 32-row LDS slot ring, labels / steps / nnz into a meta ring;
//   wave 2 (gram)    per batch: every entry is linked into a bucket table by an LDS exchange
//                    (bucket = hash(feature); the displaced tag is the entry's link) and tests a
//                    presence bitmap of the window (batches b-1, b); the few entries whose feature
//                    occurs elsewhere in the window walk their links back through it from an LDS
//                    work queue and add x_t x_r into G[t][r] for the same feature (ds_add_f32);
//   wave 3 (apply)   per batch b: the weight updates of batch b (head: ds_add_f32 into LDS; tail:
//                    buffer_atomic_add_f32 into the chain's fp32 vector), then the dots of batch
//                    b+2 against the weights after batch b (head from LDS, tail gathered from L2)
//                    with one transposed 8-row wave reduction.
// Features [0, K) are in LDS (the head, K up to ~25k), [K, d) in the chain's fp32 vector L.wf32
// (the tail; initialised by wf32_init_kernel, folded by launch_fold_f32 with the head written back).
// Tests: tests/test_sparse_gram_model.py restates this schedule (walk rules included) in numpy
// against the sequential chain; tests/test_gpu_sparse.py runs this kernel against the oracle.
// No MFMA: the work per sample is a ~100-long gather-dot and scatter.
#include "psgd_device.h"

#include <stddef.h>
#include <stdlib.h>

namespace psgd {

namespace {

constexpr int GB = 8;                 // rows per batch
constexpr int GCAP = 128;             // entries per row (two per lane)
constexpr int GSR = 32;               // row slots (4 batches)
constexpr int GPR = 16;               // link ring rows (the Gram window: 2 batches)
constexpr int GMR = 128;              // meta ring rows
constexpr int GRB = 4;                // P / C / G ring batches
constexpr int HBITS = 12;
constexpr int HSIZE = 1 << HBITS;     // bucket table entries
constexpr uint32_t kRowMask = 0xFFFFFF;
constexpr uint32_t kTagValid = 0x80000000u;
constexpr int kMaxHops = GPR * GCAP;  // a walk visits every window entry at most once
constexpr uint32_t kNoAccessG = 0x80000000u;   // buffer offset past any chain vector
constexpr int kStampLog = 14;
constexpr int kStampN = 1 << kStampLog;   // presence stamps (hashed features)
constexpr int kQCap = 1024;           // gram work queue items (a batch's entries)

struct GHeader {
    unsigned loaded;    // rows staged (loader)
    unsigned gram;      // batches whose G is complete (gram wave)
    unsigned pdone;     // batches whose P is written (apply wave)
    unsigned gathered;  // batches whose rows the apply wave holds in registers
    unsigned cdone;     // batches whose coefficients are written (chain)
    unsigned stop;
    unsigned pad[2];
};
struct GMeta {
    float y[GMR];
    float s[GMR];        // stepSize / sqrt(j), rounded (fp32 compute)
    double s64[GMR];     // the same in f64 (SquaredL2's alpha)
    int32_t nnz[GMR];
};
struct GSlot {
    int32_t col[GCAP];   // feature index (0 past the row's end)
    float val[GCAP];     // x_j (0 past the row's end)
};
struct GFixed {
    GHeader hdr;
    float dread[64];              // read target of lanes without a head entry (stays 0)
    float dwrite[64];             // write / exchange target of lanes without one (junk)
    GMeta meta;
    float P[GRB][GB];             // the batch's dots against the snapshot
    float C[GRB][GB];             // the batch's coefficients (v-space)
    float G[GRB][GB][2 * GB];     // G[t][0..7]: rows of batch b-1; G[t][8..15]: batch b
    uint32_t link[GPR][GCAP];     // the tag each entry's insertion displaced
    uint32_t bucket[HSIZE];       // latest tag per bucket (0 = empty)
    uint8_t stamp[kStampN];       // presence: batch number (mod 256) of the latest entry per hashed feature
    uint64_t queue[kQCap];        // gram work items: {link, row slot / entry / batch row}
    GSlot slot[GSR];
};
static_assert(sizeof(GFixed) % 16 == 0 && offsetof(GFixed, G) % 16 == 0 && offsetof(GFixed, slot) % 16 == 0 &&
                  offsetof(GFixed, stamp) % 8 == 0 && offsetof(GFixed, queue) % 8 == 0,
              "LDS alignment");
constexpr int64_t kGLdsCap = 160 * 1024;

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ i32x4 rsrc_of(const float* base, uint32_t bytes) {
    const uint64_t a = (uint64_t)base;
    return i32x4{__builtin_amdgcn_readfirstlane((int32_t)(uint32_t)a),
                 __builtin_amdgcn_readfirstlane((int32_t)((a >> 32) & 0xFFFF)),
                 __builtin_amdgcn_readfirstlane((int32_t)bytes), 0x00020000};
}
// Tail gathers and updates: buffer instructions with a 32-bit byte offset; lanes without a tail
// entry pass an out-of-range offset, which the bounds check drops (loads return 0).
__device__ __forceinline__ float gload_sc1(i32x4 rsrc, uint32_t off) {
    float v;
    asm volatile("buffer_load_dword %0, %1, %2, 0 offen sc1" : "=v"(v) : "v"(off), "s"(rsrc) : "memory");
    return v;
}
__device__ __forceinline__ void gatomic_add(i32x4 rsrc, uint32_t off, float v) {
    asm volatile("buffer_atomic_add_f32 %0, %1, %2, 0 offen" : : "v"(v), "v"(off), "s"(rsrc) : "memory");
}

__device__ __forceinline__ uint32_t hash_of(int32_t c) { return ((uint32_t)c * 2654435761u) >> (32 - HBITS); }

// transposed 8-value reduction: lane l ends with the total of value k(l) = l5 | l4<<1 | l3<<2
__device__ __forceinline__ float gpair32(float x, float y) {
    auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(y), false, false);
    return __uint_as_float(p[0]) + __uint_as_float(p[1]);
}
__device__ __forceinline__ float gpair16(float x, float y) {
    auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(y), false, false);
    return __uint_as_float(p[0]) + __uint_as_float(p[1]);
}
__device__ __forceinline__ float greduce8(const float (&v)[8], int lane) {
    const float a0 = gpair32(v[0], v[1]), a1 = gpair32(v[2], v[3]);
    const float a2 = gpair32(v[4], v[5]), a3 = gpair32(v[6], v[7]);
    const float b0 = gpair16(a0, a1), b1 = gpair16(a2, a3);
    const bool hi = (lane & 8) != 0;
    float r = (hi ? b1 : b0) + dpp_mov<0x140>(hi ? b0 : b1);   // row_mirror: partner l^15
    r = r + dpp_mov<0xB1>(r);                                   // l^1
    r = r + dpp_mov<0x4E>(r);                                   // l^2
    r = r + dpp_mov<0x141>(r);                                  // row_half_mirror: l^7
    return r;
}

}  // namespace

template <typename S, int GRAD, int UPD, bool TAIL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void chain_sparse_gram(
    ChainLaunch L, KParams kp, int K) {
    constexpr bool L2 = UPD == U_SQUARED_L2;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    GFixed* F = reinterpret_cast<GFixed*>(smem);
    GHeader* hdr = &F->hdr;
    float* lds = reinterpret_cast<float*>(smem);                      // dword views
    uint32_t* ldsu = reinterpret_cast<uint32_t*>(smem);
    constexpr unsigned kW = (unsigned)(sizeof(GFixed) / 4);          // dword of head weight 0
    constexpr unsigned kDread = (unsigned)(offsetof(GFixed, dread) / 4);
    constexpr unsigned kDwrite = (unsigned)(offsetof(GFixed, dwrite) / 4);
    constexpr unsigned kSlot = (unsigned)(offsetof(GFixed, slot) / 4);
    constexpr unsigned kLink = (unsigned)(offsetof(GFixed, link) / 4);
    constexpr unsigned kBucket = (unsigned)(offsetof(GFixed, bucket) / 4);
    constexpr unsigned kG = (unsigned)(offsetof(GFixed, G) / 4);
    constexpr unsigned kQueue = (unsigned)(offsetof(GFixed, queue) / 4);
    float* W = lds + kW;

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int chain = blockIdx.x;
    const ChainDesc dsc = L.descs[chain];
    const int d = kp.d;
    const int64_t n = dsc.n_rows;
    const int64_t nb = (n + GB - 1) / GB;
    const int64_t n_fill = nb * GB;          // rows past n are null: no entries, label and step 0
    float* V = L.wf32 + (int64_t)chain * L.wstride;

    for (int i = threadIdx.x; i < HSIZE; i += blockDim.x) F->bucket[i] = 0u;
    for (int i = threadIdx.x; i < kStampN / 4; i += blockDim.x) reinterpret_cast<uint32_t*>(F->stamp)[i] = 0x80808080u;
    for (int i = threadIdx.x; i < K; i += blockDim.x) W[i] = float(as_global(L.w_in)[i]);
    if (threadIdx.x < 64) {
        F->dread[threadIdx.x] = 0.0f;
        F->dwrite[threadIdx.x] = 0.0f;
    }
    if (threadIdx.x < 8) reinterpret_cast<unsigned*>(hdr)[threadIdx.x] = 0;
    __syncthreads();

    uint64_t st_wait = 0;                      // diagnostic (PSGD_STAMPS): cycles spent waiting
    uint64_t st_x[4] = {0, 0, 0, 0};           // diagnostic: per-wave sub-phase cycles / counts
    const bool stamps = L.stamps != nullptr;
    auto tick = [&]() __attribute__((always_inline)) -> uint64_t { return stamps ? __builtin_amdgcn_s_memtime() : 0; };
    const uint64_t st_begin = __builtin_amdgcn_s_memtime();
    // The flags live in LDS and are reached through an explicit address-space-3 view: a generic
    // pointer would compile to flat accesses, which count on vmcnt and make every poll and publish
    // wait for this wave's outstanding global loads and atomics.
    typedef __attribute__((address_space(3))) volatile unsigned lflag;
    lflag* FL = (lflag*)(smem);
    constexpr unsigned kLoaded = offsetof(GHeader, loaded) / 4, kGram = offsetof(GHeader, gram) / 4,
                       kPdone = offsetof(GHeader, pdone) / 4, kGathered = offsetof(GHeader, gathered) / 4,
                       kCdone = offsetof(GHeader, cdone) / 4, kStop = offsetof(GHeader, stop) / 4;
    auto wait_for = [&](unsigned& seen, unsigned flag, int64_t need, int code)
        __attribute__((always_inline)) -> bool {
        if ((int64_t)seen >= need) return true;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        const uint64_t c0 = __builtin_amdgcn_s_memtime();
        for (;;) {
            // flags and data are LDS, which one wave writes in program order
            seen = FL[flag];
            if ((int64_t)seen >= need) {
                __atomic_signal_fence(__ATOMIC_SEQ_CST);
                st_wait += __builtin_amdgcn_s_memtime() - c0;
                return true;
            }
            if (FL[kStop]) return false;
            if (__builtin_amdgcn_s_memrealtime() - t0 > kWatchdogTicks) {
                __hip_atomic_fetch_or(L.watchdog, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                FL[kStop] = 1u;
                return false;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    };
    auto publish = [&](unsigned flag, int64_t v) __attribute__((always_inline)) {
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        FL[flag] = (unsigned)v;
    };
    const i32x4 vrs = rsrc_of(V, (uint32_t)((int64_t)d * 4));   // the chain's vector [0, d)

    bool ok = true;                // chain wave: finished every batch
    double alpha = 1.0;            // SquaredL2: w = alpha v (chain wave)
    double loss_sum = 0.0;         // chain wave, lanes 0..7

    if (wave == 1) {
        // ---------------- loader: entries into slots, labels / steps / nnz into the meta ring ----
        const gptr<S> X = as_global(reinterpret_cast<const S*>(dsc.x));
        const gptr<int32_t> COL = as_global(dsc.col);
        const gptr<int64_t> RP = as_global(dsc.row_ptr);
        const gptr<double> Y = as_global(dsc.y);
        const gptr<double> STEPS = as_global(L.steps);
        const gptr<int32_t> RIDX = dsc.rows ? as_global(dsc.rows) : nullptr;
        unsigned gram = 0, gath = 0, cd = 0;
        const gptr<int32_t> dummy_i = as_global((const int32_t*)(V + d + lane));   // valid, unused
        const gptr<S> dummy_s = as_global((const S*)(V + d + 2 * lane));
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
        struct Group { int32_t ca[8], cb[8]; S xa[8], xb[8]; bool ia[8], ic[8]; };
        auto rl64 = [&](int64_t v, int i) __attribute__((always_inline)) -> int64_t {
            return (int64_t)(uint32_t)__builtin_amdgcn_readlane((int)(v & 0xffffffff), i) |
                   ((int64_t)__builtin_amdgcn_readlane((int)(v >> 32), i) << 32);
        };
        // entries of rows g + i0 .. g + i0 + 7: unconditional loads (masked-off entries read
        // valid dummy addresses), so the compiler counts them without branches
        auto load_group = [&](const Batch& bt, int i0, Group& Gr) __attribute__((always_inline)) {
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int64_t b = rl64(bt.rb, i0 + q), e = rl64(bt.re, i0 + q);
                const int64_t ka = b + lane, kc = b + 64 + lane;
                const bool ia = ka < e, ic = kc < e;
                Gr.ca[q] = *(ia ? &COL[ka] : dummy_i);
                const S xa = *(ia ? &X[ka] : dummy_s);
                Gr.cb[q] = *(ic ? &COL[kc] : dummy_i);
                const S xb = *(ic ? &X[kc] : dummy_s);
                Gr.xa[q] = ia ? xa : S(0);
                Gr.xb[q] = ic ? xb : S(0);
                Gr.ia[q] = ia;
                Gr.ic[q] = ic;
            }
        };
        // rows u0 .. u0 + 7 into their slots: the slot held row v = u - GSR, which the gram wave
        // reads until it has finished batch v/8 + 1 (the window) and the apply wave until it has
        // copied batch v/8
        auto stage_group = [&](int64_t u0, const Group& Gr) __attribute__((always_inline)) -> bool {
            if (u0 >= n_fill) return true;
            if (u0 >= GSR) {
                const int64_t vb = (u0 - GSR) / GB;
                if (!wait_for(gram, kGram, vb + 2, 16)) return false;
                if (!wait_for(gath, kGathered, vb + 1, 16)) return false;
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                GSlot& sl = F->slot[(u0 + q) & (GSR - 1)];
                sl.col[lane] = Gr.ia[q] ? Gr.ca[q] : 0;
                sl.col[lane + 64] = Gr.ic[q] ? Gr.cb[q] : 0;
                sl.val[lane] = float(Gr.xa[q]);
                sl.val[lane + 64] = float(Gr.xb[q]);
            }
            publish(kLoaded, u0 + 8);
            return true;
        };
        Batch cur = load_batch(0);
        Group GA, GB2;
        load_group(cur, 0, GA);
        for (int64_t g = 0; g < n_fill; g += 64) {
            const Batch nxt = load_batch(g + 64);
            // meta of rows g .. g + 63: their ring positions held rows g - 128 .. g - 65, which
            // the chain (their last reader) has finished with once it is past batch (g - 65) / 8
            if (g >= GMR && !wait_for(cd, kCdone, (g - 64) / GB, 16)) break;
            {
                const int m = (int)((g + lane) & (GMR - 1));
                F->meta.y[m] = float(cur.y);
                F->meta.s[m] = float(cur.s);
                F->meta.s64[m] = cur.s;
                F->meta.nnz[m] = (int32_t)(cur.re - cur.rb);
            }
            bool good = true;
            static_for<4>([&](auto kc) {
                constexpr int i0 = 16 * decltype(kc)::value;
                if (!good) return;
                load_group(cur, i0 + 8, GB2);
                good = stage_group(g + i0, GA);
                if constexpr (i0 + 16 < 64) load_group(cur, i0 + 16, GA);
                else load_group(nxt, 0, GA);
                if (good) good = stage_group(g + i0 + 8, GB2);
            });
            if (!good) break;
            cur = nxt;
        }
    } else if (wave == 2) {
        // ---------------- gram: link the batch's entries, walk the links, accumulate G ----------
        // Per batch b, rows in order: each entry tests the presence stamp of its (hashed) feature
        // -- the batch number, mod 256, of the feature's latest entry: present in the window if it
        // names batch b-1 or b (a stale or shared stamp only costs a walk) -- stamps it with b,
        // and links itself into its bucket by an exchange. Only an entry whose
        // feature is present elsewhere in the window and whose link points into the window walks:
        // it goes into an LDS work queue, which the wave drains 64 items per step (one hop each;
        // an item still inside the window goes back into the queue).
        unsigned loaded = 0, cd = 0;
        for (int64_t b = 0; b < nb; ++b) {
            if (!wait_for(loaded, kLoaded, GB * b + GB, 32)) break;
            // G[b % GRB] held batch b - GRB, which the chain has finished with
            if (b >= GRB && !wait_for(cd, kCdone, b - GRB + 1, 32)) break;
            const unsigned gbase = kG + (unsigned)(b & (GRB - 1)) * (GB * 2 * GB);
            lds[gbase + 2 * lane] = 0.0f;
            lds[gbase + 2 * lane + 1] = 0.0f;
            const uint32_t bs = (uint32_t)b & 255u, bp = (uint32_t)(b - 1) & 255u;
            typedef __attribute__((address_space(3))) volatile uint8_t lbyte;
            lbyte* SB = (lbyte*)(smem);
            uint32_t qt = 0;             // queue tail (items ever queued this batch)
            const uint64_t tA = tick();
            // the batch's columns and row lengths (one LDS round trip)
            int32_t cl[2 * GB];
            int nz[GB];
#pragma unroll
            for (int i = 0; i < GB; ++i) {
                const int64_t u = GB * b + i;
                const GSlot& sl = F->slot[u & (GSR - 1)];
                nz[i] = F->meta.nnz[u & (GMR - 1)];
                cl[2 * i] = sl.col[lane];
                cl[2 * i + 1] = sl.col[lane + 64];
            }
            uint32_t sv[2 * GB], lk[2 * GB];
            // issue, rows in order (one wave's LDS operations execute in program order): the
            // presence test (the feature's stamp names batch b-1 or b), the entry's own stamp, its
            // link; lanes without an entry use their dummy dwords
#pragma unroll
            for (int q = 0; q < 2 * GB; ++q) {
                const int i = q >> 1;
                const int e = lane + 64 * (q & 1);
                const int64_t u = GB * b + i;
                const bool on = e < nz[i];
                const int32_t c = cl[q];
                const uint32_t k = ((uint32_t)c * 2654435761u) >> (32 - kStampLog);
                const unsigned sb = on ? (unsigned)offsetof(GFixed, stamp) + k : 4 * (kDwrite + lane);
                sv[q] = SB[sb];
                SB[sb] = (uint8_t)bs;
                const uint32_t tag = kTagValid | (((uint32_t)u & kRowMask) << 7) | (uint32_t)e;
                lk[q] = __hip_atomic_exchange(ldsu + (on ? kBucket + hash_of(c) : kDwrite + lane), tag,
                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            // consume: links into the ring, walkers into the queue
#pragma unroll
            for (int q = 0; q < 2 * GB; ++q) {
                const int i = q >> 1;
                const int e = lane + 64 * (q & 1);
                const int64_t u = GB * b + i;
                const int wlim = i + (b > 0 ? GB : 0);
                const bool on = e < nz[i];
                const uint32_t l = on ? lk[q] : 0u;
                F->link[u & (GPR - 1)][e] = l;
                const bool pres = sv[q] == bs || sv[q] == bp;
                const bool act = on && pres && l != 0u && (int)(((uint32_t)u - (l >> 7)) & kRowMask) <= wlim;
                const uint64_t mk = __builtin_amdgcn_ballot_w64(act);
                if (mk) {
                    const uint32_t pos = qt + __builtin_amdgcn_mbcnt_hi((uint32_t)(mk >> 32),
                                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)mk, 0u));
                    if (act) {
                        const uint32_t me = ((uint32_t)i << 12) | ((uint32_t)(u & (GSR - 1)) << 7) | (uint32_t)e;
                        *reinterpret_cast<uint64_t*>(ldsu + kQueue + 2 * (pos & (kQCap - 1))) =
                            (uint64_t)l | ((uint64_t)me << 32);
                    }
                    qt += (uint32_t)__builtin_popcountll(mk);
                }
            }
            const uint64_t tB = tick();
            if (stamps) { st_x[0] += tB - tA; st_x[2] += qt; }
            // drain: one hop per item; a link to the same feature in an earlier row adds x_t x_r
            // to G[t][r]; an item whose next link stays inside the window (at non-decreasing
            // distance) is queued again
            uint32_t qh = 0;
            for (int it = 0; qh < qt && it < kMaxHops; ++it) {
                if (stamps) st_x[3] += 1;
                const uint32_t take = qt - qh < 64u ? qt - qh : 64u;
                const bool my = (uint32_t)lane < take;
                const uint64_t item = *reinterpret_cast<const uint64_t*>(
                    ldsu + (my ? kQueue + 2 * ((qh + lane) & (kQCap - 1)) : kDread + (lane & ~1)));
                qh += take;
                const uint32_t lk = (uint32_t)item, me = (uint32_t)(item >> 32);
                const int i = (int)(me >> 12);
                const uint32_t u = (uint32_t)(GB * b) + (uint32_t)i;
                const int dist = (int)((u - (lk >> 7)) & kRowMask);
                const uint32_t r = u - (uint32_t)dist, er = lk & 127u;
                const unsigned mine = kSlot + ((me >> 7) & (GSR - 1)) * (2 * GCAP) + (me & 127u);
                const unsigned other = kSlot + (r & (GSR - 1)) * (2 * GCAP) + er;
                const unsigned olink = kLink + (r & (GPR - 1)) * GCAP + er;
                const int32_t mc = (int32_t)ldsu[my ? mine : kDread + lane];
                const float mx = lds[my ? mine + GCAP : kDread + lane];
                const int32_t rc = (int32_t)ldsu[my ? other : kDread + lane];
                const float rx = lds[my ? other + GCAP : kDread + lane];
                const uint32_t nx = ldsu[my ? olink : kDread + lane];
                const bool match = my && dist > 0 && rc == mc;
                if (__builtin_amdgcn_ballot_w64(match)) {
                    if (match)
                        __hip_atomic_fetch_add(lds + gbase + i * (2 * GB) + (i + GB - dist), mx * rx,
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                const int wlim = i + (b > 0 ? GB : 0);
                const int nd = (int)((u - (nx >> 7)) & kRowMask);
                const bool act = my && nx != 0u && nd <= wlim && nd >= dist;
                const uint64_t mk = __builtin_amdgcn_ballot_w64(act);
                if (mk) {
                    const uint32_t pos = qt + __builtin_amdgcn_mbcnt_hi((uint32_t)(mk >> 32),
                                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)mk, 0u));
                    if (act)
                        *reinterpret_cast<uint64_t*>(ldsu + kQueue + 2 * (pos & (kQCap - 1))) =
                            (uint64_t)nx | ((uint64_t)me << 32);
                    qt += (uint32_t)__builtin_popcountll(mk);
                }
            }
            if (stamps) st_x[1] += tick() - tB;
            publish(kGram, b + 1);
        }
    } else if (wave == 3) {
        // ---------------- apply: updates of batch b, then the dots of batch b + 2 ----------------
        unsigned loaded = 0, cd = 0;
        struct Set { int32_t c[2 * GB]; float x[2 * GB]; };   // -1: no entry
        // the rows of batch b into registers
        auto copy = [&](int64_t b, Set& St) __attribute__((always_inline)) {
#pragma unroll
            for (int i = 0; i < GB; ++i) {
                const int64_t u = GB * b + i;
                const GSlot& sl = F->slot[u & (GSR - 1)];
                const int nz = F->meta.nnz[u & (GMR - 1)];
                const int32_t ca = sl.col[lane], cb = sl.col[lane + 64];
                const float xa = sl.val[lane], xb = sl.val[lane + 64];
                St.c[2 * i] = lane < nz ? ca : -1;
                St.c[2 * i + 1] = lane + 64 < nz ? cb : -1;
                St.x[2 * i] = xa;
                St.x[2 * i + 1] = xb;
            }
        };
        // P of batch b: head weights from LDS, tail from the chain's vector (after this wave's
        // earlier atomics to the same addresses: L2 sees them first), one transposed reduction
        auto dots = [&](int64_t b, const Set& St) __attribute__((always_inline)) {
            float wl[2 * GB], wt[2 * GB];
#pragma unroll
            for (int q = 0; q < 2 * GB; ++q) {
                const int32_t c = St.c[q];
                const bool head = c >= 0 && c < K;
                wl[q] = lds[head ? kW + (unsigned)c : kDread + lane];
                if constexpr (TAIL) wt[q] = gload_sc1(vrs, c >= K ? (uint32_t)c << 2 : kNoAccessG);
            }
            if constexpr (TAIL) {
                uint64_t vm0 = 0;
                if (L.stamps) vm0 = __builtin_amdgcn_s_memtime();
                asm volatile("s_waitcnt vmcnt(0)"
                             : "+v"(wt[0]), "+v"(wt[1]), "+v"(wt[2]), "+v"(wt[3]), "+v"(wt[4]), "+v"(wt[5]),
                               "+v"(wt[6]), "+v"(wt[7]), "+v"(wt[8]), "+v"(wt[9]), "+v"(wt[10]), "+v"(wt[11]),
                               "+v"(wt[12]), "+v"(wt[13]), "+v"(wt[14]), "+v"(wt[15])
                             :
                             : "memory");
                if (L.stamps) { st_wait += __builtin_amdgcn_s_memtime() - vm0; st_x[3] += __builtin_amdgcn_s_memtime() - vm0; }
            }
            float part[GB];
#pragma unroll
            for (int i = 0; i < GB; ++i) {
                // one of the two reads is the weight, the other an exact 0
                const float wa = TAIL ? wl[2 * i] + wt[2 * i] : wl[2 * i];
                const float wb = TAIL ? wl[2 * i + 1] + wt[2 * i + 1] : wl[2 * i + 1];
                part[i] = __builtin_fmaf(St.x[2 * i + 1], wb, St.x[2 * i] * wa);
            }
            const float tot = greduce8(part, lane);
            const int k = ((lane >> 5) & 1) | (((lane >> 4) & 1) << 1) | (((lane >> 3) & 1) << 2);
            if ((lane & 7) == 0) F->P[b & (GRB - 1)][k] = tot;
        };
        auto update = [&](int64_t b, const Set& St) __attribute__((always_inline)) {
            const f32x4 c0 = *reinterpret_cast<const f32x4*>(&F->C[b & (GRB - 1)][0]);
            const f32x4 c1 = *reinterpret_cast<const f32x4*>(&F->C[b & (GRB - 1)][4]);
            const float cv[GB] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
#pragma unroll
            for (int q = 0; q < 2 * GB; ++q) {
                const int32_t c = St.c[q];
                const bool head = c >= 0 && c < K;
                const float dv = cv[q >> 1] * St.x[q];
                __hip_atomic_fetch_add(lds + (head ? kW + (unsigned)c : kDwrite + lane), dv, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
                if constexpr (TAIL) gatomic_add(vrs, c >= K ? (uint32_t)c << 2 : kNoAccessG, dv);
            }
        };
        Set SA, SB;
        bool good = true;
        if (nb > 0) {
            good = wait_for(loaded, kLoaded, GB, 64);
            if (good) copy(0, SA);
            if (good && nb > 1) {
                good = wait_for(loaded, kLoaded, 2 * GB, 64);
                if (good) copy(1, SB);
            }
            if (good) {
                publish(kGathered, nb > 1 ? 2 : 1);
                dots(0, SA);
                if (nb > 1) dots(1, SB);
                publish(kPdone, nb > 1 ? 2 : 1);
            }
        }
        auto step = [&](int64_t b, Set& St) __attribute__((always_inline)) -> bool {
            if (!wait_for(cd, kCdone, b + 1, 64)) return false;
            const uint64_t t0 = tick();
            update(b, St);
            const uint64_t t1 = tick();
            if (stamps) st_x[0] += t1 - t0;
            if (b + 2 < nb) {
                if (!wait_for(loaded, kLoaded, GB * (b + 3), 64)) return false;
                const uint64_t t2 = tick();
                copy(b + 2, St);
                publish(kGathered, b + 3);
                const uint64_t t3 = tick();
                dots(b + 2, St);
                publish(kPdone, b + 3);
                if (stamps) { st_x[1] += t3 - t2; st_x[2] += tick() - t3; }
            }
            return true;
        };
        for (int64_t b = 0; good && b < nb; b += 2) {
            good = step(b, SA);
            if (good && b + 1 < nb) good = step(b + 1, SB);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
        // ---------------- chain: the scalar recurrence, lane i holds row i of the batch ----------
        const int i = lane & 7;
        float cprev[GB];
#pragma unroll
        for (int k = 0; k < GB; ++k) cprev[k] = 0.0f;
        unsigned pd = 0, gd = 0;
        for (int64_t b = 0; b < nb; ++b) {
            if (!wait_for(pd, kPdone, b + 1, 2) || !wait_for(gd, kGram, b + 1, 2)) {
                ok = false;
                break;
            }
            const int64_t u = GB * b + i;
            const int m = (int)(u & (GMR - 1));
            const int rb = (int)(b & (GRB - 1));
            const float p = F->P[rb][i];
            float G[2 * GB];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const f32x4 g4 = *reinterpret_cast<const f32x4*>(&F->G[rb][i][4 * q]);
                G[4 * q] = g4.x;
                G[4 * q + 1] = g4.y;
                G[4 * q + 2] = g4.z;
                G[4 * q + 3] = g4.w;
            }
            const float lab = F->meta.y[m], s = F->meta.s[m];
            // the cross terms with batch b-1 (their coefficients are known)
            float yv = p;
#pragma unroll
            for (int k = 0; k < GB; ++k) yv = __builtin_fmaf(cprev[k], G[k], yv);
            double al[GB + 1], inv[GB];
            if constexpr (L2) {
                const double f = 1.0 - F->meta.s64[m] * kp.reg;
                al[0] = alpha;
#pragma unroll
                for (int k = 0; k < GB; ++k) {
                    al[k + 1] = al[k] * readlane_d(f, k);
                    inv[k] = 1.0 / al[k + 1];
                }
                alpha = al[GB];
            }
            float cv[GB];
            float myloss = 0.0f, mycv = 0.0f;
#pragma unroll
            for (int k = 0; k < GB; ++k) {
                const float z = L2 ? float(al[k] * double(yv)) : yv;
                float loss;
                const float c = sparse_coef<GRAD>(z, lab, s, loss);
                const float ck = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(c), k));
                cv[k] = L2 ? float(double(ck) * inv[k]) : ck;
                myloss = i == k ? loss : myloss;
                mycv = i == k ? cv[k] : mycv;
                yv = __builtin_fmaf(cv[k], G[GB + k], yv);
            }
            if (lane < GB) F->C[rb][lane] = mycv;
            publish(kCdone, b + 1);
            if (lane < GB && u < n) loss_sum += double(myloss);
#pragma unroll
            for (int k = 0; k < GB; ++k) cprev[k] = cv[k];
        }
        // a wave that stopped early leaves the others blocked on it: wake them
        if (!ok) FL[kStop] = 1u;
    }
    if (L.stamps && lane == 0) {
        L.stamps[(size_t)chain * 16 + 2 * wave] = __builtin_amdgcn_s_memtime() - st_begin;
        L.stamps[(size_t)chain * 16 + 2 * wave + 1] = st_wait;
        if (wave >= 2)
            for (int k = 0; k < 4; ++k) L.stamps[(size_t)chain * 16 + 8 + 4 * (wave - 2) + k] = st_x[k];
    }
    __syncthreads();

    // the LDS head joins the tail in L.wf32 (the fold reads w = alpha v from there)
    for (int f = threadIdx.x; f < K; f += blockDim.x) V[f] = W[f];
    double nsq = 0.0;
    if constexpr (L2) {
        // ||v||^2 after the chain's last update (regVal, PSGD.scala:257), f64 over the floats
        for (int f = threadIdx.x; f < d; f += blockDim.x) {
            const float v = f < K ? W[f] : __hip_atomic_load(V + f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            nsq += double(v) * double(v);
        }
        nsq = wave_sum(nsq);
        double* red = reinterpret_cast<double*>(lds + kG);   // the G ring is free now
        if (lane == 0) red[wave] = nsq;
        __syncthreads();
        nsq = ((red[0] + red[1]) + red[2]) + red[3];
    }
    if (wave == 0) {
        loss_sum = wave_sum(loss_sum);
        if constexpr (GRAD == G_LEAST_SQUARES) loss_sum = loss_sum / 2.0;
        const int64_t count = ok ? n : 0;
        double rv = 0.0;
        if constexpr (L2) {
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
}

namespace {

template <typename S, int GRAD>
int gram_upd(const ChainLaunch& L, const KParams& kp, int upd, int K, size_t lds, hipStream_t st) {
    auto k = K < kp.d ? (upd == U_SIMPLE ? chain_sparse_gram<S, GRAD, U_SIMPLE, true>
                                         : chain_sparse_gram<S, GRAD, U_SQUARED_L2, true>)
                      : (upd == U_SIMPLE ? chain_sparse_gram<S, GRAD, U_SIMPLE, false>
                                         : chain_sparse_gram<S, GRAD, U_SQUARED_L2, false>);
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k, dim3(kp.n_chains), dim3(256), lds, st, L, kp, K);
    return (int)hipGetLastError();
}

template <typename S>
int gram_grad(const ChainLaunch& L, const KParams& kp, int grad, int upd, int K, size_t lds, hipStream_t st) {
    switch (grad) {
    case G_LOGISTIC: return gram_upd<S, G_LOGISTIC>(L, kp, upd, K, lds, st);
    case G_LEAST_SQUARES: return gram_upd<S, G_LEAST_SQUARES>(L, kp, upd, K, lds, st);
    case G_HINGE: return gram_upd<S, G_HINGE>(L, kp, upd, K, lds, st);
    default: return -3;
    }
}

}  // namespace

// Features [0, K) in LDS: all of them when they fit, else what the fixed part leaves.
int64_t sparse_gram_head(int64_t d) {
    const int64_t budget = (kGLdsCap - (int64_t)sizeof(GFixed)) / 4;
    return d <= budget ? d : (budget & ~int64_t(3));
}

bool sparse_gram_applies(int64_t d, int64_t max_nnz) {
    // row offsets are 32-bit in the buffer instructions: d * 4 < 2^31
    return max_nnz <= GCAP && d < ((int64_t)1 << 29);
}

int launch_sparse_gram_chains(const ChainLaunch& L, const KParams& kp, int storage, int gradient,
                              int updater, int64_t max_nnz, hipStream_t stream, int* kernel_variant) {
    if (kp.n_chains <= 0) return 0;
    if (!sparse_gram_applies(kp.d, max_nnz)) return -3;
    if (!L.wf32 || L.wstride < (int64_t)kp.d + 128 + 1024) return (int)hipErrorInvalidValue;
    int64_t K = sparse_gram_head(kp.d);
    // tests: PSGD_SPARSE_LDS_HEAD=k caps the LDS-resident head (exercises the tail at small d)
    if (const char* e = getenv("PSGD_SPARSE_LDS_HEAD"))
        if (*e) { const int64_t cap = atoll(e) & ~int64_t(3); if (cap >= 0 && cap < K) K = cap; }
    const size_t lds = sizeof(GFixed) + 4 * (size_t)K;
    if (kernel_variant) *kernel_variant = 630 + storage;
    if (storage == 1) return gram_grad<float>(L, kp, gradient, updater, (int)K, lds, stream);
    return gram_grad<double>(L, kp, gradient, updater, (int)K, lds, stream);
}

}  // namespace psgd
