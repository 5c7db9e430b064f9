// psgd_sparse_lds.hip -- the CSR chain with the chain's weights resident in LDS (gfx950): fp32
// compute (the throughput mode) and fp64 compute (the parity mode's CSR throughput kernel).
//
// Reference: ParallelizedSGD.scala:243-270 (the chain: weights read by Gradient.compute at :254,
// written by SGDUpdater.compute at :255-256), [ext] MLlib 1.6.1 Gradient.scala on SparseVector rows
// (the gradient is mult * x, non-zero only at the row's indices), SGDUpdater.scala:86-98 (Simple)
// and :163-181 (SquaredL2, alpha-scaled lazy form as in psgd_sparse.hip).
//
// T = float: weights as fp32, the tail in L.wf32, folded from there (launch_fold_f32).
// T = double: every weight, the LDS head and the HBM tail, is a double (the tail in the chain's
// slice of L.wf32 viewed as doubles); the coefficient, the loss and SquaredL2's alpha are the
// reference's Double arithmetic (only the dot's wave tree and the fused c*x + w are reassociated,
// the fp64 mode's 1e-9 bar); at the chain's end w = alpha v goes to L.w_out (the f64 fold) and
// regVal is taken from it. The alpha-scaled form runs without renormalisation, so the host
// launches it only when every prefix product of (1 - s_j lambda) stays in [2^-400, 2^400]
// (kp.alpha_ok); otherwise chain_general, which renormalises, runs.
//
// One workgroup = one chain = one CU (the 160 KiB LDS holds one chain's weights). Features
// [0, K) live in LDS as fp32 ("head"); when d does not fit, features [K, d) ("tail") stay in the
// chain's fp32 vector in HBM (L.wf32), 4 (d - K) bytes per chain instead of 4 d -- at rcv1 shape
// (d = 47,236) ~100 KB, so 32 chains per XCD fit its 4 MiB L2 where whole vectors did not.
//   * head entries: the chain reads w_j from LDS at the sample and writes the new value back
//     (one wave's LDS operations execute in program order, so row t+1 reads row t's update);
//   * tail entries: gathered from HBM SK samples ahead (sc1 loads: L2 sees this wave's earlier
//     stores first) and corrected as in chain_sparse_spec: a per-feature tag table over the tail
//     (2 B per tail feature: (row & 255) << 8 | entry of the latest row holding the feature)
//     names the latest of the SK preceding rows with the same feature, whose new value the chain
//     left in that row's LDS slot in place of x_j. Tags never alias: the tagger sweeps 1/128 of
//     the table per row and clears tags older than SK rows, so no tag outlives 256 rows.
// Three waves, one per SIMD, each a short branch-free loop:
//   wave 0 (chain)  per sample t: one LDS read per entry (head: W[j]; corrected tail: the earlier
//                   row's slot; else the gathered value), dot + wave reduction + coefficient, one
//                   LDS write per entry, the gathers of row t + SK and the row's tail stores
//                   (fixed 2 + 2 VMEM instructions: s_waitcnt vmcnt(4 SK) finds row t's gather);
//                   the next sample's slot data is read under the current sample's LDS latency;
//   wave 1 (loader) the partition's CSR entries into an SR-slot LDS ring (16 rows of loads in
//                   flight in registers, 8-row groups), labels / steps / nnz into a 128-row meta
//                   ring, 64 rows per batch;
//   wave 2 (tagger) per row: sweep a tag chunk, tail tag lookups + updates, and each entry's LDS
//                   read/write addresses (rw) into the slot.
// Rows are published through LDS counters: loaded (loader), tagged (tagger), done (chain).
// No MFMA: the work per sample is a ~100-long gather-dot and scatter.
//
// The per-sample break (tol > 0, CONV; PSGD.scala:262, :324-336): the chain wave tests
// isConverged after every sample from scalars it has -- with w' = a w + c x (a = 1 - s lambda for
// SquaredL2, else 1), z = x . w and q = x . x (one more wave sum beside the dot's),
// ||w'||^2 = a (a ||w||^2 + 2 c z) + c^2 q and ||w - w'||^2 = b (b ||w||^2 - 2 c z) + c^2 q
// (b = 1 - a), in f64 from ||w_in||^2 (L.wnsq0), as chain_block64 does; the test is
// D < tol^2 max(N, 1). After the first passing sample the rest of its unrolled group runs with
// c = 0 (no update, loss or count) and the chain ends.
#include "psgd_device.h"

#include <stdlib.h>

namespace psgd {

constexpr int LCAP = 128;                  // entries per row (two per lane)
#ifndef PSGD_LDS_TB
#define PSGD_LDS_TB 4                      // rows per tagger step (their LDS round trips overlap;
                                           // 8 measured round 5: c4 fp32 28.9 -> 43.3 ms, fp64 56.9 -> 58.0)
#endif
#ifndef PSGD_LDS_NT
#define PSGD_LDS_NT 1                      // the loader's CSR entry loads are non-temporal
#endif
#ifndef PSGD_LDS_EXP
#define PSGD_LDS_EXP 0                     // cost probes (tools/r03_c4_probe.sh, tools/r06_c4_probe.sh); 0 in the product
#endif

// The chain's tail gathers and stores are buffer instructions over its fp32 vector: a 32-bit
// byte offset per lane, and lanes without a tail entry get an out-of-range offset, which the
// hardware bounds check turns into no access at all (loads return 0, stores are dropped). EXEC
// stays full and every instruction counts once in vmcnt, with no per-lane 64-bit address or
// EXEC juggling on the chain's critical path.
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t kNoAccess = 0x80000000u;    // > any chain vector's byte size
__device__ __forceinline__ i32x4 buffer_rsrc(const float* base, uint32_t bytes) {
    const uint64_t a = (uint64_t)base;
    // dword1: base[47:32], stride 0; dword2: num_records (bytes); dword3: raw dword access (gfx9)
    return i32x4{__builtin_amdgcn_readfirstlane((int32_t)(uint32_t)a),
                 __builtin_amdgcn_readfirstlane((int32_t)((a >> 32) & 0xFFFF)),
                 __builtin_amdgcn_readfirstlane((int32_t)bytes), 0x00020000};
}
__device__ __forceinline__ float buffer_gather_sc1(i32x4 rsrc, uint32_t off) {
    float v;
    asm volatile("buffer_load_dword %0, %1, %2, 0 offen sc1" : "=v"(v) : "v"(off), "s"(rsrc) : "memory");
    return v;
}
__device__ __forceinline__ void buffer_store_f32(i32x4 rsrc, uint32_t off, float v) {
    asm volatile("buffer_store_dword %0, %1, %2, 0 offen" : : "v"(v), "v"(off), "s"(rsrc) : "memory");
}
__device__ __forceinline__ double buffer_gather_sc1(i32x4 rsrc, uint32_t off, double) {
    double v;
    asm volatile("buffer_load_dwordx2 %0, %1, %2, 0 offen sc1" : "=v"(v) : "v"(off), "s"(rsrc) : "memory");
    return v;
}
__device__ __forceinline__ float buffer_gather_sc1(i32x4 rsrc, uint32_t off, float) {
    return buffer_gather_sc1(rsrc, off);
}
__device__ __forceinline__ void buffer_store_f32(i32x4 rsrc, uint32_t off, double v) {
    asm volatile("buffer_store_dwordx2 %0, %1, %2, 0 offen" : : "v"(v), "v"(off), "s"(rsrc) : "memory");
}
constexpr int kMetaRing = 128;             // rows of label / step / nnz
constexpr int kSweepRows = 128;            // the tag table is swept once per this many rows
constexpr int64_t kLdsCap = 160 * 1024;    // LDS per CU (gfx950)

template <int SK>
struct LdsRing {
    // the chain needs rows up to t + SK + 1 staged at sample t (done = t); the loader reuses the
    // slot of row u - SR once the chain is done with row u - SR + SK (its new values are read by
    // the SK rows after it): progress needs t + SK + 1 - SR + SK + 1 <= t
    static constexpr int SR = 2 * SK + 8 <= 16 ? 16 : 32;
    static_assert(SR >= 2 * SK + 2, "ring too small for the speculation depth");
};

struct LdsHeader {
    unsigned loaded;   // rows whose entries are in their slots (loader)
    unsigned tagged;   // rows whose LDS addresses are in their slots (tagger)
    unsigned done;     // rows finished by the chain
    unsigned stop;
    unsigned dummy;    // target of inactive lanes' LDS weight reads and writes
    unsigned dtag;     // target of inactive lanes' tag reads and writes
    unsigned pad[2];
};
template <typename T>
struct LdsMeta {
    T y[kMetaRing];
    T s[kMetaRing];           // stepSize / sqrt(j) (rounded to fp32 in fp32 compute)
    double s64[kMetaRing];    // the same in f64 (SquaredL2's alpha)
    int32_t nnz[kMetaRing];
};
template <typename T>
struct LdsSlot {
    int32_t col[LCAP];   // feature index
    T val[LCAP];         // x_j; the chain replaces a tail entry's x_j by its new weight
    uint32_t rw[LCAP];   // LDS dword addresses: read (bits 0-15), write (bits 16-31)
};
// dword index of the target of inactive entries' weight reads and writes (LdsHeader::dummy; an
// 8-byte aligned pair, pad[0..1], for doubles)
template <typename T>
constexpr unsigned lds_dummy() { return sizeof(T) == 8 ? 6 : 4; }
constexpr int64_t kMetaOff = sizeof(LdsHeader);
template <typename T>
constexpr int64_t slot_off() { return kMetaOff + (int64_t)sizeof(LdsMeta<T>); }
static_assert(slot_off<float>() % 16 == 0 && sizeof(LdsSlot<float>) % 16 == 0, "alignment");
static_assert(slot_off<double>() % 16 == 0 && sizeof(LdsSlot<double>) % 16 == 0, "alignment");

template <int SK, typename T>
constexpr int64_t lds_fixed_bytes() { return slot_off<T>() + LdsRing<SK>::SR * (int64_t)sizeof(LdsSlot<T>); }
// tail tag table entries (u16), rounded for the sweep's 4-tag accesses
__host__ __device__ inline int64_t tag_entries(int64_t d, int64_t K) { return ((d - K) + 3) & ~int64_t(3); }
template <int SK, typename T>
int64_t lds_bytes(int64_t d, int64_t K) {
    return lds_fixed_bytes<SK, T>() + (int64_t)sizeof(T) * K + 2 * tag_entries(d, K);
}
// Features [0, K) in LDS: all of them when they fit, else as many as leave room for the tail's
// tag table (K a multiple of 4: the table stays 8-byte aligned); -1 when not even the table fits.
template <int SK, typename T>
int64_t lds_head(int64_t d) {
    const int64_t budget = kLdsCap - lds_fixed_bytes<SK, T>();
    if ((int64_t)sizeof(T) * d <= budget) return d;
    int64_t K = (budget - 2 * (d + 4)) / ((int64_t)sizeof(T) - 2);
    K &= ~int64_t(3);
    return K >= 0 ? K : -1;
}

// TAIL = false: every feature is in LDS (K = d), the chain issues no VMEM at all.
// T: the weights' and the arithmetic's type (float: the fp32 throughput mode; double: fp64).
template <typename S, typename T, int GRAD, int UPD, int SK, bool TAIL, bool CONV = false>
__global__ __launch_bounds__(192) void chain_sparse_lds(ChainLaunch L, KParams kp, int K) {
    constexpr bool L2 = UPD == U_SQUARED_L2;
    constexpr bool F64 = sizeof(T) == 8;
    constexpr int SR = LdsRing<SK>::SR;
    constexpr unsigned WD = sizeof(T) / 4;                       // dwords per weight
    constexpr unsigned kLdsDummy = lds_dummy<T>();
    constexpr int64_t kSlotOff = slot_off<T>();
    static_assert((SR & (SR - 1)) == 0, "slot index by mask");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    LdsHeader* hdr = reinterpret_cast<LdsHeader*>(smem);
    LdsMeta<T>* meta = reinterpret_cast<LdsMeta<T>*>(smem + kMetaOff);
    LdsSlot<T>* slots = reinterpret_cast<LdsSlot<T>*>(smem + kSlotOff);
    float* lds = reinterpret_cast<float*>(smem);                 // dword-addressed view
    // a weight (or a slot's value) at dword index i
    auto ld_w = [&](unsigned i) __attribute__((always_inline)) -> T { return *reinterpret_cast<const T*>(lds + i); };
    auto st_w = [&](unsigned i, T v) __attribute__((always_inline)) { *reinterpret_cast<T*>(lds + i) = v; };
    constexpr unsigned kWoff = (unsigned)(lds_fixed_bytes<SK, T>() / 4);
    T* W = reinterpret_cast<T*>(lds + kWoff);                    // head weights [K]
    uint16_t* tagpos = reinterpret_cast<uint16_t*>(W + K);       // tail features K .. d-1
    // dword index of val[0] of the slot holding row u
    auto val_off = [](int32_t u) __attribute__((always_inline)) -> unsigned {
        return (unsigned)((kSlotOff + (int64_t)(u & (SR - 1)) * (int64_t)sizeof(LdsSlot<T>)) / 4) + LCAP;
    };
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int chain = blockIdx.x;
    const ChainDesc dsc = L.descs[chain];
    const int d = kp.d;
    // row indices run in 32-bit: a chain's rows (>= 16 B each with the label) live in HBM, so
    // n < 2^31; the CSR offsets stay 64-bit (the loader's row_ptr values)
    const int32_t n = (int32_t)dsc.n_rows;
    const int32_t NT = (int32_t)tag_entries(d, K);
    // The chain runs n_pad samples (a multiple of its unroll SK + 1) and reads up to row
    // n_pad + SK ahead: the loader and the tagger stage n_fill rows, rows past n null (no
    // entries, label and step 0), so no read in the chain needs a condition.
    constexpr int GS = SK + 1;
    const int32_t n_pad = (n + GS - 1) / GS * GS;
    const int32_t n_fill = (n_pad + SK + 1 + 7) / 8 * 8;
    // [d] (tail used) + [128] the loader's dummy sources + [1024] the chain's dummy targets (in
    // T: for doubles the chain's slice of L.wf32 is twice as long, launch_sparse_lds64_chains)
    T* V = reinterpret_cast<T*>(L.wf32 + (int64_t)chain * L.wstride);

    for (int32_t i = threadIdx.x; i < NT; i += blockDim.x) tagpos[i] = 0xFFFF;
    for (int i = threadIdx.x; i < K; i += blockDim.x) W[i] = T(as_global(L.w_in)[i]);
    if (threadIdx.x < 8) reinterpret_cast<unsigned*>(hdr)[threadIdx.x] = 0;
    if constexpr (F64 && TAIL) {
        // the tail V[K, d) starts as w_in; the chain's gathers (sc1, through L2) must see it
        for (int i = K + threadIdx.x; i < d; i += blockDim.x) V[i] = as_global(L.w_in)[i];
        __threadfence();
    }
    // (fp32: the tail V[K, d) starts as float(w_in), wf32_init_kernel launched before this kernel)
    __syncthreads();

    uint64_t st_wait = 0;                     // diagnostic (PSGD_STAMPS): cycles spent waiting
    const uint64_t st_begin = __builtin_amdgcn_s_memtime();
    // wait until *flag >= need (cached in `seen`); false when the chain stopped or the watchdog fired
    auto wait_for = [&](unsigned& seen, const unsigned* flag, int32_t need, int code)
        __attribute__((always_inline)) -> bool {
        if ((int32_t)seen >= need) return true;
        // one LDS read first: the clocks are scalar-memory round trips (and their lgkmcnt wait
        // also drains this wave's LDS operations), paid only when the flag is not there yet
        seen = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if ((int32_t)seen >= need) {
            __atomic_signal_fence(__ATOMIC_SEQ_CST);
            return true;
        }
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        const uint64_t c0 = L.stamps ? __builtin_amdgcn_s_memtime() : 0;
        for (;;) {
            // relaxed: the flags and the data are LDS, which one wave writes in program order
            seen = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if ((int32_t)seen >= need) {
                __atomic_signal_fence(__ATOMIC_SEQ_CST);
                if (L.stamps) st_wait += __builtin_amdgcn_s_memtime() - c0;
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
    auto publish = [&](unsigned* flag, int32_t v) __attribute__((always_inline)) {
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        __hip_atomic_store(flag, (unsigned)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    auto stamp_out = [&](int k) __attribute__((always_inline)) {
        if (L.stamps && lane == 0) {
            L.stamps[(size_t)chain * 6 + 2 * k] = __builtin_amdgcn_s_memtime() - st_begin;
            L.stamps[(size_t)chain * 6 + 2 * k + 1] = st_wait;
        }
    };

    if (wave == 1) {
        // ---------------- loader: entries into slots, labels / steps / nnz into the meta ring ----
        const gptr<S> X = as_global(reinterpret_cast<const S*>(dsc.x));
        const gptr<int32_t> COL = as_global(dsc.col);
        const gptr<int64_t> RP = as_global(dsc.row_ptr);
        const gptr<double> Y = as_global(dsc.y);
        const gptr<double> STEPS = as_global(L.steps);
        const gptr<int32_t> RIDX = dsc.rows ? as_global(dsc.rows) : nullptr;
        unsigned done = 0;
        const gptr<int32_t> dummy_i = as_global((const int32_t*)(V + d + lane));   // valid, unused
        const gptr<S> dummy_s = as_global((const S*)(V + d + 2 * lane));
        struct Batch { int64_t rb, re; double y, s; };
        auto load_batch = [&](int32_t g) __attribute__((always_inline)) -> Batch {
            Batch bt{0, 0, 0.0, 0.0};
            const int32_t ti = g + lane;
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
        // entries of rows g + i0 .. g + i0 + 7 of batch bt: unconditional loads (masked-off
        // entries read valid dummy addresses), so the compiler counts them without branches. The
        // loaded values are used only when the group is staged (one group later): a select here
        // would make the compiler wait for the loads at once.
        auto load_group = [&](const Batch& bt, int i0, Group& G) __attribute__((always_inline)) {
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int64_t b = rl64(bt.rb, i0 + q), e = rl64(bt.re, i0 + q);
                const int64_t ka = b + lane, kc = b + 64 + lane;
                const bool ia = ka < e, ic = kc < e;
                // (non-temporal: the row stream is read once and must not evict the chains'
                // L2-resident tails, ~3.2 MB per XCD in its 4 MiB at c4)
                G.ca[q] = PSGD_LDS_NT ? __builtin_nontemporal_load(ia ? &COL[ka] : dummy_i) : *(ia ? &COL[ka] : dummy_i);
                G.xa[q] = PSGD_LDS_NT ? __builtin_nontemporal_load(ia ? &X[ka] : dummy_s) : *(ia ? &X[ka] : dummy_s);
                G.cb[q] = PSGD_LDS_NT ? __builtin_nontemporal_load(ic ? &COL[kc] : dummy_i) : *(ic ? &COL[kc] : dummy_i);
                G.xb[q] = PSGD_LDS_NT ? __builtin_nontemporal_load(ic ? &X[kc] : dummy_s) : *(ic ? &X[kc] : dummy_s);
                G.ia[q] = ia;
                G.ic[q] = ic;
            }
        };
        // rows u0 .. u0 + 7 (those < n_fill) into their slots, each once the chain is done with the
        // row its slot held (row u - SR, read by the chain up to row u - SR + SK), published row
        // by row: the chain at sample t waits for row t + SK + 1
        auto stage_group = [&](int32_t u0, const Group& G) __attribute__((always_inline)) -> bool {
            bool good = true;
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int32_t u = u0 + q;
                if (good && u < n_fill) {
                    good = wait_for(done, &hdr->done, u - SR + SK + 1, 16);
                    LdsSlot<T>& sl = slots[u & (SR - 1)];
                    sl.col[lane] = G.ca[q];
                    sl.col[lane + 64] = G.cb[q];
                    sl.val[lane] = G.ia[q] ? T(G.xa[q]) : T(0);
                    sl.val[lane + 64] = G.ic[q] ? T(G.xb[q]) : T(0);
                    if constexpr (!TAIL) {
                        // every feature in LDS: the entry's read and write address is W[j]
                        // (no tagger); inactive entries have x = 0 and use the dummy dword
                        const unsigned ha = G.ia[q] ? kWoff + WD * (unsigned)G.ca[q] : kLdsDummy;
                        const unsigned hb = G.ic[q] ? kWoff + WD * (unsigned)G.cb[q] : kLdsDummy;
                        sl.rw[lane] = ha | (ha << 16);
                        sl.rw[lane + 64] = hb | (hb << 16);
                        publish(&hdr->tagged, u + 1);
                    }
                    publish(&hdr->loaded, u + 1);
                }
            }
            return good;
        };
        Batch cur = load_batch(0);
        Group GA, GB;
        load_group(cur, 0, GA);
        for (int32_t g = 0; g < n_fill; g += 64) {
            const Batch nxt = load_batch(g + 64);
            // meta of rows g .. g + 63: their ring positions held rows g - 128 .. g - 65
            if (!wait_for(done, &hdr->done, g - 64, 16)) break;
            {
                const int m = (int)((g + lane) & (kMetaRing - 1));
                meta->y[m] = T(cur.y);
                meta->s[m] = T(cur.s);
                meta->s64[m] = cur.s;
                meta->nnz[m] = (int32_t)(cur.re - cur.rb);
            }
            bool ok = true;
            static_for<4>([&](auto kc) {
                // group i0 is in GA; fetch group i0 + 8 into GB, stage GA; then the other way
                constexpr int i0 = 16 * decltype(kc)::value;
                if (!ok) return;
                load_group(cur, i0 + 8, GB);
                ok = stage_group(g + i0, GA);
                if constexpr (i0 + 16 < 64) load_group(cur, i0 + 16, GA);
                else load_group(nxt, 0, GA);
                if (ok) ok = stage_group(g + i0 + 8, GB);
            });
            if (!ok) break;
            cur = nxt;
        }
        stamp_out(1);
        return;
    }

    if (wave == 2 && !TAIL) return;   // the loader writes the addresses
    if (wave == 2) {
        // ---------------- tagger: tail tags and each entry's LDS read / write address ----------
        // Four rows per step, so that their LDS round trips overlap: the rows' columns, then the
        // sweeps, then each row's tag lookups and updates in row order (one wave's LDS operations
        // execute in program order, so row u+1's lookups see row u's updates), then the rows'
        // addresses.
        constexpr int TB = PSGD_LDS_TB;
        unsigned loaded = 0;
        uint16_t* dtag = reinterpret_cast<uint16_t*>(&hdr->dtag);
        const int32_t chunk = ((NT + kSweepRows - 1) / kSweepRows + 255) & ~int32_t(255);
        static_assert(8 % TB == 0, "n_fill is a multiple of TB");
        for (int32_t u0 = 0; u0 < n_fill; u0 += TB) {
            constexpr int nb = TB;
            if (!wait_for(loaded, &hdr->loaded, u0 + nb, 32)) break;
            int nnz[TB];
            int32_t ca[TB], cb[TB];
#pragma unroll
            for (int q = 0; q < TB; ++q) {
                const int32_t u = u0 + q;
                const LdsSlot<T>& sl = slots[u & (SR - 1)];
                nnz[q] = meta->nnz[u & (kMetaRing - 1)];
                ca[q] = sl.col[lane];
                cb[q] = sl.col[lane + 64];
            }
            // the loader's count for the next step's check, read with the columns (a refresh in
            // wait_for waits for every LDS access in flight, this step's tag writes included)
            const unsigned ld_pre = __hip_atomic_load(&hdr->loaded, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            // sweep the chunks of rows u0 .. u0 + TB - 1, keeping the tags of rows u0 - SK .. u0 - 1
            // (the oldest rows this step's lookups need); each chunk is swept at least every
            // kSweepRows rows, so no tag outlives 256 rows
            auto sweep4 = [&](uint64_t v) __attribute__((always_inline)) -> uint64_t {
                uint64_t o = 0;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const unsigned tg = (unsigned)(v >> (16 * k)) & 0xFFFF;
                    const unsigned dl = ((unsigned)u0 - (tg >> 8)) & 255;
                    const bool live = tg != 0xFFFF && dl >= 1 && dl <= SK;
                    o |= (uint64_t)(live ? tg : 0xFFFFu) << (16 * k);
                }
                return o;
            };
            if (chunk <= 256) {
                // one 4-tag word per lane and row: the TB reads share one LDS round trip
                uint64_t sv[TB];
                bool sok[TB];
                int32_t si[TB];
#pragma unroll
                for (int q = 0; q < TB; ++q) {
                    const int32_t lo = ((u0 + q) & (kSweepRows - 1)) * chunk;
                    const int32_t hi = lo + chunk < NT ? lo + chunk : NT;
                    si[q] = lo + 4 * lane;
                    sok[q] = si[q] < hi;
                    sv[q] = *reinterpret_cast<const uint64_t*>(tagpos + (sok[q] ? si[q] : 0));
                }
#pragma unroll
                for (int q = 0; q < TB; ++q)
                    if (sok[q]) *reinterpret_cast<uint64_t*>(tagpos + si[q]) = sweep4(sv[q]);
            } else {
#pragma unroll
            for (int q = 0; q < TB; ++q) {
                const int32_t lo = ((u0 + q) & (kSweepRows - 1)) * chunk;
                const int32_t hi = lo + chunk < NT ? lo + chunk : NT;
                for (int32_t i = lo + 4 * lane; i < hi; i += 256) {
                    const uint64_t v = *reinterpret_cast<const uint64_t*>(tagpos + i);
                    *reinterpret_cast<uint64_t*>(tagpos + i) = sweep4(v);
                }
            }
            }
            unsigned va[TB], vb[TB];
#pragma unroll
            for (int q = 0; q < TB; ++q) {
                const int32_t u = u0 + q;
                const bool ta_on = lane < nnz[q] && ca[q] >= K, tb_on = lane + 64 < nnz[q] && cb[q] >= K;
                uint16_t* pa = ta_on ? tagpos + (ca[q] - K) : dtag;
                uint16_t* pb = tb_on ? tagpos + (cb[q] - K) : dtag;
                va[q] = *pa;
                vb[q] = *pb;
                const unsigned tag = (unsigned)(u & 255) << 8;
                *pa = (uint16_t)(tag | (unsigned)lane);
                *pb = (uint16_t)(tag | (unsigned)(lane + 64));
            }
#pragma unroll
            for (int q = 0; q < TB; ++q) {
                const int32_t u = u0 + q;
                auto rw_of = [&](int e, int32_t c, unsigned v) __attribute__((always_inline)) -> uint32_t {
                    const bool tail = c >= K;
                    const unsigned dl = ((unsigned)u - (v >> 8)) & 255;
                    const bool prev = v != 0xFFFF && dl >= 1 && dl <= SK;
                    const unsigned rd_tail = prev ? val_off(u - dl) + WD * (v & 255) : kLdsDummy;
                    const unsigned wr_tail = val_off(u) + WD * (unsigned)e;
                    const unsigned head = kWoff + WD * (unsigned)c;
                    const unsigned rd = e >= nnz[q] ? kLdsDummy : tail ? rd_tail : head;
                    const unsigned wr = e >= nnz[q] ? kLdsDummy : tail ? wr_tail : head;
                    return rd | (wr << 16);
                };
                if (q < nb) {
                    LdsSlot<T>& sl = slots[u & (SR - 1)];
                    sl.rw[lane] = rw_of(lane, ca[q], va[q]);
                    sl.rw[lane + 64] = rw_of(lane + 64, cb[q], vb[q]);
                }
            }
            publish(&hdr->tagged, u0 + nb);
            loaded = ld_pre > loaded ? ld_pre : loaded;
        }
        stamp_out(2);
        return;
    }

    // ---------------- chain ----------------
    // The per-sample code is straight-line: the flag checks come before the LDS reads they
    // guard and branch only to a spin, so no read result crosses a branch (a join would make
    // the compiler wait for it). The loop runs a multiple of SK + 1 samples; samples past n are
    // null (no entries, LDS traffic to the dummy dword, no loss), so every gather's registers
    // have a consumer: the compiler treats an asm load's result as written at issue, and a dead
    // one's registers could be reused while the load is still in flight.
    double alpha = 1.0;       // SquaredL2: w = alpha * v
    double dnsq = 0.0;        // SquaredL2, fp32: ||v||^2 - ||v_0||^2 (this lane)
    // CONV: ||w||^2 (the recurrence in the header), the break state and the samples taken
    double nsq = CONV ? *L.wnsq0 : 0.0;
    const double tol2 = kp.tol * kp.tol;
    bool brk = false;
    int32_t taken = 0;
    double loss_sum = 0.0;
    float loss_blk = 0.0f;
    int64_t count = 0;
    unsigned loaded = 0, tagged = 0;
    constexpr unsigned kShift = F64 ? 3 : 2;
    const i32x4 vrs = buffer_rsrc(reinterpret_cast<const float*>(V), (uint32_t)((int64_t)d * sizeof(T)));   // [0, d)
    auto boff = [](bool on, int32_t c) __attribute__((always_inline)) -> uint32_t {
        return on ? (uint32_t)c << kShift : kNoAccess;
    };
    // gathered tail weights: row u's in gr[u % (SK + 1)]. A gather's registers are written by
    // the load when it lands, so they are never copied before their s_waitcnt: the gather of
    // row t + SK goes to the set row t - 1 used, and the loop is unrolled SK + 1 times
    T gr[GS][2];
    bool ok = true;
    // wait until rows < nl are loaded and rows < nt tagged (the spin path only)
    auto need = [&](int32_t nl, int32_t nt) __attribute__((always_inline)) {
        nl = nl < n_fill ? nl : n_fill;
        nt = nt < n_fill ? nt : n_fill;
        if ((int32_t)loaded < nl || (int32_t)tagged < nt) {
            ok = ok && wait_for(loaded, &hdr->loaded, nl, 2);
            ok = ok && wait_for(tagged, &hdr->tagged, nt, 4);
        }
    };
    // the entries of row u a gather needs
    struct GCols { int32_t c0, c1; int nnz; };
    auto gcols = [&](int32_t u) __attribute__((always_inline)) -> GCols {
        const LdsSlot<T>& sl = slots[u & (SR - 1)];
        const int nz = meta->nnz[u & (kMetaRing - 1)];
        return GCols{sl.col[lane], sl.col[lane + 64], nz};
    };
    // Only tail entries touch memory: the other lanes get the no-access offset.
    auto gather = [&](const GCols& G, T (&g)[2]) __attribute__((always_inline)) {
#if PSGD_LDS_EXP & 2   // experiment: the tail gathers read nothing (wrong results; cost probe)
        const bool a0 = false, a1 = false;
#else
        const bool a0 = lane < G.nnz && G.c0 >= K, a1 = lane + 64 < G.nnz && G.c1 >= K;
#endif
        g[0] = buffer_gather_sc1(vrs, boff(a0, G.c0), T(0));
        g[1] = buffer_gather_sc1(vrs, boff(a1, G.c1), T(0));
    };
    // the data of sample t
    struct Row { T x0, x1; uint32_t rw0, rw1; int32_t c0, c1; int nnz; T y, s; double s64; };
    auto row_of = [&](int32_t t) __attribute__((always_inline)) -> Row {
        const LdsSlot<T>& sl = slots[t & (SR - 1)];
        const int m = (int)(t & (kMetaRing - 1));
        return Row{sl.val[lane], sl.val[lane + 64], sl.rw[lane], sl.rw[lane + 64], sl.col[lane],
                   sl.col[lane + 64], meta->nnz[m], meta->y[m], meta->s[m], L2 ? meta->s64[m] : 0.0};
    };
    // prologue: gathers of rows 0 .. SK-1, each followed by two no-access stores, the same VMEM
    // pattern as a sample of the loop; then the columns of row SK and the data of sample 0
    GCols gc{0, 0, 0};
    if constexpr (TAIL) {
        static_for<SK>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            need(q + 1, 0);
            gather(gcols(q), gr[q]);
            buffer_store_f32(vrs, kNoAccess, T(0));
            buffer_store_f32(vrs, kNoAccess, T(0));
        });
        need(SK + 1, 1);
        gc = gcols(SK);
    } else {
        need(0, 1);
    }
    Row cur = row_of(0);
    auto sample = [&](auto qc, int32_t t) __attribute__((always_inline)) {
        constexpr int Q = decltype(qc)::value;           // t % GS
        constexpr int QN = (Q + SK) % GS;                 // (t + SK) % GS
        // the rows the reads below need (a branch to the spin only)
        need(TAIL ? t + SK + 2 : 0, t + 2);
        // this sample's weight reads (after the previous sample's writes, in program order),
        // row t + SK's gather, then the columns of row t + SK + 1 and the data of sample t + 1:
        // all issued before anything waits (the scheduling barrier keeps the compiler from
        // sinking the prefetch below the arithmetic), so their LDS round trips overlap
        const unsigned r0 = cur.rw0 & 0xFFFF, r1 = cur.rw1 & 0xFFFF;
        const T l0 = ld_w(r0), l1 = ld_w(r1);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (TAIL) {
            gather(gc, gr[QN]);
            gc = gcols(t + SK + 1);
        }
        const Row nxt = row_of(t + 1);
        // the flags the next samples' need() checks, read under this sample's LDS round trip
        // (a need() that finds its cached counts short reads the flag and waits for every LDS
        // read in flight: with the tagger a few rows ahead, that happened every few samples)
        const unsigned ld_pre = TAIL ? __hip_atomic_load(&hdr->loaded, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) : 0u;
        const unsigned tg_pre = __hip_atomic_load(&hdr->tagged, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        // the counts cached from these relaxed loads let the next samples' need()
        // skip wait_for's fence and read the rows the loader / tagger published. That is sound
        // because (1) LDS operations of a workgroup execute in order (the loader and the tagger
        // write a row before its flag, this wave reads the flag before the row), and (2) no data
        // load of a later sample may be hoisted by the compiler above these flag loads: the
        // compiler-only fence below forbids it (no instruction, no lgkmcnt wait)
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        __builtin_amdgcn_sched_barrier(0);
        T w0 = l0, w1 = l1;
        if constexpr (TAIL) {
            // row t's gather: issued SK samples ago, followed by 4 SK VMEM instructions
            // (-DPSGD_STAMPS builds: the time this wait takes joins the chain's "wait" counter;
            // compiled out of the product: an s_memtime on any path into the arithmetic below
            // makes the compiler wait for every LDS read in flight, the next row's prefetch too)
            PSGD_STAMP(uint64_t vm0 = 0; if (L.stamps) vm0 = __builtin_amdgcn_s_memtime();)
#if PSGD_LDS_EXP & 16   // experiment: no wait for the row's gathers, their values unused (cost probe)
            w0 = l0;
            w1 = l1;
#else
            asm volatile("s_waitcnt vmcnt(%2)" : "+v"(gr[Q][0]), "+v"(gr[Q][1]) : "i"(4 * SK) : "memory");
            PSGD_STAMP(if (L.stamps) st_wait += __builtin_amdgcn_s_memtime() - vm0;)
            // head: W[j]; tail also in rows t-SK .. t-1: that row's new value; else the gather
            w0 = r0 == kLdsDummy ? gr[Q][0] : l0;
            w1 = r1 == kLdsDummy ? gr[Q][1] : l1;
#endif
        }
        w0 = lane < cur.nnz ? w0 : T(0);
        w1 = lane + 64 < cur.nnz ? w1 : T(0);
        T acc = cur.x0 * w0;
        acc = m_fma(cur.x1, w1, acc);
#if PSGD_LDS_EXP & 4    // experiment: no wave reduction, the lane's partial as the dot (cost probe)
        T z = acc;
#else
        T z = wave_sum_uniform(acc);
#endif
        T qx = T(0);   // CONV: x . x
        if constexpr (CONV) qx = wave_sum_uniform(m_fma(cur.x1, cur.x1, cur.x0 * cur.x0));
        // CONV: a sample after the break is not taken (c = 0, no shrink, no loss)
        [[maybe_unused]] const bool live = !CONV || !brk;
        if constexpr (L2) {
            // w = alpha v: the dot is alpha (x . v); then the L2 shrink alpha *= 1 - s lambda
            // (SGDUpdater.scala:176) and the step adds c x_j / alpha to v
            z = T(alpha * double(z));
            alpha *= live ? 1.0 - cur.s64 * kp.reg : 1.0;
        }
        T c;
        if constexpr (F64) {
            // [ext] MLlib 1.6.1 Gradient.compute in Double (the loss included); c = -s * mult
            double mult;
            const double loss = gradient_scalar<GRAD, double>(z, cur.y, mult);
            c = -cur.s * mult;
            loss_sum += t < n && live ? loss : 0.0;
        } else {
            float loss;
#if PSGD_LDS_EXP & 8    // experiment: the coefficient does not wait for the dot (cost probe)
            asm volatile("" : : "v"(z));
            c = sparse_coef<GRAD>(T(0.25) * cur.y, cur.y, cur.s, loss);
#else
            c = sparse_coef<GRAD>(z, cur.y, cur.s, loss);
#endif
            loss_blk += t < n && live ? loss : 0.0f;
            if ((t & 31) == 31) { loss_sum += double(loss_blk); loss_blk = 0.0f; }
        }
        if constexpr (CONV) {
            c = live ? c : T(0);
            // isConverged(w_t, w_{t+1}) (PSGD.scala:262, :333-335) from z, q, c (f64)
            const double cd = double(c), zd = double(z), cq = cd * cd * double(qx);
            double nn, dd;
            if constexpr (L2) {
                const double a = live ? 1.0 - cur.s64 * kp.reg : 1.0, b = 1.0 - a;
                nn = a * __builtin_fma(a, nsq, 2.0 * cd * zd) + cq;
                dd = b * __builtin_fma(b, nsq, -2.0 * cd * zd) + cq;
            } else {
                nn = __builtin_fma(cd, 2.0 * zd, nsq) + cq;
                dd = cq;
            }
            nsq = nn > 0.0 ? nn : 0.0;
            const bool pass = t < n && live && dd < tol2 * (nn > 1.0 ? nn : 1.0);
            taken = pass ? t + 1 : taken;
            brk = brk || pass;
        }
        const T cv = L2 ? T(double(c) / alpha) : c;
        const T nv0 = m_fma(cv, cur.x0, w0);
        const T nv1 = m_fma(cv, cur.x1, w1);
        if constexpr (L2 && !F64) dnsq += nsq_delta(w0, nv0) + nsq_delta(w1, nv1);
        st_w(cur.rw0 >> 16, nv0);
        st_w(cur.rw1 >> 16, nv1);
        // this row's tail stores (2 VMEM instructions)
        if constexpr (TAIL) {
            const bool a0 = lane < cur.nnz && cur.c0 >= K, a1 = lane + 64 < cur.nnz && cur.c1 >= K;
#if PSGD_LDS_EXP & 1   // experiment: the tail stores go nowhere (wrong results; cost probe)
            buffer_store_f32(vrs, kNoAccess, nv0);
            buffer_store_f32(vrs, kNoAccess, nv1);
#else
            buffer_store_f32(vrs, boff(a0, cur.c0), nv0);
            buffer_store_f32(vrs, boff(a1, cur.c1), nv1);
#endif
        }
        publish(&hdr->done, t + 1);
        cur = nxt;
        if constexpr (TAIL) loaded = ld_pre > loaded ? ld_pre : loaded;
        tagged = tg_pre > tagged ? tg_pre : tagged;
    };
    for (int32_t t = 0; ok && !brk && t < n_pad; t += GS)
        static_for<GS>([&](auto qc) { sample(qc, t + decltype(qc)::value); });
    count = ok ? (brk ? taken : n) : 0;
    __hip_atomic_store(&hdr->stop, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // the last gathers' registers stay allocated until they have landed
#pragma unroll
    for (int q = 0; q < GS; ++q) asm volatile("" : : "v"(gr[q][0]), "v"(gr[q][1]));
    stamp_out(0);
    loss_sum += double(loss_blk);
    if constexpr (GRAD == G_LEAST_SQUARES && !F64) loss_sum = loss_sum / 2.0;
    if constexpr (F64) {
        // w = alpha v into the chain's row of L.w_out (the f64 fold), regVal of the chain's last
        // update (PSGD.scala:257) from ||w||: the head from LDS, the tail from V (this wave's
        // own stores, landed above; read through L2 like its gathers)
        double* wo = L.w_out + (int64_t)chain * d;
        double nsq = 0.0;
        for (int i = lane; i < K; i += 64) {
            const double wv = L2 ? alpha * W[i] : W[i];
            wo[i] = wv;
            if constexpr (L2) nsq += wv * wv;
        }
        if constexpr (TAIL) {
            // 8 loads in flight per lane (out-of-range lanes: the no-access offset, read as 0)
            for (int i0 = K; i0 < d; i0 += 8 * 64) {
                double vv[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const int i = i0 + q * 64 + lane;
                    vv[q] = buffer_gather_sc1(vrs, i < d ? (uint32_t)i << 3 : kNoAccess, 0.0);
                }
                asm volatile("s_waitcnt vmcnt(0)" : "+v"(vv[0]), "+v"(vv[1]), "+v"(vv[2]), "+v"(vv[3]),
                             "+v"(vv[4]), "+v"(vv[5]), "+v"(vv[6]), "+v"(vv[7]) : : "memory");
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const int i = i0 + q * 64 + lane;
                    if (i < d) {
                        const double wv = L2 ? alpha * vv[q] : vv[q];
                        wo[i] = wv;
                        if constexpr (L2) nsq += wv * wv;
                    }
                }
            }
        }
        double rv = 0.0;
        if constexpr (L2) {
            nsq = wave_sum(nsq);
            if (count > 0) {
                const double nrm = sqrt(nsq);
                rv = 0.5 * kp.reg * nrm * nrm;
            }
        }
        if (lane == 0) {
            L.rv[chain] = rv;
            L.loss[chain] = loss_sum;
            L.cnt[chain] = count;
            L.cnt_d[chain] = double(count);
        }
    } else {
        // the LDS head joins the tail in L.wf32 (the fold reads w = alpha v from there); regVal
        // of the chain's last update (PSGD.scala:257) from the tracked ||v||^2
        for (int i = lane; i < K; i += 64) V[i] = W[i];
        sparse_chain_out<L2>(L, kp, chain, lane, alpha, dnsq, loss_sum, count);
    }
}

// The dispatch over every instantiation (left out of single-kernel ISA probes, tools/isa_probe.sh).
#ifndef PSGD_NO_DISPATCH
template <typename S, typename T, int GRAD, int SK, bool CONV>
static int lds_upd_c(const ChainLaunch& L, const KParams& kp, int upd, int K, size_t lds, hipStream_t st) {
    auto k = K < kp.d ? (upd == U_SIMPLE ? chain_sparse_lds<S, T, GRAD, U_SIMPLE, SK, true, CONV>
                                         : chain_sparse_lds<S, T, GRAD, U_SQUARED_L2, SK, true, CONV>)
                      : (upd == U_SIMPLE ? chain_sparse_lds<S, T, GRAD, U_SIMPLE, SK, false, CONV>
                                         : chain_sparse_lds<S, T, GRAD, U_SQUARED_L2, SK, false, CONV>);
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k, dim3(kp.n_chains), dim3(192), lds, st, L, kp, K);
    return (int)hipGetLastError();
}

// the per-sample break (tol > 0) has instances at the default depth SK = 4 only
template <typename S, typename T, int GRAD, int SK>
static int lds_upd(const ChainLaunch& L, const KParams& kp, int upd, int K, size_t lds, hipStream_t st) {
    if constexpr (SK == 4) {
        if (kp.tol > 0.0) return lds_upd_c<S, T, GRAD, SK, true>(L, kp, upd, K, lds, st);
    }
    return lds_upd_c<S, T, GRAD, SK, false>(L, kp, upd, K, lds, st);
}

template <typename S, typename T, int SK>
static int lds_grad(const ChainLaunch& L, const KParams& kp, int grad, int upd, int K, size_t lds, hipStream_t st) {
    switch (grad) {
    case G_LOGISTIC: return lds_upd<S, T, G_LOGISTIC, SK>(L, kp, upd, K, lds, st);
    case G_LEAST_SQUARES: return lds_upd<S, T, G_LEAST_SQUARES, SK>(L, kp, upd, K, lds, st);
    case G_HINGE: return lds_upd<S, T, G_HINGE, SK>(L, kp, upd, K, lds, st);
    default: return -3;
    }
}

// Variant 600 + 40 (the per-sample break, tol > 0) + 10 (SK == 8) + 20 (fp64 compute) + storage
// (1: f32 rows).
template <int SK, typename T>
static int lds_launch(const ChainLaunch& L, const KParams& kp, int storage, int gradient, int updater,
                      hipStream_t stream, int* kernel_variant) {
    int64_t K = lds_head<SK, T>(kp.d);
    if (K < 0) return -3;
    // tests: PSGD_SPARSE_LDS_HEAD=k caps the LDS-resident head (exercises the tail at small d)
    if (const char* e = getenv("PSGD_SPARSE_LDS_HEAD"))
        if (*e) { const int64_t cap = atoll(e) & ~int64_t(3); if (cap >= 0 && cap < K) K = cap; }
    const size_t lds = (size_t)lds_bytes<SK, T>(kp.d, K);
    if (kernel_variant) *kernel_variant = 600 + (kp.tol > 0.0 ? 40 : 0) + (SK == 8 ? 10 : 0) + (sizeof(T) == 8 ? 20 : 0) + storage;
    if (storage == 1) return lds_grad<float, T, SK>(L, kp, gradient, updater, (int)K, lds, stream);
    return lds_grad<double, T, SK>(L, kp, gradient, updater, (int)K, lds, stream);
}

// Speculation depth: 4 rows by default (tail gathers are L2 hits once the tails fit L2);
// PSGD_SPARSE_SK=8 for A/B measurements (read at every launch).
static int lds_depth() {
    const char* e = getenv("PSGD_SPARSE_SK");
    return (e && atoi(e) == 8) ? 8 : 4;
}

// The chain, loader and tagger waves keep row numbers in 32 bits (psgd_sparse_lds.hip: n): a
// partition of more than INT32_MAX rows (>= 32 GiB of 16-byte CSR rows, which fits in HBM) takes
// chain_sparse / chain_general instead.
bool sparse_lds_applies(int64_t d, int64_t max_nnz, int64_t n_max) {
    if (max_nnz > LCAP || n_max > (int64_t)INT32_MAX) return false;
    return (lds_depth() == 8 ? lds_head<8, float>(d) : lds_head<4, float>(d)) >= 0;
}

int64_t sparse_lds_head(int64_t d) { return lds_depth() == 8 ? lds_head<8, float>(d) : lds_head<4, float>(d); }

int launch_sparse_lds_chains(const ChainLaunch& L, const KParams& kp, int storage, int gradient,
                             int updater, int64_t max_nnz, hipStream_t stream, int* kernel_variant) {
    if (kp.n_chains <= 0) return 0;
    if (!sparse_lds_applies(kp.d, max_nnz, kp.n_max)) return -3;
    if (!L.wf32 || L.wstride < (int64_t)kp.d + 128 + 1024) return (int)hipErrorInvalidValue;
    if (kp.tol > 0.0 && !L.wnsq0) return (int)hipErrorInvalidValue;
    if (lds_depth() == 8 && kp.tol <= 0.0) return lds_launch<8, float>(L, kp, storage, gradient, updater, stream, kernel_variant);
    return lds_launch<4, float>(L, kp, storage, gradient, updater, stream, kernel_variant);
}

bool sparse_lds64_applies(int64_t d, int64_t max_nnz, int updater, bool check_conv, bool alpha_ok, int64_t n_max) {
    (void)check_conv;   // any tol: the per-sample break is a CONV instance (kp.tol > 0)
    if (max_nnz > LCAP || n_max > (int64_t)INT32_MAX) return false;
    if (updater != U_SIMPLE && !(updater == U_SQUARED_L2 && alpha_ok)) return false;
    return (lds_depth() == 8 ? lds_head<8, double>(d) : lds_head<4, double>(d)) >= 0;
}

int launch_sparse_lds64_chains(const ChainLaunch& L, const KParams& kp, int storage, int gradient,
                               int updater, int64_t max_nnz, hipStream_t stream, int* kernel_variant) {
    if (kp.n_chains <= 0) return 0;
    if (!sparse_lds64_applies(kp.d, max_nnz, updater, false, kp.alpha_ok != 0, kp.n_max)) return -3;
    // the chain's f64 vector: [d] + [128] + [1024] doubles inside its slice of L.wf32
    if (!L.wf32 || L.wstride < 2 * ((int64_t)kp.d + 128 + 1024) || (L.wstride & 3) || !L.w_out)
        return (int)hipErrorInvalidValue;
    if (kp.tol > 0.0) {
        // ||w_in||^2 for the per-sample break's norm recurrence
        if (!L.wnsq0) return (int)hipErrorInvalidValue;
        const int e = launch_wnsq0(L, kp.d, false, stream);
        if (e) return e;
    }
    if (lds_depth() == 8 && kp.tol <= 0.0) return lds_launch<8, double>(L, kp, storage, gradient, updater, stream, kernel_variant);
    return lds_launch<4, double>(L, kp, storage, gradient, updater, stream, kernel_variant);
}

#endif  // PSGD_NO_DISPATCH

}  // namespace psgd
