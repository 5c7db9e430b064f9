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
// [0, K) live in LDS ("head"); when d does not fit, features [K, d) ("tail") stay in the chain's
// vector in HBM (L.wf32), 4 (d - K) bytes per chain instead of 4 d -- at rcv1 shape (d = 47,236)
// ~100 KB, so 32 chains per XCD fit its 4 MiB L2 where whole vectors did not.
//   * head entries: the chain reads w_j from LDS at the sample and writes the new value back
//     (one wave's LDS operations execute in program order, so row t+1 reads row t's update);
//   * tail entries: gathered from HBM SK + 1 rows ahead by the tail wave into the row's LDS slot,
//     and corrected: a per-feature tag table over the tail (2 B per tail feature: (row & 255) << 8
//     | entry of the latest row holding the feature) names the latest of the SK preceding rows
//     with the same feature, whose new value the chain left in that row's slot in place of x_j;
//     such entries read that value and are not gathered. Tags never alias: the tagger sweeps
//     1/128 of the table per row and clears tags older than SK rows, so no tag outlives 256 rows.
// Four waves, one per SIMD, each a short branch-free loop (two when every feature is in LDS):
//   wave 0 (chain)  per sample t: one LDS read per entry at the address the tail wave (or the
//                   loader) wrote, dot + wave reduction + coefficient, one LDS write per entry;
//                   no VMEM at all -- the next sample's slot data is read under this one's latency;
//   wave 1 (loader) the partition's CSR entries into an SR-slot LDS ring (16 rows of loads in
//                   flight in registers, 8-row groups), labels / steps / nnz into a 128-row meta
//                   ring, 64 rows per batch;
//   wave 2 (tagger) per row: sweep a tag chunk, the tail entries' tag lookups + updates (the raw
//                   tags into the slot);
//   wave 3 (tail)   per row: the row's tail stores once the chain has its new values, a later
//                   row's LDS read / write addresses and its uncorrected tail gathers, an earlier
//                   row's gathered values into its slot.
// Rows are published through LDS counters: loaded (loader), tagged (tagger), ready (tail wave),
// done (chain), stored (tail wave).
// No MFMA: the work per sample is a ~100-long gather-dot and scatter.
#include "psgd_device.h"

#include <stddef.h>
#include <stdlib.h>

namespace psgd {

constexpr int LCAP = 128;                  // entries per row (two per lane)

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

// The ring of row slots (entries, addresses, gathered tail weights): row u's slot is reused for
// row u + SR once the chain has read row u (the tail wave and the tagger are done with a row
// before the chain may run it). The tail wave prepares row i + SK + 1 while the chain is at row
// i + 1: SR > SK + 2 plus the loader's slack.
// The ring of new tail weights (the chain's writes of a row's tail entries, read by the SK rows
// after it as corrections and by the tail wave for the row's stores): row t's entry is rewritten
// by row t + NVR once the tail wave has issued row t's stores (NVR > SK).
template <int SK>
struct LdsRing {
    static constexpr int SR = 16;
    static constexpr int NVR = 16;
    static_assert(SR >= SK + 6 && NVR > SK, "rings too small for the speculation depth");
};

struct LdsHeader {
    unsigned loaded;   // rows whose entries are in their slots (loader)
    unsigned tagged;   // rows whose raw tail tags are in their slots (tagger)
    unsigned ready;    // rows the chain may run: LDS addresses and gathered tail weights in their
                       // slots (tail wave; the loader when every feature is in LDS)
    unsigned done;     // rows finished by the chain
    unsigned stored;   // rows whose tail stores the tail wave has issued (their new-weight ring
                       // entries may be rewritten); kStoredAll: all landed
    unsigned stop;     // set by a watchdog only (normal completion needs no stop)
    unsigned dtag;     // target of inactive lanes' tag reads and writes
    unsigned pad0;
    unsigned zero[2];  // read by inactive entries: always 0 (never written)
    unsigned dummy[2]; // written by inactive entries
    unsigned pad[4];
};
constexpr unsigned kLdsZero = 8;           // dword index of LdsHeader::zero (8-byte aligned)
constexpr unsigned kLdsDummy = 10;         // dword index of LdsHeader::dummy (8-byte aligned)
constexpr unsigned kStoredAll = 0x7FFFFFFFu;
static_assert(sizeof(LdsHeader) == 64, "header layout");

template <typename T>
struct LdsMeta {
    T y[kMetaRing];
    T s[kMetaRing];           // stepSize / sqrt(j) (rounded to fp32 in fp32 compute)
    double s64[kMetaRing];    // the same in f64 (SquaredL2's alpha)
    int32_t nnz[kMetaRing];
};
template <typename T, bool TAIL>
struct LdsSlot {
    int32_t col[LCAP];   // feature index; fp32: the tail wave's gathered weights of the tail entries
                         // without correction replace it (nobody reads a row's columns after the
                         // tail wave has prepared it)
    T val[LCAP];         // x_j
    uint32_t rw[LCAP];   // the tagger's raw tag of a tail entry's feature, then LDS dword
                         // addresses: read (bits 0-15) | write (bits 16-31)
    T g[TAIL && sizeof(T) == 8 ? LCAP : 16 / sizeof(T)];   // fp64: the gathered weights (8 B each)
};
// the new tail weights of NVR rows
template <typename T>
struct LdsNv {
    T nv[LCAP];
};
constexpr int64_t kMetaOff = sizeof(LdsHeader);
template <typename T>
constexpr int64_t slot_off() { return kMetaOff + (int64_t)sizeof(LdsMeta<T>); }
static_assert(slot_off<float>() % 16 == 0 && sizeof(LdsSlot<float, true>) % 16 == 0, "alignment");
static_assert(slot_off<double>() % 16 == 0 && sizeof(LdsSlot<double, true>) % 16 == 0, "alignment");

template <int SK, typename T, bool TAIL>
constexpr int64_t nv_off() { return slot_off<T>() + LdsRing<SK>::SR * (int64_t)sizeof(LdsSlot<T, TAIL>); }
template <int SK, typename T, bool TAIL>
constexpr int64_t lds_fixed_bytes() {
    return (nv_off<SK, T, TAIL>() + (TAIL ? LdsRing<SK>::NVR * (int64_t)sizeof(LdsNv<T>) : 0) + 15) / 16 * 16;
}
// tail tag table entries (u16), rounded for the sweep's 4-tag accesses
__host__ __device__ inline int64_t tag_entries(int64_t d, int64_t K) { return ((d - K) + 3) & ~int64_t(3); }
template <int SK, typename T>
int64_t lds_bytes(int64_t d, int64_t K) {
    if (K >= d) return lds_fixed_bytes<SK, T, false>() + (int64_t)sizeof(T) * d;
    return lds_fixed_bytes<SK, T, true>() + (int64_t)sizeof(T) * K + 2 * tag_entries(d, K);
}
// Features [0, K) in LDS: all of them when they fit, else as many as leave room for the tail's
// tag table (K a multiple of 4: the table stays 8-byte aligned); -1 when not even the table fits.
template <int SK, typename T>
int64_t lds_head(int64_t d) {
    if ((int64_t)sizeof(T) * d <= kLdsCap - lds_fixed_bytes<SK, T, false>()) return d;
    const int64_t budget = kLdsCap - lds_fixed_bytes<SK, T, true>();
    int64_t K = (budget - 2 * (d + 4)) / ((int64_t)sizeof(T) - 2);
    K &= ~int64_t(3);
    return K >= 0 ? K : -1;
}

// TAIL = false: every feature is in LDS (K = d); two waves (chain, loader), no VMEM on the chain.
// TAIL = true: features [K, d) in HBM; four waves: chain, loader, tagger, tail. The chain wave
// issues no VMEM either way: every weight it reads is in LDS (the head, an earlier row's new value,
// or a tail weight the tail wave gathered into the row's slot).
// T: the weights' and the arithmetic's type (float: the fp32 throughput mode; double: fp64).
template <typename S, typename T, int GRAD, int UPD, int SK, bool TAIL>
__global__ __launch_bounds__(TAIL ? 256 : 128) void chain_sparse_lds(ChainLaunch L, KParams kp, int K) {
    constexpr bool L2 = UPD == U_SQUARED_L2;
    constexpr bool F64 = sizeof(T) == 8;
    constexpr int SR = LdsRing<SK>::SR;
    constexpr int NVR = LdsRing<SK>::NVR;
    constexpr unsigned WD = sizeof(T) / 4;                       // dwords per weight
    constexpr int64_t kSlotOff = slot_off<T>();
    using Slot = LdsSlot<T, TAIL>;
    static_assert((SR & (SR - 1)) == 0, "slot index by mask");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    LdsHeader* hdr = reinterpret_cast<LdsHeader*>(smem);
    LdsMeta<T>* meta = reinterpret_cast<LdsMeta<T>*>(smem + kMetaOff);
    Slot* slots = reinterpret_cast<Slot*>(smem + kSlotOff);
    float* lds = reinterpret_cast<float*>(smem);                 // dword-addressed view
    // a weight (or a slot's value) at dword index i
    auto ld_w = [&](unsigned i) __attribute__((always_inline)) -> T { return *reinterpret_cast<const T*>(lds + i); };
    auto st_w = [&](unsigned i, T v) __attribute__((always_inline)) { *reinterpret_cast<T*>(lds + i) = v; };
    constexpr unsigned kWoff = (unsigned)(lds_fixed_bytes<SK, T, TAIL>() / 4);
    T* W = reinterpret_cast<T*>(lds + kWoff);                    // head weights [K]
    uint16_t* tagpos = reinterpret_cast<uint16_t*>(W + K);       // tail features K .. d-1
    // dword index of val[0] / g[0] of the slot holding row u
    auto slot_dw = [](int32_t u) __attribute__((always_inline)) -> unsigned {
        return (unsigned)((kSlotOff + (int64_t)(u & (SR - 1)) * (int64_t)sizeof(Slot)) / 4);
    };
    // gathered tail weights: fp32 in place of the row's columns, fp64 in g
    constexpr unsigned kGDw = (unsigned)((F64 ? offsetof(Slot, g) : offsetof(Slot, col)) / 4);
    // dword index of nv[0] of the new-weight ring entry of row t
    auto nv_dw = [](int32_t t) __attribute__((always_inline)) -> unsigned {
        return (unsigned)((nv_off<SK, T, TAIL>() + (int64_t)(t & (NVR - 1)) * (int64_t)sizeof(LdsNv<T>)) / 4);
    };
    LdsNv<T>* nvring = reinterpret_cast<LdsNv<T>*>(smem + nv_off<SK, T, TAIL>());
    // K's bit 30 (PSGD_LDS_PROBE=1, diagnostics only): the tail wave's stores and gathers touch no
    // memory (wrong results; measures what the tail's memory traffic costs)
    const bool probe = ((K >> 30) & 1) != 0;
    K &= 0x3FFFFFFF;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int chain = blockIdx.x;
    const ChainDesc dsc = L.descs[chain];
    const int d = kp.d;
    // row indices run in 32-bit (the host runs this kernel only for n <= INT32_MAX); the CSR
    // offsets stay 64-bit (the loader's row_ptr values)
    const int32_t n = (int32_t)dsc.n_rows;
    const int32_t NT = TAIL ? (int32_t)tag_entries(d, K) : 0;
    // The chain runs n_pad samples (a multiple of its unroll) and reads row t + 1 at sample t:
    // the other waves stage n_fill rows, rows past n null (no entries, label and step 0), so no
    // read in the chain needs a condition.
    constexpr int GS = 2;
    const int32_t n_pad = (n + GS - 1) / GS * GS;
    const int32_t n_fill = (n_pad + 1 + 7) / 8 * 8;
    // [d] (tail used) + [128] the loader's dummy sources + [1024] spare (in T: for doubles the
    // chain's slice of L.wf32 is twice as long, launch_sparse_lds64_chains)
    T* V = reinterpret_cast<T*>(L.wf32 + (int64_t)chain * L.wstride);
    constexpr unsigned kShift = F64 ? 3 : 2;

    for (int32_t i = threadIdx.x; i < NT; i += blockDim.x) tagpos[i] = 0xFFFF;
    for (int i = threadIdx.x; i < K; i += blockDim.x) W[i] = T(as_global(L.w_in)[i]);
    if (threadIdx.x < 16) reinterpret_cast<unsigned*>(hdr)[threadIdx.x] = 0;
    if constexpr (F64 && TAIL) {
        // the tail V[K, d) starts as w_in; the tail wave's gathers (sc1, through L2) must see it
        for (int i = K + threadIdx.x; i < d; i += blockDim.x) V[i] = as_global(L.w_in)[i];
        __threadfence();
    }
    // (fp32: the tail V[K, d) starts as float(w_in), wf32_init_kernel launched before this kernel)
    __syncthreads();

    uint64_t st_wait = 0;                     // diagnostic (PSGD_STAMPS): cycles spent waiting
    const uint64_t st_begin = __builtin_amdgcn_s_memtime();
    // wait until *flag >= need (cached in `seen`); false when the watchdog fired (here or in
    // another wave)
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
            L.stamps[(size_t)chain * 16 + 2 * k] = __builtin_amdgcn_s_memtime() - st_begin;
            L.stamps[(size_t)chain * 16 + 2 * k + 1] = st_wait;
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
                G.ca[q] = *(ia ? &COL[ka] : dummy_i);
                G.xa[q] = *(ia ? &X[ka] : dummy_s);
                G.cb[q] = *(ic ? &COL[kc] : dummy_i);
                G.xb[q] = *(ic ? &X[kc] : dummy_s);
                G.ia[q] = ia;
                G.ic[q] = ic;
            }
        };
        // rows u0 .. u0 + 7 (those < n_fill) into their slots, each once its slot's previous row
        // u - SR is released (the chain has read it), published row by row
        auto stage_group = [&](int32_t u0, const Group& G) __attribute__((always_inline)) -> bool {
            bool good = true;
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int32_t u = u0 + q;
                if (good && u < n_fill) {
                    good = wait_for(done, &hdr->done, u - SR + 1, 16);
                    Slot& sl = slots[u & (SR - 1)];
                    sl.col[lane] = G.ca[q];
                    sl.col[lane + 64] = G.cb[q];
                    sl.val[lane] = G.ia[q] ? T(G.xa[q]) : T(0);
                    sl.val[lane + 64] = G.ic[q] ? T(G.xb[q]) : T(0);
                    if constexpr (!TAIL) {
                        // every feature in LDS: the entry's read and write address is W[j] (no
                        // tagger, no tail wave); inactive entries read the zero pair and write
                        // the dummy pair
                        const unsigned ha = kWoff + WD * (unsigned)G.ca[q], hb = kWoff + WD * (unsigned)G.cb[q];
                        sl.rw[lane] = G.ia[q] ? ha | (ha << 16) : kLdsZero | (kLdsDummy << 16);
                        sl.rw[lane + 64] = G.ic[q] ? hb | (hb << 16) : kLdsZero | (kLdsDummy << 16);
                        publish(&hdr->ready, u + 1);
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

    if constexpr (TAIL) {
    if (wave == 2) {
        // ---------------- tagger: the tail features' latest rows ----------------
        // Per row, for each tail entry, the tag of its feature -- (row & 255) << 8 | entry of the
        // latest row that held it -- is read (into the slot's rw word, for the tail wave) and
        // replaced by this row's. Four rows per step, so that their LDS round trips overlap: the
        // rows' columns, then the sweeps, then each row's lookups and updates in row order (one
        // wave's LDS operations execute in program order, so row u+1's lookups see row u's
        // updates), then the raw tags into the slots.
        constexpr int TB = 4;
        unsigned loaded = 0;
        uint16_t* dtag = reinterpret_cast<uint16_t*>(&hdr->dtag);
        const int32_t chunk = ((NT + kSweepRows - 1) / kSweepRows + 255) & ~int32_t(255);
        static_assert(8 % TB == 0, "n_fill is a multiple of TB");
        for (int32_t u0 = 0; u0 < n_fill; u0 += TB) {
            if (!wait_for(loaded, &hdr->loaded, u0 + TB, 32)) break;
            int nnz[TB];
            int32_t ca[TB], cb[TB];
#pragma unroll
            for (int q = 0; q < TB; ++q) {
                const int32_t u = u0 + q;
                const Slot& sl = slots[u & (SR - 1)];
                nnz[q] = meta->nnz[u & (kMetaRing - 1)];
                ca[q] = sl.col[lane];
                cb[q] = sl.col[lane + 64];
            }
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
                Slot& sl = slots[(u0 + q) & (SR - 1)];
                sl.rw[lane] = va[q];
                sl.rw[lane + 64] = vb[q];
            }
            publish(&hdr->tagged, u0 + TB);
        }
        stamp_out(2);
        return;
    }

    if (wave == 3) {
        // ---------------- tail wave: the tail's HBM traffic, off the chain ----------------
        // Iteration i (one per row, i from -A):
        //   1. row i + 3's gathered weights into its slot (issued WB iterations ago), publish
        //      `ready` (the chain at row t needs row t + 1); first, so that the chain never waits
        //      behind this iteration's wait for it;
        //   2. row i's new tail weights (the chain's writes into the new-weight ring) once the
        //      chain is done with row i;
        //   3. row u = i + A's LDS addresses from its raw tags, row i's tail stores, and the
        //      gathers of row u's tail entries that no row in u - SK .. u - 1 corrects. The gather
        //      follows this wave's stores of rows <= u - SK - 1 in program order, so L2 serves it
        //      after them (sc1 loads); rows u - SK .. u - 1 are the correction window (their new
        //      values, in LDS).
        // Each iteration issues exactly 2 + 2 VMEM instructions (no-access offsets where there is
        // nothing to move), so the vmcnt of step 1 is a constant.
        constexpr int A = SK + 1;
        constexpr int WB = A - 3;   // iterations a gather has to land
        static_assert(WB >= 2, "speculation depth too small for the tail wave's pipeline");
        const i32x4 vrs = buffer_rsrc(reinterpret_cast<const float*>(V), (uint32_t)((int64_t)d * sizeof(T)));
        unsigned done = 0, tagged = 0;
        bool ok = true;
        T gr[A][2];
        uint32_t so[A][2];
#pragma unroll
        for (int q = 0; q < A; ++q) so[q][0] = so[q][1] = kNoAccess;
        // The slot data of row u that its addresses and gathers need, read one iteration ahead
        // (unconditionally, past a spin-only branch: rows past n_fill read a live slot and count
        // as empty).
        struct Pre { int nz; int32_t c[2]; unsigned v[2]; };
        auto pre_read = [&](int32_t u) __attribute__((always_inline)) -> Pre {
            if (u < n_fill && (int32_t)tagged < u + 1) ok = ok && wait_for(tagged, &hdr->tagged, u + 1, 256);
            const Slot& sl = slots[u & (SR - 1)];
            return Pre{meta->nnz[u & (kMetaRing - 1)], {sl.col[lane], sl.col[lane + 64]}, {sl.rw[lane], sl.rw[lane + 64]}};
        };
        // row u's read / write addresses into its slot; its gather and store offsets
        // Branch-free (selects on 32-bit values, the row's constants uniform).
        auto prepare = [&](int32_t u, const Pre& P, uint32_t (&go)[2], uint32_t (&sv)[2]) __attribute__((always_inline)) {
            const int nz = u < n_fill ? P.nz : 0;
            const unsigned gb = slot_dw(u) + kGDw;            // this row's gathered weights
            const unsigned wb = nv_dw(u);                      // this row's new-weight entry
            constexpr unsigned kNvW = (unsigned)(sizeof(LdsNv<T>) / 4);
            constexpr unsigned kNv0 = (unsigned)(nv_off<SK, T, TAIL>() / 4);
            unsigned rwv[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const unsigned e = (unsigned)(lane + 64 * h);
                const unsigned c = (unsigned)P.c[h], v = P.v[h];
                const unsigned dl = ((unsigned)u - (v >> 8)) & 255;
                const bool prev = (v != 0xFFFFu) & (dl - 1u < (unsigned)SK);
                const bool act = e < (unsigned)nz, tail = c >= (unsigned)K;
                const unsigned head = kWoff + WD * c;
                const unsigned nvp = kNv0 + (((unsigned)u - dl) & (NVR - 1)) * kNvW + WD * (v & 255);
                const unsigned rt = prev ? nvp : gb + WD * e;
                const unsigned rd = act ? (tail ? rt : head) : kLdsZero;
                const unsigned wr = act ? (tail ? wb + WD * e : head) : kLdsDummy;
                const unsigned off = probe ? kNoAccess : c << kShift;
                const bool at = act & tail;
                sv[h] = at ? off : kNoAccess;
                go[h] = (at & !prev) ? off : kNoAccess;
                rwv[h] = rd | (wr << 16);
            }
            if (u < n_fill) {
                Slot& sl = slots[u & (SR - 1)];
                sl.rw[lane] = rwv[0];
                sl.rw[lane + 64] = rwv[1];
            }
        };
        Pre pre = pre_read(0);
        // PSGD_STAMPS: cycles of the iteration's phases (vmcnt wait of step 1, the new-weight read
        // before the stores, prepare + VMEM issue, the next row's prefetch)
        uint64_t ph[4] = {0, 0, 0, 0};
        auto tick = [&](int k, uint64_t& m) __attribute__((always_inline)) {
            if (L.stamps) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                const uint64_t now = __builtin_amdgcn_s_memtime();
                ph[k] += now - m;
                m = now;
            }
        };
        auto iteration = [&](auto qc, int32_t i) __attribute__((always_inline)) {
            uint64_t mark = L.stamps ? __builtin_amdgcn_s_memtime() : 0;
            constexpr int Q = decltype(qc)::value;            // i mod A (rows i and i + A)
            constexpr int QW = (Q + 3) % A;                   // (i + 3) mod A
            // 1. row i + 3's gathered weights into its slot, publish it: first, so that the
            //    chain's next rows never wait behind this iteration's wait for the chain. They were
            //    issued at iteration i + 3 - A; 4 (WB - 1) VMEM instructions came after them.
            const int32_t r = i + 3;
            if (r >= 0 && r < n_fill) {
                asm volatile("s_waitcnt vmcnt(%2)" : "+v"(gr[QW][0]), "+v"(gr[QW][1]) : "i"(4 * (WB - 1)) : "memory");
                tick(0, mark);
                T* gdst = reinterpret_cast<T*>(lds + slot_dw(r) + kGDw);
                gdst[lane] = gr[QW][0];
                gdst[lane + 64] = gr[QW][1];
                publish(&hdr->ready, r + 1);
            }
            // 2. row i's new tail weights, once the chain has them (read unconditionally: rows
            //    before 0 have no-access store offsets)
            if (i >= 0 && i < n_pad && (int32_t)done < i + 1) ok = ok && wait_for(done, &hdr->done, i + 1, 128);
            const LdsNv<T>& nr = nvring[i & (NVR - 1)];
            const T nv0 = nr.nv[lane], nv1 = nr.nv[lane + 64];
            if (L.stamps) { tick(3, mark); asm volatile("" : : "v"(nv0), "v"(nv1)); tick(1, mark); }
            // 3. row u = i + A's addresses and offsets (under the read above), then row i's
            //    stores and row u's gathers, in that order (the gathers must follow the stores of
            //    rows <= u - SK - 1 = i)
            const int32_t u = i + A;
            uint32_t go[2];
            const uint32_t s0 = so[Q][0], s1 = so[Q][1];
            prepare(u, pre, go, so[Q]);
            buffer_store_f32(vrs, s0, nv0);
            buffer_store_f32(vrs, s1, nv1);
            gr[Q][0] = buffer_gather_sc1(vrs, go[0], T(0));
            gr[Q][1] = buffer_gather_sc1(vrs, go[1], T(0));
            if (i >= 0) publish(&hdr->stored, i + 1);
            tick(2, mark);
            // the next row's slot data, in flight under the next iteration's first steps
            pre = pre_read(u + 1);
            tick(3, mark);
        };
        for (int32_t i0 = -A; ok && i0 < n_fill; i0 += A)
            static_for<A>([&](auto qc) {
                const int32_t i = i0 + decltype(qc)::value;
                if (ok && i < n_fill) iteration(qc, i);
            });
        // every store has landed before the chain reads the tail back (fp64) or the kernel ends
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int q = 0; q < A; ++q) asm volatile("" : : "v"(gr[q][0]), "v"(gr[q][1]));
        if (ok) publish(&hdr->stored, (int32_t)kStoredAll);
        stamp_out(3);
        if (L.stamps && lane == 0)
            for (int k = 0; k < 4; ++k) L.stamps[(size_t)chain * 16 + 8 + k] = ph[k];
        return;
    }
    }   // TAIL

    // ---------------- chain ----------------
    // Only LDS: per sample, one read per entry at its read address (head W[j]; an earlier row's
    // new value; the gathered tail weight; the zero pair), the dot, wave reduction and
    // coefficient, one write per entry at its write address (head W[j]; the slot, for the tail
    // wave's store and later rows' corrections; the dummy pair). Straight-line: the flag check
    // branches only to a spin, so no read result crosses a branch (a join would make the compiler
    // wait for it). Samples past n are null (no entries, no loss).
    double alpha = 1.0;       // SquaredL2: w = alpha * v
    double dnsq = 0.0;        // SquaredL2, fp32: ||v||^2 - ||v_0||^2 (this lane)
    double loss_sum = 0.0;
    float loss_blk = 0.0f;
    int64_t count = 0;
    unsigned ready = 0, stored = 0;
    bool ok = true;
    // rows < nr ready; with a tail, row t's new-weight ring entry free (row t - NVR stored)
    auto need = [&](int32_t nr, int32_t t) __attribute__((always_inline)) {
        nr = nr < n_fill ? nr : n_fill;
        if ((int32_t)ready < nr) ok = ok && wait_for(ready, &hdr->ready, nr, 2);
        if constexpr (TAIL)
            if ((int32_t)stored < t - NVR + 1) ok = ok && wait_for(stored, &hdr->stored, t - NVR + 1, 8);
    };
    // the data of sample t
    struct Row { T x0, x1; uint32_t rw0, rw1; T y, s; double s64; };
    auto row_of = [&](int32_t t) __attribute__((always_inline)) -> Row {
        const Slot& sl = slots[t & (SR - 1)];
        const int m = (int)(t & (kMetaRing - 1));
        return Row{sl.val[lane], sl.val[lane + 64], sl.rw[lane], sl.rw[lane + 64], meta->y[m], meta->s[m],
                   L2 ? meta->s64[m] : 0.0};
    };
    need(1, 0);
    Row cur = row_of(0);
    auto sample = [&](int32_t t) __attribute__((always_inline)) {
        need(t + 2, t);
        // this sample's weight reads (after the previous sample's writes, in program order) and
        // the data of sample t + 1, issued before anything waits (the scheduling barriers keep
        // the compiler from sinking the prefetch below the arithmetic)
        const T w0 = ld_w(cur.rw0 & 0xFFFF), w1 = ld_w(cur.rw1 & 0xFFFF);
        __builtin_amdgcn_sched_barrier(0);
        const Row nxt = row_of(t + 1);
        __builtin_amdgcn_sched_barrier(0);
        T acc = cur.x0 * w0;
        acc = m_fma(cur.x1, w1, acc);
        T z = wave_sum_uniform(acc);
        if constexpr (L2) {
            // w = alpha v: the dot is alpha (x . v); then the L2 shrink alpha *= 1 - s lambda
            // (SGDUpdater.scala:176) and the step adds c x_j / alpha to v
            z = T(alpha * double(z));
            alpha *= 1.0 - cur.s64 * kp.reg;
        }
        T c;
        if constexpr (F64) {
            // [ext] MLlib 1.6.1 Gradient.compute in Double (the loss included); c = -s * mult
            double mult;
            const double loss = gradient_scalar<GRAD, double>(z, cur.y, mult);
            c = -cur.s * mult;
            loss_sum += t < n ? loss : 0.0;
        } else {
            float loss;
            c = sparse_coef<GRAD>(z, cur.y, cur.s, loss);
            loss_blk += t < n ? loss : 0.0f;
            if ((t & 31) == 31) { loss_sum += double(loss_blk); loss_blk = 0.0f; }
        }
        const T cv = L2 ? T(double(c) / alpha) : c;
        const T nv0 = m_fma(cv, cur.x0, w0);
        const T nv1 = m_fma(cv, cur.x1, w1);
        if constexpr (L2 && !F64) dnsq += nsq_delta(w0, nv0) + nsq_delta(w1, nv1);
        st_w(cur.rw0 >> 16, nv0);
        st_w(cur.rw1 >> 16, nv1);
        publish(&hdr->done, t + 1);
        cur = nxt;
    };
    for (int32_t t = 0; ok && t < n_pad; t += GS)
        static_for<GS>([&](auto qc) { sample(t + decltype(qc)::value); });
    count = ok ? n : 0;
    stamp_out(0);
    loss_sum += double(loss_blk);
    if constexpr (GRAD == G_LEAST_SQUARES && !F64) loss_sum = loss_sum / 2.0;
    if constexpr (F64) {
        // w = alpha v into the chain's row of L.w_out (the f64 fold), regVal of the chain's last
        // update (PSGD.scala:257) from ||w||: the head from LDS, the tail from V once the tail
        // wave's stores have all landed (read through L2 like its gathers)
        double* wo = L.w_out + (int64_t)chain * d;
        double nsq = 0.0;
        for (int i = lane; i < K; i += 64) {
            const double wv = L2 ? alpha * W[i] : W[i];
            wo[i] = wv;
            if constexpr (L2) nsq += wv * wv;
        }
        if constexpr (TAIL) {
            ok = ok && wait_for(stored, &hdr->stored, (int32_t)kStoredAll, 2);
            const i32x4 vrs = buffer_rsrc(reinterpret_cast<const float*>(V), (uint32_t)((int64_t)d * sizeof(T)));
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
template <typename S, typename T, int GRAD, int SK>
static int lds_upd(const ChainLaunch& L, const KParams& kp, int upd, int K, size_t lds, hipStream_t st) {
    auto k = K < kp.d ? (upd == U_SIMPLE ? chain_sparse_lds<S, T, GRAD, U_SIMPLE, SK, true>
                                         : chain_sparse_lds<S, T, GRAD, U_SQUARED_L2, SK, true>)
                      : (upd == U_SIMPLE ? chain_sparse_lds<S, T, GRAD, U_SIMPLE, SK, false>
                                         : chain_sparse_lds<S, T, GRAD, U_SQUARED_L2, SK, false>);
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    static const bool probe = [] {
        const char* e = getenv("PSGD_LDS_PROBE");
        return e && *e == '1';
    }();
    hipLaunchKernelGGL(k, dim3(kp.n_chains), dim3(K < kp.d ? 256 : 128), lds, st, L, kp, probe ? K | (1 << 30) : K);
    return (int)hipGetLastError();
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

// Variant 600 + 10 (SK == 4) + 20 (fp64 compute) + storage (1: f32 rows).
template <int SK, typename T>
static int lds_launch(const ChainLaunch& L, const KParams& kp, int storage, int gradient, int updater,
                      hipStream_t stream, int* kernel_variant) {
    int64_t K = lds_head<SK, T>(kp.d);
    if (K < 0) return -3;
    // tests: PSGD_SPARSE_LDS_HEAD=k caps the LDS-resident head (exercises the tail at small d)
    if (const char* e = getenv("PSGD_SPARSE_LDS_HEAD"))
        if (*e) { const int64_t cap = atoll(e) & ~int64_t(3); if (cap >= 0 && cap < K) K = cap; }
    const size_t lds = (size_t)lds_bytes<SK, T>(kp.d, K);
    if (kernel_variant) *kernel_variant = 600 + (SK == 4 ? 10 : 0) + (sizeof(T) == 8 ? 20 : 0) + storage;
    if (storage == 1) return lds_grad<float, T, SK>(L, kp, gradient, updater, (int)K, lds, stream);
    return lds_grad<double, T, SK>(L, kp, gradient, updater, (int)K, lds, stream);
}

// Speculation depth (the correction window, and the tail wave's gather lead SK + 1, which leaves
// its gathers SK - 2 rows to land): 8 rows by default; PSGD_SPARSE_SK=4 for A/B measurements and
// tests (read at every launch).
static int lds_depth() {
    const char* e = getenv("PSGD_SPARSE_SK");
    return (e && atoi(e) == 4) ? 4 : 8;
}

// The chain, loader and tagger waves keep row numbers in 32 bits (psgd_sparse_lds.hip: n): a
// partition of more than INT32_MAX rows (>= 32 GiB of 16-byte CSR rows, which fits in HBM) takes
// chain_sparse / chain_general instead.
bool sparse_lds_applies(int64_t d, int64_t max_nnz, int64_t n_max) {
    if (max_nnz > LCAP || n_max > (int64_t)INT32_MAX) return false;
    return (lds_depth() == 4 ? lds_head<4, float>(d) : lds_head<8, float>(d)) >= 0;
}

int64_t sparse_lds_head(int64_t d) { return lds_depth() == 4 ? lds_head<4, float>(d) : lds_head<8, float>(d); }

int launch_sparse_lds_chains(const ChainLaunch& L, const KParams& kp, int storage, int gradient,
                             int updater, int64_t max_nnz, hipStream_t stream, int* kernel_variant) {
    if (kp.n_chains <= 0) return 0;
    if (!sparse_lds_applies(kp.d, max_nnz, kp.n_max)) return -3;
    if (!L.wf32 || L.wstride < (int64_t)kp.d + 128 + 1024) return (int)hipErrorInvalidValue;
    if (lds_depth() == 4) return lds_launch<4, float>(L, kp, storage, gradient, updater, stream, kernel_variant);
    return lds_launch<8, float>(L, kp, storage, gradient, updater, stream, kernel_variant);
}

bool sparse_lds64_applies(int64_t d, int64_t max_nnz, int updater, bool check_conv, bool alpha_ok, int64_t n_max) {
    if (max_nnz > LCAP || check_conv || n_max > (int64_t)INT32_MAX) return false;
    if (updater != U_SIMPLE && !(updater == U_SQUARED_L2 && alpha_ok)) return false;
    return (lds_depth() == 4 ? lds_head<4, double>(d) : lds_head<8, double>(d)) >= 0;
}

int launch_sparse_lds64_chains(const ChainLaunch& L, const KParams& kp, int storage, int gradient,
                               int updater, int64_t max_nnz, hipStream_t stream, int* kernel_variant) {
    if (kp.n_chains <= 0) return 0;
    if (!sparse_lds64_applies(kp.d, max_nnz, updater, false, kp.alpha_ok != 0, kp.n_max)) return -3;
    // the chain's f64 vector: [d] + [128] + [1024] doubles inside its slice of L.wf32
    if (!L.wf32 || L.wstride < 2 * ((int64_t)kp.d + 128 + 1024) || (L.wstride & 3) || !L.w_out)
        return (int)hipErrorInvalidValue;
    if (lds_depth() == 4) return lds_launch<4, double>(L, kp, storage, gradient, updater, stream, kernel_variant);
    return lds_launch<8, double>(L, kp, storage, gradient, updater, stream, kernel_variant);
}

#endif  // PSGD_NO_DISPATCH

}  // namespace psgd
