// psgd_capi.cpp -- the C ABI declared in include/psgd.h: context, partition registry, epoch
// orchestration and error reporting. The chain/fold kernels live in psgd_kernels.hip.
//
// What this replaces in the reference (paths under /root/reference,
// src/main/scala/org/apache/spark/mllib/optimization/ParallelizedSGD.scala):
//   :238      sc.broadcast(weights)            -> weights stay in HBM (d_w_in)
//   :242      data.sample(false, frac, 42+i)   -> identity for frac >= 1 - 1e-6 (Spark's
//                                                 RandomSampler.roundingEpsilon), empty for
//                                                 frac <= 1e-6; otherwise PSGD_EUNSUPPORTED
//   :243-270  mapPartitions chain              -> one chain kernel launch over all partitions
//   :271-276  treeReduce combiner              -> fold kernel in partition-index order
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/psgd.h"
#include "psgd_internal.h"

namespace {

thread_local std::string g_last_error;

int32_t fail(int32_t code, const std::string& msg) {
    g_last_error = msg;
    return code;
}
}  // namespace

namespace psgd {
// psgd_last_error() for the other translation units of the library (psgd_libsvm.cpp)
int32_t set_error(int32_t code, const std::string& msg) { return fail(code, msg); }
}  // namespace psgd

namespace {

#define HIP_TRY(expr)                                                                        \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return fail(PSGD_EDEVICE, std::string("HIP error in ") + #expr + ": " +          \
                                          hipGetErrorString(e_));                            \
    } while (0)

size_t dtype_size(int32_t dt) { return dt == PSGD_F32 ? 4 : 8; }

struct Part {
    int64_t n_rows = 0;
    int32_t d = 0;
    int32_t dtype = PSGD_F64;
    int32_t layout = psgd::kDense;
    bool owned = false;
    void* x = nullptr;        // dense rows or CSR values
    double* y = nullptr;
    int64_t* row_ptr = nullptr;
    int32_t* col = nullptr;
    int64_t ld = 0;
    int64_t max_nnz = 0;      // CSR: the longest row
};

// Device buffer that only grows.
// The seeds of RDD.sample(false, f, seed) [ext Spark 1.6.1]: PartitionwiseSampledRDD draws one
// Long per partition, in partition order, from java.util.Random(seed); BernoulliSampler.setSeed
// seeds its XORShiftRandom with hashSeed(s) = scala MurmurHash3.bytesHash of the 64-byte
// ByteBuffer.allocate(java.lang.Long.SIZE).putLong(s) (Long.SIZE is in bits; an Int result,
// sign-extended). The device walks the XORShift sequence (psgd_kernels.hip, sample_kernel).
namespace sampling {
struct JavaRandom {
    uint64_t seed;
    explicit JavaRandom(int64_t s) : seed(((uint64_t)s ^ 0x5DEECE66DULL) & ((1ULL << 48) - 1)) {}
    int32_t next(int bits) {
        seed = (seed * 0x5DEECE66DULL + 0xBULL) & ((1ULL << 48) - 1);
        return (int32_t)(uint32_t)(seed >> (48 - bits));
    }
    int64_t next_long() {
        const int64_t hi = next(32);
        const int64_t lo = next(32);
        return (int64_t)((uint64_t)hi << 32) + lo;
    }
};
inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
inline int64_t xorshift_hash_seed(int64_t s) {
    uint32_t h = 0x3c074a61u;   // MurmurHash3.arraySeed
    for (int i = 0; i < 16; ++i) {
        // little-endian words of the big-endian Long followed by 56 zero bytes
        uint32_t k = 0;
        if (i < 2) {
            const uint64_t u = (uint64_t)s;
            const int sh = 56 - 32 * i;   // byte b of the buffer is (s >> (56 - 8 b)) & 0xff
            k = (uint32_t)((u >> sh) & 0xff) | ((uint32_t)((u >> (sh - 8)) & 0xff) << 8) |
                ((uint32_t)((u >> (sh - 16)) & 0xff) << 16) | ((uint32_t)((u >> (sh - 24)) & 0xff) << 24);
        }
        k *= 0xcc9e2d51u;
        k = rotl32(k, 15);
        k *= 0x1b873593u;
        h ^= k;
        h = rotl32(h, 13);
        h = h * 5u + 0xe6546b64u;
    }
    h ^= 64u;
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return (int64_t)(int32_t)h;
}
}  // namespace sampling

// PSGD_CONTIG=1: physically contiguous device memory (hipDeviceMallocContiguous) for the CSR
// kernels' per-chain weight vectors (A/B measurements; read at every allocation; falls back to
// hipMalloc when no contiguous range is free). Off by default: measured round 5, it made c5 fp32
// 1.4 % faster and steadier (107.2 ms against 108.7) but c4 31 -> 45 ms (fp32) and c5 fp64 95 -> 117 ms
// (the chains' vectors at a regular physical stride).
static bool contig_enabled() {
    const char* e = getenv("PSGD_CONTIG");
    return e && e[0] == '1';
}

// PSGD_VMM (default 1): the CSR kernels' per-chain weight vectors of 1 GiB or more are mapped
// through the virtual memory API -- physical handles of PSGD_VMM_CHUNK_MB at a 2 GiB-aligned
// virtual range --
// rather than hipMalloc'd. Their scattered stores' rate depends on the placement the driver gives
// the buffer (profiles/r05_c5_placement.log: ~65 or ~94 ms of stores per 20M c5
// rows); mapped this way the fast placement came up in 11 of 24 measured states, hipMalloc in 1.
static bool vmm_enabled() {
    const char* e = getenv("PSGD_VMM");
    return !(e && e[0] == '0');
}
// (PSGD_VMM_MIN_MB: the smallest set mapped this way, default 1024; A/B measurements)
static size_t vmm_min() {
    const char* e = getenv("PSGD_VMM_MIN_MB");
    const long mb = e && *e ? atol(e) : 1024;
    return (size_t)(mb >= 0 ? mb : 1024) << 20;
}
constexpr size_t kVmmAlign = size_t(2) << 30;
// the physical handles' size (PSGD_VMM_CHUNK_MB, default 2048; A/B measurements)
static size_t vmm_chunk() {
    const char* e = getenv("PSGD_VMM_CHUNK_MB");
    const long mb = e && *e ? atol(e) : 2048;
    return (size_t)(mb > 0 ? mb : 2048) << 20;
}

// Process-wide counters of the VMM mappings (psgd_vmm_stats): chunks mapped and unmapped, bytes
// currently mapped, and failed unmap / release / address-free calls (each also logged to stderr).
static std::atomic<int64_t> g_vmm_mapped{0}, g_vmm_unmapped{0}, g_vmm_live_bytes{0}, g_vmm_failures{0};

static void vmm_fail(const char* what, hipError_t e) {
    g_vmm_failures.fetch_add(1);
    fprintf(stderr, "psgd: %s failed while releasing a VMM buffer: %s\n", what, hipGetErrorString(e));
    (void)hipGetLastError();
}

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    bool fresh = false;   // allocated by the last ensure() (reroll_vectors consumes it)
    // a virtual-memory mapping (vmm_map): the reservation, the physical handles and, per handle,
    // the (offset, size) it is mapped at inside the aligned range -- unmapped one by one, as mapped
    void* vres = nullptr;
    size_t vres_bytes = 0;
    std::vector<hipMemGenericAllocationHandle_t> vh;
    std::vector<std::pair<size_t, size_t>> vmaps;
    hipError_t ensure(size_t need, bool contiguous = false) {
        if (need <= bytes) return hipSuccess;
        release();
        hipError_t e = hipErrorOutOfMemory;
        if (contiguous && contig_enabled()) {
            e = hipExtMallocWithFlags(&p, need, hipDeviceMallocContiguous);
            if (e != hipSuccess) {
                (void)hipGetLastError();
                p = nullptr;
            }
        } else if (contiguous && need >= vmm_min() && vmm_enabled()) {
            e = vmm_map(need);
            if (e != hipSuccess) {
                (void)hipGetLastError();
                release();
            }
        }
        if (e != hipSuccess && !p) e = hipMalloc(&p, need);
        if (e == hipSuccess) {
            bytes = need;
            fresh = true;
        }
        return e;
    }
    char* vmm_base() const {
        return reinterpret_cast<char*>(((uintptr_t)vres + kVmmAlign - 1) / kVmmAlign * kVmmAlign);
    }
    hipError_t vmm_map(size_t need) {
        int dev = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e) return e;
        hipMemAllocationProp prop = {};
        prop.type = hipMemAllocationTypePinned;
        prop.location.type = hipMemLocationTypeDevice;
        prop.location.id = dev;
        size_t gran = 0;
        e = hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended);
        if (e) return e;
        const size_t chunk = vmm_chunk();
        if (gran == 0 || chunk % gran || kVmmAlign % gran) return hipErrorNotSupported;
        const size_t total = (need + gran - 1) / gran * gran;
        // (the runtime does not honour a large alignment argument: reserve 2 GiB more and map at
        // the first 2 GiB-aligned address inside)
        vres_bytes = total + kVmmAlign;
        e = hipMemAddressReserve(&vres, vres_bytes, 0, nullptr, 0);
        if (e) {
            vres = nullptr;
            return e;
        }
        char* va = vmm_base();
        for (size_t off = 0; off < total; off += chunk) {
            const size_t sz = std::min(chunk, total - off);
            hipMemGenericAllocationHandle_t h;
            e = hipMemCreate(&h, sz, &prop, 0);
            if (e) return e;
            vh.push_back(h);
            e = hipMemMap(va + off, sz, 0, h, 0);
            if (e) return e;
            vmaps.emplace_back(off, sz);
            g_vmm_mapped.fetch_add(1);
            g_vmm_live_bytes.fetch_add((int64_t)sz);
        }
        hipMemAccessDesc acc = {};
        acc.location = prop.location;
        acc.flags = hipMemAccessFlagsProtReadWrite;
        e = hipMemSetAccess(va, total, &acc, 1);
        if (e) return e;
        p = va;
        return hipSuccess;
    }
    void release() {
        if (vres) {
            // each handle unmapped over exactly the range it was mapped at, every
            // return code checked (a failure is counted and logged, and the rest still released)
            char* va = vmm_base();
            for (const auto& m : vmaps) {
                const hipError_t e = hipMemUnmap(va + m.first, m.second);
                if (e) {
                    vmm_fail("hipMemUnmap", e);
                } else {
                    g_vmm_unmapped.fetch_add(1);
                    g_vmm_live_bytes.fetch_sub((int64_t)m.second);
                }
            }
            for (auto h : vh) {
                const hipError_t e = hipMemRelease(h);
                if (e) vmm_fail("hipMemRelease", e);
            }
            const hipError_t e = hipMemAddressFree(vres, vres_bytes);
            if (e) vmm_fail("hipMemAddressFree", e);
        } else if (p) {
            hipFree(p);
        }
        vh.clear();
        vmaps.clear();
        vres = nullptr;
        vres_bytes = 0;
        p = nullptr;
        bytes = 0;
    }
    template <typename T>
    T* as() const { return static_cast<T*>(p); }
};

// PSGD_REROLL (default 8): how many allocations a CSR vector set below the VMM threshold is chosen
// from (<= 1: the first). Measured round 6: the rate of the chains' scattered
// read-modify-writes over their vectors is a property of the allocation (c4: 27.4 or 31.3 ms for
// the same rows, by context), and a short probe of the same access pattern tells the two kinds
// apart; the context probes a few candidates once, when it allocates the set, and keeps the fastest.
static int reroll_candidates() {
    const char* e = getenv("PSGD_REROLL");
    const int k = e && *e ? atoi(e) : 8;
    return k < 1 ? 1 : (k > 16 ? 16 : k);
}
static std::atomic<int64_t> g_reroll_sets{0}, g_reroll_swaps{0};

// b holds n_vectors vectors of d_words used 4-byte words, stride_words apart. Replaces a freshly
// hipMalloc'd b by the fastest of reroll_candidates() allocations of its size under the probe of
// words [lo_words, d_words) of every vector -- the part past the LDS head, where the chains'
// scattered accesses go (probing the whole vector separated the two kinds of allocation by ~2.5 %,
// the tail alone by ~20 %: tools/place_probe.hip, profiles/r06_c4_placement.log).
static void reroll_vectors(DevBuf& b, int64_t stride_words, int n_vectors, int d_words, int lo_words,
                           hipStream_t st) {
    if (!b.fresh) return;
    b.fresh = false;
    const int K = reroll_candidates();
    if (K <= 1 || b.vres || !b.p || b.bytes >= vmm_min() || n_vectors <= 0) return;
    if (lo_words < 0 || lo_words >= d_words) lo_words = 0;
    std::vector<void*> cand{b.p};
    for (int k = 1; k < K; ++k) {
        void* q = nullptr;
        if (hipMalloc(&q, b.bytes) != hipSuccess) {
            (void)hipGetLastError();
            break;
        }
        cand.push_back(q);
    }
    hipEvent_t e0 = nullptr, e1 = nullptr;
    size_t best = 0;
    float best_ms = 0.0f;
    std::vector<float> ms(cand.size(), -1.0f);
    if (hipEventCreate(&e0) == hipSuccess && hipEventCreate(&e1) == hipSuccess) {
        for (size_t i = 0; i < cand.size(); ++i) {
            float* w = static_cast<float*>(cand[i]) + lo_words;
            const int span = d_words - lo_words;
            if (psgd::launch_vector_probe(w, stride_words, n_vectors, span, 256, 11u, st)) break;
            (void)hipEventRecord(e0, st);
            if (psgd::launch_vector_probe(w, stride_words, n_vectors, span, 2000, 12345u, st)) break;
            (void)hipEventRecord(e1, st);
            if (hipEventSynchronize(e1) != hipSuccess || hipEventElapsedTime(&ms[i], e0, e1) != hipSuccess) break;
            if (i == 0 || ms[i] < best_ms) {
                best = i;
                best_ms = ms[i];
            }
        }
    }
    (void)hipGetLastError();
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    (void)hipStreamSynchronize(st);   // no probe still runs on a candidate that is freed below
    for (size_t i = 0; i < cand.size(); ++i)
        if (i != best) (void)hipFree(cand[i]);
    b.p = cand[best];
    g_reroll_sets.fetch_add(1);
    if (best != 0) g_reroll_swaps.fetch_add(1);
    const char* lg = getenv("PSGD_REROLL_LOG");
    if (lg && lg[0] == '1') {
        fprintf(stderr, "psgd: vector set of %zu bytes, probe ms:", b.bytes);
        for (float m : ms) fprintf(stderr, " %.3f", m);
        fprintf(stderr, " -> kept %zu\n", best);
    }
}

// Pinned staging ring of the host -> HBM ingest (registration from pageable host memory):
// kStageSlots pinned buffers; the host packs chunk k + 1 into one while chunk k's DMA runs from
// another on the context's copy stream. One Stager per registering thread at a time.
constexpr int kStageSlots = 3;
constexpr size_t kStageChunk = size_t(8) << 20;
struct Stager {
    char* buf[kStageSlots] = {};
    size_t cap = 0;
    hipEvent_t ev[kStageSlots] = {};
    bool busy[kStageSlots] = {};
    int next = 0;
    hipError_t ensure(size_t need) {
        if (!ev[0])
            for (auto& e : ev) {
                hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableTiming);
                if (r) return r;
            }
        if (need <= cap) return hipSuccess;
        drain();
        for (auto& b : buf) {
            if (b) hipHostFree(b);
            b = nullptr;
        }
        cap = 0;
        for (auto& b : buf) {
            hipError_t r = hipHostMalloc((void**)&b, need, hipHostMallocDefault);
            if (r) return r;
        }
        cap = need;
        return hipSuccess;
    }
    // the next slot, once its previous DMA has drained
    hipError_t acquire(int& k) {
        k = next;
        next = (next + 1) % kStageSlots;
        if (busy[k]) {
            hipError_t r = hipEventSynchronize(ev[k]);
            if (r) return r;
            busy[k] = false;
        }
        return hipSuccess;
    }
    void drain() {
        for (int k = 0; k < kStageSlots; ++k)
            if (busy[k]) {
                hipEventSynchronize(ev[k]);
                busy[k] = false;
            }
    }
    void release() {
        drain();
        for (auto& b : buf)
            if (b) hipHostFree(b);
        for (auto& e : ev)
            if (e) hipEventDestroy(e);
        *this = Stager{};
    }
};

}  // namespace

struct psgd_ctx {
    int32_t device = 0;
    int32_t num_cus = 256;
    hipStream_t stream = nullptr;
    // Host -> HBM registration copies run on their own stream (they overlap epochs on `stream`
    // and the caller's packing of the next partition); an epoch waits for them on the device.
    hipStream_t copy_stream = nullptr;
    hipEvent_t copy_ev = nullptr;
    bool copies_pending = false;       // copies enqueued since the last epoch (under mu)
    std::mutex stage_mu;               // guards `stagers`
    std::vector<Stager*> stagers;      // idle staging rings
    std::mutex mu;
    std::map<int64_t, Part> parts;
    bool descs_dirty = true;
    DevBuf descs, w_in, w_out, state, rv, loss, cnt_d, cnt, steps, partial, tmp, watchdog, zbuf, wf32, stamps;
    DevBuf walpha, wnsq0;                // the fp32 CSR chains' weight scale and ||float(w_in)||^2
    DevBuf sdescs, srows, sys, xstate;   // sampled epochs (miniBatchFraction < 1)
    double steps_value = NAN;
    int64_t steps_n = 0;
    int32_t last_variant = 0;
    // HIP events around the last kChainEvents chain-kernel launches, launch k in slot
    // k % kChainEvents (psgd_ctx_last_chain_ms, psgd_ctx_chain_ms): a caller that keeps several
    // epochs in flight reads each launch's time after it has enqueued later ones
    static constexpr int kChainEvents = 64;
    hipEvent_t ev_begin[kChainEvents] = {}, ev_end[kChainEvents] = {};
    int64_t chain_launches = 0;
    // The scratch buffers above belong to the context, and epochs may run on different caller
    // streams: each user of them orders its stream after the previous user's work (this event,
    // recorded on `scratch_stream`) and records the event again when it has enqueued its own.
    hipEvent_t scratch_ev = nullptr;
    hipStream_t scratch_stream = nullptr;
    bool scratch_recorded = false;
    // alpha_in_range's cached answer
    int64_t alpha_n = -1;
    double alpha_step = NAN, alpha_reg = NAN;
    bool alpha_ok = false;
    // the fp64 CSR weight-vector size whose allocation failed (0: none): not retried
    size_t wf64_failed = 0;
};

namespace {

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        hipGetDevice(&prev);
        if (prev != dev) hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        hipGetDevice(&cur);
        if (prev >= 0 && cur != prev) hipSetDevice(prev);
    }
};

void free_part(Part& p) {
    if (!p.owned) return;
    if (p.x) hipFree(p.x);
    if (p.y) hipFree(p.y);
    if (p.row_ptr) hipFree(p.row_ptr);
    if (p.col) hipFree(p.col);
    p = Part{};
}

int32_t check_compat(psgd_ctx* ctx, int32_t d, int32_t dtype, int32_t layout) {
    for (auto& kv : ctx->parts) {
        const Part& q = kv.second;
        if (q.d != d)
            return fail(PSGD_EINVAL, "requirement failed: all partitions must have the same "
                                     "number of features (got " + std::to_string(d) + " and " +
                                         std::to_string(q.d) + ")");
        if (q.dtype != dtype || q.layout != layout)
            return fail(PSGD_EUNSUPPORTED,
                        "mixing dense/CSR rows or storage dtypes across partitions is not built");
    }
    return PSGD_OK;
}

bool multinomial(const psgd_params* p) {
    return p->gradient == PSGD_GRADIENT_LOGISTIC && p->num_classes > 2;
}

int32_t validate_params(const psgd_params* p) {
    if (!p) return fail(PSGD_EINVAL, "params is null");
    if (p->gradient < PSGD_GRADIENT_LOGISTIC || p->gradient > PSGD_GRADIENT_HINGE)
        return fail(PSGD_EINVAL, "unknown gradient kind " + std::to_string(p->gradient));
    if (p->updater < PSGD_UPDATER_SIMPLE || p->updater > PSGD_UPDATER_ADAM)
        return fail(PSGD_EINVAL, "unknown updater kind " + std::to_string(p->updater));
    if (p->compute_dtype != PSGD_F64 && p->compute_dtype != PSGD_F32)
        return fail(PSGD_EINVAL, "unknown compute dtype " + std::to_string(p->compute_dtype));
    // Spark 1.6.1 BernoulliSampler: require(fraction in [0 - eps, 1 + eps]) [ext].
    const double eps = 1e-6;
    if (!(p->mini_batch_fraction >= -eps && p->mini_batch_fraction <= 1.0 + eps)) {
        char buf[160];
        snprintf(buf, sizeof buf, "requirement failed: Sampling fraction (%g) must be on interval [0, 1]",
                 p->mini_batch_fraction);
        return fail(PSGD_EINVAL, buf);
    }
    if (multinomial(p)) {
        if (p->num_classes - 1 > psgd::kMultinomialMaxBlocks)
            return fail(PSGD_EUNSUPPORTED, "LogisticGradient(numClasses = " + std::to_string(p->num_classes) +
                                               ") exceeds the built maximum of " +
                                               std::to_string(psgd::kMultinomialMaxBlocks + 1) + " classes");
        if (p->compute_dtype != PSGD_F64)
            return fail(PSGD_EUNSUPPORTED, "the multinomial LogisticGradient computes in fp64 only");
    }
    return PSGD_OK;
}

// Length of the weight vector for rows of d features: (K - 1) * d for LogisticGradient(K > 2)
// (MLlib 1.6.1: require(weights.size % dataSize == 0 && numClasses == weights.size / dataSize + 1)).
int64_t weight_dim(int32_t d, const psgd_params* p) {
    return multinomial(p) ? (int64_t)(p->num_classes - 1) * d : (int64_t)d;
}

// ---- Host -> HBM ingest (RDD partition -> pinned buffers -> HBM) ----

struct StagerLease {
    psgd_ctx* ctx;
    Stager* s;
    explicit StagerLease(psgd_ctx* c) : ctx(c), s(nullptr) {
        std::lock_guard<std::mutex> lk(ctx->stage_mu);
        if (!ctx->stagers.empty()) {
            s = ctx->stagers.back();
            ctx->stagers.pop_back();
        }
        if (!s) s = new Stager();
    }
    ~StagerLease() {
        s->drain();   // its buffers are reused by the next registration
        std::lock_guard<std::mutex> lk(ctx->stage_mu);
        ctx->stagers.push_back(s);
    }
};

// True when p is page-locked host memory the device can DMA from directly (psgd_host_alloc, or
// any hipHostMalloc / hipHostRegister'ed buffer).
bool is_pinned(const void* p) {
    if (!p) return false;
    hipPointerAttribute_t a;
    const hipError_t e = hipPointerGetAttributes(&a, p);
    if (e != hipSuccess) {
        (void)hipGetLastError();   // pageable memory: not an error for us
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// Copy `bytes` to the device at `dst` on ctx->copy_stream. Pinned sources are DMA'd directly
// (and waited for: no host pointer outlives the call); pageable ones through the staging ring,
// in chunks of whole `unit`s: fill(stage, off, len) writes bytes [off, off + len) of the device
// image into the pinned chunk and returns false to abort (validation failure, message set).
// Returns with the last chunks' DMA possibly in flight from the library's own buffers.
template <class Fill>
int32_t stage_upload(psgd_ctx* ctx, Stager& S, void* dst, size_t bytes, size_t unit, Fill fill) {
    if (bytes == 0) return PSGD_OK;
    unit = std::max<size_t>(unit, 1);
    const size_t chunk = std::max(kStageChunk / unit, size_t(1)) * unit;
    HIP_TRY(S.ensure(chunk));
    for (size_t off = 0; off < bytes; off += chunk) {
        const size_t len = std::min(chunk, bytes - off);
        int k = 0;
        HIP_TRY(S.acquire(k));
        if (!fill(S.buf[k], off, len)) {
            S.drain();
            return PSGD_EINVAL;
        }
        HIP_TRY(hipMemcpyAsync(static_cast<char*>(dst) + off, S.buf[k], len, hipMemcpyHostToDevice,
                               ctx->copy_stream));
        HIP_TRY(hipEventRecord(S.ev[k], ctx->copy_stream));
        S.busy[k] = true;
    }
    return PSGD_OK;
}

// A contiguous host array to the device: direct DMA when pinned, else staged.
int32_t upload(psgd_ctx* ctx, Stager& S, void* dst, const void* src, size_t bytes) {
    if (bytes == 0) return PSGD_OK;
    if (is_pinned(src)) {
        HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->copy_stream));
        return PSGD_OK;
    }
    const char* s = static_cast<const char*>(src);
    return stage_upload(ctx, S, dst, bytes, 1, [&](char* st, size_t off, size_t len) {
        std::memcpy(st, s + off, len);
        return true;
    });
}

// Wait for the direct (pinned-source) DMAs of this call: the caller may reuse its buffers.
int32_t finish_direct(psgd_ctx* ctx, bool any_direct) {
    if (!any_direct) return PSGD_OK;
    HIP_TRY(hipStreamSynchronize(ctx->copy_stream));
    return PSGD_OK;
}

// Order `st` after the last work enqueued on the context's scratch buffers from another stream
// (ctx->mu held).
int32_t scratch_acquire(psgd_ctx* ctx, hipStream_t st) {
    if (ctx->scratch_recorded && ctx->scratch_stream != st)
        HIP_TRY(hipStreamWaitEvent(st, ctx->scratch_ev, 0));
    return PSGD_OK;
}
// `st` now holds the newest work on the scratch buffers (ctx->mu held).
int32_t scratch_release(psgd_ctx* ctx, hipStream_t st) {
    if (!ctx->scratch_ev) HIP_TRY(hipEventCreateWithFlags(&ctx->scratch_ev, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(ctx->scratch_ev, st));
    ctx->scratch_stream = st;
    ctx->scratch_recorded = true;
    return PSGD_OK;
}

// Allocate per-chain buffers and upload descriptors (ctx->mu held).
int32_t prepare(psgd_ctx* ctx, int32_t d, int state_vectors, hipStream_t st) {
    const size_t P = ctx->parts.size();
    {
        const int32_t rc = scratch_acquire(ctx, st);
        if (rc) return rc;
    }
    if (ctx->copies_pending) {
        // registration copies still in flight on the copy stream: the epoch waits on the device
        HIP_TRY(hipEventRecord(ctx->copy_ev, ctx->copy_stream));
        HIP_TRY(hipStreamWaitEvent(st, ctx->copy_ev, 0));
        ctx->copies_pending = false;
    }
    HIP_TRY(ctx->descs.ensure(std::max<size_t>(P, 1) * sizeof(psgd::ChainDesc)));
    HIP_TRY(ctx->w_in.ensure((size_t)std::max(d, 1) * sizeof(double)));
    HIP_TRY(ctx->w_out.ensure(std::max<size_t>(P, 1) * (size_t)std::max(d, 1) * sizeof(double)));
    HIP_TRY(ctx->rv.ensure(std::max<size_t>(P, 1) * sizeof(double)));
    HIP_TRY(ctx->loss.ensure(std::max<size_t>(P, 1) * sizeof(double)));
    HIP_TRY(ctx->cnt_d.ensure(std::max<size_t>(P, 1) * sizeof(double)));
    HIP_TRY(ctx->cnt.ensure(std::max<size_t>(P, 1) * sizeof(int64_t)));
    HIP_TRY(ctx->partial.ensure(((size_t)std::max(d, 1) + 3) * sizeof(double)));
    HIP_TRY(ctx->tmp.ensure(((size_t)std::max(d, 1) + 8) * sizeof(double)));
    if (!ctx->watchdog.p) {
        // zeroed once: from then on every epoch's fold kernel clears the flags it has read
        HIP_TRY(ctx->watchdog.ensure(16));
        HIP_TRY(hipMemsetAsync(ctx->watchdog.p, 0, 16, st));
    }
    if (state_vectors > 0)
        HIP_TRY(ctx->state.ensure(std::max<size_t>(P, 1) * (size_t)state_vectors *
                                  (size_t)std::max(d, 1) * sizeof(double)));
    if (ctx->descs_dirty) {
        std::vector<psgd::ChainDesc> h;
        h.reserve(P);
        for (auto& kv : ctx->parts) {
            const Part& q = kv.second;
            psgd::ChainDesc c;
            c.x = q.x;
            c.y = q.y;
            c.row_ptr = q.row_ptr;
            c.col = q.col;
            c.n_rows = q.n_rows;
            c.ld = q.ld;
            c.rows = nullptr;   // every row (sampled epochs get descriptors of their own)
            h.push_back(c);
        }
        if (P) {
            HIP_TRY(hipMemcpyAsync(ctx->descs.p, h.data(), P * sizeof(psgd::ChainDesc),
                                   hipMemcpyHostToDevice, st));
            HIP_TRY(hipStreamSynchronize(st));
        }
        ctx->descs_dirty = false;
    }
    return PSGD_OK;
}

// SquaredL2's alpha-scaled CSR form without renormalisation (the fp64 chain_sparse_lds) is
// valid when every prefix product of (1 - s_j lambda), s_j = stepSize / sqrt(j) as the steps
// kernel computes it, stays finite, non-zero and in [2^-400, 2^400] (chain_general's
// renormalisation bounds) for j up to the longest chain. Cached per (step, lambda, n).
bool alpha_in_range(psgd_ctx* ctx, double step, double reg, int64_t n) {
    if (ctx->alpha_n == n && ctx->alpha_step == step && ctx->alpha_reg == reg) return ctx->alpha_ok;
    double a = 1.0;
    bool ok = true;
    for (int64_t j = 1; j <= n && ok; ++j) {
        a *= 1.0 - (step / std::sqrt((double)j)) * reg;
        ok = std::fabs(a) >= 0x1p-400 && std::fabs(a) <= 0x1p400;
    }
    ctx->alpha_n = n;
    ctx->alpha_step = step;
    ctx->alpha_reg = reg;
    ctx->alpha_ok = ok;
    return ok;
}

int32_t ensure_steps(psgd_ctx* ctx, double step, int64_t n, hipStream_t st) {
    n = std::max<int64_t>(n, 1);
    if (ctx->steps_n >= n && ctx->steps_value == step) return PSGD_OK;
    HIP_TRY(ctx->steps.ensure((size_t)n * sizeof(double)));
    int e = psgd::launch_steps(step, n, ctx->steps.as<double>(), st);
    if (e) return fail(PSGD_EDEVICE, "steps kernel launch failed");
    ctx->steps_value = step;
    ctx->steps_n = n;
    return PSGD_OK;
}

// Per-workgroup LDS budget for the dense chain kernel's row ring: as deep a ring as possible
// while floor(160 KiB / budget) chain workgroups fit per CU, so P chains spread evenly over
// the CUs (one per CU for P <= #CUs). PSGD_LDS_BUDGET overrides (bytes).
int lds_spread_bytes(const psgd_ctx* ctx, size_t P) {
    const char* env = getenv("PSGD_LDS_BUDGET");
    if (env) return std::max(0, atoi(env));
    if (P == 0) return 0;
    const size_t per_cu = (P + (size_t)ctx->num_cus - 1) / (size_t)ctx->num_cus;
    const size_t lds_total = 160 * 1024;
    size_t want = lds_total / std::max<size_t>(per_cu, 1) - 512;
    return (int)(want & ~(size_t)255);
}

}  // namespace

extern "C" {

int32_t psgd_abi_version(void) { return PSGD_ABI_VERSION; }

const char* psgd_last_error(void) { return g_last_error.c_str(); }

int32_t psgd_ctx_create(int32_t device, psgd_ctx** out) {
    if (!out) return fail(PSGD_EINVAL, "out is null");
    *out = nullptr;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0)
        return fail(PSGD_EDEVICE, std::string("no HIP device available: ") + hipGetErrorString(e));
    if (device < 0 || device >= n)
        return fail(PSGD_EINVAL, "device index " + std::to_string(device) + " out of range");
    DeviceGuard g(device);
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (std::string(prop.gcnArchName).rfind("gfx950", 0) != 0)
        return fail(PSGD_EUNSUPPORTED, std::string("kernels are built for gfx950, device is ") +
                                           prop.gcnArchName);
    psgd_ctx* ctx = new psgd_ctx();
    ctx->device = device;
    ctx->num_cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->copy_ev, hipEventDisableTiming);
    if (e != hipSuccess) {
        if (ctx->stream) hipStreamDestroy(ctx->stream);
        if (ctx->copy_stream) hipStreamDestroy(ctx->copy_stream);
        delete ctx;
        return fail(PSGD_EDEVICE, std::string("hipStreamCreate: ") + hipGetErrorString(e));
    }
    *out = ctx;
    return PSGD_OK;
}

int32_t psgd_ctx_destroy(psgd_ctx* ctx) {
    if (!ctx) return PSGD_OK;
    {
        DeviceGuard g(ctx->device);
        hipStreamSynchronize(ctx->copy_stream);
        hipStreamSynchronize(ctx->stream);
        for (Stager* s : ctx->stagers) {
            s->release();
            delete s;
        }
        ctx->stagers.clear();
        for (auto& kv : ctx->parts) free_part(kv.second);
        for (DevBuf* b : {&ctx->descs, &ctx->w_in, &ctx->w_out, &ctx->state, &ctx->rv, &ctx->loss,
                          &ctx->cnt_d, &ctx->cnt, &ctx->steps, &ctx->partial, &ctx->tmp, &ctx->zbuf, &ctx->wf32, &ctx->stamps, &ctx->walpha, &ctx->wnsq0,
                          &ctx->sdescs, &ctx->srows, &ctx->sys, &ctx->xstate,
                          &ctx->watchdog})
            b->release();
        for (int k = 0; k < psgd_ctx::kChainEvents; ++k) {
            if (ctx->ev_begin[k]) hipEventDestroy(ctx->ev_begin[k]);
            if (ctx->ev_end[k]) hipEventDestroy(ctx->ev_end[k]);
        }
        if (ctx->copy_ev) hipEventDestroy(ctx->copy_ev);
        if (ctx->scratch_ev) {
            hipEventSynchronize(ctx->scratch_ev);
            hipEventDestroy(ctx->scratch_ev);
        }
        hipStreamDestroy(ctx->copy_stream);
        hipStreamDestroy(ctx->stream);
    }
    delete ctx;
    return PSGD_OK;
}

int32_t psgd_register_dense(psgd_ctx* ctx, int64_t part, int64_t n_rows, int32_t d,
                            const double* labels, const void* x, int32_t dtype) {
    if (!ctx) return fail(PSGD_EINVAL, "ctx is null");
    if (part < 0) return fail(PSGD_EINVAL, "partition index must be non-negative");
    if (n_rows < 0 || d <= 0) return fail(PSGD_EINVAL, "n_rows must be >= 0 and d > 0");
    if (dtype != PSGD_F64 && dtype != PSGD_F32) return fail(PSGD_EINVAL, "unknown dtype");
    if (n_rows > 0 && (!labels || !x)) return fail(PSGD_EINVAL, "labels/x are null");
    DeviceGuard g(ctx->device);
    {
        std::lock_guard<std::mutex> lk(ctx->mu);
        int32_t rc = check_compat(ctx, d, dtype, psgd::kDense);
        if (rc) return rc;
    }
    const size_t es = dtype_size(dtype);
    const int64_t vec = (int64_t)(16 / es);
    Part p;
    p.n_rows = n_rows;
    p.d = d;
    p.dtype = dtype;
    p.layout = psgd::kDense;
    p.owned = true;
    p.ld = (d + vec - 1) / vec * vec;
    // The copies run without the context lock (Spark's N task threads register concurrently),
    // on the copy stream; the partition joins the registry once they are enqueued.
    if (n_rows > 0) {
        const size_t row_src = (size_t)d * es, row_dev = (size_t)p.ld * es;
        const size_t xbytes = (size_t)n_rows * row_dev;
        struct Undo {
            psgd_ctx* c; Part* p; bool armed = true;
            ~Undo() { if (armed) { hipStreamSynchronize(c->copy_stream); free_part(*p); } }
        } undo{ctx, &p};
        HIP_TRY(hipMalloc(&p.x, xbytes));
        HIP_TRY(hipMalloc((void**)&p.y, (size_t)n_rows * sizeof(double)));
        StagerLease lease(ctx);
        const bool pinned = is_pinned(x);
        if (pinned && row_src == row_dev) {
            HIP_TRY(hipMemcpyAsync(p.x, x, xbytes, hipMemcpyHostToDevice, ctx->copy_stream));
        } else if (pinned) {
            HIP_TRY(hipMemsetAsync(p.x, 0, xbytes, ctx->copy_stream));
            HIP_TRY(hipMemcpy2DAsync(p.x, row_dev, x, row_src, row_src, (size_t)n_rows,
                                     hipMemcpyHostToDevice, ctx->copy_stream));
        } else {
            // rows packed at the device pitch, zero padding included (no device memset)
            const char* src = static_cast<const char*>(x);
            int32_t rc = stage_upload(ctx, *lease.s, p.x, xbytes, row_dev, [&](char* st, size_t off, size_t len) {
                const size_t r0 = off / row_dev, nr = len / row_dev;
                if (row_src == row_dev) {
                    std::memcpy(st, src + r0 * row_src, nr * row_src);
                } else {
                    for (size_t r = 0; r < nr; ++r) {
                        std::memcpy(st + r * row_dev, src + (r0 + r) * row_src, row_src);
                        std::memset(st + r * row_dev + row_src, 0, row_dev - row_src);
                    }
                }
                return true;
            });
            if (rc) return rc;
        }
        int32_t rc = upload(ctx, *lease.s, p.y, labels, (size_t)n_rows * sizeof(double));
        if (rc) return rc;
        rc = finish_direct(ctx, pinned || is_pinned(labels));
        if (rc) return rc;
        undo.armed = false;
    }
    std::lock_guard<std::mutex> lk(ctx->mu);
    int32_t rc = check_compat(ctx, d, dtype, psgd::kDense);   // a concurrent registration may differ
    if (rc) {
        hipStreamSynchronize(ctx->copy_stream);
        free_part(p);
        return rc;
    }
    auto it = ctx->parts.find(part);
    if (it != ctx->parts.end()) free_part(it->second);
    ctx->parts[part] = p;
    ctx->descs_dirty = true;
    ctx->copies_pending = true;
    return PSGD_OK;
}

int32_t psgd_register_dense_device(psgd_ctx* ctx, int64_t part, int64_t n_rows, int32_t d,
                                   int64_t ld, const double* d_labels, const void* d_x,
                                   int32_t dtype) {
    if (!ctx) return fail(PSGD_EINVAL, "ctx is null");
    if (part < 0) return fail(PSGD_EINVAL, "partition index must be non-negative");
    if (n_rows < 0 || d <= 0 || ld < d) return fail(PSGD_EINVAL, "need n_rows >= 0, d > 0, ld >= d");
    if (dtype != PSGD_F64 && dtype != PSGD_F32) return fail(PSGD_EINVAL, "unknown dtype");
    const size_t es = dtype_size(dtype);
    if (((size_t)ld * es) % 16 != 0 || ((uintptr_t)d_x % 16) != 0)
        return fail(PSGD_EINVAL, "device rows must be 16-byte aligned (ld * sizeof(dtype) % 16 == 0)");
    if (n_rows > 0 && (!d_labels || !d_x)) return fail(PSGD_EINVAL, "labels/x are null");
    std::lock_guard<std::mutex> lk(ctx->mu);
    int32_t rc = check_compat(ctx, d, dtype, psgd::kDense);
    if (rc) return rc;
    Part p;
    p.n_rows = n_rows;
    p.d = d;
    p.dtype = dtype;
    p.layout = psgd::kDense;
    p.owned = false;
    p.x = const_cast<void*>(d_x);
    p.y = const_cast<double*>(d_labels);
    p.ld = ld;
    auto it = ctx->parts.find(part);
    if (it != ctx->parts.end()) free_part(it->second);
    ctx->parts[part] = p;
    ctx->descs_dirty = true;
    return PSGD_OK;
}

int32_t psgd_register_csr_device(psgd_ctx* ctx, int64_t part, int64_t n_rows, int32_t d,
                                 const double* d_labels, const int64_t* d_row_ptr,
                                 const int32_t* d_col, const void* d_val, int32_t dtype) {
    if (!ctx) return fail(PSGD_EINVAL, "ctx is null");
    if (part < 0) return fail(PSGD_EINVAL, "partition index must be non-negative");
    if (n_rows < 0 || d <= 0) return fail(PSGD_EINVAL, "n_rows must be >= 0 and d > 0");
    if (dtype != PSGD_F64 && dtype != PSGD_F32) return fail(PSGD_EINVAL, "unknown dtype");
    if (n_rows > 0 && (!d_labels || !d_row_ptr || !d_col || !d_val))
        return fail(PSGD_EINVAL, "labels/row_ptr/col/val are null");
    std::lock_guard<std::mutex> lk(ctx->mu);
    int32_t rc = check_compat(ctx, d, dtype, psgd::kCsr);
    if (rc) return rc;
    Part p;
    p.n_rows = n_rows;
    p.d = d;
    p.dtype = dtype;
    p.layout = psgd::kCsr;
    p.owned = false;
    p.x = const_cast<void*>(d_val);
    p.y = const_cast<double*>(d_labels);
    p.row_ptr = const_cast<int64_t*>(d_row_ptr);
    p.col = const_cast<int32_t*>(d_col);
    p.ld = 0;
    {
        DeviceGuard g(ctx->device);
        int e = psgd::csr_max_nnz(d_row_ptr, n_rows, &p.max_nnz, ctx->stream);
        if (e) return fail(PSGD_EDEVICE, "row length scan failed");
    }
    auto it = ctx->parts.find(part);
    if (it != ctx->parts.end()) free_part(it->second);
    ctx->parts[part] = p;
    ctx->descs_dirty = true;
    return PSGD_OK;
}

int32_t psgd_register_csr(psgd_ctx* ctx, int64_t part, int64_t n_rows, int32_t d,
                          const double* labels, const int64_t* row_ptr, const int32_t* col,
                          const void* val, int32_t dtype) {
    if (!ctx) return fail(PSGD_EINVAL, "ctx is null");
    if (part < 0) return fail(PSGD_EINVAL, "partition index must be non-negative");
    if (n_rows < 0 || d <= 0) return fail(PSGD_EINVAL, "n_rows must be >= 0 and d > 0");
    if (dtype != PSGD_F64 && dtype != PSGD_F32) return fail(PSGD_EINVAL, "unknown dtype");
    if (n_rows > 0 && (!labels || !row_ptr)) return fail(PSGD_EINVAL, "labels/row_ptr are null");
    // Validate and rebase the row pointers.
    std::vector<int64_t> rp((size_t)n_rows + 1, 0);
    const int64_t base = n_rows > 0 ? row_ptr[0] : 0;
    for (int64_t r = 0; r <= n_rows; ++r) {
        rp[(size_t)r] = row_ptr[r] - base;
        if (r > 0 && rp[(size_t)r] < rp[(size_t)r - 1])
            return fail(PSGD_EINVAL, "row_ptr must be non-decreasing");
    }
    const int64_t nnz = rp[(size_t)n_rows];
    if (nnz > 0 && (!col || !val)) return fail(PSGD_EINVAL, "col/val are null");
    DeviceGuard g(ctx->device);
    {
        std::lock_guard<std::mutex> lk(ctx->mu);
        int32_t rc = check_compat(ctx, d, dtype, psgd::kCsr);
        if (rc) return rc;
    }
    const size_t es = dtype_size(dtype);
    Part p;
    p.n_rows = n_rows;
    p.d = d;
    p.dtype = dtype;
    p.layout = psgd::kCsr;
    p.owned = true;
    for (int64_t r = 0; r < n_rows; ++r)
        p.max_nnz = std::max<int64_t>(p.max_nnz, rp[(size_t)r + 1] - rp[(size_t)r]);
    // Copies without the context lock, on the copy stream (see psgd_register_dense). The column
    // indices are validated chunk by chunk as they are packed, so a pageable partition is read
    // once; a failure drains the copies and frees the partition's buffers.
    if (n_rows > 0) {
        struct Undo {
            psgd_ctx* c; Part* p; bool armed = true;
            ~Undo() { if (armed) { hipStreamSynchronize(c->copy_stream); free_part(*p); } }
        } undo{ctx, &p};
        HIP_TRY(hipMalloc((void**)&p.row_ptr, rp.size() * sizeof(int64_t)));
        HIP_TRY(hipMalloc((void**)&p.y, (size_t)n_rows * sizeof(double)));
        StagerLease lease(ctx);
        int32_t rc = upload(ctx, *lease.s, p.row_ptr, rp.data(), rp.size() * sizeof(int64_t));
        if (rc) return rc;
        rc = upload(ctx, *lease.s, p.y, labels, (size_t)n_rows * sizeof(double));
        if (rc) return rc;
        bool direct = is_pinned(labels);
        if (nnz > 0) {
            HIP_TRY(hipMalloc((void**)&p.col, (size_t)nnz * sizeof(int32_t)));
            HIP_TRY(hipMalloc(&p.x, (size_t)nnz * es));
            const int32_t* cs = col + base;
            // entries [k0, k1): in range, strictly increasing inside a row
            int64_t row = 0;
            auto check = [&](int64_t k0, int64_t k1) -> bool {
                for (int64_t k = k0; k < k1; ++k) {
                    while (rp[(size_t)row + 1] <= k) ++row;
                    const int32_t c = cs[k];
                    if (c < 0 || c >= d) {
                        fail(PSGD_EINVAL, "requirement failed: column index " + std::to_string(c) +
                                              " out of range [0, " + std::to_string(d) + ")");
                        return false;
                    }
                    if (k > rp[(size_t)row] && c <= cs[k - 1]) {
                        fail(PSGD_EINVAL, "column indices must be strictly increasing within a row");
                        return false;
                    }
                }
                return true;
            };
            if (is_pinned(cs)) {
                if (!check(0, nnz)) return PSGD_EINVAL;
                HIP_TRY(hipMemcpyAsync(p.col, cs, (size_t)nnz * sizeof(int32_t), hipMemcpyHostToDevice,
                                       ctx->copy_stream));
                direct = true;
            } else {
                rc = stage_upload(ctx, *lease.s, p.col, (size_t)nnz * sizeof(int32_t), sizeof(int32_t),
                                  [&](char* st, size_t off, size_t len) {
                                      const int64_t k0 = (int64_t)(off / 4), k1 = (int64_t)((off + len) / 4);
                                      if (!check(k0, k1)) return false;
                                      std::memcpy(st, cs + k0, len);
                                      return true;
                                  });
                if (rc) return rc;
            }
            const char* vs = static_cast<const char*>(val) + (size_t)base * es;
            direct = direct || is_pinned(vs);
            rc = upload(ctx, *lease.s, p.x, vs, (size_t)nnz * es);
            if (rc) return rc;
        }
        rc = finish_direct(ctx, direct);
        if (rc) return rc;
        undo.armed = false;
    }
    std::lock_guard<std::mutex> lk(ctx->mu);
    int32_t rc = check_compat(ctx, d, dtype, psgd::kCsr);   // a concurrent registration may differ
    if (rc) {
        hipStreamSynchronize(ctx->copy_stream);
        free_part(p);
        return rc;
    }
    auto it = ctx->parts.find(part);
    if (it != ctx->parts.end()) free_part(it->second);
    ctx->parts[part] = p;
    ctx->descs_dirty = true;
    ctx->copies_pending = true;
    return PSGD_OK;
}

int32_t psgd_host_alloc(psgd_ctx* ctx, int64_t bytes, void** out) {
    if (!ctx || !out) return fail(PSGD_EINVAL, "ctx/out is null");
    *out = nullptr;
    if (bytes <= 0) return fail(PSGD_EINVAL, "bytes must be > 0");
    DeviceGuard g(ctx->device);
    hipError_t e = hipHostMalloc(out, (size_t)bytes, hipHostMallocDefault);
    if (e != hipSuccess) {
        *out = nullptr;
        return fail(PSGD_ENOMEM, std::string("hipHostMalloc: ") + hipGetErrorString(e));
    }
    return PSGD_OK;
}

int32_t psgd_host_free(psgd_ctx* ctx, void* p) {
    if (!ctx) return fail(PSGD_EINVAL, "ctx is null");
    if (!p) return PSGD_OK;
    DeviceGuard g(ctx->device);
    HIP_TRY(hipHostFree(p));
    return PSGD_OK;
}

int32_t psgd_register_wait(psgd_ctx* ctx) {
    if (!ctx) return fail(PSGD_EINVAL, "ctx is null");
    DeviceGuard g(ctx->device);
    HIP_TRY(hipStreamSynchronize(ctx->copy_stream));
    return PSGD_OK;
}

int32_t psgd_clear_partitions(psgd_ctx* ctx) {
    if (!ctx) return fail(PSGD_EINVAL, "ctx is null");
    std::lock_guard<std::mutex> lk(ctx->mu);
    DeviceGuard g(ctx->device);
    // epochs may run on caller streams (psgd_run_epoch_device), each ordered after the previous
    // one (scratch_acquire): the newest epoch's end and the registration copies are all that
    // can still read the partitions' buffers
    if (ctx->scratch_recorded) HIP_TRY(hipEventSynchronize(ctx->scratch_ev));
    HIP_TRY(hipStreamSynchronize(ctx->copy_stream));
    for (auto& kv : ctx->parts) free_part(kv.second);
    ctx->parts.clear();
    ctx->descs_dirty = true;
    return PSGD_OK;
}

int32_t psgd_num_partitions(psgd_ctx* ctx, int64_t* n_parts, int64_t* n_rows_total) {
    if (!ctx) return fail(PSGD_EINVAL, "ctx is null");
    std::lock_guard<std::mutex> lk(ctx->mu);
    int64_t rows = 0;
    for (auto& kv : ctx->parts) rows += kv.second.n_rows;
    if (n_parts) *n_parts = (int64_t)ctx->parts.size();
    if (n_rows_total) *n_rows_total = rows;
    return PSGD_OK;
}

// The host mirror's device address (page-locked memory from psgd_host_alloc / hipHostMalloc).
static int32_t mirror_address(psgd_ctx* ctx, double* h, double** dev) {
    *dev = nullptr;
    if (!h) return PSGD_OK;
    DeviceGuard g(ctx->device);
    void* p = nullptr;
    if (hipHostGetDevicePointer(&p, h, 0) != hipSuccess || !p) {
        (void)hipGetLastError();
        return fail(PSGD_EINVAL, "h_scalars is not page-locked host memory (psgd_host_alloc)");
    }
    *dev = static_cast<double*>(p);
    return PSGD_OK;
}

static int32_t run_epoch_device(psgd_ctx* ctx, const psgd_params* params, const double* d_w_in,
                                double* d_partial, int64_t* d_chain_counts, void* stream, double* mirror);

int32_t psgd_run_epoch_device(psgd_ctx* ctx, const psgd_params* params, const double* d_w_in,
                              double* d_partial, int64_t* d_chain_counts, void* stream) {
    return run_epoch_device(ctx, params, d_w_in, d_partial, d_chain_counts, stream, nullptr);
}

int32_t psgd_run_epoch_device_mirror(psgd_ctx* ctx, const psgd_params* params, const double* d_w_in,
                                     double* d_partial, int64_t* d_chain_counts, void* stream,
                                     double* h_scalars) {
    if (!ctx) return fail(PSGD_EINVAL, "ctx is null");
    double* mirror = nullptr;
    int32_t rc = mirror_address(ctx, h_scalars, &mirror);
    if (rc) return rc;
    return run_epoch_device(ctx, params, d_w_in, d_partial, d_chain_counts, stream, mirror);
}

static int32_t run_epoch_device(psgd_ctx* ctx, const psgd_params* params, const double* d_w_in,
                                double* d_partial, int64_t* d_chain_counts, void* stream, double* mirror) {
    if (!ctx) return fail(PSGD_EINVAL, "ctx is null");
    int32_t rc = validate_params(params);
    if (rc) return rc;
    if (!d_w_in || !d_partial) return fail(PSGD_EINVAL, "d_w_in/d_partial are null");
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (ctx->parts.empty()) return fail(PSGD_ESTATE, "no partitions registered");
    DeviceGuard g(ctx->device);
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    const Part& first = ctx->parts.begin()->second;
    const int32_t d = first.d;
    const int32_t layout = first.layout;
    const bool mn = multinomial(params);
    if (weight_dim(d, params) > INT32_MAX) return fail(PSGD_EINVAL, "(numClasses - 1) * d overflows");
    const int32_t dw = (int32_t)weight_dim(d, params);   // weights (and every weight-sized buffer)
    const bool stateful = params->updater == PSGD_UPDATER_ADAGRAD || params->updater == PSGD_UPDATER_ADAM;
    const bool conv = params->convergence_tol > 0.0;
    const bool need_state = mn || stateful || (layout == psgd::kCsr && conv);
    // weight-sized vectors of status per chain (chain_general: dense [SA|SB], CSR [SA|SB|SC];
    // chain_multinomial: [SA|SB|G])
    const int state_vectors = !need_state ? 0 : (mn || layout == psgd::kCsr) ? 3 : 2;
    rc = prepare(ctx, dw, state_vectors, st);
    if (rc) return rc;
    // from here on work may be queued on `st` (descriptor upload, sampling, a chain kernel that
    // launched before a later launch failed): every return records the scratch event, so that
    // psgd_clear_partitions (which waits on it instead of the whole device) cannot free buffers
    // under a kernel that is still running
    struct ScratchGuard {
        psgd_ctx* ctx;
        hipStream_t st;
        ~ScratchGuard() { (void)scratch_release(ctx, st); }
    } scratch_guard{ctx, st};
    int64_t n_max = 0, max_ld = 0, min_ld = INT64_MAX, max_nnz = 0;
    for (auto& kv : ctx->parts) {
        n_max = std::max(n_max, kv.second.n_rows);
        max_nnz = std::max(max_nnz, kv.second.max_nnz);
        if (kv.second.n_rows > 0) {
            max_ld = std::max(max_ld, kv.second.ld);
            min_ld = std::min(min_ld, kv.second.ld);
        }
    }
    if (max_ld == 0) max_ld = min_ld = d;
    // RDD.sample(false, f, 42 + i) (PSGD.scala:242) [ext Spark 1.6.1 BernoulliSampler]:
    // f <= 0 gives every partition empty, f >= 1 every row, else a Bernoulli batch per partition
    const bool sample_empty = params->mini_batch_fraction <= 0.0;
    const bool sampled = !sample_empty && params->mini_batch_fraction < 1.0;
    // the sampled batch's row indices are int32 (ChainDesc::rows)
    if (sampled && n_max > (int64_t)INT32_MAX)
        return fail(PSGD_EUNSUPPORTED, "miniBatchFraction < 1 on a partition of more than 2^31 - 1 rows");
    rc = ensure_steps(ctx, params->step_size, n_max, st);
    if (rc) return rc;

    const int P = (int)ctx->parts.size();
    psgd::ChainLaunch L;
    L.descs = ctx->descs.as<psgd::ChainDesc>();
    if (sampled) {
        // one XORShiftRandom per partition, seeded as PartitionwiseSampledRDD does: the p-th
        // java.util.Random(42 + i).nextLong() for partition index p, through hashSeed
        std::vector<uint64_t> xs((size_t)P);
        sampling::JavaRandom jr(42 + (int64_t)params->iteration);
        int64_t drawn = 0, s = 0;
        size_t c = 0;
        for (auto& kv : ctx->parts) {
            while (drawn <= kv.first) { s = jr.next_long(); ++drawn; }
            xs[c++] = (uint64_t)sampling::xorshift_hash_seed(s);
        }
        const int64_t stride = std::max<int64_t>(n_max, 1);
        HIP_TRY(ctx->sdescs.ensure((size_t)P * sizeof(psgd::ChainDesc)));
        HIP_TRY(ctx->srows.ensure((size_t)P * (size_t)stride * sizeof(int32_t)));
        HIP_TRY(ctx->sys.ensure((size_t)P * (size_t)stride * sizeof(double)));
        HIP_TRY(ctx->xstate.ensure((size_t)P * sizeof(uint64_t)));
        HIP_TRY(hipMemcpyAsync(ctx->xstate.p, xs.data(), (size_t)P * sizeof(uint64_t),
                               hipMemcpyHostToDevice, st));
        int e = psgd::launch_sample(L.descs, ctx->sdescs.as<psgd::ChainDesc>(),
                                    ctx->xstate.as<uint64_t>(), params->mini_batch_fraction,
                                    ctx->srows.as<int32_t>(), ctx->sys.as<double>(), stride, P, st);
        if (e) return fail(PSGD_EDEVICE, "sample kernel launch failed");
        // host data may be freed by the caller once run_epoch returns: wait for the copy
        HIP_TRY(hipStreamSynchronize(st));
        L.descs = ctx->sdescs.as<psgd::ChainDesc>();
    }
    L.w_in = d_w_in;
    L.w_out = ctx->w_out.as<double>();
    L.state = need_state ? ctx->state.as<double>() : nullptr;
    L.rv = ctx->rv.as<double>();
    L.loss = ctx->loss.as<double>();
    L.cnt_d = ctx->cnt_d.as<double>();
    L.cnt = ctx->cnt.as<int64_t>();
    L.steps = ctx->steps.as<double>();
    L.watchdog = ctx->watchdog.as<int>();
    L.stamps = nullptr;
    static const bool want_stamps = [] {
        const char* e = getenv("PSGD_STAMPS");
        return e && *e && *e != '0';
    }();
    if (want_stamps) {   // read by the CSR kernels and chain_split (and by PSGD_STAMPS builds)
        HIP_TRY(ctx->stamps.ensure((size_t)P * 16 * sizeof(unsigned long long)));
        HIP_TRY(hipMemsetAsync(ctx->stamps.p, 0, (size_t)P * 16 * sizeof(unsigned long long), st));
        L.stamps = ctx->stamps.as<unsigned long long>();
    }
    L.zbuf = nullptr;
    L.zbuf64 = nullptr;
    L.zstride = 0;
    L.wf32 = nullptr;
    L.wstride = 0;
    L.walpha = nullptr;
    L.wnsq0 = nullptr;
    if (layout == psgd::kCsr && params->compute_dtype == PSGD_F32) {
        // fp32 working weights of the CSR kernels (one d-vector per chain, HBM/L2-resident, and
        // 128 + 1024 floats the kernels' masked-off lanes load from / store to)
        // (rows 256-byte aligned: the epoch's init kernel stores 16-byte vectors)
        L.wstride = ((int64_t)d + 128 + 1024 + 63) / 64 * 64;
        HIP_TRY(ctx->wf32.ensure((size_t)P * (size_t)L.wstride * sizeof(float), true));
        // (the fp32 LDS head of chain_sparse_lds; below it the chains never touch the vector)
        reroll_vectors(ctx->wf32, L.wstride, P, d, (int)std::max<int64_t>(psgd::sparse_lds_head(d), 0), st);
        HIP_TRY(ctx->walpha.ensure((size_t)P * sizeof(double)));
        HIP_TRY(ctx->wnsq0.ensure(sizeof(double)));
        L.wf32 = ctx->wf32.as<float>();
        L.walpha = ctx->walpha.as<double>();
        L.wnsq0 = ctx->wnsq0.as<double>();
    }
    // SquaredL2's alpha-scaled CSR kernels need every prefix product of (1 - s_j lambda) in range
    const bool alpha_ok = params->updater != PSGD_UPDATER_SQUARED_L2 ||
                          alpha_in_range(ctx, params->step_size, params->reg_param, n_max);
    if (layout == psgd::kCsr && params->compute_dtype == PSGD_F64 && !mn && !psgd::per_sample_forced() &&
        (psgd::sparse_lds64_applies(d, max_nnz, params->updater, conv, alpha_ok, n_max) ||
         psgd::sparse64_path_applies(layout, 0, params->updater, conv, alpha_ok))) {
        // the fp64 CSR kernels' per-chain f64 vectors (d + 1152 doubles, in L.wf32's memory),
        // chain_sparse64's alphas, and ||w_in||^2 for the per-sample break. Only when one of those
        // kernels will run (chain_general keeps its weights in w_out, and C5's
        // vectors are ~34 GB); if HBM cannot hold them the epoch runs chain_general instead.
        const int64_t stride = 2 * (((int64_t)d + 128 + 1024 + 63) / 64 * 64);
        const size_t need = (size_t)P * (size_t)stride * sizeof(float);
        // (a size that failed once is not retried every epoch -- each retry frees the
        // old buffer and tries the VMM chunks and a hipMalloc of tens of GB again)
        if (need != ctx->wf64_failed && ctx->wf32.ensure(need, true) == hipSuccess) {
            // (the fp64 head is shorter than the fp32 one: half of it is inside the fp64 tail)
            reroll_vectors(ctx->wf32, stride, P, 2 * d, (int)std::max<int64_t>(psgd::sparse_lds_head(d), 0), st);
            HIP_TRY(ctx->walpha.ensure((size_t)P * sizeof(double)));
            HIP_TRY(ctx->wnsq0.ensure(sizeof(double)));
            L.wstride = stride;
            L.wf32 = ctx->wf32.as<float>();
            L.walpha = ctx->walpha.as<double>();
            L.wnsq0 = ctx->wnsq0.as<double>();
        } else {
            (void)hipGetLastError();   // the failed allocation is not the epoch's error
            if (need != ctx->wf64_failed)
                fprintf(stderr, "psgd: the fp64 CSR chains' weight vectors (%zu bytes) do not fit in HBM: "
                        "this epoch and later ones of this size run chain_general (variant 201)\n", need);
            ctx->wf64_failed = need;
        }
    }
    if (params->gradient == PSGD_GRADIENT_LOGISTIC && params->compute_dtype == PSGD_F32 &&
        layout == psgd::kDense) {
        // per-row margins of the fp32 Logistic block kernel (its loss is summed after the chain)
        L.zstride = std::max<int64_t>(n_max, 1);
        HIP_TRY(ctx->zbuf.ensure((size_t)P * (size_t)L.zstride * sizeof(float)));
        L.zbuf = ctx->zbuf.as<float>();
    }
    if (params->gradient == PSGD_GRADIENT_LOGISTIC && params->compute_dtype == PSGD_F64 &&
        layout == psgd::kDense && !mn) {
        // per-row dots of the fp64 per-sample kernel (its loss is summed after the chain)
        L.zstride = std::max<int64_t>(n_max, 1);
        HIP_TRY(ctx->zbuf.ensure((size_t)P * (size_t)L.zstride * sizeof(double)));
        L.zbuf64 = ctx->zbuf.as<double>();
    }
    psgd::KParams kp;
    kp.reg = params->reg_param;
    kp.tol = params->convergence_tol;
    kp.beta = params->adam_beta;
    kp.gamma = params->adam_gamma;
    kp.eps = params->adam_eps;
    kp.d = d;
    kp.n_chains = P;
    kp.nc = mn ? params->num_classes - 1 : 0;
    kp.n_max = n_max;
    kp.alpha_ok = alpha_ok;

    int weights_in = psgd::kWeightsOut;   // where the launch left the chains' weights
    if (sample_empty) {
        // RDD.sample with fraction 0: every partition is empty -> (w_in, 0, 0, 0) per chain.
        for (int p = 0; p < P; ++p)
            HIP_TRY(hipMemcpyAsync(L.w_out + (size_t)p * dw, d_w_in, (size_t)dw * sizeof(double),
                                   hipMemcpyDeviceToDevice, st));
        HIP_TRY(hipMemsetAsync(L.rv, 0, P * sizeof(double), st));
        HIP_TRY(hipMemsetAsync(L.loss, 0, P * sizeof(double), st));
        HIP_TRY(hipMemsetAsync(L.cnt_d, 0, P * sizeof(double), st));
        HIP_TRY(hipMemsetAsync(L.cnt, 0, P * sizeof(int64_t), st));
    } else {
        const int ek = (int)(ctx->chain_launches % psgd_ctx::kChainEvents);
        if (!ctx->ev_begin[ek]) {
            HIP_TRY(hipEventCreate(&ctx->ev_begin[ek]));
            HIP_TRY(hipEventCreate(&ctx->ev_end[ek]));
        }
        HIP_TRY(hipEventRecord(ctx->ev_begin[ek], st));
        int e = psgd::launch_chains(L, kp, layout, first.dtype == PSGD_F32 ? 1 : 0,
                                    params->compute_dtype == PSGD_F32 ? 1 : 0, params->gradient,
                                    params->updater, conv, min_ld, max_ld,
                                    lds_spread_bytes(ctx, (size_t)P), st, &ctx->last_variant, max_nnz,
                                    &weights_in);
        HIP_TRY(hipEventRecord(ctx->ev_end[ek], st));
        if (e == 0) ++ctx->chain_launches;
        if (L.stamps) {   // PSGD_STAMPS=1: per-chain cycle counters of the CSR fp32 kernels (stderr)
            // chain_sparse_lds: {chain, loader, tagger} x {total, waiting}; chain_sparse_spec:
            // {chain, helper} x {total, waiting}
            // chain_split: {total, row + dot + reduce, exchange wait, multiplier + update} per
            // compute wave
            const bool split = ctx->last_variant >= 800;
            const int KS = split ? 16 : ctx->last_variant >= 600 ? 6 : 4;
            const int KST = split ? 16 : KS;   // stride per chain
            std::vector<unsigned long long> h((size_t)P * 16);
            HIP_TRY(hipMemcpyAsync(h.data(), L.stamps, h.size() * 8, hipMemcpyDeviceToHost, st));
            HIP_TRY(hipStreamSynchronize(st));
            std::vector<double> v[16];
            for (int p = 0; p < P; ++p)
                for (int k = 0; k < KS; ++k)
                    v[k].push_back((double)h[(size_t)p * KST + k] / std::max<int64_t>(n_max, 1));
            const char* n4[4] = {"chain.total", "chain.wait", "helper.total", "helper.wait"};
            const char* n6[6] = {"chain.total", "chain.wait", "loader.total", "loader.wait", "tagger.total", "tagger.wait"};
            const char* ns[4] = {"total", "dot", "xwait", "update"};
            for (int k = 0; k < KS; ++k) {
                std::sort(v[k].begin(), v[k].end());
                char nm[32];
                if (split) snprintf(nm, sizeof nm, "wave%d.%s", k / 4, ns[k % 4]);
                fprintf(stderr, "psgd stamps %-18s cycles/row median %8.1f\n",
                        split ? nm : KS == 6 ? n6[k] : n4[k], v[k][v[k].size() / 2]);
            }
        }
        if (e) {
            // (no fold clears the flags of a kernel that launched before the failure)
            (void)hipMemsetAsync(L.watchdog, 0, 16, st);
            if (e == -2) return fail(PSGD_EUNSUPPORTED, "this gradient/updater/layout combination is not built");
            return fail(PSGD_EDEVICE, std::string("chain kernel launch failed: ") + hipGetErrorString((hipError_t)e));
        }
    }
    // the CSR kernels of L.wf32 leave each chain's weights there (w = alpha v, floats or doubles)
    int e = weights_in == psgd::kWeightsF32
                ? psgd::launch_fold_f32(L.wf32, L.wstride, L.walpha, L.rv, L.loss, L.cnt_d, P, dw, d_partial,
                                        L.watchdog, st, mirror)
            : weights_in == psgd::kWeightsF64
                ? psgd::launch_fold_f64(reinterpret_cast<const double*>(L.wf32), L.wstride / 2, L.walpha, L.rv,
                                        L.loss, L.cnt_d, P, dw, d_partial, L.watchdog, st, mirror)
                : psgd::launch_fold(L.w_out, dw, L.rv, L.loss, L.cnt_d, 1, P, dw, d_partial, L.watchdog, st,
                                    mirror);
    if (e) {
        (void)hipMemsetAsync(L.watchdog, 0, 16, st);
        return fail(PSGD_EDEVICE, "fold kernel launch failed");
    }
    if (d_chain_counts)
        HIP_TRY(hipMemcpyAsync(d_chain_counts, L.cnt, (size_t)P * sizeof(int64_t),
                               hipMemcpyDeviceToDevice, st));
    return PSGD_OK;   // scratch_guard records the scratch event
}

int32_t psgd_run_epoch(psgd_ctx* ctx, const psgd_params* params, const double* w_in,
                       double* w_out, double* regval_out, double* loss_sum_out,
                       int64_t* count_out, int64_t* chain_counts) {
    if (!ctx) return fail(PSGD_EINVAL, "ctx is null");
    if (!w_in || !w_out) return fail(PSGD_EINVAL, "w_in/w_out are null");
    int32_t rc0 = validate_params(params);
    if (rc0) return rc0;
    int32_t d = 0;
    size_t P = 0;
    {
        std::lock_guard<std::mutex> lk(ctx->mu);
        if (ctx->parts.empty()) return fail(PSGD_ESTATE, "no partitions registered");
        const int64_t dw = weight_dim(ctx->parts.begin()->second.d, params);
        if (dw > INT32_MAX) return fail(PSGD_EINVAL, "(numClasses - 1) * d overflows");
        d = (int32_t)dw;   // the weight vector's length from here on
        P = ctx->parts.size();
        DeviceGuard g(ctx->device);
        HIP_TRY(ctx->w_in.ensure((size_t)d * sizeof(double)));
        HIP_TRY(ctx->partial.ensure(((size_t)d + 3) * sizeof(double)));
        HIP_TRY(ctx->tmp.ensure(((size_t)d + 8) * sizeof(double)));
        HIP_TRY(hipMemcpyAsync(ctx->w_in.p, w_in, (size_t)d * sizeof(double),
                               hipMemcpyHostToDevice, ctx->stream));
    }
    int64_t* d_counts = nullptr;
    DevBuf counts;
    DeviceGuard g(ctx->device);
    if (chain_counts) {
        HIP_TRY(counts.ensure(P * sizeof(int64_t)));
        d_counts = counts.as<int64_t>();
    }
    int32_t rc = psgd_run_epoch_device(ctx, params, ctx->w_in.as<double>(),
                                       ctx->partial.as<double>(), d_counts, ctx->stream);
    if (rc) {
        counts.release();
        return rc;
    }
    std::vector<double> h((size_t)d + 3);
    HIP_TRY(hipMemcpyAsync(h.data(), ctx->partial.p, h.size() * sizeof(double),
                           hipMemcpyDeviceToHost, ctx->stream));
    if (chain_counts)
        HIP_TRY(hipMemcpyAsync(chain_counts, d_counts, P * sizeof(int64_t), hipMemcpyDeviceToHost,
                               ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    counts.release();
    std::memcpy(w_out, h.data(), (size_t)d * sizeof(double));
    if (h[(size_t)d + 2] != h[(size_t)d + 2])
        return fail(PSGD_EDEVICE, "chain kernel watchdog fired (loader/compute waves stalled)");
    if (regval_out) *regval_out = h[(size_t)d];
    if (loss_sum_out) *loss_sum_out = h[(size_t)d + 1];
    if (count_out) *count_out = (int64_t)h[(size_t)d + 2];
    return PSGD_OK;
}

int32_t psgd_fold_partials_device_mirror(psgd_ctx* ctx, int32_t n, int32_t d, const double* d_partials,
                                         double* d_out, void* stream, double* h_scalars) {
    if (!ctx) return fail(PSGD_EINVAL, "ctx is null");
    if (n <= 0 || d <= 0 || !d_partials || !d_out) return fail(PSGD_EINVAL, "bad fold arguments");
    double* mirror = nullptr;
    int32_t rc = mirror_address(ctx, h_scalars, &mirror);
    if (rc) return rc;
    DeviceGuard g(ctx->device);
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    const int64_t stride = (int64_t)d + 3;
    int e = psgd::launch_fold(d_partials, stride, d_partials + d, d_partials + d + 1,
                              d_partials + d + 2, stride, n, d, d_out, nullptr, st, mirror);
    if (e) return fail(PSGD_EDEVICE, "fold kernel launch failed");
    return PSGD_OK;
}

int32_t psgd_fold_partials_device(psgd_ctx* ctx, int32_t n, int32_t d, const double* d_partials,
                                  double* d_out, void* stream) {
    return psgd_fold_partials_device_mirror(ctx, n, d, d_partials, d_out, stream, nullptr);
}

int32_t psgd_convergence_terms_device(psgd_ctx* ctx, int32_t d, const double* d_prev,
                                      const double* d_cur, double* h_out, void* stream) {
    if (!ctx) return fail(PSGD_EINVAL, "ctx is null");
    if (d <= 0 || !d_prev || !d_cur || !h_out) return fail(PSGD_EINVAL, "bad arguments");
    std::lock_guard<std::mutex> lk(ctx->mu);
    DeviceGuard g(ctx->device);
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    int32_t rc = scratch_acquire(ctx, st);
    if (rc) return rc;
    HIP_TRY(ctx->tmp.ensure(((size_t)d + 8) * sizeof(double)));
    double* t = ctx->tmp.as<double>();
    int e = psgd::launch_sq_terms(d_prev, d_cur, d, t, st);
    if (e) return fail(PSGD_EDEVICE, "sq_terms kernel launch failed");
    HIP_TRY(hipMemcpyAsync(h_out, t, 2 * sizeof(double), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return PSGD_OK;
}

int32_t psgd_initial_regval(psgd_ctx* ctx, const psgd_params* params, int32_t d, const double* w,
                            double* regval_out) {
    if (!ctx) return fail(PSGD_EINVAL, "ctx is null");
    int32_t rc = validate_params(params);
    if (rc) return rc;
    if (d <= 0 || !w || !regval_out) return fail(PSGD_EINVAL, "bad arguments");
    if (params->updater != PSGD_UPDATER_SQUARED_L2 && params->updater != PSGD_UPDATER_L1) {
        *regval_out = 0.0;  // Simple / AdaGrad / Adam return 0 (UPD.scala:97, :214, :267)
        return PSGD_OK;
    }
    std::lock_guard<std::mutex> lk(ctx->mu);
    DeviceGuard g(ctx->device);
    rc = scratch_acquire(ctx, ctx->stream);
    if (rc) return rc;
    HIP_TRY(ctx->tmp.ensure(((size_t)d + 8) * sizeof(double)));
    double* t = ctx->tmp.as<double>();
    HIP_TRY(hipMemcpyAsync(t + 8, w, (size_t)d * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
    int e = psgd::launch_sq_terms(nullptr, t + 8, d, t, ctx->stream);
    if (e) return fail(PSGD_EDEVICE, "sq_terms kernel launch failed");
    double h[2];
    HIP_TRY(hipMemcpyAsync(h, t, sizeof h, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    if (params->updater == PSGD_UPDATER_SQUARED_L2) {
        // w' = w * (1 - 0*reg); rv = 0.5 * reg * norm * norm (UPD.scala:176-180)
        const double nrm = std::sqrt(h[0]);
        *regval_out = 0.5 * params->reg_param * nrm * nrm;
    } else {
        *regval_out = h[1] * params->reg_param;  // UPD.scala:147 with shrinkage 0
    }
    return PSGD_OK;
}

int32_t psgd_sample_partition(int32_t device, int64_t seed, int64_t n, double fraction, int32_t* rows_out,
                              int64_t* m_out) {
    if (!m_out || (n > 0 && !rows_out)) return fail(PSGD_EINVAL, "rows_out/m_out is null");
    if (n < 0 || n > INT32_MAX) return fail(PSGD_EINVAL, "n out of range");
    *m_out = 0;
    if (fraction <= 0.0 || n == 0) return PSGD_OK;
    if (fraction >= 1.0) {
        for (int64_t t = 0; t < n; ++t) rows_out[t] = (int32_t)t;
        *m_out = n;
        return PSGD_OK;
    }
    DeviceGuard g(device);
    DevBuf desc, out, rows, xs;
    struct Release {
        DevBuf* b[4];
        ~Release() {
            for (DevBuf* x : b) x->release();
        }
    } release{{&desc, &out, &rows, &xs}};
    HIP_TRY(desc.ensure(sizeof(psgd::ChainDesc)));
    HIP_TRY(out.ensure(sizeof(psgd::ChainDesc)));
    HIP_TRY(rows.ensure((size_t)n * sizeof(int32_t)));
    HIP_TRY(xs.ensure(sizeof(uint64_t)));
    psgd::ChainDesc c{};
    c.n_rows = n;
    const uint64_t s0 = (uint64_t)sampling::xorshift_hash_seed(seed);
    HIP_TRY(hipMemcpy(desc.p, &c, sizeof c, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(xs.p, &s0, sizeof s0, hipMemcpyHostToDevice));
    if (psgd::launch_sample(desc.as<psgd::ChainDesc>(), out.as<psgd::ChainDesc>(), xs.as<uint64_t>(), fraction,
                            rows.as<int32_t>(), nullptr, n, 1, nullptr))
        return fail(PSGD_EDEVICE, "sample kernel launch failed");
    HIP_TRY(hipMemcpy(&c, out.p, sizeof c, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(rows_out, rows.p, (size_t)c.n_rows * sizeof(int32_t), hipMemcpyDeviceToHost));
    *m_out = c.n_rows;
    return PSGD_OK;
}

int32_t psgd_ctx_last_kernel(psgd_ctx* ctx) { return ctx ? ctx->last_variant : 0; }

int32_t psgd_ctx_chain_ms(psgd_ctx* ctx, int64_t launch, double* ms_out) {
    if (!ctx || !ms_out) return fail(PSGD_EINVAL, "ctx/ms_out is null");
    if (ctx->chain_launches == 0) return fail(PSGD_ESTATE, "no chain kernel has been launched");
    if (launch < 0 || launch >= ctx->chain_launches || launch < ctx->chain_launches - psgd_ctx::kChainEvents)
        return fail(PSGD_EINVAL, "launch " + std::to_string(launch) + " is not among the last " +
                                     std::to_string(psgd_ctx::kChainEvents) + " of " +
                                     std::to_string(ctx->chain_launches));
    DeviceGuard g(ctx->device);
    const int ek = (int)(launch % psgd_ctx::kChainEvents);
    HIP_TRY(hipEventSynchronize(ctx->ev_end[ek]));
    float ms = 0.0f;
    HIP_TRY(hipEventElapsedTime(&ms, ctx->ev_begin[ek], ctx->ev_end[ek]));
    *ms_out = ms;
    return PSGD_OK;
}

int32_t psgd_ctx_last_chain_ms(psgd_ctx* ctx, double* ms_out) {
    if (!ctx || !ms_out) return fail(PSGD_EINVAL, "ctx/ms_out is null");
    if (ctx->chain_launches == 0) return fail(PSGD_ESTATE, "no chain kernel has been launched");
    return psgd_ctx_chain_ms(ctx, ctx->chain_launches - 1, ms_out);
}

int64_t psgd_ctx_chain_launches(psgd_ctx* ctx) { return ctx ? ctx->chain_launches : 0; }

int32_t psgd_vmm_stats(int64_t* out4) {
    if (!out4) return fail(PSGD_EINVAL, "out4 is null");
    out4[0] = g_vmm_mapped.load();
    out4[1] = g_vmm_unmapped.load();
    out4[2] = g_vmm_live_bytes.load();
    out4[3] = g_vmm_failures.load();
    return PSGD_OK;
}

int32_t psgd_reroll_stats(int64_t* out2) {
    if (!out2) return fail(PSGD_EINVAL, "out2 is null");
    out2[0] = g_reroll_sets.load();
    out2[1] = g_reroll_swaps.load();
    return PSGD_OK;
}

}  // extern "C"
