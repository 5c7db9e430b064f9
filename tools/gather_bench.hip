// gather_bench.hip -- the scattered-request ceiling behind c5 (chain_sparse at d = 2^22).
//
// c5's chain (psgd_sparse.hip) does, per sample, 100 scattered 4-byte gathers from its chain's
// 16 MiB fp32 weight vector (global_load_dword ... sc1) and 100 dependent 4-byte stores back to
// the same words (global_store_dword), one wave per chain, 1,024 chains = a 17 GB footprint.
// This kernel does that memory work and nothing else (no row stream, no dot, no reduction), with
// the product's instructions, columns drawn as c5's are (one per 1/100 of the feature range):
//   MODE 0: gathers (sc1) + stores   -- the c5 pattern
//   MODE 1: gathers (sc1) only
//   MODE 2: stores only
//   MODE 3: gathers without sc1 + stores
//   MODE 4: stores only, nt;  MODE 5: stores only, sc1 (cache-policy A/B of the scattered stores;
//   run under rocprofv3 --pmc WRITE_SIZE with a small d to see whether they stay in L2)
// DEPTH rows' gathers are in flight before the group's stores (DEPTH = 1: each row's stores
// wait for its own gathers, the chain's dependence; deeper: independent rows, the rate a deeper
// pipeline could reach). The best rate over the depths is the pattern's ceiling on this chip.
// ELEM = 8 (4th argument): the same pattern on 8-byte words (global_load_dwordx2 ... sc1 /
// global_store_dwordx2), c5's fp64 chain (chain_sparse64) -- a 34 GB footprint.
// Usage: gather_bench [rows per chain = 20000] [chains = 1024] [d = 4194304] [elem bytes = 4]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__device__ __forceinline__ unsigned mix(unsigned h) {
    h ^= h >> 16; h *= 0x7feb352du; h ^= h >> 15; h *= 0x846ca68bu; h ^= h >> 16;
    return h;
}
template <int MODE>
__device__ __forceinline__ float gather(const float* p) {
    float v;
    if constexpr (MODE == 3) asm volatile("global_load_dword %0, %1, off" : "=v"(v) : "v"(p) : "memory");
    else asm volatile("global_load_dword %0, %1, off sc1" : "=v"(v) : "v"(p) : "memory");
    return v;
}
template <int MODE>
__device__ __forceinline__ double gather(const double* p) {
    double v;
    if constexpr (MODE == 3) asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
    else asm volatile("global_load_dwordx2 %0, %1, off sc1" : "=v"(v) : "v"(p) : "memory");
    return v;
}
// POL: 0 plain, 1 nt, 2 sc1
template <int POL>
__device__ __forceinline__ void store(float* p, float v) {
    if constexpr (POL == 1) asm volatile("global_store_dword %0, %1, off nt" : : "v"(p), "v"(v) : "memory");
    else if constexpr (POL == 2) asm volatile("global_store_dword %0, %1, off sc1" : : "v"(p), "v"(v) : "memory");
    else asm volatile("global_store_dword %0, %1, off" : : "v"(p), "v"(v) : "memory");
}
template <int POL>
__device__ __forceinline__ void store(double* p, double v) {
    if constexpr (POL == 1) asm volatile("global_store_dwordx2 %0, %1, off nt" : : "v"(p), "v"(v) : "memory");
    else if constexpr (POL == 2) asm volatile("global_store_dwordx2 %0, %1, off sc1" : : "v"(p), "v"(v) : "memory");
    else asm volatile("global_store_dwordx2 %0, %1, off" : : "v"(p), "v"(v) : "memory");
}

__device__ unsigned long long* g_chain_clk = nullptr;   // [chains][2]: start / end (s_memrealtime), optional

template <typename E, int MODE, int DEPTH>
__global__ __launch_bounds__(64) void gather_store(E* W, long stride, int rows, unsigned width, int nnz) {
    const int lane = threadIdx.x;
    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
    E* base = W + (long)blockIdx.x * stride;
    const unsigned key = mix(blockIdx.x * 0x9E3779B9u + 12345u);
    // inactive lanes (entries >= nnz) use a private dummy word past the vector, as the product does
    E* dummy = base + (long)width * nnz + lane;
    E acc = 0;
    for (int r = 0; r < rows; r += DEPTH) {
        E* p0[DEPTH];
        E* p1[DEPTH];
        E g0[DEPTH], g1[DEPTH];
#pragma unroll
        for (int q = 0; q < DEPTH; ++q) {
            const unsigned h = mix(key ^ (unsigned)(r + q) * 0x85EBCA6Bu);
            p0[q] = lane < nnz ? base + (long)lane * width + mix(h + lane) % width : dummy;
            p1[q] = lane + 64 < nnz ? base + (long)(lane + 64) * width + mix(h + lane + 64) % width : dummy;
            if constexpr (MODE != 2 && MODE != 4 && MODE != 5) {
                g0[q] = gather<MODE>(p0[q]);
                g1[q] = gather<MODE>(p1[q]);
            } else {
                g0[q] = g1[q] = E(1);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int q = 0; q < DEPTH; ++q) {
            if constexpr (MODE != 1) {
                constexpr int POL = MODE == 4 ? 1 : MODE == 5 ? 2 : 0;
                store<POL>(p0[q], g0[q] + E(1));
                store<POL>(p1[q], g1[q] + E(1));
            }
            acc += g0[q] + g1[q];
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (acc == E(12345.678)) base[0] = acc;
    if (g_chain_clk && lane == 0) {
        g_chain_clk[2 * blockIdx.x] = t_start;
        g_chain_clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    }
}

// per-chain durations of the last launch (g_chain_clk), as a distribution
static void chain_spread(const char* tag, int chains) {
    std::vector<unsigned long long> h(2 * chains);
    unsigned long long* dptr;
    CK(hipMemcpyFromSymbol(&dptr, HIP_SYMBOL(g_chain_clk), sizeof(dptr)));
    CK(hipMemcpy(h.data(), dptr, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    std::vector<double> t(chains);
    unsigned long long t0 = ~0ull;
    for (int c = 0; c < chains; ++c) t0 = std::min(t0, h[2 * c]);
    for (int c = 0; c < chains; ++c) t[c] = (double)(h[2 * c + 1] - h[2 * c]) / 100.0;   // s_memrealtime: 100 MHz
    std::vector<double> u = t;
    std::sort(u.begin(), u.end());
    double xcd[8] = {0};
    for (int c = 0; c < chains; ++c) xcd[c % 8] += t[c] / (chains / 8);
    printf("    %s per-chain us: min %.0f p10 %.0f median %.0f p90 %.0f max %.0f | by XCD (c %% 8):", tag, u[0],
           u[chains / 10], u[chains / 2], u[chains * 9 / 10], u[chains - 1]);
    for (int x = 0; x < 8; ++x) printf(" %.0f", xcd[x]);
    printf("\n");
}

template <typename E, int MODE, int DEPTH>
static float run(E* W, long stride, int rows, int chains, unsigned width, int nnz) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    float best = 1e30f;
    for (int it = 0; it < 3; ++it) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL((gather_store<E, MODE, DEPTH>), dim3(chains), dim3(64), 0, 0, W, stride, rows, width, nnz);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
    }
    return best;
}

template <typename E>
static void run_all(int rows, int chains, unsigned d) {
    const int nnz = 100;
    const unsigned width = d / nnz;
    const long stride = ((long)d + 1152 + 63) / 64 * 64;   // as the product's wf32 stride (in elements)
    E* W;
    CK(hipMalloc(&W, (size_t)chains * stride * sizeof(E)));
    CK(hipMemset(W, 0, (size_t)chains * stride * sizeof(E)));
    printf("gather_bench: %d chains x %d rows x %d entries of %d bytes, d = %u (%.1f GB of weights)\n", chains,
           rows, nnz, (int)sizeof(E), d, (double)chains * stride * sizeof(E) / 1e9);
    const double R = (double)rows * chains;
    const char* names[6] = {"gather sc1 + store (c5)", "gather sc1 only", "store only", "gather plain + store",
                            "store only (nt)", "store only (sc1)"};
    auto report = [&](int mode, int depth, float ms) {
        printf("  %-24s depth %2d: %8.3f ms  %7.1f M rows/s  %6.2f G lane-requests/s\n", names[mode], depth, ms,
               R / ms / 1e3, R * (mode == 0 || mode == 3 ? 2 : 1) * nnz / ms / 1e6);
    };
#define RUN(M) \
    report(M, 1, run<E, M, 1>(W, stride, rows, chains, width, nnz)); \
    report(M, 4, run<E, M, 4>(W, stride, rows, chains, width, nnz)); \
    report(M, 16, run<E, M, 16>(W, stride, rows, chains, width, nnz));
    RUN(0) RUN(1) RUN(2) RUN(3) RUN(4) RUN(5)
#undef RUN
    CK(hipFree(W));
}

// Placement sweep (argv[1] = "place"): the c5 pattern (mode 0, depth 1) over a vector set
// allocated after PRE GB of other allocations (held while it runs) and with its base moved by OFF
// bytes -- does where the 17 / 34 GB of chain vectors land decide c5's speed?
template <typename E>
static void place_sweep(int rows, int chains, unsigned d) {
    const int nnz = 100;
    const unsigned width = d / nnz;
    const long stride = ((long)d + 1152 + 63) / 64 * 64;
    const size_t bytes = (size_t)chains * stride * sizeof(E);
    const double R = (double)rows * chains;
    const int pres[] = {0, 8, 16, 24, 32, 48, 64, 100};
    const long offs[] = {0};
    for (int pre : pres) {
        void* P = nullptr;
        if (pre) CK(hipMalloc(&P, (size_t)pre << 30));
        char* raw;
        CK(hipMalloc(&raw, bytes + (4 << 20)));
        CK(hipMemset(raw, 0, bytes + (4 << 20)));
        for (long off : offs) {
            E* W = reinterpret_cast<E*>(raw + off);
            const float ms = run<E, 0, 1>(W, stride, rows, chains, width, nnz);
            printf("  pre %3d GB  base %#14lx + %8ld: %8.3f ms  %7.1f M rows/s\n", pre, (unsigned long)(uintptr_t)raw,
                   off, ms, R / ms / 1e3);
            chain_spread("", chains);
        }
        // the same placement: gathers only, stores only
        const float m1 = run<E, 1, 1>(reinterpret_cast<E*>(raw), stride, rows, chains, width, nnz);
        const float m2 = run<E, 2, 1>(reinterpret_cast<E*>(raw), stride, rows, chains, width, nnz);
        const float m4 = run<E, 2, 16>(reinterpret_cast<E*>(raw), stride, rows, chains, width, nnz);
        printf("    gathers only %8.3f ms | stores only %8.3f ms | stores only, depth 16 %8.3f ms\n", m1, m2, m4);
        fflush(stdout);
        CK(hipFree(raw));
        if (P) CK(hipFree(P));
    }
}

// The same sweep with the vector set mapped through the virtual memory API: VA reserved at
// ALIGN_GB alignment, physical memory in handles of CH_MB (0: one handle), then mapped
// (argv[1] = "vmm", argv[2] = elem, argv[3] = ALIGN_GB, argv[4] = CH_MB); each placement is also
// run on a hipMalloc'd set in the same state, the control.
template <typename E>
static void vmm_sweep(int rows, int chains, unsigned d, size_t align_gb, size_t ch_gb) {
    const int nnz = 100;
    const unsigned width = d / nnz;
    const long stride = ((long)d + 1152 + 63) / 64 * 64;
    const double R = (double)rows * chains;
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    size_t gran = 0;
    CK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended));
    const size_t need = (size_t)chains * stride * sizeof(E);
    const size_t bytes = (need + gran - 1) / gran * gran;
    size_t ch = ch_gb ? (ch_gb << 20) : bytes;   // (argv[4] in MB)
    ch = (ch + gran - 1) / gran * gran;
    printf("vmm: granularity %zu, %zu bytes, VA alignment %zu GB, handles of %zu bytes\n", gran, bytes, align_gb, ch);
    const int pres[] = {0, 8, 16, 24, 32, 48};
    for (int pre : pres) {
        void* P = nullptr;
        if (pre) CK(hipMalloc(&P, (size_t)pre << 30));
        // (the runtime does not honour a large alignment argument: reserve ALIGN more and map at
        // the first ALIGN-aligned address inside the reservation)
        void* res = nullptr;
        const size_t al = align_gb << 30;
        CK(hipMemAddressReserve(&res, bytes + al, 0, nullptr, 0));
        void* va = (void*)(((uintptr_t)res + al - 1) / al * al);
        const size_t nh = (bytes + ch - 1) / ch;
        hipMemGenericAllocationHandle_t* h = new hipMemGenericAllocationHandle_t[nh];
        for (size_t i = 0; i < nh; ++i) {
            const size_t sz = i + 1 < nh ? ch : bytes - i * ch;
            CK(hipMemCreate(&h[i], sz, &prop, 0));
            CK(hipMemMap((char*)va + i * ch, sz, 0, h[i], 0));
        }
        hipMemAccessDesc acc = {};
        acc.location = prop.location;
        acc.flags = hipMemAccessFlagsProtReadWrite;
        CK(hipMemSetAccess(va, bytes, &acc, 1));
        CK(hipMemset(va, 0, bytes));
        const float ms = run<E, 0, 1>(reinterpret_cast<E*>(va), stride, rows, chains, width, nnz);
        E* W;
        CK(hipMalloc(&W, need));
        CK(hipMemset(W, 0, need));
        const float ms2 = run<E, 0, 1>(W, stride, rows, chains, width, nnz);
        printf("  pre %3d GB  vmm %p: %8.3f ms %7.1f M rows/s | hipMalloc %p: %8.3f ms %7.1f M rows/s\n", pre, va, ms,
               R / ms / 1e3, (void*)W, ms2, R / ms2 / 1e3);
        fflush(stdout);
        CK(hipFree(W));
        CK(hipMemUnmap(va, bytes));
        for (size_t i = 0; i < nh; ++i) CK(hipMemRelease(h[i]));
        delete[] h;
        CK(hipMemAddressFree(res, bytes + al));
        if (P) CK(hipFree(P));
    }
}

// Is "fast" a property of physical blocks? (argv[1] = "blocks", argv[2] = elem): 32 handles of
// 2 GB, each probed alone with the c5 pattern scaled to 2 GB (1,024 chains, 2,000 rows); then
// the c5 set (17 GB / 34 GB) mapped from the best-probing handles and from the worst.
template <typename E, int PM>
static void block_sweep(int nblk) {
    const int nnz = 100, chains = 1024;
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    hipMemAccessDesc acc = {};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    const size_t hb = (size_t)2 << 30;
    // the probe: per-chain vectors of d' elements inside one 2 GB handle
    const long pstride = (long)(hb / sizeof(E) / chains) / 64 * 64;
    const unsigned pd = (unsigned)(pstride - 1152 - 64) / nnz * nnz;
    std::vector<hipMemGenericAllocationHandle_t> h(nblk);
    std::vector<void*> va(nblk);
    std::vector<float> ms(nblk);
    for (int i = 0; i < nblk; ++i) {
        CK(hipMemCreate(&h[i], hb, &prop, 0));
        CK(hipMemAddressReserve(&va[i], hb, 0, nullptr, 0));
        CK(hipMemMap(va[i], hb, 0, h[i], 0));
        CK(hipMemSetAccess(va[i], hb, &acc, 1));
        CK(hipMemset(va[i], 0, hb));
    }
    for (int i = 0; i < nblk; ++i) {
        ms[i] = run<E, PM, 1>(reinterpret_cast<E*>(va[i]), pstride, 2000, chains, pd / nnz, nnz);
        printf("  block %2d at %p: %7.3f ms  %7.1f M rows/s\n", i, va[i], ms[i], 2000.0 * chains / ms[i] / 1e3);
    }
    fflush(stdout);
    std::vector<int> ord(nblk);
    for (int i = 0; i < nblk; ++i) ord[i] = i;
    std::sort(ord.begin(), ord.end(), [&](int a, int b) { return ms[a] < ms[b]; });
    const unsigned d = 1u << 22;
    const long stride = ((long)d + 1152 + 63) / 64 * 64;
    const size_t need = (size_t)chains * stride * sizeof(E);
    const int k = (int)((need + hb - 1) / hb);
    const double R = 20000.0 * chains;
    for (int pass = 0; pass < 2; ++pass) {
        if (k > nblk) break;
        void* set;
        CK(hipMemAddressReserve(&set, (size_t)k * hb, 0, nullptr, 0));
        for (int j = 0; j < k; ++j) {
            const int b = pass == 0 ? ord[j] : ord[nblk - 1 - j];
            CK(hipMemMap((char*)set + (size_t)j * hb, hb, 0, h[b], 0));
        }
        CK(hipMemSetAccess(set, (size_t)k * hb, &acc, 1));
        const float t = run<E, 0, 1>(reinterpret_cast<E*>(set), stride, 20000, chains, d / nnz, nnz);
        const float t2 = run<E, 2, 1>(reinterpret_cast<E*>(set), stride, 20000, chains, d / nnz, nnz);
        printf("  c5 set from the %s %d blocks: %8.3f ms  %7.1f M rows/s (stores only %8.3f ms)\n", pass == 0 ? "best" : "worst", k, t, R / t / 1e3, t2);
        fflush(stdout);
        CK(hipMemUnmap(set, (size_t)k * hb));
        CK(hipMemAddressFree(set, (size_t)k * hb));
    }
    for (int i = 0; i < nblk; ++i) {
        CK(hipMemUnmap(va[i], hb));
        CK(hipMemAddressFree(va[i], hb));
        CK(hipMemRelease(h[i]));
    }
}

// Placement re-roll (argv[1] = "reroll", argv[2] = elem, argv[3] = K): hold K hipMalloc'd
// candidates for the vector set, probe each with 2,000 rows of scattered stores, keep the fastest
// and free the rest; then the full c5 pattern on it. Repeated under several pre-allocations.
template <typename E>
static void reroll(int K) {
    const int nnz = 100, chains = 1024;
    const unsigned d = 1u << 22, width = d / nnz;
    const long stride = ((long)d + 1152 + 63) / 64 * 64;
    const size_t bytes = (size_t)chains * stride * sizeof(E);
    const double R = 20000.0 * chains;
    const int pres[] = {0, 8, 16, 24, 32, 48, 64, 100};
    for (int pre : pres) {
        void* P = nullptr;
        if (pre) CK(hipMalloc(&P, (size_t)pre << 30));
        std::vector<E*> cand(K);
        std::vector<float> pm(K);
        int best = 0;
        for (int k = 0; k < K; ++k) {
            CK(hipMalloc(&cand[k], bytes));
            pm[k] = run<E, 2, 1>(cand[k], stride, 2000, chains, width, nnz);
            if (pm[k] < pm[best]) best = k;
        }
        for (int k = 0; k < K; ++k) if (k != best) CK(hipFree(cand[k]));
        const float t = run<E, 0, 1>(cand[best], stride, 20000, chains, width, nnz);
        printf("  pre %3d GB: probes (ms)", pre);
        for (int k = 0; k < K; ++k) printf(" %6.3f%s", pm[k], k == best ? "*" : "");
        printf(" -> c5 pattern %8.3f ms  %7.1f M rows/s\n", t, R / t / 1e3);
        fflush(stdout);
        CK(hipFree(cand[best]));
        if (P) CK(hipFree(P));
    }
}

// Re-roll with spacers (argv[1] = "spacer", elem, ARENA_GB, K, SPACER_GB): an ARENA_GB allocation
// first (the bench's data), then K candidates with a SPACER_GB allocation after each (all held);
// the probes, and the full c5 pattern on the best candidate and on the first.
template <typename E>
static void spacer_roll(int arena_gb, int K, int spacer_gb) {
    const int nnz = 100, chains = 1024;
    const unsigned d = 1u << 22, width = d / nnz;
    const long stride = ((long)d + 1152 + 63) / 64 * 64;
    const size_t bytes = (size_t)chains * stride * sizeof(E);
    void* A = nullptr;
    if (arena_gb) CK(hipMalloc(&A, (size_t)arena_gb << 30));
    std::vector<E*> cand(K);
    std::vector<void*> sp(K, nullptr);
    std::vector<float> pm(K);
    int best = 0;
    for (int k = 0; k < K; ++k) {
        CK(hipMalloc(&cand[k], bytes));
        if (spacer_gb) CK(hipMalloc(&sp[k], (size_t)spacer_gb << 30));
        run<E, 2, 1>(cand[k], stride, 2000, chains, width, nnz);
        pm[k] = run<E, 2, 1>(cand[k], stride, 2000, chains, width, nnz);
        if (pm[k] < pm[best]) best = k;
    }
    const float t0 = run<E, 0, 1>(cand[0], stride, 20000, chains, width, nnz);
    const float tb = run<E, 0, 1>(cand[best], stride, 20000, chains, width, nnz);
    printf("  arena %3d GB, %d candidates, spacer %2d GB: probes", arena_gb, K, spacer_gb);
    for (int k = 0; k < K; ++k) printf(" %6.3f%s", pm[k], k == best ? "*" : "");
    printf(" | c5 pattern: first %8.3f ms, best %8.3f ms\n", t0, tb);
    fflush(stdout);
    for (int k = 0; k < K; ++k) {
        CK(hipFree(cand[k]));
        if (sp[k]) CK(hipFree(sp[k]));
    }
    if (A) CK(hipFree(A));
}

int main(int argc, char** argv) {
    if (argc > 1 && argv[1][0] == 's') {
        const int elem = argc > 2 ? atoi(argv[2]) : 4;
        const int arena = argc > 3 ? atoi(argv[3]) : 16;
        const int K = argc > 4 ? atoi(argv[4]) : 3;
        const int sp = argc > 5 ? atoi(argv[5]) : 0;
        if (elem == 8) spacer_roll<double>(arena, K, sp);
        else spacer_roll<float>(arena, K, sp);
        return 0;
    }
    if (argc > 1 && argv[1][0] == 'r') {
        const int elem = argc > 2 ? atoi(argv[2]) : 4;
        const int K = argc > 3 ? atoi(argv[3]) : 3;
        if (elem == 8) reroll<double>(K);
        else reroll<float>(K);
        return 0;
    }
    {
        unsigned long long* clk;
        CK(hipMalloc(&clk, 2 * 8192 * sizeof(unsigned long long)));
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_chain_clk), &clk, sizeof(clk)));
    }
    if (argc > 1 && argv[1][0] == 'b') {
        const int elem = argc > 2 ? atoi(argv[2]) : 4;
        const int nblk = argc > 3 ? atoi(argv[3]) : 32;
        const int pm = argc > 4 ? atoi(argv[4]) : 0;   // the probe: 0 gathers + stores, 2 stores only
        if (elem == 8) { if (pm == 2) block_sweep<double, 2>(nblk); else block_sweep<double, 0>(nblk); }
        else { if (pm == 2) block_sweep<float, 2>(nblk); else block_sweep<float, 0>(nblk); }
        return 0;
    }
    if (argc > 1 && argv[1][0] == 'v') {
        const int elem = argc > 2 ? atoi(argv[2]) : 4;
        const size_t al = argc > 3 ? (size_t)atol(argv[3]) : 1;
        const size_t ch = argc > 4 ? (size_t)atol(argv[4]) : 0;
        if (elem == 8) vmm_sweep<double>(20000, 1024, 1u << 22, al, ch);
        else vmm_sweep<float>(20000, 1024, 1u << 22, al, ch);
        return 0;
    }
    if (argc > 1 && argv[1][0] == 'p') {
        const int elem = argc > 2 ? atoi(argv[2]) : 4;
        if (elem == 8) place_sweep<double>(20000, 1024, 1u << 22);
        else place_sweep<float>(20000, 1024, 1u << 22);
        return 0;
    }
    const int rows = argc > 1 ? atoi(argv[1]) : 20000;
    const int chains = argc > 2 ? atoi(argv[2]) : 1024;
    const unsigned d = argc > 3 ? (unsigned)atol(argv[3]) : (1u << 22);
    const int elem = argc > 4 ? atoi(argv[4]) : 4;
    if (elem == 8) run_all<double>(rows, chains, d);
    else run_all<float>(rows, chains, d);
    return 0;
}
