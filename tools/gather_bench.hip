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

template <typename E, int MODE, int DEPTH>
__global__ __launch_bounds__(64) void gather_store(E* W, long stride, int rows, unsigned width, int nnz) {
    const int lane = threadIdx.x;
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

int main(int argc, char** argv) {
    const int rows = argc > 1 ? atoi(argv[1]) : 20000;
    const int chains = argc > 2 ? atoi(argv[2]) : 1024;
    const unsigned d = argc > 3 ? (unsigned)atol(argv[3]) : (1u << 22);
    const int elem = argc > 4 ? atoi(argv[4]) : 4;
    if (elem == 8) run_all<double>(rows, chains, d);
    else run_all<float>(rows, chains, d);
    return 0;
}
