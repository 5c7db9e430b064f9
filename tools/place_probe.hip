// place_probe.hip -- diagnostic: do allocations of c4's per-chain fp32 weight vectors (256 chains x
// 48,448 floats = 50 MB, psgd_capi.cpp wf32) differ in the rate of the chains' scattered 4-byte
// read-modify-writes, as the c4 kernel's per-context times do (tools/c4_placement.py)? Allocates
// K candidate sets and times the same random gather + store pattern on each: one workgroup (one
// wave) per chain, each lane NITER pseudo-random features of its chain's vector, past the LDS head.
// usage: place_probe [K=8] [iters=2000] [chains=256] [stride floats=48448] [head=21096] [d=47236]
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ __launch_bounds__(64) void probe(float* w, int stride, int head, int d, int iters, unsigned seed) {
    float* v = w + (size_t)blockIdx.x * stride;
    unsigned s = seed ^ (blockIdx.x * 0x9E3779B9u) ^ (threadIdx.x * 0x85EBCA6Bu);
    const unsigned span = (unsigned)(d - head);
    for (int i = 0; i < iters; ++i) {
        s ^= s << 13; s ^= s >> 17; s ^= s << 5;
        const int f = head + (int)(s % span);
        const float x = __builtin_nontemporal_load(v + f);
        v[f] = x + 1.0f;
    }
}

int main(int argc, char** argv) {
    const int K = argc > 1 ? atoi(argv[1]) : 8;
    const int iters = argc > 2 ? atoi(argv[2]) : 2000;
    const int P = argc > 3 ? atoi(argv[3]) : 256;
    const int stride = argc > 4 ? atoi(argv[4]) : 48448;
    const int head = argc > 5 ? atoi(argv[5]) : 21096;
    const int d = argc > 6 ? atoi(argv[6]) : 47236;
    std::vector<float*> bufs(K);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int k = 0; k < K; ++k) {
        CK(hipMalloc(&bufs[k], (size_t)P * stride * sizeof(float)));
        CK(hipMemset(bufs[k], 0, (size_t)P * stride * sizeof(float)));
    }
    CK(hipDeviceSynchronize());
    for (int rep = 0; rep < 3; ++rep) {
        printf("rep %d:", rep);
        for (int k = 0; k < K; ++k) {
            hipLaunchKernelGGL(probe, dim3(P), dim3(64), 0, 0, bufs[k], stride, head, d, iters, 12345u + rep);
            CK(hipEventRecord(a, 0));
            hipLaunchKernelGGL(probe, dim3(P), dim3(64), 0, 0, bufs[k], stride, head, d, iters, 777u + rep);
            CK(hipEventRecord(b, 0));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            printf(" %7.3f", ms);
        }
        printf("  ms (%d iters, %d chains)\n", iters, P);
    }
    for (auto p : bufs) CK(hipFree(p));
    return 0;
}
