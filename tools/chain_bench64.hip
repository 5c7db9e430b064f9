// chain_bench64.hip -- diagnostic: the fp64 blocked chain kernel (psgd_block64.hip, compiled here
// with -DPSGD_STAMPS) on f32 or f64 rows of the bench workload's shape, per-wave s_memtime
// counters:
//   chain wave 0: total, waiting for rows, waiting for the Gram triangle, for the other chain
//                 wave's partial dots (two chain waves)
//   loader:       total, blocked on a full ring, in its vmcnt wait
//   Gram waves:   total, waiting for rows
// Usage: chain_bench64 <rows per chain> <chains> <d> <grad 0|1|2> <upd 0|1> [storage bytes 4|8]
//                      [chain waves 1|2] [tol: > 0 runs the per-sample break instance]
#define PSGD_STAMPS 1
#define PSGD_NO_DISPATCH 1
#include "../spark-parallelized-sgd_amd/csrc/psgd_block64.hip"
// the row-loss kernel lives in psgd_kernels.hip; the diagnostic times the chain only
int psgd::launch_logistic_loss64(const psgd::ChainLaunch&, int, hipStream_t) { return 0; }

#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void fill(float* x, size_t n, unsigned seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned h = (unsigned)i * 2654435761u ^ seed;
        h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
        x[i] = (float)((int)(h & 0xffff) - 32768) / 32768.0f;
    }
}
__global__ void widen(const float* x, double* y, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        y[i] = x[i];
}
__global__ void fill_d(double* x, size_t n, double v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        x[i] = v;
}

// f64 compute on f32 rows (d = 256 / 512 / 1024: NV = 1 / 2 / 4) or f64 rows (d = 512 / 1024:
// NV = 4 / 8), full rows; H chain waves
template <typename S, int H, bool C>
static int launch_s(const psgd::ChainLaunch& L, const psgd::KParams& kp, int grad, int upd, int d) {
    const size_t lds = 160 * 1024 - 512;
    constexpr int VEC = 16 / sizeof(S);
#define NVCASE(G, U)                                                                              \
    if (grad == G && upd == U) {                                                                  \
        if constexpr (H == 1) if (d == 64 * VEC) return psgd::launch_block64<S, G, U, 1, 1, C>(L, kp, true, lds, 0); \
        if (d == 128 * VEC) return psgd::launch_block64<S, G, U, 2, H, C>(L, kp, true, lds, 0);      \
        if (d == 256 * VEC) return psgd::launch_block64<S, G, U, 4, H, C>(L, kp, true, lds, 0);      \
        if constexpr (H == 2) if (d == 512 * VEC) return psgd::launch_block64<S, G, U, 8, 2, C>(L, kp, true, lds, 0); \
    }
    NVCASE(0, 0) NVCASE(1, 0) NVCASE(0, 1) NVCASE(1, 1)
#undef NVCASE
    return -3;
}
template <bool C>
static int launch_c(const psgd::ChainLaunch& L, const psgd::KParams& kp, int grad, int upd, int d, int es, int H) {
    if (es == 4) return H == 1 ? launch_s<float, 1, C>(L, kp, grad, upd, d) : launch_s<float, 2, C>(L, kp, grad, upd, d);
    return H == 1 ? launch_s<double, 1, C>(L, kp, grad, upd, d) : launch_s<double, 2, C>(L, kp, grad, upd, d);
}
static int launch(const psgd::ChainLaunch& L, const psgd::KParams& kp, int grad, int upd, int d, int es, int H) {
    return kp.tol > 0.0 ? launch_c<true>(L, kp, grad, upd, d, es, H) : launch_c<false>(L, kp, grad, upd, d, es, H);
}

int main(int argc, char** argv) {
    const int64_t rows = argc > 1 ? atoll(argv[1]) : 39062;
    const int P = argc > 2 ? atoi(argv[2]) : 256;
    const int d = argc > 3 ? atoi(argv[3]) : 512;
    const int grad = argc > 4 ? atoi(argv[4]) : 1;
    const int upd = argc > 5 ? atoi(argv[5]) : 0;
    const int es = argc > 6 ? atoi(argv[6]) : 4;
    const int H = argc > 7 ? atoi(argv[7]) : 2;
    const double tol = argc > 8 ? atof(argv[8]) : 0.0;   // > 0: the per-sample break instance
    const size_t nx = (size_t)rows * P * d;
    float* X; double* Xd = nullptr; double *y, *steps, *w_in, *w_out, *rv, *loss, *cnt_d; int64_t* cnt; int* wd;
    unsigned long long* stamps;
    CK(hipMalloc(&X, nx * 4));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, X, nx, 12345u);
    if (es == 8) {
        CK(hipMalloc(&Xd, nx * 8));
        hipLaunchKernelGGL(widen, dim3(4096), dim3(256), 0, 0, X, Xd, nx);
        CK(hipDeviceSynchronize());
        CK(hipFree(X));
        X = nullptr;
    }
    CK(hipMalloc(&y, rows * P * 8)); hipLaunchKernelGGL(fill_d, dim3(1024), dim3(256), 0, 0, y, (size_t)rows * P, 0.5);
    CK(hipMalloc(&steps, rows * 8)); hipLaunchKernelGGL(fill_d, dim3(1024), dim3(256), 0, 0, steps, (size_t)rows, 1e-3);
    CK(hipMalloc(&w_in, d * 8)); CK(hipMemset(w_in, 0, d * 8));
    CK(hipMalloc(&w_out, (size_t)P * d * 8));
    CK(hipMalloc(&rv, P * 8)); CK(hipMalloc(&loss, P * 8)); CK(hipMalloc(&cnt_d, P * 8)); CK(hipMalloc(&cnt, P * 8));
    CK(hipMalloc(&wd, 16)); CK(hipMemset(wd, 0, 16));
    CK(hipMalloc(&stamps, (size_t)P * 16 * 8)); CK(hipMemset(stamps, 0, (size_t)P * 16 * 8));
    std::vector<psgd::ChainDesc> h(P);
    for (int p = 0; p < P; ++p) {
        h[p] = psgd::ChainDesc{};
        h[p].x = es == 8 ? (const void*)(Xd + (size_t)p * rows * d) : (const void*)(X + (size_t)p * rows * d);
        h[p].y = y + (size_t)p * rows;
        h[p].n_rows = rows;
        h[p].ld = d;
    }
    psgd::ChainDesc* dd;
    CK(hipMalloc(&dd, P * sizeof(psgd::ChainDesc)));
    CK(hipMemcpy(dd, h.data(), P * sizeof(psgd::ChainDesc), hipMemcpyHostToDevice));
    psgd::ChainLaunch L{};
    L.descs = dd; L.w_in = w_in; L.w_out = w_out; L.rv = rv; L.loss = loss; L.cnt_d = cnt_d;
    L.cnt = cnt; L.steps = steps; L.watchdog = wd; L.stamps = stamps;
    double* zbuf;
    CK(hipMalloc(&zbuf, (size_t)rows * P * 8));
    L.zbuf64 = zbuf; L.zstride = rows;
    psgd::KParams kp{};
    kp.reg = 0.01; kp.d = d; kp.n_chains = P; kp.tol = tol;
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    int variant = 0;
    float best = 1e30f;
    for (int it = 0; it < 4; ++it) {
        CK(hipEventRecord(a));
        int e = launch(L, kp, grad, upd, d, es, H);
        variant = 700 + 10 * (H - 1) + d * es / 1024;
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        if (e) { fprintf(stderr, "launch failed %d\n", e); return 1; }
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        if (it > 0) best = std::min(best, ms);
    }
    int w = 0;
    CK(hipMemcpy(&w, wd, 4, hipMemcpyDeviceToHost));
    std::vector<unsigned long long> st((size_t)P * 16);
    CK(hipMemcpy(st.data(), stamps, st.size() * 8, hipMemcpyDeviceToHost));
    const double bytes = (double)rows * P * (d + 1) * es;
    printf("variant %d  %.3f ms  %.1f GB/s  %.1f ns/row  watchdog=%d\n", variant, best, bytes / best / 1e6,
           best * 1e6 / rows, w);
    const char* names[16] = {"chain.total", "chain.wait_rows", "chain.wait_gram", "chain.p+reduce",
                             "loader.total", "loader.ring_full", "loader.vmcnt", "chain.wait_xchg",
                             "gram0.total", "gram0.wait_rows", "chain1.wait_xchg", "chain1.p+reduce",
                             "gram1.total", "gram1.wait_rows", "chain.recurrence", "chain.loss+update"};
    for (int k = 0; k < 16; ++k) {
        if (names[k][0] == '-') continue;
        std::vector<double> v(P);
        for (int p = 0; p < P; ++p) v[p] = (double)st[(size_t)p * 16 + k] / rows;
        std::sort(v.begin(), v.end());
        printf("  %-18s cycles/row  median %8.1f  min %8.1f  max %8.1f\n", names[k], v[P / 2], v[0], v[P - 1]);
    }
    return 0;
}
