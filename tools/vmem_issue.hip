// vmem_issue.hip -- what a scattered buffer instruction costs the wave that issues it (gfx950).
//
// chain_sparse_lds's tail wave issues 2 buffer stores + 2 buffer loads (sc1) per row with a
// per-lane offset each (scattered, or the no-access offset past num_records). This kernel runs
// that pattern alone, one workgroup of four waves per CU (every wave on its own SIMD, as in the
// kernel), and reports the cycles per iteration of one wave:
//   MODE 0: 2 stores + 2 loads, every lane no-access
//   MODE 1: 2 stores + 2 loads, scattered in-range offsets (a 128 KB vector per workgroup)
//   MODE 2: 1 store + 1 load (no-access)
//   MODE 3: nothing but the loop (and the same vmcnt wait)
// Usage: vmem_issue [iterations = 20000]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

typedef int i32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ i32x4 rsrc(const float* base, unsigned bytes) {
    const unsigned long long a = (unsigned long long)base;
    return i32x4{__builtin_amdgcn_readfirstlane((int)(unsigned)a), __builtin_amdgcn_readfirstlane((int)((a >> 32) & 0xFFFF)),
                 __builtin_amdgcn_readfirstlane((int)bytes), 0x00020000};
}
__device__ __forceinline__ float ld(i32x4 r, unsigned off) {
    float v;
    asm volatile("buffer_load_dword %0, %1, %2, 0 offen sc1" : "=v"(v) : "v"(off), "s"(r) : "memory");
    return v;
}
__device__ __forceinline__ void st(i32x4 r, unsigned off, float v) {
    asm volatile("buffer_store_dword %0, %1, %2, 0 offen" : : "v"(v), "v"(off), "s"(r) : "memory");
}
__device__ __forceinline__ unsigned mix(unsigned h) {
    h ^= h >> 16; h *= 0x7feb352du; h ^= h >> 15; h *= 0x846ca68bu; h ^= h >> 16;
    return h;
}

template <int MODE>
__global__ __launch_bounds__(256) void issue(float* W, int iters, unsigned long long* out) {
    const int lane = threadIdx.x & 63;
    float* base = W + (size_t)blockIdx.x * 32768;   // 128 KB per workgroup
    const i32x4 r = rsrc(base, 32768 * 4);
    float acc = 0.0f;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
        const unsigned h = mix((unsigned)(i * 0x9E3779B9u) ^ (threadIdx.x * 0x85EBCA6Bu));
        const unsigned o0 = MODE == 1 ? (h & 32767) * 4 : 0x80000000u;
        const unsigned o1 = MODE == 1 ? ((h >> 15) & 32767) * 4 : 0x80000000u;
        if constexpr (MODE != 3) {
            st(r, o0, acc);
            if constexpr (MODE != 2) st(r, o1, acc);
            float g0 = ld(r, o1);
            float g1 = MODE != 2 ? ld(r, o0) : 0.0f;
            asm volatile("s_waitcnt vmcnt(8)" : "+v"(g0), "+v"(g1) : : "memory");
            acc += g0 + g1;
        } else {
            asm volatile("s_waitcnt vmcnt(8)" : "+v"(acc) : : "memory");
            acc += 1.0f;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
    if (acc == 1234.5f) base[0] = acc;
}

template <int MODE>
static void run(float* W, int iters, unsigned long long* d_out, const char* name) {
    hipLaunchKernelGGL(issue<MODE>, dim3(256), dim3(256), 0, 0, W, iters, d_out);
    CK(hipDeviceSynchronize());
    unsigned long long h[1024];
    CK(hipMemcpy(h, d_out, sizeof h, hipMemcpyDeviceToHost));
    double s = 0;
    for (int i = 0; i < 1024; ++i) s += (double)h[i];
    printf("  %-40s %8.1f cycles per iteration per wave\n", name, s / 1024 / iters);
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 20000;
    float* W;
    unsigned long long* d_out;
    CK(hipMalloc(&W, (size_t)256 * 32768 * 4));
    CK(hipMemset(W, 0, (size_t)256 * 32768 * 4));
    CK(hipMalloc(&d_out, 1024 * 8));
    printf("vmem_issue: 256 workgroups x 4 waves, %d iterations (s_memtime cycles)\n", iters);
    for (int rep = 0; rep < 2; ++rep) {
        run<3>(W, iters, d_out, "loop only");
        run<2>(W, iters, d_out, "1 store + 1 load, no-access");
        run<0>(W, iters, d_out, "2 stores + 2 loads, no-access");
        run<1>(W, iters, d_out, "2 stores + 2 loads, scattered in range");
    }
    return 0;
}
