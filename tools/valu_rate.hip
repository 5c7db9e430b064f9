// Issue cost of a few VALU forms on gfx950 (cycles per wave-instruction, one wave per SIMD):
// v_cvt_f64_f32, v_fma_f64, v_fma_f32 and v_pk_fma_f32, each in 8 independent chains.
#include <hip/hip_runtime.h>
#include <stdio.h>
template <int OP>
__global__ __launch_bounds__(256) void k(float* out, unsigned long long* cyc, int iters) {
    float f[8]; double d[8];
    for (int i = 0; i < 8; ++i) { f[i] = threadIdx.x * 1e-3f + i; d[i] = f[i]; }
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (OP == 0) { d[i] += (double)f[i]; f[i] = (float)d[i] * 0.5f; }   // cvt f32->f64 + f64 add + cvt back + mul
            if constexpr (OP == 1) d[i] = __builtin_fma(d[i], 1.0000001, 1e-9);
            if constexpr (OP == 2) f[i] = __builtin_fmaf(f[i], 1.0000001f, 1e-9f);
            if constexpr (OP == 3) d[i] = (double)f[i] + d[i] * 0.0;                       // cvt + fma
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0; for (int i = 0; i < 8; ++i) s += f[i] + (float)d[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x % 64 == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
}
template <int OP> void run(const char* name, int per_iter) {
    float* o; unsigned long long* c; const int B = 256, iters = 4096;
    hipMalloc(&o, B * 256 * 4); hipMalloc(&c, B * 4 * 8);
    hipLaunchKernelGGL(k<OP>, dim3(B), dim3(256), 0, 0, o, c, iters);
    hipLaunchKernelGGL(k<OP>, dim3(B), dim3(256), 0, 0, o, c, iters);
    unsigned long long h[4]; hipMemcpy(h, c, 32, hipMemcpyDeviceToHost);
    printf("%-28s %.2f cycles per loop-body instruction (per wave)\n", name, (double)h[0] / iters / (8.0 * per_iter));
    hipFree(o); hipFree(c);
}
int main() {
    run<0>("cvt64+add64+cvt32+mul32", 4);
    run<1>("fma_f64", 1);
    run<2>("fma_f32", 1);
    run<3>("cvt64+fma64", 2);
    return 0;
}
