// newton_check.hip -- relative error of gfx950's v_rcp_f64 / v_rsq_f64 alone and after one and
// two Newton steps, against host IEEE 1/x and 1/sqrt(x), over 4M inputs in [1, 1e6) (the ranges
// of 1 + exp(m) and AdaGrad's accum + 1). Decides how many Newton steps the fp64 kernels need for
// their 1e-9 bar (psgd_device.h recip_one_plus_exp, rsqrt_newton).
// build: hipcc --offload-arch=gfx950 -O3 -o tools/newton_check tools/newton_check.hip
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

__global__ void k(const double* x, double* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double d = x[i];
    double r = __builtin_amdgcn_rcp(d);
    out[6 * i + 0] = r;
    r = __builtin_fma(r, __builtin_fma(-d, r, 1.0), r);
    out[6 * i + 1] = r;
    r = __builtin_fma(r, __builtin_fma(-d, r, 1.0), r);
    out[6 * i + 2] = r;
    double y = __builtin_amdgcn_rsq(d);
    out[6 * i + 3] = y;
    double e = __builtin_fma(-(d * y), y, 1.0);
    y = __builtin_fma(0.5 * y, e, y);
    out[6 * i + 4] = y;
    e = __builtin_fma(-(d * y), y, 1.0);
    y = __builtin_fma(0.5 * y, e, y);
    out[6 * i + 5] = y;
}

int main() {
    const int n = 1 << 22;
    double *x, *o;
    hipMallocManaged(&x, n * 8);
    hipMallocManaged(&o, 6 * (size_t)n * 8);
    srand(7);
    for (int i = 0; i < n; ++i) x[i] = 1.0 + pow(10.0, 6.0 * rand() / RAND_MAX) * ((double)rand() / RAND_MAX);
    hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, x, o, n);
    hipDeviceSynchronize();
    double worst[6] = {0, 0, 0, 0, 0, 0};
    for (int i = 0; i < n; ++i) {
        const double rr = 1.0 / x[i], rs = 1.0 / sqrt(x[i]);
        for (int j = 0; j < 6; ++j) {
            const double ref = j < 3 ? rr : rs;
            const double e = fabs(o[6 * (size_t)i + j] - ref) / ref;
            if (e > worst[j]) worst[j] = e;
        }
    }
    printf("v_rcp_f64: raw %.3g, 1 Newton %.3g, 2 Newton %.3g (max relative error, %d inputs in [1, 1e6))\n",
           worst[0], worst[1], worst[2], n);
    printf("v_rsq_f64: raw %.3g, 1 Newton %.3g, 2 Newton %.3g\n", worst[3], worst[4], worst[5]);
    return 0;
}
