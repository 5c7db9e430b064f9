// sigmoid_check.hip -- accuracy of chain_block64's short-chain 1/(1+exp(m)) (recip_one_plus_exp) against
// host libm and against the device library exp + IEEE division, over 1M margins incl. the edges.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <math.h>
#include <stdlib.h>
#define PSGD_NO_DISPATCH 1
#include "../spark-parallelized-sgd_amd/csrc/psgd_block64.hip"
int psgd::launch_logistic_loss64(const psgd::ChainLaunch&, int, hipStream_t) { return 0; }
__global__ void k(const double* m, double* a, double* b, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { a[i] = psgd::recip_one_plus_exp(m[i]); b[i] = 1.0 / (1.0 + exp(m[i])); }
}
int main() {
    const int n = 1 << 20;
    double *m, *a, *b;
    hipMallocManaged(&m, n * 8); hipMallocManaged(&a, n * 8); hipMallocManaged(&b, n * 8);
    srand(1);
    for (int i = 0; i < n; ++i) m[i] = (i < 16) ? (double[]){0, 1e-300, -1e-300, 709, 710, 800, -745, -746, -800, 30, -30, 0.5, -0.5, 1e-17, NAN, INFINITY}[i] : ((double)rand() / RAND_MAX - 0.5) * (i % 3 == 0 ? 100 : 4);
    hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, m, a, b, n);
    hipDeviceSynchronize();
    double worst = 0, worst_host = 0; int wi = 0;
    for (int i = 0; i < n; ++i) {
        double ref = 1.0 / (1.0 + exp(m[i]));   // host libm
        if (isnan(ref)) { if (!isnan(a[i])) printf("NaN mismatch at %d\n", i); continue; }
        double e = ref == 0 ? fabs(a[i]) : fabs(a[i] - ref) / ref;
        if (e > worst) { worst = e; wi = i; }
        double eh = ref == 0 ? fabs(b[i]) : fabs(b[i] - ref) / ref;
        if (eh > worst_host) worst_host = eh;
    }
    printf("fast vs host libm: worst rel %.3g at m=%.17g (%.17g vs %.17g); ocml vs host: %.3g\n", worst, m[wi], a[wi], 1.0/(1.0+exp(m[wi])), worst_host);
    for (int i = 0; i < 16; ++i) printf("m=%g fast=%.17g ocml=%.17g\n", m[i], a[i], b[i]);
    return 0;
}
