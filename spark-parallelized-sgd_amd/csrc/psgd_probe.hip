// psgd_probe.hip -- the placement probe of the CSR chains' per-chain weight vectors (gfx950).
//
// The CSR kernels keep each chain's weights (or their tail past the LDS head) in one vector of
// the context's wf32 buffer and read-modify-write 4 / 8-byte words of it at the row's columns
// (ParallelizedSGD.scala:254-255: the gradient's axpy into the chain's local weights). Measured
// round 6 (tools/c4_placement.py, tools/place_probe.hip): the rate of those
// scattered accesses is a property of the allocation the buffer received -- the same rows run the
// c4 launch in 27.4 or 31.3 ms depending only on which allocation of the 50 MB vector set the
// context holds, repeatably -- and a short random read-modify-write pattern over each chain's
// vector separates the two kinds of allocation the same way (~1.13 against ~1.38 ms). The
// context re-rolls such a buffer once, when it allocates it (psgd_capi.cpp, reroll_vectors):
// a few candidates are probed with this kernel and the fastest is kept.
#include "psgd_internal.h"

namespace psgd {

namespace {
// One wave per chain (the chain kernels' workgroup -> chain mapping); each lane `iters`
// xorshift-random words of the chain's vector [0, d) (the kernels' vectors are stride words
// apart); the words' contents are garbage afterwards (every epoch re-initialises the vectors).
__global__ __launch_bounds__(64) void vector_probe_kernel(float* __restrict__ w, int64_t stride, int d,
                                                          int iters, unsigned seed) {
    float* v = w + (int64_t)blockIdx.x * stride;
    unsigned s = seed ^ (blockIdx.x * 0x9E3779B9u) ^ (threadIdx.x * 0x85EBCA6Bu) ^ 1u;
    const unsigned span = (unsigned)(d > 0 ? d : 1);
    for (int i = 0; i < iters; ++i) {
        s ^= s << 13;
        s ^= s >> 17;
        s ^= s << 5;
        const int f = (int)(s % span);
        const float x = __builtin_nontemporal_load(v + f);
        v[f] = x + 1.0f;
    }
}
}  // namespace

int launch_vector_probe(float* w, int64_t stride_words, int n_vectors, int d_words, int iters, unsigned seed,
                        hipStream_t st) {
    if (n_vectors <= 0) return 0;
    hipLaunchKernelGGL(vector_probe_kernel, dim3(n_vectors), dim3(64), 0, st, w, stride_words, d_words, iters, seed);
    return (int)hipGetLastError();
}

}  // namespace psgd
