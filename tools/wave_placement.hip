// wave_placement.hip -- which SIMD each wave of a one-workgroup-per-CU launch lands on (gfx950).
// The chain kernels give each wave one role (chain, loader, Gram ...) and assume the roles that
// must not share a SIMD do not; this reads HW_REG_HW_ID (SIMD_ID = bits 5:4, CU_ID = 11:8) per
// wave and prints, per workgroup size, how often each wave-to-SIMD pattern occurs.
// Usage: wave_placement [workgroups = 256]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <map>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void probe(unsigned* out, int spin) {
    extern __shared__ char smem[];
    unsigned id;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(id));
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 16 + (threadIdx.x >> 6)] = id;
    smem[threadIdx.x] = 0;
    // stay resident a while so that the workgroups overlap as the chain kernels' do
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)spin) {}
}

int main(int argc, char** argv) {
    const int wgs = argc > 1 ? atoi(argv[1]) : 256;
    unsigned* d;
    CK(hipMalloc(&d, (size_t)wgs * 16 * 4));
    const size_t lds = 150 * 1024;   // one workgroup per CU
    CK(hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    for (int waves = 3; waves <= 8; ++waves) {
        CK(hipMemset(d, 0xff, (size_t)wgs * 16 * 4));
        hipLaunchKernelGGL(probe, dim3(wgs), dim3(64 * waves), lds, 0, d, 100000);
        CK(hipDeviceSynchronize());
        std::vector<unsigned> h((size_t)wgs * 16);
        CK(hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost));
        std::map<std::string, int> pat;
        for (int b = 0; b < wgs; ++b) {
            std::string s;
            const unsigned s0 = (h[(size_t)b * 16] >> 4) & 3;
            for (int w = 0; w < waves; ++w) {
                const unsigned simd = (h[(size_t)b * 16 + w] >> 4) & 3;
                s += char('0' + ((simd - s0) & 3));   // relative to wave 0's SIMD
            }
            pat[s]++;
        }
        printf("%d waves per workgroup: wave -> SIMD (relative to wave 0's), count of %d workgroups\n", waves, wgs);
        for (auto& kv : pat) printf("   %s  %d\n", kv.first.c_str(), kv.second);
    }
    return 0;
}
