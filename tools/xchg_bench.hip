// xchg_bench.hip -- cost of chain_split's per-sample cross-wave exchange on gfx950: H waves of a
// workgroup (one per SIMD) each publish a tagged 64-bit word in LDS and poll until all H words of
// the round carry the round's tag (the same code as psgd_split.hip's exchange), N rounds.
// Variants (argv[1]): 0 exchange only; 1 + a 6-step DPP wave reduction before it; 2 + a
// ds_read_b128 whose result feeds the reduction (a row prefetch); 3 = 2 + 8 dependent VALU ops
// after it (the multiplier); 4: a wave-local LDS write->read round trip alone (no other wave).
// One workgroup per CU (256), s_memtime cycles per round, median over workgroups.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/xchg_bench tools/xchg_bench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <vector>
#include <algorithm>

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL, int ROWS>
__device__ __forceinline__ float dpp_rows(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROWS, 0xF, false));
}
__device__ __forceinline__ float wsum(float v) {
    v = v + dpp<0xB1>(v);
    v = v + dpp<0x4E>(v);
    v = v + dpp<0x141>(v);
    v = v + dpp<0x140>(v);
    v = v + dpp_rows<0x142, 0xA>(v);
    v = v + dpp_rows<0x143, 0xC>(v);
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
__device__ __forceinline__ void wr64(uint64_t* p, uint64_t v) {
    asm volatile("ds_write_b64 %0, %1" : : "v"((unsigned)(uintptr_t)p), "v"(v) : "memory");
}
__device__ __forceinline__ uint64_t rd64(const uint64_t* p) {
    uint64_t v;
    asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"((unsigned)(uintptr_t)p) : "memory");
    return v;
}

template <int H, int VAR>
__global__ __launch_bounds__(64 * H) void xchg(int rounds, float* out, unsigned long long* cyc) {
    __shared__ uint64_t xw[2 * H];
    __shared__ float rowbuf[H][256];
    const int lane = threadIdx.x & 63, h = threadIdx.x >> 6;
    if (threadIdx.x < 2 * H) xw[threadIdx.x] = 0;
    for (int i = threadIdx.x; i < H * 256; i += blockDim.x) rowbuf[i / 256][i % 256] = 1.0f + i;
    __syncthreads();
    float acc = 0.0f, z = 1.0f;
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    for (int t = 0; t < rounds; ++t) {
        float part = z * 0.5f + (float)lane;
        if constexpr (VAR >= 2) {
            const float4 x = *reinterpret_cast<const float4*>(&rowbuf[h][(lane * 4) & 255]);
            part = part * x.x + x.y * x.z + x.w;
        }
        if constexpr (VAR >= 1) part = wsum(part);
        if constexpr (VAR == 4) {
            uint64_t* my = xw + h;
            if (lane == 0) wr64(my, ((uint64_t)(t + 1) << 32) | __float_as_uint(part));
            const uint64_t v = rd64(my);
            z = __uint_as_float((uint32_t)v) * 1e-3f;
        } else {
            const uint32_t tag = (uint32_t)(t + 1);
            uint64_t* slot = xw + (t & 1) * H;
            if (lane == 0) wr64(slot + h, ((uint64_t)tag << 32) | __float_as_uint(part));
            const uint64_t* src = slot + (lane < H ? lane : 0);
            constexpr uint64_t mask = (1ull << H) - 1;
            uint64_t v = rd64(src);
            while ((__ballot((uint32_t)(v >> 32) == tag) & mask) != mask) v = rd64(src);
            const int lo = (int)(uint32_t)v;
            float s = __int_as_float(__builtin_amdgcn_readlane(lo, 0));
#pragma unroll
            for (int g = 1; g < H; ++g) s = s + __int_as_float(__builtin_amdgcn_readlane(lo, g));
            z = s * 1e-3f;
        }
        if constexpr (VAR == 3) {
#pragma unroll
            for (int k = 0; k < 8; ++k) z = __builtin_fmaf(z, 0.999f, 1e-4f);
        }
        acc += z;
    }
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) {
        out[blockIdx.x * H + h] = acc;
        cyc[blockIdx.x * H + h] = c1 - c0;
    }
}

template <int H, int VAR>
double run(int blocks, int rounds) {
    float* out;
    unsigned long long* cyc;
    hipMalloc(&out, blocks * H * sizeof(float));
    hipMalloc(&cyc, blocks * H * 8);
    for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL((xchg<H, VAR>), dim3(blocks), dim3(64 * H), 0, 0, rounds, out, cyc);
    hipDeviceSynchronize();
    std::vector<unsigned long long> h(blocks * H);
    hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost);
    std::sort(h.begin(), h.end());
    hipFree(out);
    hipFree(cyc);
    return (double)h[h.size() / 2] / rounds;
}

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 200000;
    const int blocks = 256;
    printf("cycles per round (median over %d workgroups x waves, %d rounds)\n", blocks, rounds);
    printf("H=4 exchange only          %8.1f\n", run<4, 0>(blocks, rounds));
    printf("H=4 + DPP reduce           %8.1f\n", run<4, 1>(blocks, rounds));
    printf("H=4 + row read + reduce    %8.1f\n", run<4, 2>(blocks, rounds));
    printf("H=4 + read + reduce + 8 op %8.1f\n", run<4, 3>(blocks, rounds));
    printf("H=2 exchange only          %8.1f\n", run<2, 0>(blocks, rounds));
    printf("H=1 exchange only          %8.1f\n", run<1, 0>(blocks, rounds));
    printf("H=4 own write->read only   %8.1f\n", run<4, 4>(blocks, rounds));
    printf("H=4 reduce + own round trip%8.1f\n", run<4, 4>(blocks, rounds));
    return 0;
}
