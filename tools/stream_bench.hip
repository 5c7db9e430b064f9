// stream_bench.hip -- ceilings for the chain kernels' row stream on MI355X (diagnostic tool, not
// part of the product). Every workgroup streams its own contiguous partition of `rows` rows of
// `rowbytes` bytes, the chain kernels' access pattern (one partition per CU):
//   plain    : 4 waves per workgroup, global_load_dwordx4 into registers, rows split over waves
//   plain1   : 1 wave per workgroup, global_load_dwordx4, 8 rows in flight
//   ldsdma   : ring_loader (the chain kernels' loader) + a consumer wave that hands every slot
//              straight back (no compute): the loader/handshake ceiling
// Usage: stream_bench <rows per partition> <partitions> <R ring rows> <D depth> [nv]
#include "../spark-parallelized-sgd_amd/csrc/psgd_device.h"

#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

using namespace psgd;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ __launch_bounds__(256) void plain(const float4* __restrict__ X, int64_t rows_per, int nv,
                                             float* out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const float4* base = X + (int64_t)blockIdx.x * rows_per * nv * 64;
    float4 acc = {0, 0, 0, 0};
    for (int64_t r = wave; r < rows_per; r += 4) {
        for (int v = 0; v < nv; ++v) {
            float4 x = base[(r * nv + v) * 64 + lane];
            acc.x += x.x; acc.y += x.y; acc.z += x.z; acc.w += x.w;
        }
    }
    if (acc.x == 1234.5f) out[0] = acc.y + acc.z + acc.w;
}

__global__ __launch_bounds__(64) void plain1(const float4* __restrict__ X, int64_t rows_per, int nv,
                                             float* out) {
    const int lane = threadIdx.x & 63;
    const float4* base = X + (int64_t)blockIdx.x * rows_per * nv * 64;
    float4 acc = {0, 0, 0, 0};
    const int64_t total = rows_per * nv;
    int64_t i = 0;
    for (; i + 16 <= total; i += 16) {
        float4 x[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) x[k] = base[(i + k) * 64 + lane];
#pragma unroll
        for (int k = 0; k < 16; ++k) { acc.x += x[k].x; acc.y += x[k].y; acc.z += x[k].z; acc.w += x[k].w; }
    }
    if (acc.x == 1234.5f) out[0] = acc.y + acc.z + acc.w;
}


// NW waves per workgroup, each streaming a contiguous share of the partition with U 16-byte
// loads per lane in flight (loads to registers).
template <int NW, int U>
__global__ __launch_bounds__(NW * 64) void regstream(const float4* __restrict__ X, int64_t rows_per,
                                                     int nv, float* out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t total = rows_per * nv;          // 1 KiB pieces in the partition
    const int64_t a = total * wave / NW, b = total * (wave + 1) / NW;
    const float4* base = X + (int64_t)blockIdx.x * total * 64;
    float4 acc = {0, 0, 0, 0};
    int64_t i = a;
    for (; i + U <= b; i += U) {
        float4 x[U];
#pragma unroll
        for (int k = 0; k < U; ++k) x[k] = base[(i + k) * 64 + lane];
#pragma unroll
        for (int k = 0; k < U; ++k) { acc.x += x[k].x; acc.y += x[k].y; acc.z += x[k].z; acc.w += x[k].w; }
    }
    for (; i < b; ++i) { float4 x = base[i * 64 + lane]; acc.x += x.x; }
    if (acc.x == 1234.5f) out[0] = acc.y + acc.z + acc.w;
}

// NW loader waves per workgroup, each LDS-DMAing its contiguous share of the partition into its
// own 32 KiB LDS region (overwritten, no consumer), keeping D pieces (1 KiB each) in flight.
template <int NW, int D>
__global__ __launch_bounds__(NW * 64) void dmaraw(const float4* __restrict__ X, int64_t rows_per, int nv) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t total = rows_per * nv;
    const int64_t a = total * wave / NW, b = total * (wave + 1) / NW;
    const float4* base = X + (int64_t)blockIdx.x * total * 64;
    char* region = smem + wave * 32768;
    int slot = 0;
    for (int64_t i = a; i < b; ++i) {
        __builtin_amdgcn_global_load_lds((const void*)(as_global(base + i * 64 + lane)),
                                         (__attribute__((address_space(3))) void*)(region + slot * 1024), 16, 0, 0);
        slot = (slot + 1) & 31;
        wait_vmcnt_le(D);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// dmaraw with the partitions' rows interleaved in HBM: groups of G rows (nv 1 KiB pieces each)
// round-robin over the P partitions, so at any moment the CUs read neighbouring addresses.
template <int NW, int D>
__global__ __launch_bounds__(NW * 64) void dmaint(const float4* __restrict__ X, int64_t rows_per, int nv, int G) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t P = gridDim.x, gp = (int64_t)G * nv;   // pieces per group
    // whole groups only: piece index ((i / gp) P + p) gp + i % gp stays below P * total
    const int64_t total = rows_per * nv / gp * gp;
    const int64_t a = total * wave / NW, b = total * (wave + 1) / NW;
    char* region = smem + wave * 32768;
    int slot = 0;
    for (int64_t i = a; i < b; ++i) {
        const int64_t piece = ((i / gp) * P + blockIdx.x) * gp + i % gp;
        __builtin_amdgcn_global_load_lds((const void*)(as_global(X + piece * 64 + lane)),
                                         (__attribute__((address_space(3))) void*)(region + slot * 1024), 16, 0, 0);
        slot = (slot + 1) & 31;
        wait_vmcnt_le(D);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int NV>
__global__ __launch_bounds__(128) void ldsdma(ChainLaunch L, RingGeom geom) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    RingHeader* hdr = reinterpret_cast<RingHeader*>(smem);
    char* meta_ring = smem + sizeof(RingHeader);
    char* ring = meta_ring + geom.meta_blocks * kMetaBlockBytes;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const ChainDesc dsc = L.descs[blockIdx.x];
    if (threadIdx.x == 0) { hdr->ready = 0; hdr->consumed = 0; hdr->stop = 0; }
    __syncthreads();
    if (wave == 1) {
        ring_loader<float, NV, true, 8>(L, dsc, hdr, meta_ring, ring, geom, lane);
        return;
    }
    const int64_t n = dsc.n_rows;
    unsigned ready = 0;
    while ((int64_t)ready < n) {
        ready = __hip_atomic_load(&hdr->ready, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_store(&hdr->consumed, ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __builtin_amdgcn_s_sleep(1);
    }
}


// ring_loader variants: PUB = rows per `ready` publish (0: only at the end), DC = compile-time
// depth (0: runtime switch), META = meta DMA on/off, CONS = consult `consumed` (ring flow control).
template <int PUB, int DC, bool META, bool CONS>
__device__ void loader_var(const ChainLaunch& L, const ChainDesc& dsc, RingHeader* hdr, char* meta_ring,
                           char* ring, const RingGeom& geom, int lane) {
    constexpr int NV = 2;
    using V = f32x4;
    constexpr int ROW_BYTES = NV * 1024;
    const int64_t n = dsc.n_rows;
    const int R = geom.rows, MB = geom.meta_blocks;
    const int D = DC ? DC : geom.depth;
    const float* X = reinterpret_cast<const float*>(dsc.x);
    const int64_t ld = dsc.ld;
    const unsigned* msrc = reinterpret_cast<const unsigned*>((lane & 2) ? L.steps : dsc.y) + (lane & 1);
    const int mrow = lane >> 2;
    unsigned consumed = 0;
    int slot = 0, mslot = 0;
    for (int64_t t = 0; t < n; ++t) {
        if (CONS && t >= (int64_t)consumed + R) {
            for (;;) {
                consumed = lds_load_u32_asm(&hdr->consumed);
                if (t < (int64_t)consumed + R) break;
                __builtin_amdgcn_s_sleep(1);
            }
        }
        if (META && (t & (kMetaRows - 1)) == 0) {
            int64_t r = t + mrow;
            if (r >= n) r = n - 1;
            __builtin_amdgcn_global_load_lds((const void*)(as_global(msrc + 2 * r)),
                (__attribute__((address_space(3))) void*)(meta_ring + mslot * kMetaBlockBytes), 4, 0, 0);
            if (++mslot == MB) mslot = 0;
        }
        char* dst = ring + slot * ROW_BYTES;
        const V* row = reinterpret_cast<const V*>(X + t * ld);
#pragma unroll
        for (int v = 0; v < NV; ++v)
            __builtin_amdgcn_global_load_lds((const void*)(as_global(row + v * 64 + lane)),
                                             (__attribute__((address_space(3))) void*)(dst + v * 1024), 16, 0, 0);
        if (++slot == R) slot = 0;
        if (t >= D) {
            if (DC) wait_vmcnt_le(DC * NV); else wait_vmcnt_le(D * NV);
            if (PUB && ((t + 1) % PUB) == 0) lds_store_u32_asm(&hdr->ready, (unsigned)(t - D + 1));
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" : : : "memory");
    lds_store_u32_asm(&hdr->ready, (unsigned)n);
}

template <int PUB, int DC, bool META, bool CONS>
__global__ __launch_bounds__(128) void ldsvar(ChainLaunch L, RingGeom geom) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    RingHeader* hdr = reinterpret_cast<RingHeader*>(smem);
    char* meta_ring = smem + sizeof(RingHeader);
    char* ring = meta_ring + geom.meta_blocks * kMetaBlockBytes;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const ChainDesc dsc = L.descs[blockIdx.x];
    if (threadIdx.x == 0) { hdr->ready = 0; hdr->consumed = 0; hdr->stop = 0; }
    __syncthreads();
    if (wave == 1) {
        loader_var<PUB, DC, META, CONS>(L, dsc, hdr, meta_ring, ring, geom, lane);
        return;
    }
    const int64_t n = dsc.n_rows;
    unsigned ready = 0;
    while ((int64_t)ready < n) {
        ready = __hip_atomic_load(&hdr->ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_store(&hdr->consumed, ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __builtin_amdgcn_s_sleep(8);
    }
}

// the buffer through the virtual memory API: 2 GiB handles at a 2 GiB-aligned range (libpsgd's
// DevBuf::vmm_map for the CSR weight vectors)
static void* vmm_alloc(size_t bytes) {
    const size_t chunk = size_t(2) << 30;
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    const size_t total = (bytes + chunk - 1) / chunk * chunk;
    void* res;
    CK(hipMemAddressReserve(&res, total + chunk, 0, nullptr, 0));
    char* va = (char*)(((uintptr_t)res + chunk - 1) / chunk * chunk);
    for (size_t off = 0; off < total; off += chunk) {
        hipMemGenericAllocationHandle_t h;
        CK(hipMemCreate(&h, chunk, &prop, 0));
        CK(hipMemMap(va + off, chunk, 0, h, 0));
    }
    hipMemAccessDesc acc = {};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    CK(hipMemSetAccess(va, total, &acc, 1));
    return va;
}

int main(int argc, char** argv) {
    const int64_t rows = argc > 1 ? atoll(argv[1]) : 39062;
    const int P = argc > 2 ? atoi(argv[2]) : 256;
    const int R = argc > 3 ? atoi(argv[3]) : 64;
    const int D = argc > 4 ? atoi(argv[4]) : 28;
    const int nv = argc > 5 ? atoi(argv[5]) : 2;  // 1 KiB vectors per row: 2 = d 512 f32 (c2), 4 = c3
    const int64_t rowbytes = nv * 1024;
    const size_t bytes = (size_t)rows * P * rowbytes;
    // [6] GB allocated, written and freed before the stream's buffer (a process that ran another
    // workload first); [7] 1: the stream's buffer from hipExtMallocWithFlags(hipDeviceMallocContiguous),
    // 2: mapped through the virtual memory API (vmm_alloc)
    const double pre_gb = argc > 6 ? atof(argv[6]) : 0.0;
    const int contig = argc > 7 ? atoi(argv[7]) : 0;
    if (pre_gb > 0) {
        void* T;
        const size_t tb = (size_t)(pre_gb * 1e9);
        CK(hipMalloc(&T, tb));
        CK(hipMemset(T, 1, tb));
        CK(hipDeviceSynchronize());
        CK(hipFree(T));
    }
    void* X;
    if (contig == 2) {
        X = vmm_alloc(bytes);
        printf("vmm mapping of %.1f GB at %p\n", bytes / 1e9, X);
    } else if (contig) {
        hipError_t e = hipExtMallocWithFlags(&X, bytes, hipDeviceMallocContiguous);
        printf("contiguous allocation of %.1f GB: %s\n", bytes / 1e9, hipGetErrorString(e));
        if (e != hipSuccess) { (void)hipGetLastError(); CK(hipMalloc(&X, bytes)); }
    } else {
        CK(hipMalloc(&X, bytes));
    }
    CK(hipMemset(X, 0, bytes));
    double* y; double* steps; int* wd; float* out;
    CK(hipMalloc(&y, rows * P * 8)); CK(hipMemset(y, 0, rows * P * 8));
    CK(hipMalloc(&steps, rows * 8)); CK(hipMemset(steps, 0, rows * 8));
    CK(hipMalloc(&wd, 4)); CK(hipMemset(wd, 0, 4));
    CK(hipMalloc(&out, 4));
    ChainDesc* h = (ChainDesc*)calloc(P, sizeof(ChainDesc));
    for (int p = 0; p < P; ++p) {
        h[p].x = (char*)X + (size_t)p * rows * rowbytes;
        h[p].y = y + (size_t)p * rows;
        h[p].n_rows = rows;
        h[p].ld = nv * 256;
    }
    ChainDesc* dd;
    CK(hipMalloc(&dd, P * sizeof(ChainDesc)));
    CK(hipMemcpy(dd, h, P * sizeof(ChainDesc), hipMemcpyHostToDevice));
    ChainLaunch L{};
    L.descs = dd; L.steps = steps; L.watchdog = wd;
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    auto timeit = [&](const char* name, auto launch) {
        launch();
        CK(hipDeviceSynchronize());
        float best = 1e30f;
        for (int it = 0; it < 3; ++it) {
            CK(hipEventRecord(a));
            launch();
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms; CK(hipEventElapsedTime(&ms, a, b));
            if (ms < best) best = ms;
        }
        printf("%-10s %8.3f ms  %8.1f GB/s  (%.1f ns/row/CU)\n", name, best, bytes / best / 1e6,
               best * 1e6 / rows);
        fflush(stdout);
    };
    timeit("plain", [&] { hipLaunchKernelGGL(plain, dim3(P), dim3(256), 0, 0, (const float4*)X, rows, nv, out); });
    timeit("plain1", [&] { hipLaunchKernelGGL(plain1, dim3(P), dim3(64), 0, 0, (const float4*)X, rows, nv, out); });
#define RS(NW, U) timeit("reg" #NW "x" #U, [&] { hipLaunchKernelGGL((regstream<NW, U>), dim3(P), dim3(NW * 64), 0, 0, (const float4*)X, rows, nv, out); });
    RS(1, 32) RS(2, 16) RS(4, 8) RS(4, 16) RS(8, 8) RS(8, 16) RS(16, 4) RS(16, 8)
#define DR(NW, D) CK(hipFuncSetAttribute((const void*)dmaraw<NW, D>, hipFuncAttributeMaxDynamicSharedMemorySize, NW * 32768)); \
    timeit("dma" #NW "x" #D, [&] { hipLaunchKernelGGL((dmaraw<NW, D>), dim3(P), dim3(NW * 64), NW * 32768, 0, (const float4*)X, rows, nv); });
    DR(1, 16) DR(1, 32) DR(1, 56) DR(2, 16) DR(2, 28) DR(2, 56) DR(4, 8) DR(4, 14) DR(4, 28)
    // host check of the interleaved kernel's largest piece index (whole groups of G rows only)
    for (int G : {1, 8, 64, 512}) {
        const int64_t gp = (int64_t)G * nv, tot = rows * nv / gp * gp;
        const int64_t maxp = (((tot - 1) / gp) * P + (P - 1)) * gp + (tot - 1) % gp;
        if (tot <= 0 || maxp >= (int64_t)rows * nv * P) { fprintf(stderr, "dmaint bounds G=%d\n", G); return 1; }
    }
#define DI(NW, D, G) CK(hipFuncSetAttribute((const void*)dmaint<NW, D>, hipFuncAttributeMaxDynamicSharedMemorySize, NW * 32768)); \
    timeit("int" #NW "x" #D "g" #G, [&] { hipLaunchKernelGGL((dmaint<NW, D>), dim3(P), dim3(NW * 64), NW * 32768, 0, (const float4*)X, rows, nv, G); });
    DI(1, 56, 8) DI(2, 28, 8) DI(4, 14, 8) DI(2, 28, 1) DI(2, 28, 64) DI(2, 28, 512)
    DR(2, 28) DR(4, 14)
    if (nv != 2) return 0;   // the ring-loader variants below are NV = 2 instances
    // (and they need a ring deeper than their depth plus two groups: a shallower ring with the
    // consumed check can wait forever -- R = 32 with D = 28 hung, r05)
    if (R < D + 16) return 0;
    const int MB = (R + kMetaRows - 1) / kMetaRows + 2;
    RingGeom g{R, MB, D, 0};
    const size_t lds = sizeof(RingHeader) + (size_t)MB * kMetaBlockBytes + (size_t)R * rowbytes;
    CK(hipFuncSetAttribute((const void*)ldsdma<2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    timeit("ldsdma", [&] { hipLaunchKernelGGL(ldsdma<2>, dim3(P), dim3(128), lds, 0, L, g); });
#define LV(PUB, DC, META, CONS) CK(hipFuncSetAttribute((const void*)ldsvar<PUB, DC, META, CONS>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); \
    timeit("v" #PUB "_" #DC "_" #META "_" #CONS, [&] { hipLaunchKernelGGL((ldsvar<PUB, DC, META, CONS>), dim3(P), dim3(128), lds, 0, L, g); });
    LV(1, 0, true, true) LV(1, 28, true, true) LV(8, 28, true, true) LV(0, 28, true, false)
    LV(0, 28, false, false) LV(8, 28, false, true) LV(1, 28, false, false) LV(8, 28, true, false)
    int w = 0;
    CK(hipMemcpy(&w, wd, 4, hipMemcpyDeviceToHost));
    printf("watchdog=%d R=%d D=%d lds=%zu\n", w, R, D, lds);
    return 0;
}
