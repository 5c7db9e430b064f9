// psgd_internal.h -- structures shared by the C-ABI layer (psgd_capi.cpp) and the HIP kernels
// (psgd_kernels.hip). Not part of the public ABI (include/psgd.h is).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace psgd {

// One chain = one registered partition (its RDD partition index is its chain id, PSGD.scala:243).
struct ChainDesc {
    const void* x;           // dense rows (storage dtype) or CSR values
    const double* y;         // labels[n_rows]
    const int64_t* row_ptr;  // CSR: absolute offsets into col/x, [n_rows+1]; null for dense
    const int32_t* col;      // CSR column indices
    int64_t n_rows;
    int64_t ld;              // dense: leading dimension in elements (>= d, multiple of 16B/elt)
    const int32_t* rows;     // sampled epoch: the chain's t-th sample is partition row rows[t]
                             // (y is then the sampled rows' labels); null: row t
};

// Per-launch scalars (hyper-parameters of ParallelizedSGD, PSGD.scala:46-50).
struct KParams {
    double reg;
    double tol;
    double beta, gamma, eps;  // AdamSGDUpdater (UPD.scala:241-244)
    int32_t d;                // features per row
    int32_t n_chains;
    int32_t nc = 0;           // multinomial LogisticGradient: K - 1 weight blocks of d; 0: binary
    // SquaredL2's alpha-scaled CSR form without renormalisation is valid for this epoch: every
    // prefix product of (1 - s_j lambda), j <= the longest chain, is finite, non-zero and within
    // [2^-400, 2^400] (set by the host; chain_sparse_lds in fp64 runs only then)
    int32_t alpha_ok = 0;
    // the longest chain of the epoch (before sampling): kernels that count rows in 32 bits apply
    // only while it is <= INT32_MAX
    int64_t n_max = 0;
};

// LogisticGradient(numClasses = K): at most this many weight blocks (K - 1), the chain keeps
// the K-1 margins and multipliers in LDS (16 bytes a class).
constexpr int kMultinomialMaxBlocks = 4096;

enum Layout { kDense = 0, kCsr = 1 };
enum WeightsIn { kWeightsOut = 0, kWeightsF32 = 1, kWeightsF64 = 2 };

// Everything a chain launch needs (device pointers).
struct ChainLaunch {
    const ChainDesc* descs;  // [n_chains]
    const double* w_in;      // [d]
    double* w_out;           // [n_chains * d]   per-chain final weights (also the general
                             //                  kernel's working copy)
    double* state;           // [n_chains * 2 * d] AdaGrad/Adam status (general kernel) or null
    double* rv;              // [n_chains]  localRegVal
    double* loss;            // [n_chains]  localLossSum
    double* cnt_d;           // [n_chains]  count as double (exact < 2^53) for the fold
    int64_t* cnt;            // [n_chains]  count
    const double* steps;     // [n_max] stepSize / sqrt(j), j = 1..n_max
    int* watchdog;           // set by a wave whose partner stopped making progress
    unsigned long long* stamps;  // per-wave cycle counters, diagnostic builds only (PSGD_STAMPS)
    float* zbuf;             // [n_chains * zstride] per-row margins (fp32 Logistic block kernel)
    double* zbuf64;          // [n_chains * zstride] per-row dots (fp64 Logistic chain_dense)
    int64_t zstride;
    float* wf32;             // [n_chains * wstride] fp32 working weights (CSR fp32 kernel)
    int64_t wstride;
    // CSR fp32 kernels: the chain's weights are w = walpha[chain] * wf32[chain] (SquaredL2's
    // alpha-scaled form; 1 otherwise), folded straight from wf32 (launch_fold_f32); wnsq0 =
    // ||float(w_in)||^2, the start of the chain's incrementally tracked ||v||^2.
    double* walpha;          // [n_chains]
    double* wnsq0;           // [1]
};

// Diagnostic builds (-DPSGD_STAMPS, tools/chain_bench.hip) count s_memtime cycles per wave.
#ifdef PSGD_STAMPS
#define PSGD_STAMP(...) __VA_ARGS__
#else
#define PSGD_STAMP(...)
#endif

// Host-side launchers implemented in psgd_kernels.hip. Return hipError_t as int.
// storage: 0 = f64, 1 = f32; compute: 0 = f64, 1 = f32.
// Kernel variants (*kernel_variant, psgd_ctx_last_kernel): 100 + NV chain_dense, 200 + LAYOUT
// chain_general, 300 + NV chain_block, 400 + storage chain_sparse, 410 + storage chain_sparse_spec,
// 420 + storage chain_sparse64, 500 + LAYOUT chain_multinomial, 600 + 10 (SK 8) + 20 (fp64) + storage chain_sparse_lds,
// 700 + 10 (H - 1) + NV chain_block64, 800 + 10 H + NV chain_split.
// *weights_in (nullable): where the launch left each chain's weights -- kWeightsOut: L.w_out
// (launch_fold); kWeightsF32: L.wf32 as floats, w = walpha v (the fp32 CSR kernels,
// launch_fold_f32); kWeightsF64: L.wf32 as doubles, w = walpha v (chain_sparse64, launch_fold_f64).
int launch_chains(const ChainLaunch& L, const KParams& kp, int layout, int storage, int compute,
                  int gradient, int updater, bool check_conv, int64_t min_ld, int64_t max_ld,
                  int lds_spread, hipStream_t stream, int* kernel_variant, int64_t max_nnz = 0,
                  int* weights_in = nullptr);
// The blocked fp32 kernel (psgd_block.hip): dense rows, Simple/SquaredL2, no per-sample
// convergence test. launch_block_chains returns -3 when it does not apply.
bool block_path_applies(int layout, int compute, int updater, bool check_conv, int storage,
                        int64_t max_ld);
int launch_block_chains(const ChainLaunch& L, const KParams& kp, int storage, int gradient,
                        int updater, int64_t min_ld, int64_t max_ld, int lds_spread,
                        hipStream_t stream, int* kernel_variant);
// The blocked fp64 kernel (psgd_block64.hip): dense rows, Simple/SquaredL2, fp64 compute, no
// per-sample convergence test (the parity mode's throughput kernel). -3 when it does not apply.
bool block64_path_applies(int layout, int compute, int updater, bool check_conv, int storage,
                          int64_t max_ld);
int launch_block64_chains(const ChainLaunch& L, const KParams& kp, int storage, int gradient,
                          int updater, int64_t min_ld, int64_t max_ld, int lds_spread,
                          hipStream_t stream, int* kernel_variant);
// lossSum of fp64 Logistic chains from the per-row dots in L.zbuf64 (psgd_kernels.hip).
int launch_logistic_loss64(const ChainLaunch& L, int n_chains, hipStream_t stream);
// lossSum of fp32 Logistic chains from the per-row margins in L.zbuf (psgd_block.hip).
int launch_margin_loss(const ChainLaunch& L, int n_chains, hipStream_t stream);
// The fold kernels read the epoch's watchdog flags (a set flag poisons the count) and clear them
// for the next epoch; mirror (nullable, device-visible page-locked host memory) also receives
// {regVal, lossSum, count}.
int launch_fold(const double* w, int64_t w_stride, const double* rv, const double* loss,
                const double* cnt, int64_t s_stride, int n, int d, double* out,
                int* watchdog, hipStream_t stream, double* mirror = nullptr);
// The combiner over the CSR fp32 kernels' outputs: w_p = walpha[p] * double(wf32[p][i]).
int launch_fold_f32(const float* wf32, int64_t wstride, const double* walpha, const double* rv,
                    const double* loss, const double* cnt, int n, int d, double* out,
                    int* watchdog, hipStream_t stream, double* mirror = nullptr);
int launch_sq_terms(const double* a, const double* b, int d, double* out2, hipStream_t stream);
int launch_steps(double step, int64_t n, double* steps, hipStream_t stream);
// The fp32 CSR kernel (psgd_sparse.hip): weights as fp32 vectors in HBM (L.wf32).
bool sparse_path_applies(int layout, int compute, int updater, bool check_conv);
int launch_sparse_chains(const ChainLaunch& L, const KParams& kp, int storage, int gradient,
                         int updater, int64_t max_nnz, hipStream_t stream, int* kernel_variant);
// *L.wnsq0 = ||w_in||^2 in f64 (round_f32: of float(w_in), the fp32 kernels' weights).
int launch_wnsq0(const ChainLaunch& L, int d, bool round_f32, hipStream_t st);
// The fp64 CSR chain with HBM-resident weights (psgd_sparse.hip, chain_sparse64): Simple, and
// SquaredL2 when kp.alpha_ok; the chain's double vector lives in its slice of L.wf32 (>= 2 (d +
// 1152) floats), its alpha in L.walpha; weights end there (w = walpha v, launch_fold_f64).
bool sparse64_path_applies(int layout, int compute, int updater, bool check_conv, bool alpha_ok);
// PSGD_PER_SAMPLE=1 (tests, A/B): launch_chains keeps the per-sample kernels
bool per_sample_forced();
int launch_sparse64_chains(const ChainLaunch& L, const KParams& kp, int storage, int gradient,
                           int updater, hipStream_t stream, int* kernel_variant);
// The combiner over chain_sparse64's vectors: w_p = walpha[p] * v_p[i] (v_p doubles).
int launch_fold_f64(const double* wv, int64_t wstride_d, const double* walpha, const double* rv,
                    const double* loss, const double* cnt, int n, int d, double* out,
                    int* watchdog, hipStream_t stream, double* mirror = nullptr);
// The fp32 CSR kernel with LDS-resident weights (psgd_sparse_lds.hip): rows of <= 128 non-zeros,
// features [0, K) in LDS and [K, d) in L.wf32; -3 when it does not apply.
bool sparse_lds_applies(int64_t d, int64_t max_nnz, int64_t n_max);
int64_t sparse_lds_head(int64_t d);
int launch_sparse_lds_chains(const ChainLaunch& L, const KParams& kp, int storage, int gradient,
                             int updater, int64_t max_nnz, hipStream_t stream, int* kernel_variant);
// The same kernel in fp64 compute (the parity mode's CSR throughput kernel): Simple, and
// SquaredL2 when kp.alpha_ok; the chain's f64 vector lives in its slice of L.wf32, which must be
// >= 2 (d + 1152) floats; weights end in L.w_out. -3 when it does not apply.
bool sparse_lds64_applies(int64_t d, int64_t max_nnz, int updater, bool check_conv, bool alpha_ok,
                          int64_t n_max);
int launch_sparse_lds64_chains(const ChainLaunch& L, const KParams& kp, int storage, int gradient,
                               int updater, int64_t max_nnz, hipStream_t stream, int* kernel_variant);
// Longest row of a device-resident CSR partition (synchronises `st`).
// Placement probe of the CSR chains' weight vectors (psgd_probe.hip): n_vectors waves, each
// `iters` random 4-byte read-modify-writes per lane over its vector's first d_words words.
int launch_vector_probe(float* w, int64_t stride_words, int n_vectors, int d_words, int iters, unsigned seed,
                        hipStream_t st);
int csr_max_nnz(const int64_t* d_row_ptr, int64_t n, int64_t* out, hipStream_t st);
// RDD.sample(false, fraction, seed) per partition (PSGD.scala:242): from the registered
// descriptors `base`, the epoch's descriptors `out` (rows/y/n_rows of the sampled subsequence;
// rows and labels in `rows`/`ys`, `stride` entries per chain). xs_state[c] is the chain's
// XORShiftRandom state (hashSeed of its partition seed, computed by the host).
// The multinomial LogisticGradient chain (psgd_multinomial.hip): fp64 compute, any updater,
// dense or CSR rows. L.w_out holds n_chains * nc * d doubles, L.state 3 * nc * d per chain.
int launch_multinomial_chains(const ChainLaunch& L, const KParams& kp, int layout, int storage, int updater,
                              bool check_conv, hipStream_t stream, int* kernel_variant);

int launch_sample(const ChainDesc* base, ChainDesc* out, const uint64_t* xs_state, double fraction,
                  int32_t* rows, double* ys, int64_t stride, int n_chains, hipStream_t stream);

}  // namespace psgd
