// psgd_split.h -- launcher of the feature-split per-sample chain (psgd_split.hip), called by the
// dispatcher in psgd_kernels.hip. Not part of the public ABI (include/psgd.h is).
#pragma once
#include "psgd_internal.h"

namespace psgd {

// Dense rows, rows of 2 .. 8 KiB (f32 rows: d <= 2,048; f64 rows: d <= 1,024), fp32 or fp64
// compute: AdaGrad / Adam / L1 (SGDUpdater.scala:120-148, :193-286) with or without the
// per-sample convergence test, Simple / SquaredL2 only with it (tol > 0; without it the 8-row
// Gram-block kernels are faster).
bool split_path_applies(int layout, int updater, bool check_conv, int storage, int64_t max_ld);
// Kernel variant 800 + 10 H + NV (H compute waves, NV 1-KiB row vectors). -3 when it does not apply.
int launch_split_chains(const ChainLaunch& L, const KParams& kp, int storage, int compute, int gradient,
                        int updater, int64_t min_ld, int64_t max_ld, int lds_spread, hipStream_t stream,
                        int* kernel_variant);

}  // namespace psgd
