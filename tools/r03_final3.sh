#!/bin/bash
# Close-out after the 32-bit bookkeeping changes: the GPU suite, smoke, the default bench line,
# and fresh profiles of the lines whose kernels changed (c4, the chain_split lines).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/r03_check.sh > gpurun_out/r03_final3_check.log 2>&1 || exit 1
bash tools/profile_r03.sh c4_f32 c4_f64 c3_f32_adagrad c3_f32_adam c3_f64_adagrad c3_f64_adam > gpurun_out/r03_final3_prof.log 2>&1
