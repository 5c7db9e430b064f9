#!/bin/bash
# Final close-out: the GPU suite, smoke, the default bench line, and fresh profiles of the
# chain_split lines (their kernel names carry the CONV parameter since the per-sample break).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/r03_check.sh > gpurun_out/r03_final2_check.log 2>&1 || exit 1
bash tools/profile_r03.sh c3_f32_adagrad c3_f32_adam c3_f64_adagrad c3_f64_adam > gpurun_out/r03_final2_prof.log 2>&1
