#!/bin/bash
# Round-3 close-out on one box: the GPU suite, smoke and the default bench line (what the driver
# runs), then the rocprofv3 kernel traces + PMC passes of every bench line (tools/profile_r03.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/r03_check.sh > gpurun_out/r03_final_check.log 2>&1 || exit 1
bash tools/profile_r03.sh c2 c2_f64 c3_f32 c3_f64 c3_f64rows c4_f32 c4_f64 c5 c3_f32_adagrad c3_f32_adam c3_f64_adagrad c3_f64_adam c1 > gpurun_out/r03_final_prof.log 2>&1
