#!/bin/bash
# Device ISA of one kernel instance, without the dispatch over every instantiation (seconds
# instead of minutes): tools/isa_probe.sh FILE.hip 'template-instance' OUT.s ['kernel params']
#   e.g. tools/isa_probe.sh psgd_sparse_lds.hip 'chain_sparse_lds<float, float, 2, 0, 4, true>' /tmp/c4.s
#        tools/isa_probe.sh psgd_split.hip 'chain_split<float, float, 0, 3, false, 4, true, 4>' /tmp/s.s \
#            'ChainLaunch, KParams, RingGeom'
set -e
SRC=$1; INST=$2; OUT=$3; PARAMS=${4:-ChainLaunch, KParams, int}
D=$(cd "$(dirname "$0")/../spark-parallelized-sgd_amd/csrc" && pwd)
T=$(mktemp /tmp/isa_probeXXXX.hip)
cat > $T <<EOT
#define PSGD_NO_DISPATCH
#include "$D/$SRC"
namespace psgd { template __global__ void $INST($PARAMS); }
EOT
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off --cuda-device-only -S -I$D -o $OUT $T
rm -f $T
