#!/bin/bash
# Build a variant of libslamhip with sift_band.hip compiled under extra -D flags:
#   scripts/diag/build_sift_variant.sh NAME -DSIFT_BAND_PAIR2=1 ...
# -> scripts/diag/lib_sift_NAME.so (the other objects from the in-tree build)
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
N=$1; shift
P=$R/slam-indoor-code_amd
make -s -C $P
O=/tmp/sv_build_$N
mkdir -p $O
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -munsafe-fp-atomics -Wall \
    -Wno-unused-function -I$R/include "$@" -x hip -c $P/csrc/sift_band.hip -o $O/sift_band.hip.o
objs=$(ls $P/build/*.o | grep -v sift_band.hip.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $R/scripts/diag/lib_sift_$N.so $objs $O/sift_band.hip.o
echo built scripts/diag/lib_sift_$N.so
