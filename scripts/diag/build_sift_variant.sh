#!/bin/bash
# Build a variant of libslamhip with one source (env SRC, default sift_band.hip)
# compiled under extra -D flags:
#   scripts/diag/build_sift_variant.sh NAME -DSIFT_BAND_TPREF=0 ...
#   SRC=knn.hip scripts/diag/build_sift_variant.sh knn_q4m2 -DKNN_QT=4 -DKNN_MINB=2
# -> scripts/diag/lib_sift_NAME.so (the other objects from the in-tree build)
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
N=$1; shift
SRC=${SRC:-sift_band.hip}
P=$R/slam-indoor-code_amd
make -s -C $P
O=/tmp/sv_build_$N
mkdir -p $O
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -munsafe-fp-atomics -Wall \
    -Wno-unused-function -I$R/include "$@" -x hip -c $P/csrc/$SRC -o $O/$SRC.o
objs=$(ls $P/build/*.o | grep -v "/$SRC.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $R/scripts/diag/lib_sift_$N.so $objs $O/$SRC.o
echo built scripts/diag/lib_sift_$N.so
