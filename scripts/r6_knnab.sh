#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
LIB=$R/slam-indoor-code_amd/slamhip/libslamhip.so
cp $LIB /tmp/lib_base.so
for v in ${VARS:-k512_2_64 k512_2_128}; do
    cp $R/scripts/diag/lib_sift_$v.so $LIB
    timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_parity.py -q -x -k "knn or match or batch_pipeline or 4k" --timeout 200 --timeout-method thread -p no:cacheprovider > $R/gpurun_out/knnab_$v.log 2>&1
    rc=$?; echo "$v tests rc=$rc $(tail -1 $R/gpurun_out/knnab_$v.log)"
    [ $rc -eq 0 ] || { cp /tmp/lib_base.so $LIB; exit 1; }
done
cp /tmp/lib_base.so $LIB
BATCHES="210 27" bash $R/scripts/r6_kab.sh ${TAG:-r6knn} base:A=1 $(for v in ${VARS:-k512_2_64 k512_2_128}; do echo -n "$v:A=1 "; done)
