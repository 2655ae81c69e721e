#!/bin/bash
# each detector variant library swapped in: the detector parity tests, then the batch timing
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cp $R/slam-indoor-code_amd/slamhip/libslamhip.so /tmp/libslamhip_orig.so
for v in "$@"; do
    cp $R/scripts/diag/lib_sift_$v.so $R/slam-indoor-code_amd/slamhip/libslamhip.so || exit 1
    timeout -k 10 300 python -u -m pytest $R/tests -m gpu -q -x -k "sift_detect" --timeout 200 --timeout-method thread \
        > $R/gpurun_out/dvc_$v.log 2>&1
    rc=$?
    echo "$v tests rc=$rc $(tail -1 $R/gpurun_out/dvc_$v.log)"
    [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
    timeout -k 10 200 python3 $R/scripts/diag/det_time.py 2>&1 | tail -1 || exit 1
done
cp /tmp/libslamhip_orig.so $R/slam-indoor-code_amd/slamhip/libslamhip.so
